#!/usr/bin/env bash
# Round 5, part G: the first shared-launch call's phases (coalescer creation, first batches'
# close / launch / done) on the coalescer path.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05g}"
mkdir -p "$E"
cd "$ROOT"
for i in 1 2; do
  QUICFEC_RESIDENT=0 QUICFEC_COALESCE_STAMPS=1 timeout -k 10 120 ./quic-test_amd/lib/batcher_latency legacy_raw 5000 > "$E/legacy_coalescer_$i.json" 2> "$E/legacy_coalescer_$i.err"
  grep coalescer_ "$E/legacy_coalescer_$i.err" || true
  python -c "import json,sys; d=json.loads(open('$E/legacy_coalescer_$i.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('max_at_call','first_call_us','max_after_first_us','delay_us','errors')})"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/coalesce.log" 2>&1 || { tail -60 "$E/coalesce.log"; exit 1; }
tail -1 "$E/coalesce.log"
QUICFEC_RESIDENT=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$E/prof_legacy_coalescer" -o run --output-format csv -- \
  ./quic-test_amd/lib/batcher_latency legacy_raw 5000 > "$E/prof_legacy_coalescer.json" 2> "$E/prof_legacy_coalescer.err"
python -c "import json,sys; d=json.loads(open('$E/prof_legacy_coalescer.json').read().strip().splitlines()[-1]); print('rocprof', {k: d[k] for k in ('max_at_call','first_call_us','max_after_first_us','delay_us','errors')})"
QUICFEC_RESIDENT=0 timeout -k 10 120 ./quic-test_amd/lib/batcher_latency legacy 16 0 2 > "$E/legacy_coalescer_s16.json" 2>&1
tail -1 "$E/legacy_coalescer_s16.json" | cut -c1-400
