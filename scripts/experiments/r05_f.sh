#!/usr/bin/env bash
# Round 5, part F: the shared-launch path after dropping the coalescer's own context and stream
# (VERDICT r04 item 8): the coalesce GPU tests, legacy_raw on the coalescer path plain and under
# rocprofv3 (its slowest call against p99), and the exit-path programs.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05f}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py tests/test_gpu_batcher.py tests/test_host_mirror.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/coalesce.log" 2>&1 || { tail -60 "$E/coalesce.log"; exit 1; }
tail -1 "$E/coalesce.log"
for i in 1 2; do
  QUICFEC_RESIDENT=0 QUICFEC_COALESCE_STAMPS=1 timeout -k 10 120 ./quic-test_amd/lib/batcher_latency legacy_raw 5000 > "$E/legacy_coalescer_$i.json" 2> "$E/legacy_coalescer_$i.err"
  grep coalescer_create "$E/legacy_coalescer_$i.err" || true
  python -c "import json,sys; d=json.loads(open('$E/legacy_coalescer_$i.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('max_at_call','first_call_us','max_after_first_us','delay_us','errors')})"
done
QUICFEC_RESIDENT=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$E/prof_legacy_coalescer" -o run --output-format csv -- \
  ./quic-test_amd/lib/batcher_latency legacy_raw 5000 > "$E/prof_legacy_coalescer.json" 2> "$E/prof_legacy_coalescer.err"
python -c "import json,sys; d=json.loads(open('$E/prof_legacy_coalescer.json').read().strip().splitlines()[-1]); print('rocprof', {k: d[k] for k in ('max_at_call','first_call_us','max_after_first_us','delay_us','errors')})"
for m in coalescer pageable; do
  timeout -k 10 120 ./quic-test_amd/lib/exit_path_test $m 300 > "$E/exit_$m.json"
  tail -1 "$E/exit_$m.json"
done
for s in 16; do
  QUICFEC_RESIDENT=0 timeout -k 10 120 ./quic-test_amd/lib/batcher_latency legacy $s 2 > "$E/legacy_coalescer_s$s.json" 2>&1 || true
  tail -1 "$E/legacy_coalescer_s$s.json"
done
