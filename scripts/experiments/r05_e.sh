#!/usr/bin/env bash
# Round 5, part E: (1) where the shared-launch path's first call goes (coalescer creation
# stamps); (2) VERDICT r04 item 7: the C4 mix (24 GB read + 6 GB written) by LDS-DMA vs register
# loads (probe_glds); (3) the C5 tile recover's store policy on one more box (probe_runs);
# (4) the --gpus 2 rehearsal (two gloo ranks on the card) at the driver's default sizes, with
# the line's wall_s phases (the N = 8 budget).
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05e}"
mkdir -p "$E"
cd "$ROOT"
for i in 1 2; do
  QUICFEC_RESIDENT=0 QUICFEC_COALESCE_STAMPS=1 timeout -k 10 120 ./quic-test_amd/lib/batcher_latency legacy_raw 5000 > "$E/legacy_coalescer_$i.json" 2> "$E/legacy_coalescer_$i.err"
  grep coalescer_create "$E/legacy_coalescer_$i.err" || true
  python -c "import json,sys; d=json.loads(open('$E/legacy_coalescer_$i.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('max_at_call','first_call_us','max_after_first_us','delay_us')})"
done
timeout -k 10 300 ./quic-test_amd/lib/probe_glds 24000000000 > "$E/probe_glds_c4.txt" 2>&1
cat "$E/probe_glds_c4.txt"
timeout -k 10 300 ./quic-test_amd/lib/probe_runs 1000000 9 0.01 > "$E/probe_runs_c5.txt" 2>&1
tail -14 "$E/probe_runs_c5.txt"
QUICFEC_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 > "$E/bench_gpus2_gloo_rehearsal.json" 2> "$E/bench_gpus2.err"
python -c "import json; d=json.loads(open('$E/bench_gpus2_gloo_rehearsal.json').read().strip().splitlines()[-1]); print('gpus2', d['n_gpus'], d['value'], d['verified'], d.get('wall_s'), {s: (d[s]['ranks'], d[s]['value'], d[s]['verified']) for s in ('c4', 'c5_e2e')}, d['c5_e2e']['e2e_pinned'].get('decode_GiBps'))"
