#!/usr/bin/env bash
# Round 4, evidence part B (one gpurun call): PMC traffic per config on this build (recorded with
# its workload; copied into profiles/ so the benches below read this build's bytes), rocprofv3
# kernel statistics of the default bench, the default bench line, the other configs' legs, and
# the --gpus 2 rehearsal (two gloo ranks sharing the card) carrying the C4 and C5 sections.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r04}"
mkdir -p "$E"
cd "$ROOT"
CFGS="${PMC_CFGS:-c2c3 c5 c4}" bash scripts/gpu_pmc.sh > "$E/pmc.log" 2>&1
for c in ${PMC_CFGS:-c2c3 c5 c4}; do cp "$ROOT/gpurun_out/pmc_$c.json" "$ROOT/profiles/pmc_$c.json"; cp "$ROOT/gpurun_out/pmc_$c.json" "$E/pmc_$c.json"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$E/prof" -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$E/prof_bench.json" 2> "$E/prof_bench.err"
find "$E/prof" -name "*kernel_stats.csv" -exec cp {} "$E/kernel_stats.csv" \;
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$E/bench.json" 2> "$E/bench.err"
python -c "import json; d=json.loads(open('$E/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
mkdir -p "$E/legs"
T="timeout -k 10 300"
$T python bench.py --config c4 --no-cpu-baseline > "$E/legs/c4.json" 2> /dev/null
$T python bench.py --config c5 --e2e --no-cpu-baseline > "$E/legs/c5_satellite.json" 2> /dev/null
for f in "$E"/legs/*.json; do
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); k=d['kernels']; print('$f'.split('/')[-1], d['value'], d['verified'], {n: (v['ms'], v['achieved_GBps']) for n, v in k.items()}, d['roofline']['frac'], d['roofline']['traffic'])"
done
QUICFEC_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 2 --groups 500000 --leg-groups 500000 > "$E/bench_gpus2_gloo_rehearsal.json" 2> "$E/bench_gpus2.err"
python -c "import json; d=json.loads(open('$E/bench_gpus2_gloo_rehearsal.json').read().strip().splitlines()[-1]); print('gpus2', d['n_gpus'], d['value'], d['verified'], {s: (d[s]['ranks'], d[s]['value'], d[s]['verified']) for s in ('c4', 'c5_e2e')}, d['c5_e2e']['e2e_pinned'].get('decode_GiBps'))"
