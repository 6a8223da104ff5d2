#!/usr/bin/env bash
# Round-end evidence on the current build, in one gpurun call: GPU suite, smoke, PMC traffic
# per config (copied into profiles/ so the bench below reads this build's bytes), rocprofv3
# kernel statistics of the default bench, the default bench line, and the extra legs.
# Everything lands in gpurun_out/${EVID:-final}/.  Any failure ends the script.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-final}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/pytest_gpu.log" 2>&1
tail -1 "$E/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$E/smoke.log" 2>&1
tail -1 "$E/smoke.log"
CFGS="c2c3 c5 c4 c4d" bash scripts/gpu_pmc.sh > "$E/pmc.log" 2>&1
for c in c2c3 c5 c4 c4d; do cp "$ROOT/gpurun_out/pmc_$c.json" "$ROOT/profiles/pmc_$c.json"; cp "$ROOT/gpurun_out/pmc_$c.json" "$E/pmc_$c.json"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$E/prof" -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$E/prof_bench.json" 2> "$E/prof_bench.err"
find "$E/prof" -name "*kernel_stats.csv" -exec cp {} "$E/kernel_stats.csv" \;
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$E/bench.json" 2> "$E/bench.err"
python -c "import json; d=json.loads(open('$E/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
mkdir -p "$E/legs"
T="timeout -k 10 300"
$T python bench.py --config c4 --no-cpu-baseline > "$E/legs/c4.json" 2> /dev/null
$T python bench.py --config c4d --no-cpu-baseline > "$E/legs/c4d.json" 2> /dev/null
$T python bench.py --config c5 --no-cpu-baseline > "$E/legs/c5_satellite.json" 2> /dev/null
$T python bench.py --config c5 --loss 0.05 --no-cpu-baseline > "$E/legs/c5_mobile.json" 2> /dev/null
$T python bench.py --config c2c3 --shape 10,1,1200 --no-cpu-baseline > "$E/legs/k10r1.json" 2> /dev/null
for f in "$E"/legs/*.json; do
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); k=d['kernels']; print('$f'.split('/')[-1], d['value'], d['verified'], {n: (v['ms'], v['achieved_GBps']) for n, v in k.items()}, d['roofline']['frac'], d['roofline']['traffic'])"
done
