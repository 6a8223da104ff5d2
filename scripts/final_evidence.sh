set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -2 gpurun_out/smoke.log
CFGS="c2c3 c5 c4 c4d" bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1
tail -1 gpurun_out/pmc.log
# the bench below reads profiles/pmc_<config>.json; these were measured on this very build
for c in c2c3 c5 c4 c4d; do cp gpurun_out/pmc_$c.json profiles/pmc_$c.json; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['roofline'], d['cpu_baseline']['value'])"
