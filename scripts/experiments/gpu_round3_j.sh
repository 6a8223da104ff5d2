# decode-API A/B (another box), PMC per API for every config, kernel trace, default bench, extra legs
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ab_decode_api.jsonl
timeout -k 10 900 bash scripts/ab_decode_api.sh > /dev/null || exit 1
python3 -c "
import json
for l in open('gpurun_out/ab_decode_api.jsonl'): d=json.loads(l); print(d['config'], d['api'], d['rep'], d['value'], d['decode_ms_in_step'], d['decode_ms_isolated'], d['other_api'])
"
CFGS="c2c3 c5 c4 c4d" timeout -k 10 1200 bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail gpurun_out/pmc.log; exit 1; }
for c in c2c3 c5 c4 c4d; do cp gpurun_out/pmc_$c.json profiles/pmc_$c.json; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit 1
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -3 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['roofline'])"
timeout -k 10 900 bash scripts/extra_legs.sh || exit 1
