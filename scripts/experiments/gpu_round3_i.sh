# full GPU suite, smoke, legacy sweep, decode-API A/B, default bench
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 bash scripts/legacy_sweep.sh > gpurun_out/legacy_i.jsonl 2> gpurun_out/legacy_i.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/legacy_i.jsonl'):
    d=json.loads(l)
    if d.get('mode')=='cpu_one_core': print(l.strip()[:150]); continue
    if d.get('mode')=='legacy_raw': print('raw', d['coalesce'], d['resident'], d['delay_us']['p50'], d['delay_us']['p99'], d['errors']); continue
    print(d['streams'], d['rate_pps'], 'coal',d['coalesce'],'res',d['resident'], int(d['groups_per_s']), d['delay_us']['p50'], d['delay_us']['p99'], d['cpu_us_per_group'], d['errors'])
"
timeout -k 10 900 bash scripts/ab_decode_api.sh > /dev/null || exit 1
python3 -c "
import json
for l in open('gpurun_out/ab_decode_api.jsonl'): d=json.loads(l); print(d['config'], d['api'], d['rep'], d['value'], d['decode_ms_in_step'], d['decode_ms_isolated'], d['other_api'])
"
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
cut -c1-600 gpurun_out/bench.json
