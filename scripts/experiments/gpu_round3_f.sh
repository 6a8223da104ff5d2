# pointer-attribute cost + ping-pong floor, then resident encoder tests and the legacy sweep
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 ./quic-test_amd/lib/probe_pingpong 5000 > gpurun_out/pingpong2.jsonl 2>&1 || exit 1
head -4 gpurun_out/pingpong2.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py tests/test_host_mirror.py tests/test_gpu_parity.py -k "legacy or coalesce or resident or mirror or context" -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_coalesce.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_coalesce.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash scripts/legacy_sweep.sh > gpurun_out/legacy_f.jsonl 2> gpurun_out/legacy_f.err
rc=$?; python3 -c "
import json
for l in open('gpurun_out/legacy_f.jsonl'):
    d=json.loads(l)
    if d.get('mode')!='legacy': print(l.strip()); continue
    print(d['streams'], d['rate_pps'], 'coal',d['coalesce'],'res',d['resident'], int(d['groups_per_s']), d['delay_us']['p50'], d['delay_us']['p99'], d['cpu_us_per_group'])
"; exit $rc
timeout -k 10 900 bash scripts/ab_decode_api.sh > /dev/null || exit 1
