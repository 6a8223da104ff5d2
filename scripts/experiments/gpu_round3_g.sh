set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=./quic-test_amd/lib/batcher_latency
QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy_raw 20000 > gpurun_out/stamps_raw.json 2> gpurun_out/stamps_raw.err || exit 1
cut -c1-330 gpurun_out/stamps_raw.json; grep resident_stamps gpurun_out/stamps_raw.err
QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy 16 0 2 > gpurun_out/stamps_16.json 2> gpurun_out/stamps_16.err || exit 1
cut -c1-200 gpurun_out/stamps_16.json; grep resident_stamps gpurun_out/stamps_16.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py tests/test_host_mirror.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_coalesce.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_coalesce.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash scripts/legacy_sweep.sh > gpurun_out/legacy_g.jsonl 2> gpurun_out/legacy_g.err
rc=$?; python3 -c "
import json
for l in open('gpurun_out/legacy_g.jsonl'):
    d=json.loads(l)
    if d.get('mode')=='cpu_one_core': print(l.strip()[:150]); continue
    if d.get('mode')=='legacy_raw': print('raw', d['coalesce'], d['resident'], d['delay_us']['p50'], d['delay_us']['p99'], d['errors']); continue
    print(d['streams'], d['rate_pps'], 'coal',d['coalesce'],'res',d['resident'], int(d['groups_per_s']), d['delay_us']['p50'], d['delay_us']['p99'], d['cpu_us_per_group'], d['errors'])
"; exit $rc
