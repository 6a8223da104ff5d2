# resident exit + coalesce tests, host sanitizers over the coalescer, decode-API A/B on a third box
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_coalesce.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_coalesce.log; [ $rc -eq 0 ] || exit $rc
SAN=address timeout -k 10 900 bash scripts/asan_host.sh run > gpurun_out/asan_r03.log 2>&1; rc=$?; echo "asan rc=$rc"; grep -E "PASS|ERROR: AddressSanitizer|errors|groups_per_s" gpurun_out/asan_r03.log | cut -c1-200 | head; [ $rc -eq 0 ] || exit $rc
SAN=thread timeout -k 10 900 bash scripts/asan_host.sh run > gpurun_out/tsan_r03.log 2>&1; rc=$?; echo "tsan rc=$rc"; grep -cE "WARNING: ThreadSanitizer" gpurun_out/tsan_r03.log; grep -E "PASS|groups_per_s" gpurun_out/tsan_r03.log | cut -c1-200 | head
rm -f gpurun_out/ab_decode_api.jsonl
timeout -k 10 900 bash scripts/ab_decode_api.sh > /dev/null || exit 1
python3 -c "
import json
for l in open('gpurun_out/ab_decode_api.jsonl'): d=json.loads(l); print(d['config'], d['api'], d['rep'], d['value'], d['decode_ms_in_step'], d['decode_ms_isolated'], d['other_api'])
"
