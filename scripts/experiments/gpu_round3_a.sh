set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash scripts/legacy_sweep.sh > gpurun_out/legacy.jsonl 2> gpurun_out/legacy.err
rc=$?; cat gpurun_out/legacy.jsonl; tail -5 gpurun_out/legacy.err; exit $rc
