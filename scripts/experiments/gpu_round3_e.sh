# resident legacy encoder: its GPU tests first, then the legacy sweep
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_coalesce.log 2>&1
rc=$?; tail -20 gpurun_out/pytest_coalesce.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash scripts/legacy_sweep.sh > gpurun_out/legacy_e.jsonl 2> gpurun_out/legacy_e.err
rc=$?; cat gpurun_out/legacy_e.jsonl; tail -3 gpurun_out/legacy_e.err; exit $rc
