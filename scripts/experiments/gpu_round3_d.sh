# round-3 evidence batch: GPU tests, coalescer sweep, per-API PMC (c2c3, c5), SQ counters (c4, c2c3)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash scripts/experiments/gpu_round3_c.sh > /dev/null || exit 1
CFGS="c2c3 c5" timeout -k 10 900 bash scripts/gpu_pmc.sh || exit 1
timeout -k 10 600 bash scripts/gpu_sq.sh || exit 1
