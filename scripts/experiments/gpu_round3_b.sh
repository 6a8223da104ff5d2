# coalescer A/B: GPU coalesce tests, then the legacy sweep at several in-flight depths
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "legacy or coalesce" > gpurun_out/pytest_coalesce.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_coalesce.log; [ $rc -eq 0 ] || exit $rc
B=./quic-test_amd/lib/batcher_latency
for inf in 1 2 3; do
  for s in 1 16 100; do
    QUICFEC_COALESCE_INFLIGHT=$inf timeout -k 10 60 $B legacy $s 0 2 >> gpurun_out/legacy_b.jsonl || exit 1
  done
done
for s in 16 100; do QUICFEC_COALESCE=0 timeout -k 10 60 $B legacy $s 0 2 >> gpurun_out/legacy_b.jsonl || exit 1; done
cat gpurun_out/legacy_b.jsonl
# two ranks on the one GPU (gloo): the C5 line with aggregate host-resident legs
QUICFEC_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --config c5 --e2e --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5_gpus2_gloo.json 2> gpurun_out/c5_gpus2_gloo.err
rc=$?; cat gpurun_out/c5_gpus2_gloo.json; tail -3 gpurun_out/c5_gpus2_gloo.err; exit $rc
