set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batcher.py tests/test_host_mirror.py tests/test_abi.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1 || { tail -40 gpurun_out/pytest_multi.log; exit 1; }
tail -2 gpurun_out/pytest_multi.log
B=./quic-test_amd/lib/batcher_latency
export QUICFEC_SKIP_COPY=1
for d in "" "0,0"; do
  for s in 8 16; do
    QUICFEC_BATCHER_DEVICES=$d timeout -k 10 60 $B raw $s 2 1 1000 4096 1024 >> gpurun_out/multi.jsonl
    QUICFEC_BATCHER_DEVICES=$d timeout -k 10 60 $B raw $s 2 3 1000 4096 1024 >> gpurun_out/multi.jsonl
    QUICFEC_BATCHER_DEVICES=$d timeout -k 10 60 $B decode $s 2 3 1000 4096 1024 >> gpurun_out/multi.jsonl
  done
done
cat gpurun_out/multi.jsonl
