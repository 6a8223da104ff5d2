set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_limits.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab3.log 2>&1 || { tail -30 gpurun_out/pytest_ab3.log; exit 1; }
tail -1 gpurun_out/pytest_ab3.log
VAR=QUICFEC_ENCODE_RUNTIME_K VALUES="1 0" ROUNDS=2 BENCH_ARGS="--shape 10,2,1200" bash scripts/ab_env.sh > gpurun_out/ab3.txt 2>&1
VAR=QUICFEC_ENCODE_BLOCKS VALUES="2 3 4 0" ROUNDS=2 BENCH_ARGS="--shape 10,2,1200" bash scripts/ab_env.sh >> gpurun_out/ab3.txt 2>&1
VAR=QUICFEC_ENCODE_WAVES VALUES="10 15" ROUNDS=2 BENCH_ARGS="--shape 10,1,1200" bash scripts/ab_env.sh >> gpurun_out/ab3.txt 2>&1
VAR=QUICFEC_ENCODE_WAVES VALUES="10 15" ROUNDS=2 BENCH_ARGS="--shape 10,2,700" bash scripts/ab_env.sh >> gpurun_out/ab3.txt 2>&1
grep -o "QUICFEC_ENCODE_[A-Z_]*=[0-9].\{0,120\}encode.: ([0-9.]*" gpurun_out/ab3.txt | sed 's/C2 encode.*encode/ encode/'
