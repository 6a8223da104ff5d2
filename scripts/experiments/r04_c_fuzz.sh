# Long random sweeps on the current build: every API incl. the packed recover's two forms.
set -e
QUICFEC_FUZZ_SEED=0x5EED4000 QUICFEC_FUZZ_BLOCKS=150 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_fuzz.log 2>&1
tail -3 gpurun_out/r04_fuzz.log
