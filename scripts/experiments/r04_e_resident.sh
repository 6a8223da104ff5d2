# The resident encoder after the load fix: its phase stamps, the raw call latency and the
# unchanged call site at 1 / 16 streams; then its GPU tests.
set -e
B=./quic-test_amd/lib/batcher_latency
for s in 1 16; do
  QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy $s 0 2 > gpurun_out/stampsC_$s.json 2> gpurun_out/stampsC_$s.err || [ $? -eq 1 ]
  cat gpurun_out/stampsC_$s.json; grep resident_stamps gpurun_out/stampsC_$s.err || true
done
QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy_raw 20000 > gpurun_out/stampsC_raw.json 2> gpurun_out/stampsC_raw.err || [ $? -eq 1 ]
cat gpurun_out/stampsC_raw.json; grep resident_stamps gpurun_out/stampsC_raw.err || true
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/coalesceC.log 2>&1; tail -2 gpurun_out/coalesceC.log
