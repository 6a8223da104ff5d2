# The resident encoder's own phase stamps (QUICFEC_RESIDENT_STAMPS) under 1 and 16 streams of the
# unchanged call site, to see whether the device loop or the callers bound the throughput.
set -e
B=./quic-test_amd/lib/batcher_latency
for s in 1 16; do
  QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy $s 0 2 > gpurun_out/stamps_$s.json 2> gpurun_out/stamps_$s.err || [ $? -eq 1 ]
  cat gpurun_out/stamps_$s.json; grep resident_stamps gpurun_out/stamps_$s.err || true
done
QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy_raw 5000 > gpurun_out/stamps_raw.json 2> gpurun_out/stamps_raw.err || [ $? -eq 1 ]
cat gpurun_out/stamps_raw.json; grep resident_stamps gpurun_out/stamps_raw.err || true
