# The resident encoder's VRAM ring: the legacy-call tests first (both ring kinds), then an A/B
# on one box, alternating (QUICFEC_RESIDENT_VRAM=1/0): raw one-stream calls and the unchanged
# call site at 1 / 4 / 8 / 16 streams.  Output: gpurun_out/r04h/.
set -e
mkdir -p gpurun_out/r04h
timeout -k 10 400 python -u -m pytest tests/test_gpu_coalesce.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r04h/pytest_coalesce.log 2>&1
B=./quic-test_amd/lib/batcher_latency
for rep in 1 2; do
  for v in 1 0; do
    QUICFEC_RESIDENT_VRAM=$v timeout -k 10 60 $B legacy_raw 20000 | sed "s/^{/{\"vram\": $v, /" \
      >> gpurun_out/r04h/ab.jsonl || [ $? -eq 1 ]
    for s in 1 4 8 16; do
      QUICFEC_RESIDENT_VRAM=$v timeout -k 10 60 $B legacy $s 0 2 | sed "s/^{/{\"vram\": $v, /" \
        >> gpurun_out/r04h/ab.jsonl || [ $? -eq 1 ]
    done
  done
done
cat gpurun_out/r04h/ab.jsonl
# the server's phase stamps on the VRAM ring, one stream and 16
QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy_raw 5000 > gpurun_out/r04h/stamps_raw.json 2> gpurun_out/r04h/stamps_raw.err || [ $? -eq 1 ]
QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy 16 0 1 > gpurun_out/r04h/stamps_s16.json 2> gpurun_out/r04h/stamps_s16.err || [ $? -eq 1 ]
grep -h resident_stamps gpurun_out/r04h/stamps_*.err
