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
