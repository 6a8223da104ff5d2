# The resident encoder's speculative poll, A/B on one box (QUICFEC_RESIDENT_SPEC=1/0, alternating):
# raw one-stream calls and the unchanged call site at 4 / 8 / 16 streams.
# (QUICFEC_RESIDENT_SPEC existed only until the VRAM ring; the speculative poll was removed)
set -e
B=./quic-test_amd/lib/batcher_latency
for rep in 1 2; do
  for sp in 1 0; do
    QUICFEC_RESIDENT_SPEC=$sp timeout -k 10 60 $B legacy_raw 20000 | sed "s/^{/{\"spec\": $sp, /" || [ $? -eq 1 ]
    for s in 4 8 16; do
      QUICFEC_RESIDENT_SPEC=$sp timeout -k 10 60 $B legacy $s 0 2 | sed "s/^{/{\"spec\": $sp, /" || [ $? -eq 1 ]
    done
  done
done
