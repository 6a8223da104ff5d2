B=./quic-test_amd/lib/batcher_latency
for rep in 1 2; do
  for m in high plain; do
    for s in 1 16; do
      QUICFEC_RESIDENT_STREAM=$m QUICFEC_COALESCE=1 QUICFEC_RESIDENT=1 timeout -k 10 60 $B legacy $s 0 2 | sed "s/^{/{\"stream_mode\": \"$m\", /" || true
    done
  done
done
