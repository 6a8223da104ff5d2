# A single stream at the reference's 100 packets/s (a group every 100 ms) with the resident
# instance's default bounds (2-ms idle, 50-ms life: a relaunch per call) and with them raised
# so one instance stays (QUICFEC_RESIDENT_IDLE_US / _LIFE_US); also 100 streams at that rate.
set -e
B=./quic-test_amd/lib/batcher_latency
for s in 1 100; do
  timeout -k 10 60 $B legacy $s 100 3 | sed "s/^{/{\"policy\": \"default\", /" || [ $? -eq 1 ]
  QUICFEC_RESIDENT_IDLE_US=2000000 QUICFEC_RESIDENT_LIFE_US=10000000 timeout -k 10 60 $B legacy $s 100 3 \
    | sed "s/^{/{\"policy\": \"resident 2 s idle\", /" || [ $? -eq 1 ]
done
