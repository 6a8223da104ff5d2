# Soak of the resident encoder's VRAM ring: the unchanged call site back to back, every repair
# checked against the AVX2 XOR -- millions of calls, so the slots' 8-bit header lap tags wrap
# (every 262,144 calls) many times.  16 streams for 30 s, 100 streams for 20 s.
set -e
B=./quic-test_amd/lib/batcher_latency
timeout -k 10 90 $B legacy 16 0 30
timeout -k 10 90 $B legacy 100 0 20
