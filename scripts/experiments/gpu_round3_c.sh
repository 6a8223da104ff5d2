# coalescer tuning sweep: in-flight depth x waiter spin budget, 16 and 100 streams, vs the per-context path
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=./quic-test_amd/lib/batcher_latency
O=gpurun_out/legacy_c.jsonl
run() { timeout -k 10 60 "$@" >> $O || exit 1; }
for s in 16 100; do
  QUICFEC_COALESCE=0 run $B legacy $s 0 2
  for inf in 2 3 4; do
    QUICFEC_COALESCE_INFLIGHT=$inf run $B legacy $s 0 2
    QUICFEC_COALESCE_INFLIGHT=$inf QUICFEC_COALESCE_SPIN_PAUSE=64 QUICFEC_COALESCE_SPIN_YIELD=0 run $B legacy $s 0 2
    QUICFEC_COALESCE_INFLIGHT=$inf QUICFEC_COALESCE_SPIN_PAUSE=0 QUICFEC_COALESCE_SPIN_YIELD=0 run $B legacy $s 0 2
  done
done
QUICFEC_COALESCE_INFLIGHT=3 run $B legacy 1 0 2
cat $O
