#!/usr/bin/env bash
# The reference's unchanged call site (every stream its own HybridFECEncoder -> fec_encode_batch
# with one group per call) at 1 / 16 / 100 streams, back to back and at the reference's 100
# packets/s, with the library's legacy-call coalescing on and off (QUICFEC_COALESCE), next to
# one CPU core.  One JSON object per line on stdout.
# GPU box: bash scripts/legacy_sweep.sh > gpurun_out/legacy.jsonl
set -euo pipefail
B=./quic-test_amd/lib/batcher_latency
T="timeout -k 10 60"
SECS=${SECS:-2}
run() { "$@" || [ $? -eq 1 ]; }  # a run reporting errors exits 1 after its line; a hang still ends it
run $T $B cpu
for rep in ${REPS:-1}; do
  for s in 1 16 100; do
    for c in 1 0; do
      QUICFEC_COALESCE=$c run $T $B legacy $s 0 "$SECS"
    done
  done
  for s in 1 100; do
    for c in 1 0; do
      QUICFEC_COALESCE=$c run $T $B legacy $s 100 "$SECS"
    done
  done
done
