#!/usr/bin/env bash
# The reference's unchanged call site (every stream its own HybridFECEncoder -> fec_encode_batch
# with one group per call, page-locked slab and repair buffer as FECEncoderCXX allocates them) at
# 1 / 16 / 100 streams, back to back and at the reference's 100 packets/s, through the library's
# three paths -- resident encoder (default), shared launches (QUICFEC_RESIDENT=0), one launch per
# call on the caller's context (QUICFEC_COALESCE=0) -- next to one CPU core.  One JSON object per
# line on stdout.  GPU box: bash scripts/legacy_sweep.sh > gpurun_out/legacy.jsonl
set -euo pipefail
B=./quic-test_amd/lib/batcher_latency
T="timeout -k 10 60"
SECS=${SECS:-2}
run() { "$@" || [ $? -eq 1 ]; }  # a run reporting errors exits 1 after its line; a hang still ends it
run $T $B cpu
for e in "QUICFEC_RESIDENT=1" "QUICFEC_RESIDENT=0" "QUICFEC_COALESCE=0"; do env $e $T $B legacy_raw 20000 || [ $? -eq 1 ]; done
for rep in $(seq 1 "${REPS:-1}"); do
  for s in 1 16 100; do
    for mode in resident batches percontext; do
      case $mode in
        resident) e="QUICFEC_COALESCE=1 QUICFEC_RESIDENT=1" ;;
        batches) e="QUICFEC_COALESCE=1 QUICFEC_RESIDENT=0" ;;
        percontext) e="QUICFEC_COALESCE=0" ;;
      esac
      env $e $T $B legacy $s 0 "$SECS" || [ $? -eq 1 ]
    done
  done
  for s in 1 100; do
    for mode in resident percontext; do
      e=$([ $mode = resident ] && echo "QUICFEC_COALESCE=1 QUICFEC_RESIDENT=1" || echo "QUICFEC_COALESCE=0")
      env $e $T $B legacy $s 100 "$SECS" || [ $? -eq 1 ]
    done
  done
done
