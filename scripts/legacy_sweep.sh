#!/usr/bin/env bash
# The reference's unchanged call site (every stream its own HybridFECEncoder -> fec_encode_batch
# with one group per call, page-locked slab and repair buffer as FECEncoderCXX allocates them) at
# 1 / 16 / 100 streams, back to back and at the reference's 100 packets/s, through the library's
# paths -- resident encoder (default: its ring in VRAM), the same with the page-locked ring
# (QUICFEC_RESIDENT_VRAM=0), shared launches (QUICFEC_RESIDENT=0), one launch per call on the
# caller's context (QUICFEC_COALESCE=0) -- next to one CPU core.  One JSON object per
# line on stdout.  GPU box: bash scripts/legacy_sweep.sh > gpurun_out/legacy.jsonl
set -euo pipefail
B=./quic-test_amd/lib/batcher_latency
T="timeout -k 10 60"
SECS=${SECS:-2}
run() { "$@" || [ $? -eq 1 ]; }  # a run reporting errors exits 1 after its line; a hang still ends it
run $T $B cpu
for e in "QUICFEC_RESIDENT=1" "QUICFEC_RESIDENT_VRAM=0" "QUICFEC_RESIDENT=0" "QUICFEC_COALESCE=0"; do env $e $T $B legacy_raw 20000 | sed "s/^{/{\"env\": \"$e\", /" || [ $? -eq 1 ]; done
for rep in $(seq 1 "${REPS:-1}"); do
  for s in 1 16 100; do
    for mode in resident hostring batches percontext; do
      case $mode in
        resident) e="QUICFEC_COALESCE=1 QUICFEC_RESIDENT=1" ;;
        hostring) e="QUICFEC_COALESCE=1 QUICFEC_RESIDENT=1 QUICFEC_RESIDENT_VRAM=0" ;;
        batches) e="QUICFEC_COALESCE=1 QUICFEC_RESIDENT=0" ;;
        percontext) e="QUICFEC_COALESCE=0" ;;
      esac
      env $e $T $B legacy $s 0 "$SECS" | sed "s/^{/{\"path\": \"$mode\", /" || [ $? -eq 1 ]
    done
  done
  for s in 1 100; do
    for mode in resident hostring percontext; do
      case $mode in
        resident) e="QUICFEC_COALESCE=1 QUICFEC_RESIDENT=1" ;;
        hostring) e="QUICFEC_COALESCE=1 QUICFEC_RESIDENT=1 QUICFEC_RESIDENT_VRAM=0" ;;
        percontext) e="QUICFEC_COALESCE=0" ;;
      esac
      env $e $T $B legacy $s 100 "$SECS" | sed "s/^{/{\"path\": \"$mode\", /" || [ $? -eq 1 ]
    done
  done
done
