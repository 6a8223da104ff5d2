#!/usr/bin/env bash
# What bounds the encode kernels: SQ instruction / cycle counters and the GRBM clock, one counter
# group per rocprofv3 pass (<= 8 SQ, <= 2 GRBM), for C4 (k=20 r=5) and C2 (k=10 r=3) encode.
# SQ_CONFIGS narrows the configs, SQ_TAG suffixes the output directory (A/B of a switch such
# as QUICFEC_ENCODE_BITS, which the bench processes inherit).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
# the tuning switches live in the test library (quic-test_amd/csrc/fec_knobs.hpp); bench.py loads it through quicfec
export QUICFEC_LIB="${QUICFEC_LIB:-$ROOT/quic-test_amd/lib/libfec_hip_test.so}"
OUT="$ROOT/gpurun_out/sq${SQ_TAG:-}"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
grep -oE "SQ_[A-Z_0-9]+|GRBM_[A-Z_0-9]+" "$OUT/counters_list.txt" | sort -u > "$OUT/counter_names.txt" || true
for CFG in ${SQ_CONFIGS:-c4 c2c3}; do
  i=0
  for group in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
               "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VALU" \
               "GRBM_GUI_ACTIVE GRBM_COUNT" \
               "FETCH_SIZE"; do
    i=$((i + 1))
    ok=1
    for c in $group; do grep -qx "$c" "$OUT/counter_names.txt" || { echo "skip pass $i ($c not listed)"; ok=0; }; done
    [ $ok = 1 ] || continue
    echo "== $CFG pass $i: $group"
    timeout -s KILL 120 rocprofv3 --pmc $group -d "$OUT/${CFG}_p$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-other-api \
      > "$OUT/${CFG}_p$i.json" 2> "$OUT/${CFG}_p$i.err" || { echo "pass failed rc=$?"; tail -3 "$OUT/${CFG}_p$i.err"; exit 1; }
  done
  python3 "$ROOT/scripts/pmc_generic.py" "$OUT/sq_$CFG.json" "$OUT/${CFG}_p"* > /dev/null
done
ls "$OUT"
