#!/usr/bin/env bash
# Any rocprofv3 --pmc counter groups over bench.py runs, one group per pass (each group within
# the per-block limits: <= 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 GRBM), summarised per kernel by
# scripts/pmc_generic.py into gpurun_out/pmc<TAG>/pmc_<config>.json.
#   PMC_GROUPS  groups separated by ';'      PMC_CONFIGS  bench configs (default c2c3)
#   PMC_TAG     output directory suffix      other env (QUICFEC_*) passes through to bench.py
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/pmc${PMC_TAG:-}"
mkdir -p "$OUT"
export TMPDIR=/tmp
IFS=';' read -ra GROUPS_ARR <<< "${PMC_GROUPS:?}"
for CFG in ${PMC_CONFIGS:-c2c3}; do
  i=0
  for group in "${GROUPS_ARR[@]}"; do
    i=$((i + 1))
    echo "== $CFG pass $i: $group"
    timeout -s KILL 120 rocprofv3 --pmc $group -d "$OUT/${CFG}_p$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-other-api \
      > "$OUT/${CFG}_p$i.json" 2> "$OUT/${CFG}_p$i.err" || { echo "pass failed rc=$?"; tail -3 "$OUT/${CFG}_p$i.err"; exit 1; }
  done
  python3 "$ROOT/scripts/pmc_generic.py" "$OUT/pmc_$CFG.json" "$OUT/${CFG}_p"* > /dev/null
done
