#!/usr/bin/env bash
# rocprofv3 PMC passes (one counter per pass, nothing else alongside) for each config in
# $CFGS, summarised per kernel into gpurun_out/pmc_<config>.json with the library hash
# (bench.py only uses a file whose lib_sha256 matches the .so it loads).
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
for CFG in ${CFGS:-c2c3}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $CFG $c"
    timeout -s KILL 240 rocprofv3 --pmc "$c" -d "$OUT/pmc_${CFG}_$c" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-verify \
      > "$OUT/pmc_${CFG}_$c.json" 2> "$OUT/pmc_${CFG}_$c.err"
  done
  python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_${CFG}_FETCH_SIZE" "$OUT/pmc_${CFG}_WRITE_SIZE" "$CFG" "$OUT/pmc_$CFG.json" > /dev/null
  echo "wrote $OUT/pmc_$CFG.json"
done
