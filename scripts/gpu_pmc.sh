#!/usr/bin/env bash
# rocprofv3 PMC passes (one counter group per pass, kernel trace only alongside).
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"
CFG="${CFG:-c2c3}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c"
  timeout -k 10 400 rocprofv3 --pmc "$c" -d "$OUT/pmc_$c" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-verify > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err"
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_FETCH_SIZE" "$OUT/pmc_WRITE_SIZE" "$CFG" "$OUT/pmc_$CFG.json"
