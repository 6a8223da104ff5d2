#!/usr/bin/env bash
# rocprofv3 PMC passes (one counter per pass, nothing else alongside), summarised per kernel
# into gpurun_out/pmc_<config>.json with the library hash (bench.py only uses a file whose
# lib_sha256 matches the .so it loads).  Configs with a decode get one pass pair per decode API
# (bench.py --decode-api X --no-other-api), stored as recover_packed / recover_slots.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # tag config extra-bench-args...
  local tag=$1 cfg=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $cfg $tag $c"
    timeout -s KILL 240 rocprofv3 --pmc "$c" -d "$OUT/pmc_${cfg}_${tag}_$c" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config "$cfg" --steps 3 --warmup 1 --no-cpu-baseline --no-verify "$@" \
      > "$OUT/pmc_${cfg}_${tag}_$c.json" 2> "$OUT/pmc_${cfg}_${tag}_$c.err"
  done
}
for CFG in ${CFGS:-c2c3}; do
  rm -f "$OUT/pmc_$CFG.json"
  case "$CFG" in
    c4)
      pass all c4
      python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_c4_all_FETCH_SIZE" "$OUT/pmc_c4_all_WRITE_SIZE" c4 "$OUT/pmc_c4.json" > /dev/null ;;
    c4d)
      pass inplace c4d --decode-api in-place --no-other-api
      python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_c4d_inplace_FETCH_SIZE" "$OUT/pmc_c4d_inplace_WRITE_SIZE" c4d "$OUT/pmc_c4d.json" > /dev/null
      pass slots c4d --decode-api recover --no-other-api
      python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_c4d_slots_FETCH_SIZE" "$OUT/pmc_c4d_slots_WRITE_SIZE" c4d "$OUT/pmc_c4d.json" --tag slots > /dev/null ;;
    *)
      for api in packed slots; do
        a=$([ "$api" = slots ] && echo recover || echo packed)
        pass "$api" "$CFG" --decode-api "$a" --no-other-api
        python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_${CFG}_${api}_FETCH_SIZE" "$OUT/pmc_${CFG}_${api}_WRITE_SIZE" \
          "$CFG" "$OUT/pmc_$CFG.json" --tag "$api" > /dev/null
      done ;;
  esac
  echo "wrote $OUT/pmc_$CFG.json"
done
