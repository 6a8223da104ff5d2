#!/usr/bin/env bash
# A/B of the bit-sliced encode against the table form, alternating runs.  Each spec is
# config:bits:window:waves (QUICFEC_ENCODE_BITS, QUICFEC_ENCODE_BITS_WINDOW, QUICFEC_ENCODE_WAVES
# = waves per CU cap, 0 = none); SPECS overrides the default list, REPS the repeats.
# One JSON line per run in gpurun_out/ab_bits.jsonl.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
# the tuning switches live in the test library (quic-test_amd/csrc/fec_knobs.hpp); bench.py loads it through quicfec
export QUICFEC_LIB="${QUICFEC_LIB:-$ROOT/quic-test_amd/lib/libfec_hip_test.so}"
OUT="$ROOT/gpurun_out/ab_bits.jsonl"
: > "$OUT"
run() {  # config bits window waves
  local line wv=()
  [ "$4" != 0 ] && wv=(QUICFEC_ENCODE_WAVES="$4")
  line=$(env QUICFEC_ENCODE_BITS="$2" QUICFEC_ENCODE_BITS_WINDOW="$3" "${wv[@]}" timeout -k 10 150 python3 "$ROOT/bench.py" \
         --config "$1" --steps 20 --warmup 3 --no-cpu-baseline --no-other-api 2>/dev/null | tail -1) || return 1
  python3 - "$1" "$2" "$3" "$4" "$line" >> "$OUT" <<'PY'
import json, sys
cfg, bits, win, waves, line = sys.argv[1:6]
d = json.loads(line)
e = d["kernels"]["encode"]
print(json.dumps({"config": cfg, "bits": int(bits), "window": int(win), "waves_per_cu": int(waves), "encode_ms": e["ms"],
                  "encode_GBps": e["achieved_GBps"], "box_copy_GBps": d["roofline"].get("box_copy_GBps"),
                  "verified": d["verified"]}))
PY
}
SPECS="${SPECS:-c4:1:4:0 c4:1:8:0 c4:0:0:0 c2c3:1:4:0 c2c3:0:0:0}"
for rep in $(seq "${REPS:-2}"); do
  for s in $SPECS; do
    IFS=: read -r c b w v <<< "$s"
    run "$c" "$b" "$w" "$v" || exit 1
  done
done
cat "$OUT"
