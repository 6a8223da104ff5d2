#!/usr/bin/env bash
# Same-box A/B of two library builds on the default bench (QUICFEC_LIB selects the .so),
# alternating; one JSON summary line per run in gpurun_out/ab_lib.jsonl.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/ab_lib.jsonl"
: > "$OUT"
for rep in $(seq "${REPS:-3}"); do
  for lib in ${LIBS:-quic-test_amd/lib/libfec_hip.so quic-test_amd/lib/old/libfec_hip.so}; do
    line=$(QUICFEC_LIB="$ROOT/$lib" timeout -k 10 200 python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null | tail -1) || exit 1
    python3 - "$lib" "$line" >> "$OUT" <<'PY'
import json, sys
lib, line = sys.argv[1:3]
d = json.loads(line)
k = d["kernels"]
print(json.dumps({"lib": lib, "value": d["value"], "encode_ms": k["encode"]["ms"], "decode_ms": k.get("decode", {}).get("ms"),
                  "decode_isolated_ms": k.get("decode", {}).get("isolated", {}).get("ms_median"),
                  "box_copy_GBps": d["roofline"].get("box_copy_GBps")}))
PY
  done
done
cat "$OUT"
