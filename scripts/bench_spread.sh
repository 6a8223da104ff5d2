#!/usr/bin/env bash
# The default bench (and C4) in N separate processes on one box: the per-process spread that
# buffer placement adds (DESIGN §5 "Recover time by box").  gpurun_out/bench_spread.jsonl
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/bench_spread.jsonl"
: > "$OUT"
for cfg in ${CFGS:-c2c3 c4}; do
  for i in $(seq "${N:-6}"); do
    line=$(timeout -k 10 200 python3 "$ROOT/bench.py" --config "$cfg" --steps 20 --warmup 5 --no-cpu-baseline --no-other-api 2>/dev/null | tail -1) || exit 1
    python3 - "$cfg" "$line" >> "$OUT" <<'PY'
import json, sys
cfg, line = sys.argv[1:3]
d = json.loads(line)
k = d["kernels"]
print(json.dumps({"config": cfg, "value": d["value"], "encode_ms": k["encode"]["ms"],
                  "decode_ms": k.get("decode", {}).get("ms"), "frac": d["roofline"]["frac"],
                  "box_copy_GBps": d["roofline"]["box_copy_GBps"], "verified": d["verified"]}))
PY
  done
done
cat "$OUT"
