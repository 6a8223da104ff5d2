#!/usr/bin/env bash
# The default bench in N separate processes (fresh allocations each), buffer addresses logged:
# does the recover's time depend on where its buffers land?  gpurun_out/placement_runs.jsonl
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/placement_runs.jsonl"
: > "$OUT"
for i in $(seq "${N:-8}"); do
  line=$(QUICFEC_BENCH_ADDRS=1 timeout -k 10 200 python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-other-api ${BENCH_ARGS:-} 2>/dev/null | tail -1) || exit 1
  python3 - "$line" >> "$OUT" <<'PY'
import json, sys
d = json.loads(sys.argv[1])
k = d["kernels"]
print(json.dumps({"value": d["value"], "encode_ms": k["encode"]["ms"], "decode_ms": k["decode"]["ms"],
                  "decode_isolated_ms": k["decode"]["isolated"]["ms_median"], "buffers": d.get("buffers")}))
PY
done
cat "$OUT"
