#!/usr/bin/env bash
# the C5 (satellite iid loss) recover's form on this build, in the bench's own
# step -- packed rows (recover_runs, one launch) vs slot rows (decode_fused, 8 groups per wave) --
# alternating, ROUNDS rounds, one JSON line per run into gpurun_out/${EVID}/ab_c5_api.jsonl.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r06}"
mkdir -p "$E"
cd "$ROOT"
for rd in $(seq 1 "${ROUNDS:-3}"); do
  for api in packed recover; do
    timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-call-site \
      --decode-api $api --no-other-api > "$E/ab_c5_$api.json" 2> /dev/null
    python - "$E/ab_c5_$api.json" "$api" "$rd" >> "$E/ab_c5_api.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]["decode"]
print(json.dumps({"api": sys.argv[2], "round": int(sys.argv[3]), "value": d["value"], "verified": d["verified"],
                  "decode_ms": k["ms"], "decode_isolated_ms": k["isolated"]["ms_median"],
                  "encode_ms": d["kernels"]["encode"]["ms"], "box_copy_GBps": d["roofline"]["box_copy_GBps"]}))
PY
  done
done
tail -n $((2 * ${ROUNDS:-3})) "$E/ab_c5_api.jsonl"
