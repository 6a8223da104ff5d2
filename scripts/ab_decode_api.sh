#!/usr/bin/env bash
# Decode API A/B on one box: bench.py --decode-api packed vs recover (slot rows), alternating,
# C3 (c2c3) and C5; every run also times the other API isolated (kernels.decode.other_api).
# One JSON line per run: gpurun_out/ab_decode_api.jsonl
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in c2c3 c5; do
    for api in packed recover; do
      timeout -k 10 240 python3 bench.py --config $cfg --decode-api $api --steps 20 --warmup 3 --no-cpu-baseline --no-verify \
        > gpurun_out/ab_api_tmp.json 2> gpurun_out/ab_api_tmp.err || { tail -3 gpurun_out/ab_api_tmp.err; exit 1; }
      python3 - "$cfg" "$api" "$rep" <<'PY' >> gpurun_out/ab_decode_api.jsonl
import json, sys
d = json.loads(open("gpurun_out/ab_api_tmp.json").read().strip().splitlines()[-1])
k = d["kernels"]["decode"]
print(json.dumps({"config": sys.argv[1], "api": sys.argv[2], "rep": int(sys.argv[3]), "value": d["value"],
                  "decode_ms_in_step": k["ms"], "decode_ms_isolated": k["isolated"]["ms_median"],
                  "other_api": k.get("other_api"), "encode_ms": d["kernels"]["encode"]["ms"],
                  "box_copy_GBps": d["roofline"]["box_copy_GBps"]}))
PY
    done
  done
done
cat gpurun_out/ab_decode_api.jsonl
