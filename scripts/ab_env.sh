#!/usr/bin/env bash
# A/B of a library environment switch inside one box: alternating bench runs.
# usage: VAR=QUICFEC_ENCODE_PAIR VALUES="0 1" CFG=c4 ROUNDS=2 bash scripts/ab_env.sh
set -euo pipefail
# the tuning switches live in the test library (quic-test_amd/csrc/fec_knobs.hpp); bench.py loads it through quicfec
export QUICFEC_LIB="${QUICFEC_LIB:-$(pwd)/quic-test_amd/lib/libfec_hip_test.so}"
for rd in $(seq 1 "${ROUNDS:-2}"); do
  for v in ${VALUES:-0 1}; do
    env "$VAR=$v" timeout -k 10 200 python bench.py --config "${CFG:-c2c3}" --steps "${STEPS:-10}" --warmup 2 \
      --no-cpu-baseline --no-verify ${BENCH_ARGS:-} > /tmp/ab.json
    python - "$VAR=$v" <<'PY'
import json, sys
d = json.load(open("/tmp/ab.json"))
print(sys.argv[1], d["config"]["workload"][:40], "value", d["value"],
      {k: (v["ms"], v["achieved_GBps"], v.get("isolated", {}).get("ms_median"), v.get("api"),
           (v.get("other_api") or {}).get("ms_median")) for k, v in d["kernels"].items()})
PY
  done
done
