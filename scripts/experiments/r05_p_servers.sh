#!/usr/bin/env bash
# Round 5, part P: the resident encoder with several serving workgroups (QUICFEC_RESIDENT_SERVERS,
# one per seq class).  (1) the coalesce GPU suite (default, plus every ring-protocol run with 2
# and 4 classes); (2) the call site at 1/4/16/64 streams with 1, 2 and 4 classes, alternating.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05p}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_coalesce.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/coalesce.log" 2>&1 || { tail -80 "$E/coalesce.log"; exit 1; }
tail -3 "$E/coalesce.log"
T=quic-test_amd/lib/call_site
: > "$E/ab_servers.jsonl"
for rep in 1 2 3; do
  for sv in 1 2 4; do
    for argv in "raw 20000" "streams 1 1" "streams 4 1" "streams 16 2" "streams 64 2"; do
      line=$(QUICFEC_RESIDENT_SERVERS=$sv timeout -k 10 120 $T $argv | grep '^{' | tail -1)
      echo "{\"servers\": $sv, \"argv\": \"$argv\", \"rec\": $line}" >> "$E/ab_servers.jsonl"
    done
  done
  echo "rep $rep done"
done
python - "$E/ab_servers.jsonl" <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["rec"]
    assert r["errors"] == 0, d
    agg[(d["argv"], d["servers"])].append((round(r["groups_per_s"]), r["delay_us"]["p50"], r["delay_us"]["p99"], r.get("resident_servers")))
for k in sorted(agg):
    print(k, agg[k])
PY
for sv in 1 2 4; do
  QUICFEC_RESIDENT_SERVERS=$sv timeout -k 10 90 ./quic-test_amd/lib/batcher_latency legacy 16 0 5 > "$E/legacy16_servers$sv.json"
  cat "$E/legacy16_servers$sv.json"
done
