#!/usr/bin/env bash
# Round 5, part S: serving classes with the shared words read by every 8th poll: class 0's
# stamps at one stream (1 / 4 / 8 classes), then the call site at 1, 16 and 64 streams, alternating.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05s}"
mkdir -p "$E"
cd "$ROOT"
T=quic-test_amd/lib/call_site
for sv in 1 4 8; do
  echo "== servers $sv streams 1"
  QUICFEC_RESIDENT_STAMPS=1 QUICFEC_RESIDENT_SERVERS=$sv timeout -k 10 120 $T streams 1 1 2>&1 | grep '^{'
done > "$E/stamps.txt"
cat "$E/stamps.txt"
: > "$E/ab_servers.jsonl"
for rep in 1 2 3; do
  for sv in 1 4 8; do
    for argv in "raw 20000" "streams 1 1" "streams 16 2" "streams 64 2"; do
      line=$(QUICFEC_RESIDENT_SERVERS=$sv timeout -k 10 120 $T $argv | grep '^{' | tail -1)
      echo "{\"servers\": $sv, \"argv\": \"$argv\", \"rec\": $line}" >> "$E/ab_servers.jsonl"
    done
  done
  echo "rep $rep done"
done
python - "$E/ab_servers.jsonl" <<'PY'
import json, sys, collections, statistics
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["rec"]
    assert r["errors"] == 0, d
    agg[(d["argv"], d["servers"])].append((round(r["groups_per_s"]), r["delay_us"]["p50"]))
for k in sorted(agg):
    v = agg[k]
    print(k, "median rate", statistics.median(x[0] for x in v), "median p50", statistics.median(x[1] for x in v), v)
PY
