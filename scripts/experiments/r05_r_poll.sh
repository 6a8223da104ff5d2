#!/usr/bin/env bash
# Round 5, part R: serving classes x poll width (QUICFEC_RESIDENT_SERVERS x QUICFEC_RESIDENT_POLL),
# the call site at 1, 16 and 64 streams, alternating, four rounds; class 0's stamps at one stream.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05r}"
mkdir -p "$E"
cd "$ROOT"
T=quic-test_amd/lib/call_site
: > "$E/ab_poll.jsonl"
for rep in 1 2 3 4; do
  for cfg in "1 16" "4 16" "4 4" "8 16" "8 4" "8 2"; do
    set -- $cfg
    for argv in "raw 20000" "streams 1 1" "streams 16 2" "streams 64 2"; do
      line=$(QUICFEC_RESIDENT_SERVERS=$1 QUICFEC_RESIDENT_POLL=$2 timeout -k 10 120 $T $argv | grep '^{' | tail -1)
      echo "{\"servers\": $1, \"poll\": $2, \"argv\": \"$argv\", \"rec\": $line}" >> "$E/ab_poll.jsonl"
    done
  done
  echo "rep $rep done"
done
python - "$E/ab_poll.jsonl" <<'PY'
import json, sys, collections, statistics
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["rec"]
    assert r["errors"] == 0, d
    agg[(d["argv"], d["servers"], d["poll"])].append((round(r["groups_per_s"]), r["delay_us"]["p50"]))
for k in sorted(agg):
    v = agg[k]
    print(k, "median rate", statistics.median(x[0] for x in v), "median p50", statistics.median(x[1] for x in v), v)
PY
for cfg in "1 16" "4 4" "8 4" "8 2"; do
  set -- $cfg
  echo "== servers $1 poll $2 streams 1"
  QUICFEC_RESIDENT_STAMPS=1 QUICFEC_RESIDENT_SERVERS=$1 QUICFEC_RESIDENT_POLL=$2 timeout -k 10 120 $T streams 1 1 2>&1 | grep '^{'
done > "$E/stamps.txt"
cat "$E/stamps.txt"
