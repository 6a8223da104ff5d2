#!/usr/bin/env bash
# Round 5, part Q: serving classes (QUICFEC_RESIDENT_SERVERS) 1/2/4/8 at 1, 16 and 64 streams,
# alternating, five rounds; then class 0's server stamps at one stream and at 16 (1 vs 4 classes).
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05q}"
mkdir -p "$E"
cd "$ROOT"
T=quic-test_amd/lib/call_site
: > "$E/ab_servers.jsonl"
for rep in 1 2 3 4 5; do
  for sv in 1 2 4 8; do
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
for sv in 1 2 4; do
  for argv in "streams 1 1" "streams 16 1"; do
    echo "== servers $sv $argv"
    QUICFEC_RESIDENT_STAMPS=1 QUICFEC_RESIDENT_SERVERS=$sv timeout -k 10 120 $T $argv 2>&1 | grep '^{'
  done
done > "$E/stamps.txt"
cat "$E/stamps.txt"
