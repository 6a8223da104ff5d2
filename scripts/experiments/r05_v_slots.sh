#!/usr/bin/env bash
# Round 5, part V: each serving class's slots as one block of consecutive slots (server_slot)
# against the interleaved slots of the previous build (quic-test_amd/lib/ab_prev), the call site
# alternating; the coalesce suite on the new build first; class 0's stamps at one stream.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05v}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_coalesce.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/coalesce.log" 2>&1 || { tail -80 "$E/coalesce.log"; exit 1; }
tail -2 "$E/coalesce.log"
: > "$E/ab_slots.jsonl"
for rep in 1 2 3 4; do
  for lib in prev new; do
    T=quic-test_amd/lib/call_site; [ $lib = prev ] && T=quic-test_amd/lib/ab_prev/call_site
    for argv in "raw 20000" "streams 1 1" "streams 4 1" "streams 16 2" "streams 64 2"; do
      line=$(timeout -k 10 120 $T $argv | grep '^{' | tail -1)
      echo "{\"lib\": \"$lib\", \"argv\": \"$argv\", \"rec\": $line}" >> "$E/ab_slots.jsonl"
    done
  done
  echo "rep $rep done"
done
python - "$E/ab_slots.jsonl" <<'PY'
import json, sys, collections, statistics
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["rec"]
    assert r["errors"] == 0, d
    agg[(d["argv"], d["lib"])].append((round(r["groups_per_s"]), r["delay_us"]["p50"]))
for k in sorted(agg):
    v = agg[k]
    print(k, "median rate", statistics.median(x[0] for x in v), "median p50", statistics.median(x[1] for x in v), v)
PY
for lib in prev new; do
  T=quic-test_amd/lib/call_site; [ $lib = prev ] && T=quic-test_amd/lib/ab_prev/call_site
  echo "== $lib streams 1"
  QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 120 $T streams 1 1 2>&1 | grep '^{'
  echo "== $lib streams 16"
  QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 120 $T streams 16 1 2>&1 | grep '^{'
done > "$E/stamps.txt"
cat "$E/stamps.txt"
