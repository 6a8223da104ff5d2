#!/usr/bin/env bash
# Round 5, part N: the resident encoder's inline copy against device reads of the page-locked
# slab (QUICFEC_RESIDENT_INLINE 1 = always copy, 0 = never for a page-locked slab, N = copy only
# while fewer than N calls are in flight), the call site at 1/4/16 streams, alternating.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05n}"
mkdir -p "$E"
cd "$ROOT"
T=quic-test_amd/lib/call_site
: > "$E/ab_inline.jsonl"
for rep in 1 2 3; do
  for mode in 1 0 3 6; do
    for argv in "raw 20000" "streams 1 1" "streams 4 1" "streams 16 2" "streams 64 2"; do
      line=$(QUICFEC_RESIDENT_INLINE=$mode timeout -k 10 120 $T $argv | grep '^{' | tail -1)
      echo "{\"inline\": $mode, \"argv\": \"$argv\", \"rec\": $line}" >> "$E/ab_inline.jsonl"
    done
  done
  echo "rep $rep done"
done
python - "$E/ab_inline.jsonl" <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["rec"]
    assert r["errors"] == 0, d
    agg[(d["argv"], d["inline"])].append((round(r["groups_per_s"]), r["delay_us"]["p50"], r["delay_us"]["p99"]))
for k in sorted(agg):
    print(k, agg[k])
PY
for mode in 1 0 3; do
  QUICFEC_RESIDENT_INLINE=$mode timeout -k 10 90 ./quic-test_amd/lib/batcher_latency legacy 16 0 5 > "$E/legacy16_inline$mode.json"
  cat "$E/legacy16_inline$mode.json"
done
