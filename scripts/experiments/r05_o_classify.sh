#!/usr/bin/env bash
# Round 5, part O: what the per-call pointer classification of the legacy call's offsets array
# (pageable: a HIP runtime pointer lookup per call) costs the call site, alternating.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05o}"
mkdir -p "$E"
cd "$ROOT"
T=quic-test_amd/lib/call_site
: > "$E/ab_classify.jsonl"
for rep in 1 2 3; do
  for skip in 0 1; do
    for argv in "raw 20000" "streams 1 1" "streams 16 2" "streams 64 2"; do
      line=$(QUICFEC_PROBE_SKIP_OFFSETS=$skip timeout -k 10 120 $T $argv | grep '^{' | tail -1)
      echo "{\"skip\": $skip, \"argv\": \"$argv\", \"rec\": $line}" >> "$E/ab_classify.jsonl"
    done
  done
  echo "rep $rep done"
done
python - "$E/ab_classify.jsonl" <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["rec"]
    assert r["errors"] == 0, d
    agg[(d["argv"], d["skip"])].append((round(r["groups_per_s"]), r["delay_us"]["p50"], r["delay_us"]["p99"]))
for k in sorted(agg):
    print(k, agg[k])
PY
for skip in 0 1; do
  QUICFEC_PROBE_SKIP_OFFSETS=$skip timeout -k 10 90 ./quic-test_amd/lib/batcher_latency legacy 16 0 5 > "$E/legacy16_skip$skip.json"
  cat "$E/legacy16_skip$skip.json"
done
