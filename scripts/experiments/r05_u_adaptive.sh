#!/usr/bin/env bash
# Round 5, part U: the serving class chosen by the calls in flight (a lone caller's calls all to
# class 0, idle classes polling slowly) against round-robin over all 8 classes (QUICFEC_RESIDENT_SPREAD=1,
# slow polling off) and one class; the coalesce suite first.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05u}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_coalesce.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/coalesce.log" 2>&1 || { tail -80 "$E/coalesce.log"; exit 1; }
tail -3 "$E/coalesce.log"
T=quic-test_amd/lib/call_site
: > "$E/ab_adaptive.jsonl"
for rep in 1 2 3 4; do
  for cfg in adaptive spread one; do
    case $cfg in
      adaptive) envs="" ;;
      spread) envs="QUICFEC_RESIDENT_SPREAD=1 QUICFEC_RESIDENT_SLOW_US=100000000" ;;
      one) envs="QUICFEC_RESIDENT_SERVERS=1" ;;
    esac
    for argv in "raw 20000" "streams 1 1" "streams 2 1" "streams 4 1" "streams 16 2" "streams 64 2"; do
      line=$(env $envs timeout -k 10 120 $T $argv | grep '^{' | tail -1)
      echo "{\"cfg\": \"$cfg\", \"argv\": \"$argv\", \"rec\": $line}" >> "$E/ab_adaptive.jsonl"
    done
  done
  echo "rep $rep done"
done
python - "$E/ab_adaptive.jsonl" <<'PY'
import json, sys, collections, statistics
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["rec"]
    assert r["errors"] == 0, d
    agg[(d["argv"], d["cfg"])].append((round(r["groups_per_s"]), r["delay_us"]["p50"]))
for k in sorted(agg):
    v = agg[k]
    print(k, "median rate", statistics.median(x[0] for x in v), "median p50", statistics.median(x[1] for x in v), v)
PY
for cfg in adaptive spread; do
  envs=""; [ $cfg = spread ] && envs="QUICFEC_RESIDENT_SPREAD=1 QUICFEC_RESIDENT_SLOW_US=100000000"
  echo "== $cfg streams 1"
  env QUICFEC_RESIDENT_STAMPS=1 $envs timeout -k 10 120 $T streams 1 1 2>&1 | grep '^{'
done > "$E/stamps.txt"
cat "$E/stamps.txt"
QUICFEC_RESIDENT_STAMPS=0 timeout -k 10 90 ./quic-test_amd/lib/batcher_latency legacy 16 0 5 > "$E/legacy16.json"
cat "$E/legacy16.json"
