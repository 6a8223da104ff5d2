#!/usr/bin/env bash
# Round 5, part L: inline chunks with 7 payload bytes + a tag byte per 8-B half (14 per 16 B over
# the BAR instead of 12): the coalesce GPU tests and exit-path hooks on it, then the call site
# alternating over three libraries -- round 4 (lib/old), round 5's first form (lib/r5a: 6 + 2 per
# half), this one -- raw calls, 16 and 100 streams.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05l}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py tests/test_host_mirror.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/coalesce.log" 2>&1 || { tail -60 "$E/coalesce.log"; exit 1; }
tail -1 "$E/coalesce.log"
for m in tear epoch poison_mt mixed; do
  n=300; case $m in epoch) n=6144;; poison_mt) n=2400;; mixed) n=360;; esac
  timeout -k 10 120 ./quic-test_amd/lib/exit_path_test $m $n > "$E/exit_$m.json"
  tail -1 "$E/exit_$m.json"
done
: > "$E/ab_call_site.jsonl"
for rep in 1 2 3; do
  for lib in old r5a new; do
    tool=quic-test_amd/lib/call_site; [ $lib != new ] && tool=quic-test_amd/lib/$lib/call_site
    for argv in "raw 20000" "streams 16 2" "streams 100 2"; do
      line=$(timeout -k 10 120 $tool $argv | grep '^{' | tail -1)
      echo "{\"lib\": \"$lib\", \"argv\": \"$argv\", \"rec\": $line}" >> "$E/ab_call_site.jsonl"
    done
  done
done
python - "$E/ab_call_site.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["rec"]
    print(d["lib"], d["argv"], round(r["groups_per_s"]), r["delay_us"]["p50"], r["errors"])
PY
