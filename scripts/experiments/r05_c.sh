#!/usr/bin/env bash
# Round 5, part C: (1) coalesce GPU tests on the power-of-two tag epochs; (2) the call site,
# round-4 library vs this one, alternating; (3) the shared-launch legacy path's slowest call
# (legacy_raw, QUICFEC_RESIDENT=0; plain and under rocprofv3); (4) the C3 recover against the
# parity -> rebuilt distance (scripts/probe_recover_delta.py).
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05c}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/coalesce.log" 2>&1 || { tail -60 "$E/coalesce.log"; exit 1; }
tail -1 "$E/coalesce.log"
: > "$E/ab_call_site.jsonl"
for rep in 1 2 3; do
  for lib in old new; do
    tool=quic-test_amd/lib/call_site; [ $lib = old ] && tool=quic-test_amd/lib/old/call_site
    for argv in "raw 20000" "streams 16 2"; do
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
for i in 1 2; do
  QUICFEC_RESIDENT=0 timeout -k 10 120 ./quic-test_amd/lib/batcher_latency legacy_raw 5000 > "$E/legacy_coalescer_$i.json"
  cat "$E/legacy_coalescer_$i.json"
done
QUICFEC_RESIDENT=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$E/prof_legacy_coalescer" -o run --output-format csv -- \
  ./quic-test_amd/lib/batcher_latency legacy_raw 5000 > "$E/prof_legacy_coalescer.json" 2> "$E/prof_legacy_coalescer.err"
cat "$E/prof_legacy_coalescer.json"
timeout -k 10 400 python -u scripts/probe_recover_delta.py --alloc contiguous > "$E/delta_contiguous.jsonl"
cat "$E/delta_contiguous.jsonl"
timeout -k 10 400 python -u scripts/probe_recover_delta.py --alloc torch > "$E/delta_torch.jsonl"
cat "$E/delta_torch.jsonl"
# the one-launch tile recover with the next group's loads in flight
# (kRunPipe), dense (C3: several groups per wave) and sparse (C5), against the library's forms
timeout -k 10 300 ./quic-test_amd/lib/probe_runs 1000000 7 0 > "$E/probe_runs_c3.txt" 2>&1
tail -25 "$E/probe_runs_c3.txt"
timeout -k 10 300 ./quic-test_amd/lib/probe_runs 1000000 9 0.01 > "$E/probe_runs_c5.txt" 2>&1
tail -25 "$E/probe_runs_c5.txt"
