#!/usr/bin/env bash
# Round 5, part B: (1) the gfx950 counter list; (2) staged parity rows A/B on a second box;
# (3) the call site, round-4 library (lib/old: one tag word per 16-B chunk) vs this one (two
# tagged 8-B halves, epochs), alternating on one box; (4) one raw per-instance TCC counter over
# the placement probe, to see how rocprofv3 reports instances; (5) the default bench line.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05b}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 120 rocprofv3 -L > "$E/counters.txt" 2>&1 || echo "rocprofv3 -L rc=$?"
timeout -k 10 300 python -u scripts/ab_stage_rows.py > "$E/ab_stage_rows.jsonl"
cat "$E/ab_stage_rows.jsonl"
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
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ -d "$E/pmc_inst" -o run --output-format csv -- \
  python3 scripts/probe_recover_placement.py --trials 2 --reps 3 > "$E/pmc_inst.jsonl" 2> "$E/pmc_inst.err" || { echo "pmc rc=$?"; tail -5 "$E/pmc_inst.err"; }
timeout -k 10 600 python -u bench.py > "$E/bench_default.json" 2> "$E/bench_default.err"
python - "$E/bench_default.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["kernels"]
print("value", d["value"], "encode", k["encode"]["ms"], "decode", k["decode"]["ms"], "frac", d["roofline"]["frac"],
      "traffic", d["roofline"]["traffic"], "wall", d.get("wall_s"))
PY
