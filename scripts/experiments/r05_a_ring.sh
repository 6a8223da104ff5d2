#!/usr/bin/env bash
# Round 5, part A (one gpurun call): the resident ring's per-8-B tags, epoch scrubs and poisoning
# (ADVICE r04), then the whole GPU suite, smoke (prints the library's source
# hash), and the default bench line (its call_site section: raw call p50 and 16 streams against
# round 4's 6.98 us / 0.849 M groups/s).  Everything lands in gpurun_out/r05a/.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05a}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/coalesce.log" 2>&1 || { tail -60 "$E/coalesce.log"; exit 1; }
tail -1 "$E/coalesce.log"
for m in tear epoch epoch_hostring poison_mt; do
  n=300; case $m in epoch*) n=6144;; poison_mt) n=2400;; esac
  timeout -k 10 120 ./quic-test_amd/lib/exit_path_test $m $n > "$E/exit_$m.json"
  tail -1 "$E/exit_$m.json"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/pytest_gpu.log" 2>&1 || { tail -40 "$E/pytest_gpu.log"; exit 1; }
tail -1 "$E/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$E/smoke.log" 2>&1
tail -2 "$E/smoke.log"
timeout -k 10 600 python -u bench.py > "$E/bench_default.json" 2> "$E/bench_default.err"
python - "$E/bench_default.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
cs = d.get("call_site", {})
print("value", d["value"], "frac", d["roofline"]["frac"], "call_site raw", cs.get("raw"), "s16", cs.get("streams_16"))
PY
# staged parity rows, A/B in one process, then write counters per mode
timeout -k 10 300 python -u scripts/ab_stage_rows.py > "$E/ab_stage_rows.jsonl"
cat "$E/ab_stage_rows.jsonl"
for st in 0 1; do
  QUICFEC_ENCODE_STAGE=$st PMC_TAG="/r05a_stage$st" PMC_CONFIGS="c2c3 c4" \
    PMC_GROUPS="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum;WRITE_SIZE" timeout -k 10 600 bash scripts/pmc_passes.sh > "$E/pmc_stage$st.log" 2>&1 || { tail -20 "$E/pmc_stage$st.log"; exit 1; }
done
