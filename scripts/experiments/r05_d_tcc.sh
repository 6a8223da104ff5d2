#!/usr/bin/env bash
# Round 5, part D: per-TCC-channel DRAM request and credit-stall counters of
# the C3 recover into fast and slow rebuilt buffers (scripts/probe_recover_placement.py: several
# torch buffers, plain hipMalloc and physically contiguous ones in one process), one base
# counter per rocprofv3 pass, its 16 instances as derived counters (scripts/pmc_tcc_instances.py).
set -uo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05d}"
mkdir -p "$E"
cd "$ROOT"
DEFS="$E/tccdefs"
i=0
python3 scripts/pmc_tcc_instances.py defs "$DEFS" TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_DRAM > "$E/passes.txt"
echo "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum" >> "$E/passes.txt"
while read -r counters; do
  i=$((i + 1))
  echo "== pass $i: ${counters%% *} ..."
  ROCPROFILER_METRICS_PATH="$DEFS" timeout -s KILL 150 rocprofv3 --pmc $counters -d "$E/p$i" -o run --output-format csv -- \
    python3 scripts/probe_recover_placement.py --trials 2 --reps 2 > "$E/p$i.jsonl" 2> "$E/p$i.err"
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$E/p$i.err"; exit 1; fi
  f=$(find "$E/p$i" -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_tcc_instances.py summary "$f" > "$E/p${i}_summary.jsonl"
  head -3 "$E/p${i}_summary.jsonl" | cut -c1-400
done < "$E/passes.txt"
