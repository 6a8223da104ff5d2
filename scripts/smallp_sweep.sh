#!/usr/bin/env bash
# Recover (compact rows) vs in-place decode for small packets, device-resident, same box.
# Usage (GPU box): bash scripts/smallp_sweep.sh [k,r,P ...] > gpurun_out/smallp.txt
set -euo pipefail
SHAPES=${*:-"10,3,256 10,3,200 10,3,128 10,1,128 20,5,200 4,2,256 10,2,256 10,3,64"}
for S in $SHAPES; do
  IFS=, read -r K R P <<< "$S"
  G=$((6000000000 / (K * P)))
  for API in recover in-place; do
    printf "%s %s " "$S" "$API"
    timeout -k 10 120 python bench.py --config c2c3 --shape "$S" --groups "$G" --steps 10 --warmup 2 \
        --no-cpu-baseline --decode-api "$API" | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['kernels']; print(d['verified'], 'dec', e['decode']['ms'], e['decode']['achieved_GBps'])"
  done
done
