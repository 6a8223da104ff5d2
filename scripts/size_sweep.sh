#!/usr/bin/env bash
# Packet-size sweep of the device-resident kernels at k=10 r=3 (~12 GB of data per size).
# Each line: P, verified, encode ms and algorithmic GB/s, decode (2 erasures/group) ms and GB/s.
# Usage (GPU box): bash scripts/size_sweep.sh [P ...] > gpurun_out/size_sweep.txt
set -euo pipefail
SIZES=${*:-"64 128 256 384 512 768 1024 1200 1201 1350 1400 1452 1472 1500 1800 2048"}
for P in $SIZES; do
  G=$((12000000000 / (10 * P)))
  printf "P=%s " "$P"
  timeout -k 10 120 python bench.py --config c2c3 --shape 10,3,"$P" --groups "$G" --steps 10 --warmup 2 \
      --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['kernels']; print(d['verified'], 'enc', e['encode']['ms'], e['encode']['achieved_GBps'], 'dec', e['decode']['ms'], e['decode']['achieved_GBps'])"
done
