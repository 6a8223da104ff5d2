#!/usr/bin/env bash
# Encode k=10 r=3 1200 B: groups per workgroup (QUICFEC_ENCODE_TILE) x workgroups per CU
# (QUICFEC_ENCODE_BLOCKS), alternating runs in one box.  "tile blocks" pairs; waves/CU = blocks x ceil(75 tile / 64).
set -euo pipefail
for rd in 1 2; do
  for tb in "4 2" "3 2" "3 3" "2 4" "5 2" "6 1" "6 2" "2 5" "1 8"; do
    set -- $tb
    QUICFEC_ENCODE_TILE=$1 QUICFEC_ENCODE_BLOCKS=$2 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify > /tmp/abt.json
    python -c "import json; d=json.load(open('/tmp/abt.json')); print('tile $1 blocks $2', d['kernels']['encode']['ms'], d['kernels']['encode']['achieved_GBps'])"
  done
done
