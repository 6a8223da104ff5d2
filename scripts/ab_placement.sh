#!/usr/bin/env bash
# Buffer placement A/B: decode time vs the rebuilt buffer's offset from an allocation start
# (parity row g and rebuilt row g share the same stride), each offset in several processes.
set -euo pipefail
for rd in 1 2 3; do
  for off in 0 4096 65536 300000 1048576 1200; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify --rebuilt-offset $off > /tmp/abp.json 2>/dev/null
    python -c "import json; d=json.load(open('/tmp/abp.json')); k=d['kernels']; print('rebuilt-offset $off', 'value', d['value'], {n: (v['ms'], v['isolated']['ms_median']) for n, v in k.items()})"
  done
done
