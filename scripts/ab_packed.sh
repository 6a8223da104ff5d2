#!/usr/bin/env bash
# Packed vs slot recover rows in the bench (C3 dense, C5 sparse), alternating runs on one box.
set -euo pipefail
for rd in 1 2; do
  for cfg in c2c3 c5; do
    for api in packed recover; do
      timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-verify --decode-api $api > /tmp/abpk.json 2>/dev/null
      python -c "import json; d=json.load(open('/tmp/abpk.json')); k=d['kernels']['decode']; print('$cfg $api', 'value', d['value'], 'decode', k['ms'], k['isolated']['ms_median'])"
    done
  done
done
