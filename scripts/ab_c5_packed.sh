#!/usr/bin/env bash
# C5 (sparse loss) recover: packed vs slot rows x one wave per group vs 8 groups per wave.
set -euo pipefail
for rd in 1 2; do
  for api in packed recover; do
    for sc in 1 8; do
      QUICFEC_DECODE_SCAN=$sc timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-verify --decode-api $api > /tmp/abc5.json 2>/dev/null
      python -c "import json; d=json.load(open('/tmp/abc5.json')); k=d['kernels']['decode']; print('$api scan$sc', 'value', d['value'], 'decode', k['ms'], k['isolated']['ms_median'], round(k['achieved_GBps']))"
    done
  done
done
