#!/usr/bin/env bash
# Timing-setup A/B: kernels and events on one torch stream (default) vs stream handle 0
# (--null-stream: kernels on the context's stream, events on torch's default stream).
set -euo pipefail
for rd in 1 2; do
  for cfg in c2c3 c5; do
    for mode in "" "--null-stream"; do
      timeout -k 10 200 python bench.py --config $cfg --steps 20 --no-cpu-baseline $mode > /tmp/abs.json 2>/dev/null
      python -c "import json; d=json.load(open('/tmp/abs.json')); k=d['kernels']; print('$cfg', '${mode:-one-stream}', 'value', d['value'], 'ms_per_step', d['ms_per_step'], {n: (v['ms'], v['isolated']['ms_median']) for n, v in k.items()}, 'verified', d['verified'])"
    done
  done
done
