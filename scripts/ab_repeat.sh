#!/usr/bin/env bash
# The same bench in separate processes on one box: per-process spread of the kernel times.
set -euo pipefail
for i in 1 2 3 4 5 6; do
  for v in "--no-verify" ""; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $v > /tmp/abr.json 2>/dev/null
    python -c "import json; d=json.load(open('/tmp/abr.json')); k=d['kernels']; print('run $i ${v:-verify}', 'value', d['value'], {n: (v['ms'], v['isolated']['ms_median'], v.get('other_api', {}).get('ms_median')) for n, v in k.items()})"
  done
done
