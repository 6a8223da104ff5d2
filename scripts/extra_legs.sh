#!/usr/bin/env bash
# Extra device-resident bench legs on the current build (one JSON line each under gpurun_out/legs/):
# C4 encode, C4-shape 5-erasure decode, C5 satellite and mobile loss, and the reference's own
# computation (k=10 r=1: XOR row only) at C2 size.
set -euo pipefail
mkdir -p gpurun_out/legs
T="timeout -k 10 300"
$T python bench.py --config c4 --no-cpu-baseline > gpurun_out/legs/c4.json
$T python bench.py --config c4d --no-cpu-baseline > gpurun_out/legs/c4d.json
$T python bench.py --config c5 --no-cpu-baseline > gpurun_out/legs/c5_satellite.json
$T python bench.py --config c5 --loss 0.05 --no-cpu-baseline > gpurun_out/legs/c5_mobile.json
$T python bench.py --config c2c3 --shape 10,1,1200 --no-cpu-baseline > gpurun_out/legs/k10r1.json
for f in gpurun_out/legs/*.json; do
  python -c "import json,sys; d=json.load(open('$f')); k=d['kernels']; print('$f', d['value'], {n: (v['ms'], v['achieved_GBps']) for n, v in k.items()}, d['roofline']['frac'], d['roofline']['box_copy_GBps'])"
done
