#!/usr/bin/env bash
# Shared-batcher repair delay and throughput (quic-test_amd/lib/batcher_latency) at the
# reference's call pattern: 1 / 10 / 100 streams x 100 packets/s, and saturating streams.
# One JSON object per line on stdout.  GPU box: bash scripts/batcher_sweep.sh > gpurun_out/batcher.jsonl
set -euo pipefail
B=./quic-test_amd/lib/batcher_latency
T="timeout -k 10 60"
# a run that reports errors exits 1 after printing its line; keep going (a hang still ends it)
run() { "$@" || [ $? -eq 1 ]; }
run $T $B cpu
run $T $B single 2000
for r in 1 3; do
  for s in 1 10 100; do
    run $T $B paced $s 100 5 $r 1000
  done
  run $T $B paced 100 100 5 $r 200
  run $T $B paced 100 100 5 $r 0
done
for r in 1 3; do
  run $T $B saturate 16 3 $r 1000 4096
  run $T $B saturate 16 3 $r 1000 512
done
# the C-ABI alone (submit by pointers, collect by ticket), 1024 groups outstanding per stream
for s in 1 4 8 16; do
  run $T $B raw $s 2 1 1000 4096 1024
done
run $T $B raw 16 2 3 1000 4096 1024
# the decoder batcher (receivers' recoveries shared across connections), every packet checked
for s in 1 4 8 16; do
  run $T $B decode $s 2 3 1000 4096 1024
done
run $T $B decode 16 2 1 1000 4096 1024
