#!/usr/bin/env bash
# Shared-batcher repair delay and throughput (quic-test_amd/lib/batcher_latency) at the
# reference's call pattern: 1 / 10 / 100 streams x 100 packets/s, and saturating streams.
# One JSON object per line on stdout.  GPU box: bash scripts/batcher_sweep.sh > gpurun_out/batcher.jsonl
set -euo pipefail
B=./quic-test_amd/lib/batcher_latency
T="timeout -k 10 60"
$T $B cpu
$T $B single 2000
for r in 1 3; do
  for s in 1 10 100; do
    $T $B paced $s 100 5 $r 1000
  done
  $T $B paced 100 100 5 $r 200
  $T $B paced 100 100 5 $r 0
done
for r in 1 3; do
  $T $B saturate 16 3 $r 1000 4096
  $T $B saturate 16 3 $r 1000 512
done
