#!/usr/bin/env bash
# Round 5, part W: a long soak of the final build's resident encoder at its production tag epoch
# (32,768 laps): 16 streams for 120 s (~140 M calls, ~130 k laps of every slot: four epochs with
# real scrubs), then 100 streams for 40 s -- every repair checked against the AVX2 XOR.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05w}"
mkdir -p "$E"
cd "$ROOT"
B=./quic-test_amd/lib/batcher_latency
timeout -k 10 200 $B legacy 16 0 120 > "$E/soak16.json"
cat "$E/soak16.json"
timeout -k 10 100 $B legacy 100 0 40 > "$E/soak100.json"
cat "$E/soak100.json"
