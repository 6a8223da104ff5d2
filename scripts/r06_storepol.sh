#!/usr/bin/env bash
# tools/probe_storepol.hip on the box: the encode's memory replica under each cache policy, next to
# the product encode and the 16-B copy, two processes; into gpurun_out/${EVID}/.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r06s}"
mkdir -p "$E"
# built here, not by the csrc Makefile (the Makefile is part of the library's source hash)
cd "$ROOT/quic-test_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I. -o ../lib/probe_storepol tools/probe_storepol.hip \
  -L../lib -lfec_hip -Wl,-rpath,'$ORIGIN' > "$E/build.log" 2>&1
cd "$ROOT"
for i in 1 2; do
  timeout -k 10 240 "$ROOT/quic-test_amd/lib/probe_storepol" 1000000 5 10 > "$E/storepol_$i.jsonl" 2>&1
done
echo "storepol: 2 processes"
