#!/usr/bin/env bash
# Round 6's final-build evidence in one gpurun call: scripts/r06_evidence.sh parts 1 and 2 into
# gpurun_out/${EVID}/, then the placement probe (tools/probe_placement.cpp) in three processes.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
PART=1 bash scripts/r06_evidence.sh
PART=2 bash scripts/r06_evidence.sh
E="$ROOT/gpurun_out/${EVID:-r06}/placement"
mkdir -p "$E"
(cd quic-test_amd/csrc && g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I../../include -I/opt/rocm/include \
   -o ../lib/probe_placement tools/probe_placement.cpp -L../lib -lfec_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN')
for i in 1 2 3; do
  timeout -k 10 150 quic-test_amd/lib/probe_placement > "$E/process$i.jsonl" 2>&1
done
echo "placement probe: 3 processes"
