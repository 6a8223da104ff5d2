#!/usr/bin/env bash
# Round 6 A/Bs on one box: the C5 decode-form A/B in the bench's step (scripts/ab_c5_api.sh),
# then the C3 recover placement probe (tools/probe_placement.cpp, three processes).
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r06b}"
mkdir -p "$E"
cd "$ROOT"
EVID="$(basename "$E")" ROUNDS="${ROUNDS:-3}" bash scripts/ab_c5_api.sh
(cd quic-test_amd/csrc && g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I../../include -I/opt/rocm/include \
   -o ../lib/probe_placement tools/probe_placement.cpp -L../lib -lfec_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN')
for i in 1 2 3; do
  timeout -k 10 150 quic-test_amd/lib/probe_placement > "$E/placement_$i.jsonl" 2>&1
done
echo "placement probe: 3 processes"
