#!/usr/bin/env bash
# The C3 recover's occupancy against buffer placement (tools/probe_placement.cpp --waves, built
# against the test library whose QUICFEC_DECODE_WAVES caps the recover's waves per CU), two
# processes, into gpurun_out/${EVID}/.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r06w}"
mkdir -p "$E"
cd "$ROOT/quic-test_amd/csrc"
g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I../../include -I/opt/rocm/include -o ../lib/probe_placement_hooks \
  tools/probe_placement.cpp -L../lib -lfec_hip_test -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN'
cd "$ROOT"
for i in 1 2; do
  timeout -k 10 200 quic-test_amd/lib/probe_placement_hooks --waves --skip-delta > "$E/waves_process$i.jsonl" 2>&1
done
echo "waves sweep: 2 processes"
