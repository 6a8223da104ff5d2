#!/usr/bin/env bash
# Round 6 quick check on the GPU box: the GPU suite (both libraries), smoke, and the C3 recover
# placement probe (tools/probe_placement.cpp) in three processes.  Output in gpurun_out/${EVID}/.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r06a}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/pytest_gpu.log" 2>&1 || { tail -40 "$E/pytest_gpu.log"; exit 1; }
tail -1 "$E/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$E/smoke.log" 2>&1
tail -2 "$E/smoke.log"
if [ "${PROBE:-1}" = 1 ]; then
  (cd quic-test_amd/csrc && g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I../../include -I/opt/rocm/include \
     -o ../lib/probe_placement tools/probe_placement.cpp -L../lib -lfec_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN')
  for i in 1 2 3; do
    timeout -k 10 150 quic-test_amd/lib/probe_placement > "$E/placement_$i.jsonl" 2>&1
  done
  echo "placement probe: 3 processes"
fi
