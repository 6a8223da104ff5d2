#!/usr/bin/env bash
# Round 4, evidence part A (one gpurun call): the GPU suite and smoke on this build, then the
# exit path under the profiler -- the legacy call site (batcher_latency legacy_raw: resident
# encoder with its VRAM ring and with the page-locked ring, and the shared-launch path) and tests/csrc/exit_path_test run under rocprofv3 --kernel-trace --stats,
# each of which must exit 0 (the round-3 abort, f13ed47, was a HIP call after the profiler had
# finalised).  Everything lands in gpurun_out/${EVID:-r04}/.  Any failure ends the script.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r04}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > "$E/pytest_gpu.log" 2>&1 || { tail -40 "$E/pytest_gpu.log"; exit 1; }
tail -1 "$E/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$E/smoke.log" 2>&1
tail -1 "$E/smoke.log"
for m in resident hostring coalescer; do
  case $m in resident) e="QUICFEC_RESIDENT=1";; hostring) e="QUICFEC_RESIDENT_VRAM=0";; *) e="QUICFEC_RESIDENT=0";; esac
  env $e timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$E/prof_legacy_$m" -o run --output-format csv -- \
    ./quic-test_amd/lib/batcher_latency legacy_raw 5000 > "$E/prof_legacy_$m.json" 2> "$E/prof_legacy_$m.err"
  echo "legacy_raw $m under rocprofv3: exit 0"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$E/prof_exit_path" -o run --output-format csv -- \
  ./quic-test_amd/lib/exit_path_test resident 300 > "$E/prof_exit_path.json" 2> "$E/prof_exit_path.err"
cat "$E/prof_exit_path.json"
