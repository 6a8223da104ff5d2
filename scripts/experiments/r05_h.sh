#!/usr/bin/env bash
# Round 5, part H: the staged encodes' workgroup shape (tile x occupancy), swept in one process
# (scripts/sweep_encode_tiles.py), then the staged-rows GPU tests.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05h}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 600 python -u scripts/sweep_encode_tiles.py > "$E/sweep_encode_tiles.jsonl"
cat "$E/sweep_encode_tiles.jsonl"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bits.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/bits.log" 2>&1 || { tail -40 "$E/bits.log"; exit 1; }
tail -1 "$E/bits.log"
