#!/usr/bin/env bash
# Round 5, part I: C4's staged encode under occupancy caps (second box), and the C5 tile
# recover's store policy by path (image copy-out vs rows past the image) and image size.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05i}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 600 python -u scripts/sweep_encode_tiles.py --configs c4 > "$E/sweep_encode_tiles_c4.jsonl"
cat "$E/sweep_encode_tiles_c4.jsonl"
timeout -k 10 300 ./quic-test_amd/lib/probe_runs 1000000 9 0.01 > "$E/probe_runs_c5.txt" 2>&1
tail -20 "$E/probe_runs_c5.txt"
