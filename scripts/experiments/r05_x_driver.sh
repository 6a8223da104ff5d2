#!/usr/bin/env bash
# Round 5, part X: the driver's round-end sequence on the final tree: the GPU suite, smoke, and
# the default bench line.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05x}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > "$E/pytest_gpu.log" 2>&1 || { tail -60 "$E/pytest_gpu.log"; exit 1; }
tail -1 "$E/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$E/smoke.log" 2>&1 || { tail -30 "$E/smoke.log"; exit 1; }
tail -2 "$E/smoke.log"
timeout -k 10 600 python bench.py > "$E/bench.json" 2> "$E/bench.err" || { tail -30 "$E/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$E/bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['call_site']['streams_16']['groups_per_s'])"
