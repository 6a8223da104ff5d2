#!/usr/bin/env bash
# Round 5, part J: the new defaults in the bench's own legs, alternating in one box: C5's tile
# recover with plain vs non-temporal row stores (QUICFEC_RUNS_NT_STORE), C4's staged encode at 2
# workgroups per CU vs uncapped (QUICFEC_ENCODE_WAVES=0); then the packed / bits GPU tests.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05j}"
mkdir -p "$E"
cd "$ROOT"
: > "$E/ab_legs.jsonl"
for rep in 1 2 3; do
  for v in 0 1; do
    line=$(QUICFEC_RUNS_NT_STORE=$v timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-other-api 2>/dev/null | tail -1)
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'leg': 'c5', 'nt_store': $v, 'decode_ms': d['kernels']['decode']['ms'], 'encode_ms': d['kernels']['encode']['ms'], 'verified': d['verified']}))" "$line" >> "$E/ab_legs.jsonl"
  done
  for w in default 0; do
    if [ $w = default ]; then line=$(timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline 2>/dev/null | tail -1)
    else line=$(QUICFEC_ENCODE_WAVES=0 timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline 2>/dev/null | tail -1); fi
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'leg': 'c4', 'waves': '$w', 'encode_ms': d['kernels']['encode']['ms'], 'verified': d['verified']}))" "$line" >> "$E/ab_legs.jsonl"
  done
done
cat "$E/ab_legs.jsonl"
timeout -k 10 400 python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_bits.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/packed_bits.log" 2>&1 || { tail -40 "$E/packed_bits.log"; exit 1; }
tail -1 "$E/packed_bits.log"
