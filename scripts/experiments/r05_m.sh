#!/usr/bin/env bash
# Round 5, part M: the C3 slot recover's cache policy in the bench's own step (encode then
# recover), alternating on one box: QUICFEC_DECODE_MEMPOL 0 (NT loads + NT stores, the default),
# 1 (NT loads, plain stores), 2 (plain loads, NT stores), 3 (plain both).
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05m}"
mkdir -p "$E"
cd "$ROOT"
: > "$E/ab_decode_mempol.jsonl"
for rep in 1 2 3; do
  for v in 0 1 2 3; do
    line=$(QUICFEC_DECODE_MEMPOL=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-api 2>/dev/null | tail -1)
    python -c "import json,sys; d=json.loads(sys.argv[1]); k=d['kernels']; print(json.dumps({'mempol': $v, 'value': d['value'], 'encode_ms': k['encode']['ms'], 'decode_ms': k['decode']['ms'], 'decode_isolated_ms': k['decode']['isolated']['ms_median'], 'verified': d['verified']}))" "$line" >> "$E/ab_decode_mempol.jsonl"
  done
done
cat "$E/ab_decode_mempol.jsonl"
