#!/usr/bin/env bash
# Round 5, part K: the staged encodes' cache policy (QUICFEC_ENCODE_MEMPOL: nt stores / plain /
# nt loads + nt stores / nt loads + plain), one process, interleaved; then the host code under
# AddressSanitizer and ThreadSanitizer (scripts/asan_host.sh: the mirror suite, 16 legacy streams
# on every path, the mixed shapes, and round 5's ring hooks and poisoning).
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05k}"
mkdir -p "$E"
cd "$ROOT"
timeout -k 10 600 python -u scripts/sweep_encode_tiles.py --configs c2pol,c4pol > "$E/sweep_mempol.jsonl"
cat "$E/sweep_mempol.jsonl"
bash scripts/asan_host.sh run > "$E/asan_host.log" 2>&1 || { echo "asan rc=$?"; tail -30 "$E/asan_host.log"; exit 1; }
grep -c '^{' "$E/asan_host.log"; grep -E "PASS|ERROR|SUMMARY" "$E/asan_host.log" | head -5
SAN=thread bash scripts/asan_host.sh run > "$E/tsan_host.log" 2>&1 || { echo "tsan rc=$?"; tail -30 "$E/tsan_host.log"; exit 1; }
grep -E "PASS|WARNING: ThreadSanitizer|SUMMARY" "$E/tsan_host.log" | head -5 || true
# the other compile-time encodes staged (k=10 r=1 -- the reference's XOR row -- k=10 r=2, k=4 r=2)
timeout -k 10 400 python -u scripts/ab_stage_rows.py --configs k10r1,k10r2,k4r2 > "$E/ab_stage_rows_other.jsonl"
cat "$E/ab_stage_rows_other.jsonl"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coalesce.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/parity_coalesce.log" 2>&1 || { tail -40 "$E/parity_coalesce.log"; exit 1; }
tail -1 "$E/parity_coalesce.log"
