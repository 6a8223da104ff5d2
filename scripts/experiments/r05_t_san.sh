#!/usr/bin/env bash
# Round 5, part T: the final build's host code under AddressSanitizer and ThreadSanitizer
# (scripts/asan_host.sh: the mirror suite, 16 legacy streams on every path, the mixed shapes, the
# ring's tag hooks, poisoning under 8 threads, relaunch cycles with 8 serving classes).
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r05t}"
mkdir -p "$E"
cd "$ROOT"
bash scripts/asan_host.sh run > "$E/asan_host.log" 2>&1 || { echo "asan rc=$?"; tail -30 "$E/asan_host.log"; exit 1; }
grep -c '^{' "$E/asan_host.log"; grep -E "PASS|ERROR|SUMMARY" "$E/asan_host.log" | head -5 || true
SAN=thread bash scripts/asan_host.sh run > "$E/tsan_host.log" 2>&1 || { echo "tsan rc=$?"; tail -30 "$E/tsan_host.log"; exit 1; }
grep -c '^{' "$E/tsan_host.log"; grep -E "PASS|WARNING: ThreadSanitizer|SUMMARY" "$E/tsan_host.log" | head -5 || true
