#!/usr/bin/env bash
# Per-call latency of the host-resident C-ABI at small batches (tools/latency.cpp), with the
# zero-copy small-call path off (0), at its defaults (64 MiB page-locked, 2 MiB staged) and
# for every size (1e12).
# Usage (GPU box): bash scripts/latency_sweep.sh > gpurun_out/latency.txt
set -euo pipefail
for t in ${THRESHOLDS:-0 default 1000000000000}; do
  echo "== QUICFEC_SMALL_CALL_BYTES=$t"
  if [ "$t" = default ]; then unset QUICFEC_SMALL_CALL_BYTES; else export QUICFEC_SMALL_CALL_BYTES=$t; fi
  timeout -k 10 200 quic-test_amd/lib/latency "${CALLS:-200}" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['api'][:40].ljust(40), d['host_memory'].ljust(8), str(d['groups']).rjust(6),
          'median_us', d.get('median_us'), 'p99_us', d.get('p99_us'), 'GiB/s', d.get('payload_GiBps'))
"
done
