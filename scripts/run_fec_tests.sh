#!/usr/bin/env bash
# FEC campaign over BASELINE.json's configs, for the MI355X engine.
#
# The reference's scripts/run_fec_tests.sh drives ./bin/quic-test runs with FEC levels on
# the mobile / satellite network profiles (its --fec flag is a bool, main.go:49, and the
# binary path does not exist in the snapshot: SURVEY.md §2).  This campaign measures the
# FEC engine itself on the same loss profiles:
#
#   C1  k=4 r=2, 256 B, 1k groups      host CPU only (the CPU checker, plumbing; no GPU)
#   C2  k=10 r=3, 1200 B, 1M groups    encode, device-resident           } bench.py c2c3
#   C3  same, 2 erasures per group      decode, bit-exact vs the original }
#   C4  k=20 r=5, 1200 B, 1M groups per GPU, encode                         bench.py c4
#   C5  k=10 r=3, 1200 B, satellite loss p=0.01 (and mobile p=0.05),
#       encode + decode, also timed host-resident with pinned H2D/D2H       bench.py c5 --e2e
#
# usage: scripts/run_fec_tests.sh [--gpus N] [--cpu-only] [--out DIR]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
GPUS=1
CPU_ONLY=0
OUT="$ROOT/gpurun_out/fec_campaign"
while [ $# -gt 0 ]; do
  case "$1" in
    --gpus) GPUS="$2"; shift 2 ;;
    --cpu-only) CPU_ONLY=1; shift ;;
    --out) OUT="$2"; shift 2 ;;
    *) echo "unknown argument $1" >&2; exit 2 ;;
  esac
done
mkdir -p "$OUT"
cd "$ROOT"

echo "== build"
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1

echo "== C1 (host CPU, k=4 r=2, 256 B, 1k groups)"
python - <<'EOF' | tee "$OUT/c1.json"
import json, sys, time
sys.path.insert(0, "oracle")
import numpy as np, oracle
k, r, P, G = 4, 2, 256, 1024
d = oracle.splitmix_bytes(G * k * P, 0x5EED0001)
t0 = time.perf_counter(); par = oracle.rs_encode(d, G, k, r, P); t = time.perf_counter() - t0
row0 = par.reshape(G, r, P)[:, 0, :].reshape(-1)
xr = np.concatenate([oracle.xor_packets([d[(g*k+j)*P:(g*k+j+1)*P] for j in range(k)], P) for g in range(G)])
ref = oracle.ref_lib()
print(json.dumps({"config": "C1", "k": k, "r": r, "P": P, "groups": G, "encode_GiBps": round(G*k*P/t/2**30, 3),
                  "row0_equals_xor": bool((row0 == xr).all()), "reference_lib_present": ref is not None}))
EOF
[ "$CPU_ONLY" = "1" ] && exit 0

run_bench() {
  local tag="$1"; shift
  echo "== $tag (gpus=$GPUS)"
  if [ "$GPUS" -gt 1 ]; then
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$GPUS" \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$GPUS" "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  else
    timeout -k 10 900 python bench.py "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  fi
  cat "$OUT/$tag.json"
}
run_bench c2c3 --config c2c3 --steps 30 --warmup 5
run_bench c4 --config c4 --steps 30 --warmup 5 --no-cpu-baseline
run_bench c5_satellite --config c5 --steps 30 --warmup 5 --no-cpu-baseline --e2e
run_bench c5_mobile --config c5 --loss 0.05 --steps 30 --warmup 5 --no-cpu-baseline --e2e
