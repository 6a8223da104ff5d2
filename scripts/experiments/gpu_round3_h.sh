# resident store A/B on one box: plain stores + release fence (0) vs system-coherent stores + vmcnt (1)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=./quic-test_amd/lib/batcher_latency
for rep in 1 2; do
  for sm in 0 1; do
    QUICFEC_RESIDENT_STORE=$sm QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy_raw 20000 > gpurun_out/h.json 2> gpurun_out/h.err || exit 1
    echo "store=$sm raw $(python3 -c "import json; d=json.load(open('gpurun_out/h.json')); print(d['delay_us']['p50'], d['errors'])") $(grep -o '"us": {[^}]*}' gpurun_out/h.err)"
    QUICFEC_RESIDENT_STORE=$sm QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy 16 0 2 > gpurun_out/h.json 2> gpurun_out/h.err || exit 1
    echo "store=$sm s16 $(python3 -c "import json; d=json.load(open('gpurun_out/h.json')); print(int(d['groups_per_s']), d['delay_us']['p50'], d['errors'])") $(grep -o '"us": {[^}]*}' gpurun_out/h.err)"
  done
done
