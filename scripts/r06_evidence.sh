#!/usr/bin/env bash
# Round 6 evidence on the current build, in two gpurun calls (PART=1: A-C, PART=2: D, PART=3: D
# without PMC; everything in gpurun_out/${EVID}/):
#  A. the GPU suite and smoke (prints the library's source hash against the tree's);
#  B. the legacy call site and the exit-path program under rocprofv3 (each must exit 0);
#  C. a soak of the resident ring (16 and 100 streams, every repair
#     checked) and a 12,000-case random sweep against the oracle;
#  D. PMC traffic per config on this build (copied into profiles/ so the benches read this
#     build's bytes), rocprofv3 kernel statistics of the default bench, the default bench line as
#     the driver runs it, and the other configs' legs.
# Any failure ends the script.
set -euo pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
E="$ROOT/gpurun_out/${EVID:-r06}"
mkdir -p "$E"
cd "$ROOT"
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$E/pytest_gpu.log" 2>&1 || { tail -40 "$E/pytest_gpu.log"; exit 1; }
tail -1 "$E/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$E/smoke.log" 2>&1
tail -2 "$E/smoke.log"
for m in resident hostring coalescer; do
  case $m in resident) e="QUICFEC_RESIDENT=1";; hostring) e="QUICFEC_RESIDENT_VRAM=0";; *) e="QUICFEC_RESIDENT=0";; esac
  env $e timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$E/prof_legacy_$m" -o run --output-format csv -- \
    ./quic-test_amd/lib/batcher_latency legacy_raw 5000 > "$E/prof_legacy_$m.json" 2> "$E/prof_legacy_$m.err"
  echo "legacy_raw $m under rocprofv3: exit 0"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$E/prof_exit_path" -o run --output-format csv -- \
  ./quic-test_amd/lib/exit_path_test resident 300 > "$E/prof_exit_path.json" 2> "$E/prof_exit_path.err"
tail -1 "$E/prof_exit_path.json"
B=./quic-test_amd/lib/batcher_latency
timeout -k 10 90 $B legacy 16 0 30 > "$E/soak.jsonl" 2>&1
timeout -k 10 90 $B legacy 100 0 20 >> "$E/soak.jsonl" 2>&1
grep '^{' "$E/soak.jsonl" | cut -c1-200
QUICFEC_FUZZ_SEED=0x5EED5000 QUICFEC_FUZZ_BLOCKS=1200 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > "$E/fuzz_12000.log" 2>&1 || { tail -20 "$E/fuzz_12000.log"; exit 1; }
tail -1 "$E/fuzz_12000.log"
exit 0
fi
# PART=3: D on another box without the PMC passes (profiles/pmc_*.json stay as they are)
if [ "${PART}" != 3 ]; then
CFGS="${PMC_CFGS:-c2c3 c5 c4}" bash scripts/gpu_pmc.sh > "$E/pmc.log" 2>&1
for c in ${PMC_CFGS:-c2c3 c5 c4}; do cp "$ROOT/gpurun_out/pmc_$c.json" "$ROOT/profiles/pmc_$c.json"; cp "$ROOT/gpurun_out/pmc_$c.json" "$E/pmc_$c.json"; done
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$E/prof" -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$E/prof_bench.json" 2> "$E/prof_bench.err"
find "$E/prof" -name "*kernel_stats.csv" -exec cp {} "$E/kernel_stats.csv" \;
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$E/bench.json" 2> "$E/bench.err"
python -c "import json; d=json.loads(open('$E/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'], d['cpu_baseline']['value'], d['call_site']['raw'], d['call_site']['streams_16'], d['call_site'].get('batcher_16_r1'), d['call_site'].get('batcher_16_r3'), d['wall_s'])"
mkdir -p "$E/legs"
T="timeout -k 10 300"
$T python bench.py --config c4 --no-cpu-baseline > "$E/legs/c4.json" 2> /dev/null
$T python bench.py --config c5 --e2e --no-cpu-baseline > "$E/legs/c5_satellite.json" 2> /dev/null
for f in "$E"/legs/*.json; do
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); k=d['kernels']; print('$f'.split('/')[-1], d['value'], d['verified'], {n: (v['ms'], v['achieved_GBps']) for n, v in k.items()}, d['roofline']['frac'], d['roofline']['traffic'])"
done
# the --gpus 2 rehearsal (two gloo ranks sharing the card) at the driver's default sizes: every
# section verified, traffic from this build's PMC (1M groups per rank = the PMC workload), wall_s
QUICFEC_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 > "$E/bench_gpus2_gloo_rehearsal.json" 2> "$E/bench_gpus2.err"
python -c "import json; d=json.loads(open('$E/bench_gpus2_gloo_rehearsal.json').read().strip().splitlines()[-1]); print('gpus2', d['n_gpus'], d['value'], d['verified'], d['roofline']['traffic'], d.get('wall_s'), {s: (d[s]['ranks'], d[s]['value'], d[s]['verified'], d[s]['roofline']['traffic']) for s in ('c4', 'c5_e2e')})"
