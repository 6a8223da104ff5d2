#!/usr/bin/env python3
"""bench.py — device-resident FEC encode+decode throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2c3|c4]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

Workload (one "step" = one pass of the hot path over one batch):
  c2c3 (default; BASELINE.json configs[1] + configs[2]): per GPU 1,000,000 groups of
       k=10 data packets x 1200 B (12.0 GB resident in HBM).  A step encodes every group
       (r=3 parity rows) and then rebuilds every group with 2 erased shards (positions
       uniform over the 13 shards, seeded): fec_recover_batch_rs_dev returns the rebuilt
       packets back to back, as the reference decoder returns Recovered buffers
       (decoder.go:29-34); --decode-api in-place rebuilds them inside the data instead (both
       timed, the other one as kernels.decode.other_api).  value = payload GiB (k*P*G, all
       ranks) / step time: the rate at which data goes through encode AND decode.
  c4   (configs[3]): per GPU 1,000,000 groups of k=20 x 1200 B, r=5 encode only.

Multi-GPU: one process per GPU, each with its own contiguous range of the global group
stream; no data-path collective (groups are independent), a barrier and a MAX
all-reduce of the elapsed time only.  scaling = "weak".

Prints ONE JSON line on rank 0.  Extra keys: per-kernel timings ("kernels"), the HBM
roofline of the dominant kernel ("roofline") and the CPU baseline ("cpu_baseline",
rank 0 at N=1 only; the oracle restatement timed on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

T_START = time.monotonic()  # this process's start: the line's wall_s phases are measured from it

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "quic-test_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
SEED = 0x5EED0000

CONFIGS = {
    "c2c3": dict(k=10, r=3, P=1200, groups=1_000_000, erasures=2, decode=True,
                 workload="C2 encode + C3 decode: k=10 r=3, 1200 B packets, 1M groups/GPU, 2 erasures/group"),
    "c4": dict(k=20, r=5, P=1200, groups=1_000_000, erasures=0, decode=False,
               workload="C4 encode: k=20 r=5, 1200 B packets, 1M groups/GPU (8M over 8 GPUs)"),
    # k=20 r=5 with 5 erasures per group (the C4 shape's worst recoverable decode; evidence
    # config, not a BASELINE line)
    "c4d": dict(k=20, r=5, P=1200, groups=500_000, erasures=5, decode=True,
                workload="C4 shape encode + 5-erasure decode: k=20 r=5, 1200 B packets, 500k groups/GPU"),
    # satellite profile: iid loss 0.01 per packet (internal/network_profiles.go:78)
    "c5": dict(k=10, r=3, P=1200, groups=1_000_000, erasures=0, loss=0.01, decode=True,
               workload="C5 encode + decode, satellite loss (iid p=0.01 per shard): k=10 r=3, 1200 B, 1M groups/GPU"),
}


# ----------------------------------------------------------------------------- launch
def dist_backend() -> str:
    """RCCL ("nccl") unless QUICFEC_DIST_BACKEND overrides it (gloo: multi-rank rehearsal
    on a one-GPU box, where several ranks share the card)."""
    return os.environ.get("QUICFEC_DIST_BACKEND", "nccl")


def launch_plan(gpus: int, env) -> tuple[str, int]:
    """How this process runs `--gpus N`:
      ("run", W)   this process is one rank of W (WORLD_SIZE from torch.distributed.run, or
                   W = 1 for a plain single-GPU run);
      ("spawn", N) no WORLD_SIZE and N > 1: start N rank processes here (spawn_ranks).
    A WORLD_SIZE that disagrees with --gpus is an error, never silently one of the two."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    w = env.get("WORLD_SIZE")
    if w is not None and w != "":
        world = int(w)
        if world != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} disagrees with WORLD_SIZE={world} from the launcher")
        return "run", world
    return ("run", 1) if gpus == 1 else ("spawn", gpus)


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
VISIBLE_VARS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def visible_gpus(env=None, nodes: str = KFD_NODES) -> int:
    """Visible GPU count without loading the HIP runtime in this process: the KFD topology's
    GPU nodes (gpu_id != 0; CPU nodes have 0), narrowed by ROCR_/HIP_/CUDA_VISIBLE_DEVICES
    (each lists the devices the next layer sees; set but empty = none).  The spawning parent
    of `bench.py --gpus N` must stay off the GPU (its children bind their devices; a process
    that initialised the GPU must never fork-exec), so it never imports torch."""
    env = os.environ if env is None else env
    phys = None
    try:
        ids = []
        for nd in sorted(os.listdir(nodes)):
            try:
                ids.append(int(open(os.path.join(nodes, nd, "gpu_id")).read().split()[0]))
            except (OSError, ValueError, IndexError):
                pass
        phys = sum(1 for i in ids if i != 0)
    except OSError:
        pass
    n = phys
    for var in VISIBLE_VARS:
        v = env.get(var)
        if v is None:
            continue
        listed = len([x for x in v.split(",") if x.strip()])
        n = listed if n is None else min(n, listed)
    return n or 0


def hip_runtime_mapped() -> bool:
    """Whether this process has the HIP runtime (libamdhip64) mapped, e.g. through torch."""
    try:
        with open("/proc/self/maps") as f:
            return any("libamdhip64" in ln for ln in f)
    except OSError:
        return False


def bind_local_device(local: int, world: int, ndev: int) -> int:
    """The device of local rank `local`: one process per GPU.  Ranks beyond the visible
    devices are an error under RCCL; the gloo rehearsal shares the card (local % ndev)."""
    if ndev <= 0:
        raise SystemExit("bench.py: no GPU visible")
    if local < ndev:
        return local
    if dist_backend() == "gloo":
        return local % ndev
    raise SystemExit(f"bench.py: local rank {local} of {world} needs GPU {local}, only {ndev} visible")


def parse_cpulist(text: str) -> set:
    """CPUs of a sysfs cpulist ("0-7,16-23")."""
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def bind_host_to_gpu(local: int, sysfs: Path = Path("/sys/bus/pci/devices")) -> dict:
    """One rank of N > 1: confine this process's threads (and so the node its page-locked host
    buffers are allocated on) to the CPUs local to its GPU's PCIe link, as sysfs lists them, within
    the CPUs it may already use.  On a two-socket node half the GPUs hang off each socket; without
    this the host-resident legs (c5_e2e) of some ranks would read and write memory of the other
    socket across the inter-socket link.  Returns what was done (the line's `host_binding`)."""
    import torch
    p = torch.cuda.get_device_properties(local)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    out = {"gpu": local, "pci": bdf}
    try:
        cpus = parse_cpulist((sysfs / bdf / "local_cpulist").read_text())
        node = int((sysfs / bdf / "numa_node").read_text())
    except (OSError, ValueError):
        return {**out, "bound": False, "why": "no sysfs entry"}
    cur = set(os.sched_getaffinity(0))
    want = cpus & cur
    out.update({"numa_node": node, "local_cpus": len(want), "allowed_cpus": len(cur)})
    if not want or want == cur:
        return {**out, "bound": False, "why": "no local CPU allowed" if not want else "already local"}
    os.sched_setaffinity(0, want)
    return {**out, "bound": True}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str], check_devices: bool = True) -> int:
    """`bench.py --gpus N` run directly (no torch.distributed.run): start N rank processes
    of this script on 127.0.0.1, one per GPU, and return the worst exit code.  This parent
    makes no GPU call (children bind their device before RCCL init); only rank 0 prints."""
    import subprocess
    if hip_runtime_mapped():
        raise SystemExit("bench.py: the spawning parent has the HIP runtime loaded; it must make no GPU call")
    if check_devices and dist_backend() != "gloo":
        ndev = visible_gpus()
        if n > ndev:
            raise SystemExit(f"bench.py: --gpus {n} but only {ndev} GPU(s) visible")
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv], env=env))
    rc = 0
    try:
        for p in procs:
            code = p.wait()
            if code != 0 and rc == 0:
                rc = code
                for q in procs:          # a failed rank would leave the others in a collective
                    if q.poll() is None:
                        q.terminate()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 1


# ----------------------------------------------------------------------------- helpers
def shard_range(total_groups: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [g0, g1) slice of the global group stream owned by `rank`."""
    g0 = total_groups * rank // world
    g1 = total_groups * (rank + 1) // world
    return g0, g1


def reduce_max(x: float) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(x: float) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def reduce_min(x: float) -> float:
    return -reduce_max(-x)


def barrier() -> None:
    import torch
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def erasure_masks(G: int, n_shards: int, erasures: int, seed: int):
    """Exactly `erasures` distinct shards lost per group, uniform over n_shards."""
    import numpy as np
    rng = np.random.default_rng(seed)
    out = np.zeros(G, dtype=np.uint64)
    chunk = 1 << 18
    for c0 in range(0, G, chunk):
        c1 = min(G, c0 + chunk)
        pos = np.argsort(rng.random((c1 - c0, n_shards)), axis=1)[:, :erasures].astype(np.uint64)
        out[c0:c1] = np.left_shift(np.uint64(1), pos).sum(axis=1, dtype=np.uint64)
    return out


def iid_masks(G: int, n_shards: int, p: float, seed: int):
    """Every shard lost independently with probability p (network_profiles.go:73-82)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    out = np.zeros(G, dtype=np.uint64)
    chunk = 1 << 18
    w = np.left_shift(np.uint64(1), np.arange(n_shards, dtype=np.uint64))
    for c0 in range(0, G, chunk):
        c1 = min(G, c0 + chunk)
        lost = rng.random((c1 - c0, n_shards)) < p
        out[c0:c1] = (lost * w).sum(axis=1, dtype=np.uint64)
    return out


def make_masks(cfg: dict, G: int, seed: int):
    if cfg.get("loss"):
        return iid_masks(G, cfg["k"] + cfg["r"], cfg["loss"], seed)
    return erasure_masks(G, cfg["k"] + cfg["r"], cfg["erasures"], seed)


def unrecoverable_count(masks, k: int, r: int) -> int:
    """Groups with more lost data shards than surviving parity rows."""
    import numpy as np
    e = _popcount(masks & np.uint64((1 << k) - 1))
    lost_par = _popcount((masks >> np.uint64(k)) & np.uint64((1 << r) - 1))
    return int(((e > 0) & (e > r - lost_par)).sum())


def _popcount(x):
    import numpy as np
    c = np.zeros(len(x), dtype=np.int64)
    y = x.copy()
    while y.any():
        c += (y & np.uint64(1)).astype(np.int64)
        y >>= np.uint64(1)
    return c


def decode_algorithmic_bytes(masks, k: int, r: int, P: int, reads_only: bool = False) -> int:
    """Sum over groups with lost data shards of (k + e) * P (read k survivors, write e);
    reads_only: the k * P read part alone."""
    import numpy as np
    m = masks & np.uint64((1 << k) - 1)
    e = np.zeros(len(m), dtype=np.int64)
    mm = m.copy()
    while mm.any():
        e += (mm & np.uint64(1)).astype(np.int64)
        mm >>= np.uint64(1)
    pm = (masks >> np.uint64(k)) & np.uint64((1 << r) - 1)
    alive = np.full(len(m), r, dtype=np.int64)
    pp = pm.copy()
    while pp.any():
        alive -= (pp & np.uint64(1)).astype(np.int64)
        pp >>= np.uint64(1)
    ok = (e > 0) & (e <= alive)
    if reads_only:
        return int(ok.sum()) * k * P
    return int(((k + e[ok]) * P).sum())


def cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 quota (cpu.max), or None when unlimited/unknown."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) / int(period)))
    except (OSError, ValueError):
        pass
    return None


def host_threads() -> int:
    """Every core this process may run on: the sched_getaffinity set, bounded by the cgroup
    CPU quota when one is set (more threads than the quota only time-slice)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    q = cgroup_cpu_quota()
    return max(1, min(aff, q) if q else aff)


def _rate(fn, nbytes: int, seconds: float) -> float:
    """GiB/s of `nbytes` per call of fn(), repeated for about `seconds`."""
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return reps * nbytes / dt / 2**30


def _threaded(n: int, G: int, body) -> None:
    """body(g0, g1) over n Python threads on disjoint group ranges; the ctypes calls inside
    release the GIL, so the threads run the C code in parallel."""
    import threading
    th = [threading.Thread(target=body, args=(G * t // n, G * (t + 1) // n)) for t in range(1, n)]
    for t in th:
        t.start()
    body(0, G // n)
    for t in th:
        t.join()


def cpu_baseline(cfg: dict, seconds: float = 10.0) -> dict:
    """The same workload on this host's CPU cores, timed on a bounded sample (test
    infrastructure, oracle/; never the product path).

    value: the GF(2^8) restatement in its fast form (oracle_rs_encode_fast /
    oracle_rs_decode_fast: GFNI affine multiply, 64 B per instruction with AVX-512,
    recovery rows cached per erasure pattern -- how a tuned CPU library does it), byte-equal
    to the table restatement (tests/test_oracle_golden.py), on every core of this process's
    affinity.  The reference itself has no GF(2^8) code, so the reference
    numbers beside it are its XOR row only: the reference library (oracle/_ref, compiled from
    /root/reference's fec_xor_simd.cpp) fec_encode_batch single-threaded as written, and on
    every core over disjoint group ranges, plus the AVX2 restatement."""
    import numpy as np
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    k, r, P = cfg["k"], cfg["r"], cfg["P"]
    threads = host_threads()
    G = min(200_000, max(20_000, 1250 * threads))   # ~15 MB of data per thread: out of cache
    data = oracle.splitmix_bytes(G * k * P, SEED + 2)
    masks = make_masks(cfg, G, SEED + 3) if cfg["decode"] else None
    par = oracle.rs_encode_fast(data, G, k, r, P, nthreads=threads)
    done, t_enc, t_dec = 0, 0.0, 0.0
    while t_enc + t_dec < seconds:
        t0 = time.perf_counter()
        oracle.rs_encode_fast(data, G, k, r, P, nthreads=threads)
        t1 = time.perf_counter()
        if cfg["decode"]:
            oracle.rs_decode_fast(data, par, masks, G, k, r, P, nthreads=threads)
        t_enc += t1 - t0
        t_dec += time.perf_counter() - t1
        done += G
    value = done * k * P / (t_enc + t_dec) / 2**30
    leg = max(1.0, seconds / 5)
    port_1 = _rate(lambda: oracle.rs_encode_fast(data[: 2000 * k * P], 2000, k, r, P, nthreads=1),
                   2000 * k * P, leg)
    xor1 = _rate(lambda: oracle.xor_encode_contig(data, G, k, P, nthreads=1), G * k * P, leg)
    xorn = _rate(lambda: oracle.xor_encode_contig(data, G, k, P, nthreads=threads), G * k * P, leg)
    ref_block = None
    ref = oracle.ref_lib()
    if ref is not None:
        # fec_encode_batch takes 10 packets per group (fec_xor_simd.cpp:580): the slab read
        # as G*k/10 groups of ten 1200-B packets, the same bytes
        Gr = G * k // 10
        offs = (np.arange(Gr * 10, dtype=np.uint64) * P).astype(np.uint32)
        rep = np.zeros(Gr * P, dtype=np.uint8)
        h = ref.fec_encoder_new(0.10, 1024)

        def ref_range(g0, g1):
            if g1 > g0:
                ref.fec_encode_batch(h, data.ctypes.data, offs[g0 * 10:].ctypes.data, g1 - g0, P,
                                     rep[g0 * P:].ctypes.data)

        ref1 = _rate(lambda: ref_range(0, Gr), Gr * 10 * P, leg)
        refn = _rate(lambda: _threaded(threads, Gr, ref_range), Gr * 10 * P, leg)
        ref.fec_encoder_free(h)
        ref_block = (round(ref1, 3), round(refn, 3))
    cpu_model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu_model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    isa = {2: "AVX-512+GFNI", 1: "AVX2+GFNI", 0: "scalar tables"}[oracle.fast_isa()]
    return {
        "value": round(value, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "sample": f"{done} groups ({G} per pass) of k={k} r={r} P={P}: GF(2^8) restatement, fast form "
                  f"({isa}) rs_encode_fast"
                  + (f" + rs_decode_fast ({'iid loss p=%g' % cfg['loss'] if cfg.get('loss') else '%d erasures/group' % cfg['erasures']})"
                     if cfg["decode"] else "")
                  + f", {threads} threads, {t_enc + t_dec:.1f} s",
        "encode_GiBps": round(done * k * P / t_enc / 2**30, 3),
        "decode_GiBps": round(done * k * P / t_dec / 2**30, 3) if cfg["decode"] else None,
        "port_encode_threads_1_GiBps": round(port_1, 3),
        "cpu_model": cpu_model, "nproc": os.cpu_count(),
        "affinity_cores": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
        "cgroup_cpu_quota": cgroup_cpu_quota(),
        # the reference itself (XOR parity row 0 only, its whole computation): oracle/_ref =
        # /root/reference internal/fec/fec_xor_simd.cpp compiled by oracle/Makefile,
        # fec_encode_batch on 1 thread as written and on every core over disjoint group ranges
        "ref_encode_batch_1t_GiBps": ref_block[0] if ref_block else None,
        "ref_encode_batch_nt_GiBps": ref_block[1] if ref_block else None,
        "ref_encode_batch_threads": threads if ref_block else None,
        # AVX2 restatement of xor_packets_avx2 (fec_xor_simd.cpp:74-204), bit-identical to it
        # (tests/test_oracle_golden.py)
        "xor_avx2_row0_1t_GiBps": round(xor1, 3),
        "xor_avx2_row0_nt_GiBps": round(xorn, 3),
        "ref_note": ("ref_encode_batch_*: the reference library (oracle/_ref, built from /root/reference's "
                     "internal/fec/fec_xor_simd.cpp) fec_encode_batch, XOR row 0 only, 1 thread and "
                     f"{threads} threads; value: the GF(2^8) port, r={r} rows"
                     + (" + decode" if cfg["decode"] else "")),
    }


def e2e_pinned(ctx, d_data, d_parity, d_masks, G: int, cfg: dict, reps: int = 3) -> dict:
    """The path as the QUIC client/server sees it: packets start and end in host memory.
    Page-locked host buffers (the same allocator kind as fec_alloc_slab) go through the
    synchronous API, whose kernels then read and write them in place over PCIe (zero-copy;
    QUICFEC_SMALL_CALL_BYTES=0 selects the 3-stream H2D -> kernel -> D2H pipeline instead).

    Every rank runs each leg after a barrier; a leg's job time is the MAX over ranks and its
    rate the payload of ALL ranks over that time (best of `reps`), with the per-rank rates'
    spread beside it -- with N GPUs this is the node's host-resident rate, each GPU on its own
    PCIe link.  Never `value`."""
    import torch
    k, r, P = cfg["k"], cfg["r"], cfg["P"]
    h_data = torch.empty(d_data.numel(), dtype=torch.uint8, pin_memory=True)
    h_par = torch.empty(d_parity.numel(), dtype=torch.uint8, pin_memory=True)
    h_data.copy_(d_data)
    torch.cuda.synchronize()
    payload = k * P * G
    total = reduce_sum(float(payload))
    ranks = int(reduce_sum(1.0))

    def leg(fn, nbytes_local: float, nbytes_total: float) -> dict:
        best = None
        for _ in range(reps):
            barrier()
            t0 = time.perf_counter()
            fn()
            t = time.perf_counter() - t0
            tj = reduce_max(t)
            if best is None or tj < best[0]:
                best = (tj, t)
        tj, t = best
        mine = nbytes_local / t / 2**30
        return {"job_s": tj, "GiBps": nbytes_total / tj / 2**30,
                "rank_GiBps": {"min": round(reduce_min(mine), 2), "max": round(reduce_max(mine), 2)}}

    def sync_copy(dst, src):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()

    out = {"ranks": ranks}
    nb = float(h_data.numel())
    nb_all = reduce_sum(nb)
    for name, dst, src in (("h2d", d_data, h_data), ("d2h", h_data, d_data)):
        x = leg(lambda: sync_copy(dst, src), nb, nb_all)
        out[f"{name}_GBps"] = round(x["GiBps"] * 2**30 / 1e9, 2)
    enc = leg(lambda: ctx.encode(h_data, k, r, P, h_par, num_groups=G), payload, total)
    out["encode_GiBps"] = round(enc["GiBps"], 2)
    out["encode_ms"] = round(enc["job_s"] * 1e3, 2)
    out["encode_rank_GiBps"] = enc["rank_GiBps"]
    if d_masks is not None:
        h_masks = d_masks.cpu().numpy().view("uint64")
        dec = leg(lambda: ctx.decode(h_data, h_par, h_masks, k, r, P, num_groups=G), payload, total)
        out["decode_GiBps"] = round(dec["GiBps"], 2)
        out["decode_ms"] = round(dec["job_s"] * 1e3, 2)
        out["decode_rank_GiBps"] = dec["rank_GiBps"]
        out["roundtrip_GiBps"] = round(total / (enc["job_s"] + dec["job_s"]) / 2**30, 2)
    out["note"] = (f"payload k*P*G of all {ranks} rank(s) per second of the slowest rank (barrier before "
                   f"each leg), host page-locked in/out, best of {reps}; *_rank_GiBps = per-rank spread")
    del h_data, h_par
    return out


CALL_SITE_TOOL = REPO / "quic-test_amd" / "lib" / "call_site"


def call_site(ref_1t_GiBps=None, seconds: float = 2.0) -> dict:
    """The reference's unchanged product call site next to the headline: every QUIC stream's own
    HybridFECEncoder making one fec_encode_batch call per group of 10 x 1200 B
    (encoder_hybrid.go:115 -> fec_cgo.go:138), through the C++ mirror, measured by
    quic-test_amd/lib/call_site (tools/call_site.cpp) in a process of its own, as a Go binary
    would be: raw calls with FECEncoderCXX's buffers, then 1 and 16 streams back to back.  Then
    the opt-in integration that changes the call site: 16 streams' BatchedFECEncoders
    on one shared batcher, r = 1 (the reference's row) and r = 3.  Every repair row is checked
    inside the tool (no oracle).  ref_1t_GiBps (cpu_baseline's ref_encode_batch_1t_GiBps, the
    reference library on one core) is quoted beside them in groups/s.  Not the headline metric."""
    import subprocess
    if not CALL_SITE_TOOL.exists():
        return {"skipped": "quic-test_amd/lib/call_site not built (__graft_entry__.build())"}
    out = {"reference_call": "encoder_hybrid.go:115 -> fec_cgo.go:138 fec_encode_batch, 1 group of 10 x 1200 B per call",
           "tool": "quic-test_amd/lib/call_site"}
    if ref_1t_GiBps:
        out["ref_encode_batch_1t_groups_per_s"] = round(ref_1t_GiBps * 2**30 / (10 * 1200), 1)
    for name, argv in (("raw", ["raw", "20000"]), ("streams_1", ["streams", "1", str(seconds)]),
                       ("streams_16", ["streams", "16", str(seconds)]),
                       ("batcher_16_r1", ["batcher", "16", str(seconds), "1"]),
                       ("batcher_16_r3", ["batcher", "16", str(seconds), "3"])):
        try:
            p = subprocess.run([str(CALL_SITE_TOOL), *argv], capture_output=True, text=True, timeout=120)
        except subprocess.TimeoutExpired:
            out[name] = {"error": "timed out"}
            break
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if not lines:
            out[name] = {"error": f"exit {p.returncode}: {p.stderr.strip()[-300:]}"}
            break
        rec = json.loads(lines[-1])
        out[name] = {k: rec[k] for k in ("groups_per_s", "delay_us", "errors", "expired", "resident_inline",
                                         "resident_vram", "batches", "max_batch") if k in rec}
        if ref_1t_GiBps and "groups_per_s" in rec:
            out[name]["vs_ref_1t"] = round(rec["groups_per_s"] / out["ref_encode_batch_1t_groups_per_s"], 3)
    return out


def packed_supported(k: int, r: int, P: int) -> bool:
    """Shapes with a mask-addressed (inline-classify) recover form, which the packed API needs
    (include/fec_hip.h fec_recover_batch_rs_dev_packed)."""
    return ((k == 10 and r <= 3) or (k == 4 and r == 2)) and 256 < P < 2048


def pmc_key(kernel: str, api: str) -> str:
    """Key of a kernel's entry in profiles/pmc_<config>.json (scripts/pmc_summary.py --tag)."""
    if kernel != "decode":
        return kernel
    return {"packed": "recover_packed", "recover": "recover_slots"}.get(api, "decode")


def lib_sha256() -> str:
    """Hash of the libfec_hip.so this process loads (the build being timed)."""
    import hashlib
    import quicfec
    # the library quicfec.load_library() loads: QUICFEC_LIB when set (tuning runs against the test
    # library), else libfec_hip.so
    return hashlib.sha256(Path(os.environ.get("QUICFEC_LIB", quicfec.LIB_PATH)).read_bytes()).hexdigest()


def workload_key(cfg: dict, G: int) -> dict:
    """What a PMC file's bytes were measured on: the code shape, groups per GPU and loss model.
    roofline.traffic is taken from a profiles/pmc_<config>.json only when its recorded workload
    equals this one field for field (a --shape / --groups / --loss override gets null)."""
    return {"k": int(cfg["k"]), "r": int(cfg["r"]), "P": int(cfg["P"]), "groups": int(G),
            "erasures": int(cfg["erasures"]) if cfg.get("erasures") else None,
            "loss": float(cfg["loss"]) if cfg.get("loss") else None}


def workload_of_line(line: dict) -> dict:
    """workload_key() of the run that printed this bench JSON line (scripts/pmc_summary.py)."""
    c = line["config"]
    return {"k": int(c["k"]), "r": int(c["r"]), "P": int(c["packet_bytes"]), "groups": int(c["groups_per_gpu"]),
            "erasures": int(c["erasures_per_group"]) if c.get("erasures_per_group") else None,
            "loss": float(c["iid_loss"]) if c.get("iid_loss") else None}


def load_pmc_traffic(config: str, workload: dict, path=None, sha: str | None = None):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (profiles/pmc_<config>.json,
    scripts/gpu_pmc.sh), used only when they were measured on this very library build (the
    file's lib_sha256 equals the loaded .so's) AND on this exact workload (the file's `workload`,
    recorded by scripts/pmc_summary.py from the profiled bench line, equals `workload`).
    Returns (pmc dict or None, note naming the source or the mismatch)."""
    p = Path(path) if path is not None else REPO / "profiles" / f"pmc_{config}.json"
    name = f"profiles/{p.name}"
    if not p.exists():
        return None, f"no {name}"
    try:
        pmc = json.loads(p.read_text())
    except (OSError, ValueError):
        return None, f"unreadable {name}"
    if pmc.get("lib_sha256") != (sha if sha is not None else lib_sha256()):
        return None, f"{name} was measured on another build of libfec_hip.so"
    wl = pmc.get("workload")
    if not isinstance(wl, dict):
        return None, f"{name} records no workload: not attributable to this run"
    diff = [f"{f}={wl.get(f)!r} there vs {workload[f]!r} here" for f in workload if wl.get(f) != workload[f]]
    if diff:
        return None, f"{name} was measured on another workload ({'; '.join(diff)})"
    return pmc, f"{name} (rocprofv3 PMC on this build, lib_sha256 {pmc['lib_sha256'][:16]}, same workload)"


# ----------------------------------------------------------------------------- main
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2c3", choices=sorted(CONFIGS))
    ap.add_argument("--groups", type=int, default=0, help="groups per GPU (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--loss", type=float, default=None,
                    help="iid per-shard loss probability (c5; 0.05 = mobile profile)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--shape", default=None,
                    help="k,r,P override of the config's code shape (tuning sweeps; not the headline)")
    ap.add_argument("--e2e", action="store_true",
                    help="also time the host-resident path (pinned buffers, H2D -> kernel -> D2H)")
    ap.add_argument("--decode-api", default="auto", choices=("auto", "packed", "recover", "in-place"),
                    help="packed: fec_recover_batch_rs_dev_packed (all groups' rebuilt packets back to back, as "
                         "the reference decoder returns its Recovered list); recover: fec_recover_batch_rs_dev "
                         "((g*r + m)*P slots); in-place: fec_decode_batch_rs_dev; auto: packed for sparse loss "
                         "(a loss profile), else recover")
    ap.add_argument("--null-stream", action="store_true",
                    help="launch through stream handle 0 (the context's own stream) with events on torch's "
                         "default stream, as round-1/2 benches did (A/B of the timing setup)")
    ap.add_argument("--parity-offset", type=int, default=0, help="parity buffer placement (bytes past an allocation start)")
    ap.add_argument("--rebuilt-offset", type=int, default=0, help="rebuilt-packet buffer placement (bytes)")
    ap.add_argument("--no-other-api", action="store_true",
                    help="skip the comparison run of the other decode API (PMC passes keyed per API)")
    ap.add_argument("--legs", default="auto", choices=("auto", "on", "off"),
                    help="after the headline, measure the other multi-GPU BASELINE configs in the same ranks: "
                         "C4 (k=20 r=5 encode) and C5 (satellite loss, device-resident and host-resident with "
                         "H2D/D2H); auto = on when N > 1")
    ap.add_argument("--leg-groups", type=int, default=0, help="groups per GPU of the legs (default: each config's)")
    ap.add_argument("--e2e-groups", type=int, default=0,
                    help="groups per rank of the host-resident legs (default: all at N = 1, 250k per rank at N > 1, "
                         "so N ranks' page-locked buffers stay within one node's RAM)")
    ap.add_argument("--no-call-site", action="store_true",
                    help="skip the call_site section (the reference's one-group-per-call site; N = 1, runs with "
                         "the cpu_baseline leg, so --no-cpu-baseline skips it too)")
    ap.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# The other multi-GPU BASELINE lines, measured after the headline when N > 1 (--legs): C4
# (configs[3], 8M groups over 8 GPUs = 1M per GPU, encode) and C5 (configs[4], satellite loss,
# "timed with H2D/D2H copies": device-resident step plus the host-resident legs).
LEGS = (("c4", "c4", False), ("c5_e2e", "c5", True))


def legs_enabled(args, world: int) -> bool:
    return args.legs == "on" or (args.legs == "auto" and world > 1)


def leg_section(res: dict) -> dict:
    """A leg's entry in rank 0's JSON line: the same quantities as the headline (payload of all
    ranks / the slowest rank's time, per-kernel timings, roofline) for that config."""
    keep = ("workload", "value", "unit", "ranks", "groups_per_gpu", "steps", "warmup", "ms_per_step", "verified",
            "decode_api", "kernels", "roofline", "e2e_pinned")
    return {k: res[k] for k in keep if k in res}


def run_legs(measure_leg) -> dict:
    """measure_leg(config) -> result dict, on every rank in the same order (its collectives
    line up); returns {section: leg_section(...)}."""
    return {section: leg_section(measure_leg(config, e2e)) for section, config, e2e in LEGS}


def launch_selftest(args) -> int:
    """CPU-only check of the launch path (tests/test_distributed.py): every rank joins a
    gloo group, reduces like the bench does (headline and legs), and rank 0 prints one JSON
    line with the same sections as the real bench."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="gloo", init_method="env://")
    G = 1000
    g0, g1 = shard_range(G * world, rank, world)
    mx = reduce_max(0.25 * (rank + 1))
    total = reduce_sum(float(g1 - g0))

    def fake_leg(config: str, e2e: bool) -> dict:
        cfg = CONFIGS[config]
        barrier()
        t = reduce_max(0.01 * (rank + 1))
        ranks = int(reduce_sum(1.0))
        res = {"workload": cfg["workload"], "value": ranks * G * cfg["k"] * cfg["P"] / t / 2**30, "unit": "GiB/s",
               "ranks": ranks, "groups_per_gpu": G, "ms_per_step": t * 1e3, "verified": True}
        if e2e:
            res["e2e_pinned"] = {"ranks": ranks}
        return res

    legs = run_legs(fake_leg) if legs_enabled(args, world) else None
    barrier()
    if rank == 0:
        line = {"selftest": True, "n_gpus": world, "gpus_arg": args.gpus, "max_elapsed": mx, "total_groups": total}
        if legs:
            line.update(legs)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


class Bench:
    """One rank's measurement state: context, stream, the rank's place in the job."""

    def __init__(self, args, rank: int, world: int, local: int):
        import torch
        import quicfec
        self.args, self.rank, self.world = args, rank, world
        self.ctx = quicfec.Context(device=local)
        # One stream for everything: the library's launches, torch's ops and the timing events.
        # torch's default stream has handle 0, which the C-ABI reads as "the context's own
        # stream" (a blocking stream); launching there while recording events on the default
        # stream made every event an implicit cross-stream synchronisation inside the timed steps
        # (~15-60 us per kernel, profiles/r02_stream_ab.txt).  --null-stream keeps that old setup.
        if args.null_stream:
            self.stream = torch.cuda.current_stream()
        else:
            self.stream = torch.cuda.Stream()
            torch.cuda.set_stream(self.stream)
        self.sp = self.stream.cuda_stream
        self.copy = None  # the box's copy rate (measured once per process)

    def measure(self, config: str, cfg: dict, G: int, steps: int, warmup: int, api: str, verify: bool,
                other_api: bool, e2e: bool) -> dict:
        """One workload on this rank: verify, W untimed + K timed steps between barriers, per-kernel
        timings, roofline.  Every rank calls it with the same arguments (collectives line up)."""
        import numpy as np
        import torch
        args, rank, world, ctx, stream, sp = self.args, self.rank, self.world, self.ctx, self.stream, self.sp
        k, r, P = cfg["k"], cfg["r"], cfg["P"]
        g0, _ = shard_range(G * world, rank, world)

        def dev_buffer(nbytes: int, offset: int):
            """nbytes of HBM starting `offset` bytes into a fresh allocation (buffer placement A/B)."""
            if offset <= 0:
                return torch.empty(nbytes, dtype=torch.uint8, device="cuda")
            return torch.empty(nbytes + offset, dtype=torch.uint8, device="cuda")[offset:]

        data = torch.empty(G * k * P, dtype=torch.uint8, device="cuda")
        parity = dev_buffer(G * r * P, args.parity_offset)
        # this rank's slice of one global synthetic stream
        ctx.fill_random_dev(data, data.numel(), SEED + 2, byte_offset=g0 * k * P, stream=sp)
        dec_bytes = dec_read = 0
        if api == "auto":
            # The slot rows (fec_recover_batch_rs_dev) at every density.  Dense loss (C3): never
            # more than 4% behind the packed rows on any box measured, same HBM bytes by PMC
            # (profiles/r03_final/ab_decode_api_box*.jsonl).  Sparse loss (C5, the 8-groups-per-wave
            # form by the loss hint) against the packed rows' one-launch recover_runs, this build,
            # in this step, two boxes x 3 rounds (scripts/ab_c5_api.sh, profiles/r06/ab_c5_api_box*.jsonl):
            # median 0.2410 vs 0.2437 ms in the step, 0.2392 vs 0.2443 ms isolated.
            api = "recover"
        recover = cfg["decode"] and api in ("recover", "packed")
        rebuilt = dev_buffer(G * r * P, args.rebuilt_offset) if recover else None
        row_start = torch.empty(G, dtype=torch.int32, device="cuda") if cfg["decode"] and api == "packed" else None
        masks = None

        def decode_call(api: str, status=None):
            if api == "packed":
                ctx.recover_packed_dev(data, parity, masks, G, k, r, P, rebuilt, row_start, None, status, stream=sp)
            elif api == "recover":
                ctx.recover_dev(data, parity, masks, G, k, r, P, rebuilt, status, stream=sp)
            else:
                ctx.decode_dev(data, parity, masks, G, k, r, P, status, stream=sp)

        if cfg["decode"]:
            masks_h = make_masks(cfg, G, SEED + 3 + rank)
            dec_bytes = decode_algorithmic_bytes(masks_h, k, r, P)
            dec_read = decode_algorithmic_bytes(masks_h, k, r, P, reads_only=True)
            masks = torch.from_numpy(masks_h.view(np.int64)).to("cuda")
            ctx.decode_prepare(k, r)
            # the receiver knows its loss profile: share of groups that lose a data shard (a
            # dense caller says so too: the library's scan form is for sparse loss only)
            ctx.decode_loss_hint(1.0 - (1.0 - cfg["loss"]) ** k if cfg.get("loss") else -1.0)
        torch.cuda.synchronize()

        verified = None
        if verify:
            # correctness of this exact configuration before timing: encode, poison the erased
            # data shards, rebuild, compare with the untouched copy; sampled groups vs oracle
            # parity are covered by tests/test_gpu_parity.py.
            orig = data.clone()
            ctx.encode_dev(data, G, k, r, P, parity, stream=sp)
            if cfg["decode"]:
                bits = torch.arange(k, device="cuda", dtype=torch.int64)
                lost = ((masks.view(G, 1) >> bits.view(1, k)) & 1).bool()
                data.view(G, k, P)[lost] = 0xEE
                st = torch.zeros(G, dtype=torch.uint8, device="cuda")
                decode_call(api, st)
                torch.cuda.synchronize()
                bad_exp = unrecoverable_count(masks_h, k, r)
                n_bad = int(st.sum().item())
                ok_rows = st == 0
                if api == "packed":
                    # rows back to back in (g, j ascending) order: boolean indexing's order
                    want = orig.view(G, k, P)[lost & ok_rows.view(G, 1)]
                    got = rebuilt.view(-1, P)[:want.shape[0]]
                    verified = bool(torch.equal(got, want)) and n_bad == bad_exp
                    data.copy_(orig)
                elif recover:
                    # slot m of group g = its m-th lost data shard: the same (g, j ascending) order
                    # as boolean indexing of the lost shards
                    e_g = lost.sum(dim=1, keepdim=True)
                    slots = torch.arange(r, device="cuda").view(1, r) < e_g
                    got = rebuilt.view(G, r, P)[slots & ok_rows.view(G, 1)]
                    want = orig.view(G, k, P)[lost & ok_rows.view(G, 1)]
                    verified = bool(torch.equal(got, want)) and n_bad == bad_exp
                    data.copy_(orig)
                elif n_bad == 0:
                    verified = bool(torch.equal(data, orig)) and bad_exp == 0
                else:
                    verified = bool(torch.equal(data.view(G, -1)[ok_rows], orig.view(G, -1)[ok_rows])) and n_bad == bad_exp
            else:
                # encode-only config: the library's decoder (separate kernels, table arithmetic)
                # rebuilds r erased shards of every group, data and parity mixed, from the parity
                # just written -- a size-independent round trip of every parity row (the encode
                # against the oracle on sampled groups is in tests/)
                vm_h = erasure_masks(G, k + r, r, SEED + 7 + rank)
                vm = torch.from_numpy(vm_h.view(np.int64)).to("cuda")
                ctx.decode_prepare(k, r)
                bits = torch.arange(k, device="cuda", dtype=torch.int64)
                lost = ((vm.view(G, 1) >> bits.view(1, k)) & 1).bool()
                data.view(G, k, P)[lost] = 0xEE
                st = torch.zeros(G, dtype=torch.uint8, device="cuda")
                rb = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
                ctx.recover_dev(data, parity, vm, G, k, r, P, rb, st, stream=sp)
                torch.cuda.synchronize()
                e_g = lost.sum(dim=1, keepdim=True)
                slots = torch.arange(r, device="cuda").view(1, r) < e_g
                verified = bool(torch.equal(rb.view(G, r, P)[slots], orig.view(G, k, P)[lost])) and int(st.sum().item()) == 0
                data.copy_(orig)
                del rb, vm, lost, slots, st
            del orig
            torch.cuda.empty_cache()

        def step(ev=None):
            if ev is not None:
                ev[0].record(stream)
            ctx.encode_dev(data, G, k, r, P, parity, stream=sp)
            if ev is not None:
                ev[1].record(stream)
            if cfg["decode"]:
                decode_call(api)
                if ev is not None:
                    ev[2].record(stream)

        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(events[i])
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        enc_ms = sum(e[0].elapsed_time(e[1]) for e in events) / steps
        dec_ms = (sum(e[1].elapsed_time(e[2]) for e in events) / steps) if cfg["decode"] else 0.0

        elapsed_max = reduce_max(elapsed)
        if verified is not None:  # every rank must have rebuilt its shard exactly
            verified = reduce_max(0.0 if verified else 1.0) == 0.0
        total_groups = reduce_sum(float(G))
        ranks = int(reduce_sum(1.0))
        payload = total_groups * k * P * steps
        value = payload / elapsed_max / 2**30
        ms_per_step = elapsed_max / steps * 1e3

        enc_bytes = (k + r) * P * G
        enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
        kernels = {"encode": {"ms": round(enc_ms, 4), "algorithmic_bytes": enc_bytes,
                              "achieved_GBps": round(enc_gbs, 1),
                              "payload_GiBps": round(k * P * G / (enc_ms * 1e-3) / 2**30, 2)}}
        if cfg["decode"]:
            dec_gbs = dec_bytes / (dec_ms * 1e-3) / 1e9
            kernels["decode"] = {"ms": round(dec_ms, 4), "algorithmic_bytes": dec_bytes,
                                 "achieved_GBps": round(dec_gbs, 1),
                                 "payload_GiBps": round(k * P * G / (dec_ms * 1e-3) / 2**30, 2)}
        # Each kernel alone, back to back (decode is idempotent on rebuilt data): its own time,
        # without the write-back of the other kernel's output still draining from the caches
        # when it starts (which the in-step times above include).
        reps = max(5, steps // 4)

        def isolated(fn, nbytes):
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
            evs[0].record(stream)
            for i in range(reps):
                fn()
                evs[i + 1].record(stream)
            torch.cuda.synchronize()
            ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(reps))[reps // 2]
            return {"ms_median": round(ms, 4), "achieved_GBps": round(nbytes / (ms * 1e-3) / 1e9, 1)}

        kernels["encode"]["isolated"] = isolated(lambda: ctx.encode_dev(data, G, k, r, P, parity, stream=sp), enc_bytes)
        if cfg["decode"]:
            kernels["decode"]["api"] = api
            kernels["decode"]["isolated"] = isolated(lambda: decode_call(api), dec_bytes)
            # the other decode API on the same buffers, for comparison (not in `value`)
            # (sparse loss: the packed rows, the form the slot rows were chosen over)
            other = {"packed": "recover",
                     "recover": "packed" if cfg.get("loss") and packed_supported(k, r, P) else "in-place"}.get(api, "recover")
            if other_api:
                if other == "recover" and rebuilt is None:
                    rebuilt = dev_buffer(G * r * P, args.rebuilt_offset)
                if other == "packed" and row_start is None:
                    row_start = torch.empty(G, dtype=torch.int32, device="cuda")
                kernels["decode"]["other_api"] = {"api": other, **isolated(lambda: decode_call(other), dec_bytes)}
        # The box's own HBM copy rate (fec_copy_dev: the encode's 16-B-per-lane pattern, no
        # arithmetic), measured the same way once per process: box-to-box spread is a few
        # percent, so the kernels are also quoted against it.
        if self.copy is None:
            half = (data.numel() // 2) // 16 * 16
            scratch = torch.empty(half, dtype=torch.uint8, device="cuda")
            self.copy = isolated(lambda: ctx.copy_dev(data, scratch, half, stream=sp), 2 * half)
            del scratch
            torch.cuda.empty_cache()
        copy = self.copy
        dom = max(kernels, key=lambda n: kernels[n]["ms"])
        dom_read = k * P * G if dom == "encode" else dec_read
        wl = workload_key(cfg, G)
        pmc, pmc_note = load_pmc_traffic(config, wl)
        pmc = pmc or {}
        roofline = {"bound": "hbm", "kernel": dom, "achieved": kernels[dom]["achieved_GBps"],
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(kernels[dom]["achieved_GBps"] / HBM_PEAK_GBS, 4),
                    # PMC entries are keyed per decode API (recover_packed / recover_slots / decode)
                    "traffic": pmc.get(pmc_key(dom, api) if cfg["decode"] else dom, {}).get("hbm_bytes_per_launch"),
                    "algorithmic_bytes_per_launch": kernels[dom]["algorithmic_bytes"],
                    "traffic_source": pmc_note,
                    "read_frac": round(dom_read / (kernels[dom]["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "read_frac_of_box_copy": round(dom_read / (kernels[dom]["ms"] * 1e-3) / 1e9 / copy["achieved_GBps"], 4),
                    # north_star's "70% of the HBM-read roofline": reads at 0.70 x 8 TB/s while this
                    # kernel also writes its bytes needs this much total traffic -- above the box's
                    # copy ceiling (box_copy_GBps), so that literal target is out of reach
                    "read_target_total_GBps": round(0.70 * HBM_PEAK_GBS * kernels[dom]["algorithmic_bytes"] / dom_read, 1),
                    "box_copy_GBps": copy["achieved_GBps"],
                    "frac_of_box_copy": round(kernels[dom]["achieved_GBps"] / copy["achieved_GBps"], 4),
                    "timing": ("torch.cuda.Event on torch's default stream, kernels on the context's stream"
                               if args.null_stream else
                               "torch.cuda.Event on the launch stream (one torch stream for launches, ops and "
                               "events), averaged over the timed steps")}
        res = {"workload": cfg["workload"], "value": round(value, 3), "unit": "GiB/s", "ranks": ranks,
               "groups_per_gpu": G, "steps": steps, "warmup": warmup, "ms_per_step": round(ms_per_step, 4),
               "verified": verified, "decode_api": api if cfg["decode"] else None,
               "kernels": kernels, "roofline": roofline, "workload_key": wl}
        if e2e:
            # host-resident legs on the first Ge groups: the whole batch at N = 1 (15.6 GB page-locked
            # at C5), --e2e-groups (default 250k, ~3.9 GB) per rank when N ranks share one node's RAM
            Ge = min(G, args.e2e_groups if args.e2e_groups else (G if world == 1 else 250_000))
            k_, r_, P_ = cfg["k"], cfg["r"], cfg["P"]
            res["e2e_pinned"] = e2e_pinned(ctx, data[:Ge * k_ * P_], parity[:Ge * r_ * P_],
                                           masks[:Ge] if cfg["decode"] else None, Ge, cfg)
            res["e2e_pinned"]["groups_per_rank"] = Ge
        if os.environ.get("QUICFEC_BENCH_ADDRS") == "1":  # placement diagnostics (A/B runs)
            res["buffers"] = {n: hex(t.data_ptr()) for n, t in (("data", data), ("parity", parity), ("rebuilt", rebuilt))
                              if t is not None}
        del data, parity, rebuilt, row_start, masks
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        return res


DECODE_API_TEXT = {"packed": "fec_recover_batch_rs_dev_packed (rebuilt packets of all groups back to back with "
                             "per-group row starts, decoder.go Recovered list)",
                   "recover": "fec_recover_batch_rs_dev (rebuilt packets at (g*r + m)*P slots)",
                   "in-place": "fec_decode_batch_rs_dev (in place)"}


def main() -> int:
    args = parse_args()
    mode, n = launch_plan(args.gpus, os.environ)
    if mode == "spawn":
        return spawn_ranks(n, sys.argv[1:])
    if args.launch_selftest:
        return launch_selftest(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; bind the GPU before RCCL creates its communicator.
    local = bind_local_device(local, world, torch.cuda.device_count())
    torch.cuda.set_device(local)
    host_binding = None
    if world > 1:
        # before any host allocation (N = 1 keeps every core: its cpu_baseline uses them)
        host_binding = bind_host_to_gpu(local)
        dist.init_process_group(backend=dist_backend(), init_method="env://")
    cfg = dict(CONFIGS[args.config])
    if args.loss is not None:
        cfg["loss"] = args.loss
        cfg["decode"] = True
        cfg["workload"] += f" (loss override p={args.loss})"
    if args.shape:
        cfg["k"], cfg["r"], cfg["P"] = (int(x) for x in args.shape.split(","))
        cfg["erasures"] = min(cfg["erasures"], cfg["r"])
        cfg["workload"] += f" (shape override k={cfg['k']} r={cfg['r']} P={cfg['P']})"
    G = args.groups or cfg["groups"]
    if args.groups:
        cfg["workload"] += f" (groups override: {G}/GPU)"

    wall = {"setup": round(time.monotonic() - T_START, 2)}  # rank 0's wall-clock seconds per phase
    bench = Bench(args, rank, world, local)
    t = time.monotonic()
    head = bench.measure(args.config, cfg, G, args.steps, args.warmup, args.decode_api, not args.no_verify,
                         not args.no_other_api, args.e2e)
    wall["headline"] = round(time.monotonic() - t, 2)

    legs = None
    if legs_enabled(args, world):
        def measure_leg(config: str, e2e: bool) -> dict:
            lc = dict(CONFIGS[config])
            lg = args.leg_groups or lc["groups"]
            if args.leg_groups:
                lc["workload"] += f" (groups override: {lg}/GPU)"
            t0 = time.monotonic()
            res = bench.measure(config, lc, lg, min(args.steps, 20), min(args.warmup, 2), "auto",
                                not args.no_verify, False, e2e)
            wall["leg_" + config] = round(time.monotonic() - t0, 2)
            return res
        legs = run_legs(measure_leg)

    cpu = None
    t = time.monotonic()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg)
        wall["cpu_baseline"] = round(time.monotonic() - t, 2)
    site = None  # beside the headline like cpu_baseline, and skipped with it (profiled and A/B runs)
    t = time.monotonic()
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.no_call_site:
        site = call_site(cpu.get("ref_encode_batch_1t_GiBps") if cpu else None)
        wall["call_site"] = round(time.monotonic() - t, 2)
    wall["total"] = round(time.monotonic() - T_START, 2)

    if rank == 0:
        k, r, P = cfg["k"], cfg["r"], cfg["P"]
        out = {
            "metric": "FEC encode+decode GiB/s (device-resident), k=10 r=3 1200B pkts, 1/2/4/8 GPU",
            "value": head["value"], "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (counter-based splitmix64 bytes generated in HBM; seeded erasure masks)",
            "config": {"workload": cfg["workload"], "k": k, "r": r, "packet_bytes": P,
                       "groups_per_gpu": G, "erasures_per_group": cfg["erasures"] or None,
                       "iid_loss": cfg.get("loss"),
                       "decode_api": DECODE_API_TEXT[head["decode_api"]] if cfg["decode"] else None,
                       "parallelism": f"group-sharded x{world} (no collective)"},
            "verified": head["verified"],
            "kernels": head["kernels"],
            "roofline": head["roofline"],
            "cpu_baseline": cpu,
        }
        if "e2e_pinned" in head:
            out["e2e_pinned"] = head["e2e_pinned"]
        if site is not None:
            out["call_site"] = site
        if "buffers" in head:
            out["buffers"] = head["buffers"]
        if legs:
            out.update(legs)
        if host_binding is not None:
            out["host_binding"] = host_binding  # rank 0's (every rank binds to its own GPU's CPUs)
        out["wall_s"] = wall
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    bench.ctx.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
