"""Multi-process path of bench.py on CPU (gloo, world_size 2, 127.0.0.1).

The FEC path shards by group with no data-path collective: each rank owns a contiguous
slice of the global group stream, and only the elapsed time (MAX) and the group counts
(SUM) are reduced.  This checks the sharding and the reductions exactly as bench.py runs
them under torch.distributed.run."""
import os
import socket
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, str(REPO))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    import bench
    G_total = 1_000_003
    g0, g1 = bench.shard_range(G_total, rank, world)
    elapsed = 0.5 + rank                      # rank 1 is the slow one
    mx = bench.reduce_max(elapsed)
    total = bench.reduce_sum(float(g1 - g0))
    bench.barrier()
    # the stream offset each rank would pass to fec_fill_random_dev
    q.put((rank, g0, g1, mx, total, g0 * 10 * 1200))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_group_sharding_and_reductions(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spans = [(g0, g1) for _, g0, g1, *_ in res]
    assert spans[0][0] == 0 and spans[-1][1] == 1_000_003
    assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))      # contiguous, disjoint
    assert max(g1 - g0 for g0, g1 in spans) - min(g1 - g0 for g0, g1 in spans) <= 1
    for _, g0, g1, mx, total, off in res:
        assert mx == pytest.approx(0.5 + (world - 1))
        assert total == pytest.approx(1_000_003)
        assert off == g0 * 12000


def test_launch_plan_gpus_vs_world_size():
    sys.path.insert(0, str(REPO))
    import bench
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}) == ("run", 4)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == ("run", 1)
    with pytest.raises(SystemExit, match="disagrees"):
        bench.launch_plan(8, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit, match="disagrees"):
        bench.launch_plan(1, {"WORLD_SIZE": "8"})
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


def test_bind_local_device(monkeypatch):
    sys.path.insert(0, str(REPO))
    import bench
    monkeypatch.setenv("QUICFEC_DIST_BACKEND", "nccl")
    assert bench.bind_local_device(3, 8, 8) == 3
    with pytest.raises(SystemExit, match="only 1 visible"):
        bench.bind_local_device(1, 2, 1)
    with pytest.raises(SystemExit):
        bench.bind_local_device(0, 1, 0)
    monkeypatch.setenv("QUICFEC_DIST_BACKEND", "gloo")      # one-GPU rehearsal shares the card
    assert bench.bind_local_device(1, 2, 1) == 0


@pytest.mark.parametrize("world", [1, 3])
def test_bench_gpus_n_spawns_n_ranks(world):
    """`python bench.py --gpus N` with no WORLD_SIZE starts N ranks itself (gloo, CPU)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["QUICFEC_DIST_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", str(world), "--launch-selftest"],
                         env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout                       # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == world and rec["gpus_arg"] == world
    assert rec["max_elapsed"] == pytest.approx(0.25 * world)
    assert rec["total_groups"] == pytest.approx(1000 * world)
    # the multi-GPU BASELINE legs (C4, C5 with H2D/D2H) run after the headline when N > 1 only
    assert ("c4" in rec) == (world > 1) and ("c5_e2e" in rec) == (world > 1)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_gpus_n_carries_every_multi_gpu_config(world):
    """One `bench.py --gpus N` invocation reports the C4 and C5 lines beside the headline, each
    reduced over all N ranks (barrier, MAX time, SUM of payload) like the headline.  N = 8 is the
    driver's scaling run: eight gloo ranks spawned by the GPU-free parent."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["QUICFEC_DIST_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", str(world), "--launch-selftest"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == world and rec["gpus_arg"] == world
    assert rec["max_elapsed"] == pytest.approx(0.25 * world)          # MAX over ranks
    assert rec["total_groups"] == pytest.approx(1000 * world)         # SUM over ranks
    for sec in ("c4", "c5_e2e"):
        assert rec[sec]["ranks"] == world, sec
        assert rec[sec]["ms_per_step"] == pytest.approx(10.0 * world)  # MAX over ranks (rank i: 0.01 (i + 1) s)
        assert rec[sec]["verified"] is True
    assert rec["c5_e2e"]["e2e_pinned"]["ranks"] == world
    if world != 2:
        return
    assert "C4" in rec["c4"]["workload"] and "C5" in rec["c5_e2e"]["workload"]
    # --legs off drops them
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--legs", "off", "--launch-selftest"],
                         env=env, capture_output=True, text=True, timeout=180)
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert "c4" not in rec and "c5_e2e" not in rec


def test_bench_gpus_disagreeing_world_size_fails():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "4", "--launch-selftest"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "disagrees" in out.stderr


def test_shard_range_single():
    sys.path.insert(0, str(REPO))
    import bench
    assert bench.shard_range(10, 0, 1) == (0, 10)
    assert bench.shard_range(0, 0, 4) == (0, 0)


def test_bench_decode_api_shapes():
    """bench.py's packed-recover shape rule mirrors the library's mask-addressed forms
    (fec_kernels.hip try_decode_fused QFEC_FUSED_DS / _D; tests/test_gpu_packed.py checks the
    library refuses the rest)."""
    import bench
    assert bench.packed_supported(10, 3, 1200) and bench.packed_supported(10, 1, 700)
    assert bench.packed_supported(10, 2, 1400) and bench.packed_supported(4, 2, 513)
    assert not bench.packed_supported(20, 5, 1200)      # record-addressed LDS-table form
    assert not bench.packed_supported(10, 3, 200)       # tiled form (P <= 256)
    assert not bench.packed_supported(10, 3, 2048)      # no fused piece layout past 2047 B
    assert not bench.packed_supported(6, 3, 1200)       # runtime-k wave kernel


def test_visible_gpus_without_hip(tmp_path):
    """The spawning parent counts GPUs from the KFD topology and the *_VISIBLE_DEVICES lists,
    never through the HIP runtime."""
    import bench
    nodes = tmp_path / "nodes"
    for i, gid in enumerate((0, 4321, 8765, 0, 1111)):      # CPU nodes have gpu_id 0
        (nodes / str(i)).mkdir(parents=True)
        (nodes / str(i) / "gpu_id").write_text(f"{gid}\n")
    assert bench.visible_gpus({}, str(nodes)) == 3
    assert bench.visible_gpus({"HIP_VISIBLE_DEVICES": "1"}, str(nodes)) == 1
    assert bench.visible_gpus({"ROCR_VISIBLE_DEVICES": "0,2", "HIP_VISIBLE_DEVICES": "0,1"}, str(nodes)) == 2
    assert bench.visible_gpus({"ROCR_VISIBLE_DEVICES": ""}, str(nodes)) == 0
    assert bench.visible_gpus({"CUDA_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}, str(tmp_path / "absent")) == 8
    assert bench.visible_gpus({}, str(tmp_path / "absent")) == 0


def test_spawn_parent_never_maps_hip_runtime():
    """`bench.py --gpus 2` under RCCL: the parent checks the device count and starts the ranks
    with libamdhip64 unmapped (spawn_ranks refuses otherwise); here the ranks run the gloo
    launch self-test."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "QUICFEC_DIST_BACKEND")}
    env["HIP_VISIBLE_DEVICES"] = "0,1"
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--launch-selftest"],
                         env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 2
    # a parent that did load the runtime (torch) is refused before any rank starts
    code = ("import sys; sys.path.insert(0, %r); import torch, bench; bench.spawn_ranks(2, ['--launch-selftest'])"
            % str(REPO))
    bad = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert bad.returncode != 0 and "HIP runtime" in bad.stderr


def test_rank_binds_host_threads_to_its_gpu(monkeypatch, tmp_path):
    """bench.py ranks of N > 1 confine their threads to the CPUs sysfs lists as local to their
    GPU (within the CPUs they may use), so each rank's page-locked buffers sit on its GPU's
    socket; nothing changes when none of those CPUs is allowed or all already are."""
    import os
    import types
    import torch
    import bench
    assert bench.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    dev = tmp_path / "0000:c1:00.0"
    dev.mkdir()
    (dev / "numa_node").write_text("1\n")
    props = types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0xC1, pci_device_id=0)
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: props)
    allowed = set(range(16))
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(allowed))
    calls = []
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: calls.append(set(cpus)))
    (dev / "local_cpulist").write_text("8-23\n")
    rec = bench.bind_host_to_gpu(3, sysfs=tmp_path)
    assert rec["bound"] and rec["numa_node"] == 1 and rec["pci"] == "0000:c1:00.0" and rec["local_cpus"] == 8
    assert calls == [set(range(8, 16))]
    (dev / "local_cpulist").write_text("32-47\n")                 # none of them allowed: leave it
    assert not bench.bind_host_to_gpu(3, sysfs=tmp_path)["bound"] and len(calls) == 1
    (dev / "local_cpulist").write_text("0-63\n")                  # every allowed CPU is local already
    assert not bench.bind_host_to_gpu(3, sysfs=tmp_path)["bound"] and len(calls) == 1
    props.pci_bus_id = 0x05                                       # no sysfs entry for the device
    assert bench.bind_host_to_gpu(3, sysfs=tmp_path)["why"] == "no sysfs entry"


@pytest.mark.gpu
def test_rccl_group_runs_the_bench_reductions():
    """The reductions of a multi-GPU bench run (barrier with the rank's device, MAX and SUM of a
    float64 on the GPU) over a real RCCL communicator: one rank on this box's GPU, in a child
    process so the communicator does not outlive the test.  The driver's N = 2/4/8 runs use the
    same calls; this is the part of them a one-GPU box can run."""
    import json
    import subprocess
    code = f"""
import json, os, sys
sys.path.insert(0, {str(REPO)!r})
import torch, torch.distributed as dist
import bench
torch.cuda.set_device(0)
dist.init_process_group(backend=bench.dist_backend(), init_method="env://")
bench.barrier()
mx = bench.reduce_max(1.25)
sm = bench.reduce_sum(3.0)
mn = bench.reduce_min(0.5)
bench.barrier()
print(json.dumps({{"backend": dist.get_backend(), "max": mx, "sum": sm, "min": mn}}), flush=True)
dist.destroy_process_group()
"""
    env = {k: v for k, v in os.environ.items() if k != "QUICFEC_DIST_BACKEND"}
    env.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, (out.stdout, out.stderr[-2000:])
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec == {"backend": "nccl", "max": 1.25, "sum": 3.0, "min": 0.5}, rec
