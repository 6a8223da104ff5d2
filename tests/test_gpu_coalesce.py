"""Legacy-call coalescing (fec_coalesce.cpp): the reference's unchanged call pattern -- one
group per fec_encode_batch call, every stream on its own context (encoder_hybrid.go:115 via
fec_cgo.go:138) -- from many threads at once, joined into shared launches.

Row 0 is pinned by the reference: the expected repair rows are the golden fixture
`batch_k10_p1200_g64` that `tests/golden/make_golden.py` produced with the reference's own
fec_encode_batch (oracle/_ref); other sizes are checked against the oracle's XOR restatement.
"""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pinned_copy(lib, arr):
    p = lib.fec_alloc_slab(max(arr.nbytes, 1))
    assert p
    ctypes.memmove(p, arr.ctypes.data, arr.nbytes)
    return p


def _read(p, n):
    return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p)).copy()


def _run_threads(n, fn):
    errs = []

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]


@pytest.mark.parametrize("pinned,resident", [(True, True), (True, False), (False, True)],
                         ids=["pinned_slab_resident", "pinned_slab_batches", "pageable_slab"])
def test_concurrent_one_group_calls_match_reference(quicfec_mod, oracle_mod, xor_golden, manifest, pinned, resident,
                                                    monkeypatch):
    """16 streams, each with its own context (the Go wrapper's FECEncoderCXX), 1 group per call:
    page-locked slabs go to the resident encoder (QUICFEC_RESIDENT=0: shared launches);
    pageable ones too when its ring is in device memory (the packets copied into the slot),
    else to shared launches."""
    monkeypatch.setenv("QUICFEC_COALESCE", "1")
    monkeypatch.setenv("QUICFEC_RESIDENT", "1" if resident else "0")
    c = next(c for c in manifest["cases"] if c["name"] == "batch_k10_p1200_g64")
    G, P = c["G"], c["P"]
    slab = oracle_mod.splitmix_bytes(G * 10 * P, c["seed"])
    exp = xor_golden["batch_k10_p1200_g64"].reshape(G, P)
    lib = quicfec_mod.load_library()
    quicfec_mod.coalesce_stats(reset=True)
    S, CALLS = 16, 96

    def stream(i):
        ctx = quicfec_mod.Context(device=0)
        rng = np.random.default_rng(100 + i)
        # the Go wrapper packs the group's 10 packets back to back into its page-locked slab
        sp = lib.fec_alloc_slab(10 * P) if pinned else None
        rp = lib.fec_alloc_repair_buffer(P)
        host = np.zeros(10 * P, dtype=np.uint8)
        offs = (np.arange(10, dtype=np.uint32) * P).astype(np.uint32)
        try:
            for _ in range(CALLS):
                g = int(rng.integers(G))
                grp = slab[g * 10 * P:(g + 1) * 10 * P]
                if pinned:
                    ctypes.memmove(sp, grp.ctypes.data, grp.nbytes)
                    src = sp
                else:
                    host[:] = grp
                    src = host.ctypes.data
                assert lib.fec_encode_batch(ctx.handle, src, offs.ctypes.data, 1, P, rp) == 0
                assert np.array_equal(_read(rp, P), exp[g]), (i, g)
        finally:
            if sp:
                lib.fec_free_slab(sp)
            lib.fec_free_repair_buffer(rp)
            ctx.close()

    _run_threads(S, stream)
    st = quicfec_mod.coalesce_stats()
    vram = st["resident_vram"] > 0
    if resident and (pinned or vram):
        # every call served by the resident encoder (the ring of 1024 slots wrapped), a
        # launch only when no instance was running; in a VRAM ring every call (1 group,
        # 1200 B) has its packets inline
        assert st["resident_calls"] == S * CALLS and st["calls"] == 0, st
        assert 1 <= st["resident_launches"] < S * CALLS // 8, st
        assert st["resident_inline"] == (S * CALLS if vram else 0), st
    else:
        assert st["calls"] == S * CALLS and st["groups"] == S * CALLS
        # calls from different contexts shared launches
        assert st["batches"] < st["calls"] and st["max_calls"] >= 2, st


@pytest.mark.parametrize("P", [8, 17, 100, 1200, 1201, 1500])
def test_concurrent_mixed_calls_match_oracle(quicfec_mod, oracle_mod, P, monkeypatch):
    """Calls of 1..64 groups, scattered u32 offsets, pinned and pageable slabs, one batch."""
    monkeypatch.setenv("QUICFEC_COALESCE", "1")
    lib = quicfec_mod.load_library()
    quicfec_mod.coalesce_stats(reset=True)
    S = 8

    def stream(i):
        ctx = quicfec_mod.Context(device=0)
        rng = np.random.default_rng(7 * P + i)
        try:
            for call in range(24):
                G = int(rng.integers(1, 65))
                slab = oracle_mod.splitmix_bytes(G * 10 * P + 4096, 1000 * P + 37 * i + call)
                # each packet at an arbitrary byte offset (packet_size bytes read from each)
                offs = rng.integers(0, slab.nbytes - P + 1, size=G * 10).astype(np.uint32)
                pk = [[slab[o:o + P] for o in offs[g * 10:(g + 1) * 10]] for g in range(G)]
                exp = np.concatenate([oracle_mod.xor_packets(p, P) for p in pk])
                pinned = bool(call % 2)
                if pinned:
                    sp, rp = _pinned_copy(lib, slab), lib.fec_alloc_repair_buffer(G * P)
                    try:
                        assert lib.fec_encode_batch(ctx.handle, sp, offs.ctypes.data, G, P, rp) == 0
                        got = _read(rp, G * P)
                    finally:
                        lib.fec_free_slab(sp)
                        lib.fec_free_repair_buffer(rp)
                else:
                    got = np.full(G * P, 0xEE, dtype=np.uint8)
                    assert ctx.encode_batch_legacy(slab, offs, G, P, got) == 0
                assert np.array_equal(got, exp), (i, call, G, pinned)
        finally:
            ctx.close()

    _run_threads(S, stream)
    st = quicfec_mod.coalesce_stats()
    assert st["calls"] + st["resident_calls"] == S * 24, st
    if P >= 16:
        assert st["resident_calls"] > 0, st          # pinned calls of <= 8 groups


@pytest.mark.parametrize("coalesce", ["0", "1"])
def test_coalesce_switch_same_bytes(gpu_ctx, oracle_mod, xor_golden, manifest, coalesce, monkeypatch, quicfec_mod):
    """QUICFEC_COALESCE=0 runs the call alone on its context; both give the reference's bytes."""
    monkeypatch.setenv("QUICFEC_COALESCE", coalesce)
    quicfec_mod.coalesce_stats(reset=True)
    c = next(c for c in manifest["cases"] if c["name"] == "batch_scattered_p100_g16")
    slab = oracle_mod.splitmix_bytes(c["slab_bytes"], c["seed"])
    offs = xor_golden["batch_scattered_p100_g16_offsets"]
    rep = np.zeros(c["G"] * c["P"], dtype=np.uint8)
    assert gpu_ctx.encode_batch_legacy(slab, offs, c["G"], c["P"], rep) == 0
    assert np.array_equal(rep, xor_golden["batch_scattered_p100_g16"])
    assert quicfec_mod.coalesce_stats()["calls"] == (1 if coalesce == "1" else 0)


def test_large_and_device_calls_bypass(gpu_ctx, oracle_mod, quicfec_mod, torch_cuda, monkeypatch):
    """Calls above QUICFEC_COALESCE_MAX_GROUPS and device-resident calls run alone."""
    monkeypatch.setenv("QUICFEC_COALESCE", "1")
    monkeypatch.setenv("QUICFEC_COALESCE_MAX_GROUPS", "4")
    quicfec_mod.coalesce_stats(reset=True)
    G, P = 5, 300
    slab = oracle_mod.splitmix_bytes(G * 10 * P, 99)
    offs = (np.arange(G * 10, dtype=np.uint32) * P).astype(np.uint32)
    exp = np.concatenate([oracle_mod.xor_packets([slab[(g * 10 + j) * P:(g * 10 + j + 1) * P] for j in range(10)], P)
                          for g in range(G)])
    rep = np.zeros(G * P, dtype=np.uint8)
    assert gpu_ctx.encode_batch_legacy(slab, offs, G, P, rep) == 0
    assert np.array_equal(rep, exp)
    ds = torch_cuda.from_numpy(slab).cuda()
    do = torch_cuda.from_numpy(offs.view(np.int32)).cuda()
    dr = torch_cuda.zeros(4 * P, dtype=torch_cuda.uint8, device="cuda")
    assert gpu_ctx.encode_batch_legacy(ds, do, 4, P, dr) == 0
    assert np.array_equal(dr.cpu().numpy(), exp[:4 * P])
    assert quicfec_mod.coalesce_stats()["calls"] == 0
    rep4 = np.zeros(4 * P, dtype=np.uint8)
    assert gpu_ctx.encode_batch_legacy(slab, offs, 4, P, rep4) == 0
    assert np.array_equal(rep4, exp[:4 * P])
    st = quicfec_mod.coalesce_stats()
    # shared launches, or (VRAM ring: 4 groups of 300 B go inline) the resident encoder
    assert st["calls"] + st["resident_calls"] == 1
    assert st["resident_calls"] == (1 if st["resident_vram"] else 0), st


def test_resident_encoder_leaves_when_idle_and_comes_back(quicfec_mod, oracle_mod, monkeypatch):
    """The resident instance leaves after its idle time (default 2 ms); the next call launches
    the next one from the served-up-to mark and is served like the first."""
    import time
    monkeypatch.setenv("QUICFEC_COALESCE", "1")
    monkeypatch.setenv("QUICFEC_RESIDENT", "1")
    lib = quicfec_mod.load_library()
    P = 1200
    ctx = quicfec_mod.Context(device=0)
    sp, rp = lib.fec_alloc_slab(10 * P), lib.fec_alloc_repair_buffer(P)
    offs = (np.arange(10, dtype=np.uint32) * P).astype(np.uint32)
    try:
        time.sleep(0.05)  # an instance an earlier test's last call launched has left
        quicfec_mod.coalesce_stats(reset=True)
        for rnd in range(4):
            grp = oracle_mod.splitmix_bytes(10 * P, 4242 + rnd)
            ctypes.memmove(sp, grp.ctypes.data, grp.nbytes)
            assert lib.fec_encode_batch(ctx.handle, sp, offs.ctypes.data, 1, P, rp) == 0
            exp = oracle_mod.xor_packets([grp[j * P:(j + 1) * P] for j in range(10)], P)
            assert np.array_equal(_read(rp, P), exp), rnd
            time.sleep(0.05)                                   # well past the idle time
        st = quicfec_mod.coalesce_stats()
        assert st["resident_calls"] == 4 and st["resident_launches"] == 4, st
    finally:
        lib.fec_free_slab(sp)
        lib.fec_free_repair_buffer(rp)
        ctx.close()


def test_resident_repair_to_pageable_buffer(quicfec_mod, oracle_mod, monkeypatch):
    """Page-locked slab, pageable repair buffer: rows staged in the slot, copied out; 1..8 groups."""
    monkeypatch.setenv("QUICFEC_COALESCE", "1")
    monkeypatch.setenv("QUICFEC_RESIDENT", "1")
    lib = quicfec_mod.load_library()
    ctx = quicfec_mod.Context(device=0)
    quicfec_mod.coalesce_stats(reset=True)
    try:
        for G, P in ((1, 16), (3, 1201), (8, 1500), (8, 2048), (5, 333)):
            slab = oracle_mod.splitmix_bytes(G * 10 * P, 77 + G + P)
            offs = (np.arange(G * 10, dtype=np.uint32) * P).astype(np.uint32)[::-1].copy()   # any order
            sp = _pinned_copy(lib, slab)
            rep = np.full(G * P, 0xEE, dtype=np.uint8)
            try:
                assert lib.fec_encode_batch(ctx.handle, sp, offs.ctypes.data, G, P, rep.ctypes.data) == 0
            finally:
                lib.fec_free_slab(sp)
            exp = np.concatenate([oracle_mod.xor_packets([slab[o:o + P] for o in offs[g * 10:(g + 1) * 10]], P)
                                  for g in range(G)])
            assert np.array_equal(rep, exp), (G, P)
        assert quicfec_mod.coalesce_stats()["resident_calls"] == 5
    finally:
        ctx.close()


def test_process_exits_promptly_with_resident_instance(tmp_path):
    """A process that used the resident encoder exits at once: its exit handler stores the stop
    word and the instance leaves (no kernel outlives its process's last call by more than the
    poll it is in)."""
    import subprocess
    import sys
    import time
    from pathlib import Path
    repo = Path(__file__).resolve().parent.parent
    code = f"""
import ctypes, sys, numpy as np
sys.path.insert(0, {str(repo / 'quic-test_amd')!r})
import quicfec
lib = quicfec.load_library()
ctx = quicfec.Context(device=0)
P = 1200
sp, rp = lib.fec_alloc_slab(10 * P), lib.fec_alloc_repair_buffer(P)
ctypes.memset(sp, 7, 10 * P)
offs = (np.arange(10, dtype=np.uint32) * P).astype(np.uint32)
for _ in range(100):
    assert lib.fec_encode_batch(ctx.handle, sp, offs.ctypes.data, 1, P, rp) == 0
st = quicfec.coalesce_stats()
assert st["resident_calls"] == 100, st
print("CALLS_DONE", flush=True)
"""
    env = {**__import__("os").environ, "QUICFEC_COALESCE": "1", "QUICFEC_RESIDENT": "1",
           "QUICFEC_RESIDENT_IDLE_US": "10000000", "QUICFEC_RESIDENT_LIFE_US": "10000000"}
    t0 = time.monotonic()
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0 and "CALLS_DONE" in out.stdout, out.stdout + out.stderr
    # with a 10-s idle time the instance would still run at exit: only the stop word ends it
    assert time.monotonic() - t0 < 60


def test_resident_does_not_hold_up_other_streams(quicfec_mod, torch_cuda, monkeypatch):
    """While the resident encoder serves legacy calls (a persistent kernel on its own
    high-priority stream), kernels the same process launches on its other streams run at once:
    on a plain stream the runtime's queue pool put some of them behind the resident instance
    for up to its life bound (p99 33 ms, profiles/r03_probe_resident_interference.txt)."""
    import time
    monkeypatch.setenv("QUICFEC_COALESCE", "1")
    monkeypatch.setenv("QUICFEC_RESIDENT", "1")
    torch = torch_cuda
    lib = quicfec_mod.load_library()
    bg = quicfec_mod.Context(device=0)
    ctx = quicfec_mod.Context(device=0)
    G, k, r, P = 500, 10, 3, 1200
    data = torch.randint(0, 256, (G * k * P,), dtype=torch.uint8, device="cuda")
    par = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(8)]
    for s in streams:  # warm: module load, first launches
        ctx.encode_dev(data, G, k, r, P, par, stream=s.cuda_stream)
        s.synchronize()
    slab = lib.fec_alloc_slab(10 * P)
    rep = lib.fec_alloc_repair_buffer(P)
    offs = (np.arange(10, dtype=np.uint32) * P).astype(np.uint32)
    stop = threading.Event()
    calls = [0]

    def background():
        while not stop.is_set():
            assert lib.fec_encode_batch(bg.handle, slab, offs.ctypes.data, 1, P, rep) == 0
            calls[0] += 1

    th = threading.Thread(target=background)
    th.start()
    try:
        time.sleep(0.05)
        lat = []
        for i in range(96):
            s = streams[i % len(streams)]
            t0 = time.perf_counter()
            ctx.encode_dev(data, G, k, r, P, par, stream=s.cuda_stream)
            s.synchronize()
            lat.append(time.perf_counter() - t0)
            time.sleep(0.001)
    finally:
        stop.set()
        th.join()
        lib.fec_free_slab(slab)
        lib.fec_free_repair_buffer(rep)
        bg.close()
        ctx.close()
    assert calls[0] > 100, calls[0]  # the resident path was busy the whole time
    slow = [x for x in lat if x > 0.02]
    assert len(slow) <= 1, f"{len(slow)} of {len(lat)} launches took > 20 ms: {sorted(lat)[-5:]}"


def test_first_legacy_call_of_a_process_is_not_a_spike(tmp_path):
    """The first context on a device loads the kernels and sets up the resident ring, so the
    first fec_encode_batch of a fresh process (the first repair packet of the first stream)
    does not pay ~26 ms for them (profiles/r03_first_call_warmup.jsonl)."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parent.parent
    code = r'''
import ctypes, sys, time
import numpy as np
sys.path.insert(0, sys.argv[1])
import quicfec
lib = quicfec.load_library()
ctx = lib.fec_encoder_new(0.1, 64)
assert ctx
P = 1200
slab = lib.fec_alloc_slab(10 * P)
rep = lib.fec_alloc_repair_buffer(P)
offs = (np.arange(10, dtype=np.uint32) * P).astype(np.uint32)
t0 = time.perf_counter()
rc = lib.fec_encode_batch(ctx, slab, offs.ctypes.data, 1, P, rep)
dt = time.perf_counter() - t0
assert rc == 0, rc
print(f"{dt * 1e6:.1f}")
lib.fec_free_slab(slab)
lib.fec_free_repair_buffer(rep)
lib.fec_encoder_free(ctx)
'''
    env = {k: v for k, v in os.environ.items() if not k.startswith("QUICFEC_")}
    out = subprocess.run([sys.executable, "-c", code, str(repo / "quic-test_amd")], capture_output=True, text=True,
                         timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    first_us = float(out.stdout.strip().splitlines()[-1])
    assert first_us < 5000, f"first legacy call took {first_us:.0f} us"


# modes that inject faults (tests/csrc/exit_path_test.cpp): they run the program linked against
# the test library (libfec_hip_test.so, csrc/fec_knobs.hpp), the others the product library
_HOOK_MODES = ("nolaunch", "tear", "epoch", "epoch_hostring", "poison_mt")


def _exit_path_run(mode, calls=300, servers=None, product=None):
    """product: run the program linked against libfec_hip.so (default: unless the mode injects faults)."""
    import json
    import os
    import subprocess
    from pathlib import Path
    if product is None:
        product = mode not in _HOOK_MODES
    name = "exit_path_test" if product else "exit_path_test_hooks"
    exe = Path(__file__).resolve().parents[1] / "quic-test_amd" / "lib" / name
    assert exe.exists(), f"build() makes quic-test_amd/lib/{name} (csrc Makefile target tests)"
    env = dict(os.environ)
    if servers is not None:
        env["QUICFEC_RESIDENT_SERVERS"] = str(servers)
    out = subprocess.run([str(exe), mode, str(calls)], capture_output=True, text=True, timeout=90, env=env)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert out.returncode == 0 and lines, (out.returncode, out.stdout, out.stderr)
    return json.loads(lines[-1])


@pytest.mark.parametrize("mode", ["resident", "hostring", "coalescer", "pageable"])
def test_exit_makes_no_hip_call(mode):
    """A process that made legacy calls on each path (resident encoder, shared launches,
    pageable slab + repair buffer) and returns from main with its encoders alive exits with no
    HIP call from libfec_hip.so after exit began (the program counts them through its own
    definitions of the runtime entry points; tests/csrc/exit_path_test.cpp).  A HIP call there
    aborted a process under rocprofv3 (f13ed47)."""
    rec = _exit_path_run(mode)
    if "skip" in rec:
        pytest.skip(rec["skip"])
    assert rec["repairs_ok"] is True and rec["calls"] == 300
    assert rec["calls_after_exit"] == 0, rec["names"]


def test_never_serving_resident_poisons_itself():
    """A resident instance that never serves (QUICFEC_RESIDENT_TEST_NOLAUNCH: a launch is recorded
    but nothing runs) fails the call that waited on it within the deadline (200 ms here) and takes
    itself out of service: every later call -- past the ring's 1,024 slots -- completes on the
    shared-launch path with the right bytes instead of hanging, and the exit stays HIP-free."""
    import time
    t0 = time.monotonic()
    rec = _exit_path_run("nolaunch", calls=1_500)
    assert time.monotonic() - t0 < 60
    assert rec["first_rc"] == -2                        # FEC_ERR_HIP
    assert rec["repairs_ok"] is True and rec["calls"] == 1_500
    assert rec["calls_after_exit"] == 0, rec["names"]


@pytest.mark.parametrize("mode", ["mixed", "mixed_hostring"])
def test_resident_ring_kinds_mixed_shapes(mode):
    """Both resident ring kinds, each in a process of its own (the kind is fixed per process):
    360 calls cycling through shapes on both sides of the VRAM ring's inline bounds (1..8
    groups; P 16, 20, 100, 333, 1200, 1201, 1500, 1536, 1538, 2048; scattered offsets) over
    page-locked and pageable slabs and repair buffers -- every repair row checked against the
    XOR on the CPU.  In the VRAM ring the inline calls take the resident path from pageable
    slabs too; in the page-locked ring none is inline."""
    rec = _exit_path_run(mode, calls=360)
    if "skip" in rec:
        pytest.skip(rec["skip"])
    assert rec["repairs_ok"] is True and rec["calls"] == 360, rec
    assert rec["calls_after_exit"] == 0, rec["names"]
    assert rec["resident_calls"] > 0, rec
    if mode == "mixed_hostring":
        assert rec["resident_vram"] == 0 and rec["resident_inline"] == 0, rec
    elif rec["resident_vram"]:
        # inline shapes: (1,1200) (4,1536) (2,16) (3,100) (4,20) (1,1500) -- 6 of every 12 calls,
        # whatever the slab; page-locked slabs add the rest of the <= 8-group shapes
        assert rec["resident_inline"] == 180, rec
        assert rec["resident_calls"] > rec["resident_inline"], rec


def test_resident_serves_no_torn_chunk_or_late_address_word():
    """The VRAM ring's tags are per 8-B word (fec_kernels.hpp server_tag):
    with QUICFEC_RESIDENT_TEST_TEAR every inline call stores one chunk's tagged high half first
    and its low half ~100 us after the slot's header -- a 16-B write-combined store reaching the
    device as two pieces -- and every addressed call of several groups stores its later groups'
    address words ~100 us after the header.  The server must see those slots as not yet landed
    (resident_bad_slots > 0: it retried them) and serve every one only once both halves / every
    word arrived: each repair row equals the XOR of its ten packets (the reference's
    xor_packets_scalar, fec_xor_simd.cpp:411-427), computed on the CPU."""
    rec = _exit_path_run("tear", calls=300)
    if "skip" in rec:
        pytest.skip(rec["skip"])
    assert rec["repairs_ok"] is True and rec["calls"] == 300, rec
    assert rec["calls_after_exit"] == 0, rec["names"]
    if rec["resident_vram"]:  # pageable slabs take the resident path only inline (VRAM ring)
        assert rec["resident_calls"] == 300, rec
    assert rec["bad_slots"] > 0, rec


@pytest.mark.parametrize("mode", ["epoch", "epoch_hostring"])
def test_resident_tag_epoch_scrub_under_mixed_calls(mode):
    """a later group's address word written by an 8-group call and not since
    (one-group inline calls write none) carries the same tag again one tag epoch later.  With an
    epoch of 2 laps, slots 0, 5, 10, ... take 8-group addressed calls on even laps and one-group
    inline calls on odd laps over 6 laps (6,144 calls), and the tear hook stores the later groups'
    words ~100 us late, so the server reads the words two laps old first.  The server zeroes each
    slot after the last lap of an epoch (scrubs > 0), so those words never match: every row
    equals the CPU XOR.  Both ring kinds (VRAM; page-locked host memory, where no call is inline)."""
    rec = _exit_path_run(mode, calls=6 * 1024)
    if "skip" in rec:
        pytest.skip(rec["skip"])
    assert rec["repairs_ok"] is True and rec["calls"] == 6 * 1024, rec
    assert rec["calls_after_exit"] == 0, rec["names"]
    assert rec["resident_calls"] == 6 * 1024, rec
    # epochs end after laps 1 and 3 (and 5, if the last lap's calls were served before the read)
    assert rec["scrubs"] >= 2 * 1024, rec
    assert rec["bad_slots"] > 0, rec


def test_poisoned_resident_fails_no_in_flight_call():
    """when one call poisons the Resident (its deadline passed), the calls
    other threads have in flight must not fail with it.  8 threads with a context each make
    one-group calls; the 601st fails at once (QUICFEC_RESIDENT_TEST_FAIL_AT).  Its slot and every
    other published slot are either served before the instance leaves or, once it has left
    without serving them, run on the coalescer path: all 2,400 calls return 0 with the right row."""
    rec = _exit_path_run("poison_mt", calls=2_400)
    if "skip" in rec:
        pytest.skip(rec["skip"])
    assert rec["repairs_ok"] is True and rec["calls"] == 2_400, rec
    assert rec["calls_after_exit"] == 0, rec["names"]
    assert 600 <= rec["resident_calls"] < 2_400, rec


def test_resident_relaunch_cycles_under_concurrent_calls():
    """4 threads with a context each make one-group calls in bursts of 8 with 2-ms pauses, the
    idle bound at 300 us: resident instances leave and are relaunched many times while other
    threads' calls are in flight (each of the 8 serving classes resumes from its own progress
    mark), and every row equals the CPU XOR."""
    rec = _exit_path_run("cycles_mt", calls=2_000)
    if "skip" in rec:
        pytest.skip(rec["skip"])
    assert rec["resident_servers"] == (8 if rec["resident_vram"] else 1), rec  # the defaults per ring kind
    assert rec["repairs_ok"] is True and rec["calls"] == 2_000, rec
    assert rec["calls_after_exit"] == 0, rec["names"]
    assert rec["resident_calls"] == 2_000 and rec["resident_launches"] > 5, rec


def test_product_library_ignores_fault_injection():
    """The fault-injection switches exist only in the test library: the same poisoning run
    (QUICFEC_RESIDENT_TEST_FAIL_AT=600, which the program sets) against libfec_hip.so serves
    every one of the 2,400 calls on the resident encoder -- nothing fails, nothing is poisoned."""
    rec = _exit_path_run("poison_mt", calls=2_400, product=True)
    if "skip" in rec:
        pytest.skip(rec["skip"])
    assert rec["repairs_ok"] is True and rec["calls"] == 2_400, rec
    assert rec["resident_calls"] == 2_400, rec


# (mode, calls) of the runs above, repeated with several serving workgroups per resident instance
_SERVER_MODES = [("resident", 300), ("mixed", 360), ("mixed_hostring", 360), ("tear", 300), ("epoch", 6 * 1024),
                 ("poison_mt", 2_400), ("cycles_mt", 2_000)]


@pytest.mark.parametrize("servers", [1, 2, 4])
@pytest.mark.parametrize("mode,calls", _SERVER_MODES, ids=[m for m, _ in _SERVER_MODES])
def test_resident_serving_classes(mode, calls, servers):
    """QUICFEC_RESIDENT_SERVERS: the resident instance is `servers` workgroups (default 8 on the
    VRAM ring, which the runs above use, 1 on the page-locked ring), workgroup c serving the seqs of class c (seq % servers == c) with its own
    poll, run, done words and progress mark (fec_kernels.hip legacy_server).  Every ring-protocol
    run above -- mixed shapes on both ring kinds, torn chunks and late address words, epoch scrubs,
    poisoning under 8 threads, relaunch cycles under 4 -- gives every row equal to the CPU XOR
    with one, two and four classes too, and the exit stays HIP-free."""
    rec = _exit_path_run(mode, calls=calls, servers=servers)
    if "skip" in rec:
        pytest.skip(rec["skip"])
    assert rec["repairs_ok"] is True and rec["calls"] == calls, rec
    assert rec["calls_after_exit"] == 0, rec["names"]
    assert rec["resident_servers"] == servers, rec
    if mode == "poison_mt":
        assert 600 <= rec["resident_calls"] < calls, rec
    elif mode in ("tear", "epoch") and rec["resident_vram"]:
        assert rec["resident_calls"] == calls and rec["bad_slots"] > 0, rec
        if mode == "epoch":
            assert rec["scrubs"] >= 2 * 1024, rec
    elif mode == "cycles_mt":
        assert rec["resident_calls"] == calls and rec["resident_launches"] > 5, rec
    else:
        assert rec["resident_calls"] > 0, rec
