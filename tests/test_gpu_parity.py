"""GPU parity tests: libfec_hip.so (through its C-ABI) against the oracle and the
reference-generated golden fixtures.  Bit-exact everywhere (byte arithmetic).

Small cases compare every byte with the oracle; BASELINE.json's full sizes (1M groups,
k=10 r=3 / k=20 r=5, 1200 B) are checked through sampled groups against the oracle and
the size-independent encode -> erase -> decode round trip.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED0000


def _dev(torch, arr):
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


# ---------------- reference ABI: fec_encode_batch, xor_packets_* ----------------

def test_legacy_batch_golden_host_pinned_device(gpu_ctx, quicfec_mod, oracle_mod, xor_golden, manifest, torch_cuda):
    c = next(c for c in manifest["cases"] if c["name"] == "batch_k10_p1200_g64")
    G, P = c["G"], c["P"]
    slab = oracle_mod.splitmix_bytes(G * 10 * P, c["seed"])
    offs = (np.arange(G * 10, dtype=np.uint32) * P).astype(np.uint32)
    exp = xor_golden["batch_k10_p1200_g64"]
    # pageable host memory
    rep = np.zeros(G * P, dtype=np.uint8)
    assert gpu_ctx.encode_batch_legacy(slab, offs, G, P, rep) == 0
    assert np.array_equal(rep, exp)
    # pinned slab + repair from fec_alloc_slab / fec_alloc_repair_buffer (the Go wrapper's path)
    lib = quicfec_mod.load_library()
    ps = lib.fec_alloc_slab(slab.nbytes)
    pr = lib.fec_alloc_repair_buffer(rep.nbytes)
    assert ps and pr and ps % 64 == 0
    import ctypes
    ctypes.memmove(ps, slab.ctypes.data, slab.nbytes)
    assert lib.fec_encode_batch(gpu_ctx.handle, ps, offs.ctypes.data, G, P, pr) == 0
    got = np.ctypeslib.as_array((ctypes.c_uint8 * rep.nbytes).from_address(pr)).copy()
    lib.fec_free_slab(ps)
    lib.fec_free_repair_buffer(pr)
    assert np.array_equal(got, exp)
    # device pointers
    ds, do, dr = _dev(torch_cuda, slab), _dev(torch_cuda, offs.view(np.int32)), torch_cuda.zeros(G * P, dtype=torch_cuda.uint8, device="cuda")
    assert gpu_ctx.encode_batch_legacy(ds, do, G, P, dr) == 0
    assert np.array_equal(dr.cpu().numpy(), exp)


def test_legacy_batch_scattered_unaligned(gpu_ctx, oracle_mod, xor_golden, manifest):
    c = next(c for c in manifest["cases"] if c["name"] == "batch_scattered_p100_g16")
    slab = oracle_mod.splitmix_bytes(c["slab_bytes"], c["seed"])
    offs = xor_golden["batch_scattered_p100_g16_offsets"]
    rep = np.zeros(c["G"] * c["P"], dtype=np.uint8)
    assert gpu_ctx.encode_batch_legacy(slab, offs, c["G"], c["P"], rep) == 0
    assert np.array_equal(rep, xor_golden["batch_scattered_p100_g16"])


def test_legacy_return_codes(gpu_ctx, manifest):
    codes = manifest["legacy_return_codes"]
    buf = np.zeros(64, dtype=np.uint8)
    off = np.zeros(10, dtype=np.uint32)
    rep = np.full(8, 0xAB, dtype=np.uint8)
    assert gpu_ctx.encode_batch_legacy(None, off, 1, 8, rep) == codes["null_slab"]
    assert gpu_ctx.encode_batch_legacy(buf, None, 1, 8, rep) == codes["null_offsets"]
    assert gpu_ctx.encode_batch_legacy(buf, off, 1, 8, None) == codes["null_repair"]
    assert gpu_ctx.encode_batch_legacy(buf, off, 0, 8, rep) == codes["zero_groups"]
    assert gpu_ctx.encode_batch_legacy(buf, off, 1, 0, rep) == codes["zero_size"]
    assert (rep == 0xAB).all()


@pytest.mark.parametrize("variant", ["avx2", "scalar", "avx512", "neon"])
def test_xor_packets_entry_points_golden(quicfec_mod, oracle_mod, xor_golden, manifest, variant):
    n = 0
    for c in manifest["cases"]:
        if c["api"] != "xor_packets_avx2" or "G" not in c:
            continue
        data = oracle_mod.splitmix_bytes(c["G"] * c["k"] * c["P"], c["seed"])
        got = []
        for g in range(c["G"]):
            pk = [data[(g * c["k"] + j) * c["P"]:(g * c["k"] + j + 1) * c["P"]] for j in range(c["k"])]
            out = np.zeros(c["P"], dtype=np.uint8)
            quicfec_mod.xor_packets(pk, c["P"], out, variant=variant)
            got.append(out)
        assert np.array_equal(np.concatenate(got), xor_golden[c["name"]]), (variant, c["name"])
        n += 1
    assert n >= 12
    pk = [np.full(1200, i, dtype=np.uint8) for i in range(10)]
    out = np.zeros(1200, dtype=np.uint8)
    quicfec_mod.xor_packets(pk, 1200, out, variant=variant)
    assert np.array_equal(out, xor_golden["kat_encoder_test"])
    pre = np.full(16, 0x5A, dtype=np.uint8)
    quicfec_mod.xor_packets([], 16, pre, variant=variant)
    assert (pre == 0x5A).all()


def test_select_xor_impl_is_callable(quicfec_mod, oracle_mod):
    lib = quicfec_mod.load_library()
    fn = quicfec_mod.XOR_IMPL_FN(lib.fec_select_xor_impl())
    pk = [oracle_mod.splitmix_bytes(300, s) for s in range(5)]
    import ctypes
    arr = (ctypes.c_void_p * 5)(*[p.ctypes.data for p in pk])
    out = np.zeros(300, dtype=np.uint8)
    fn(arr, 5, 300, out.ctypes.data)
    assert np.array_equal(out, oracle_mod.xor_packets(pk, 300))


# ---------------- batch GF(2^8) API ----------------

SHAPES = [(4, 2, 256), (10, 3, 1200), (20, 5, 1200), (10, 1, 1200), (7, 4, 48), (12, 9, 64),
          (3, 1, 16), (10, 3, 100), (5, 3, 33), (1, 1, 7), (30, 20, 32), (10, 2, 1200), (10, 2, 700)]


@pytest.mark.parametrize("k,r,P", SHAPES)
def test_rs_encode_matches_oracle(gpu_ctx, oracle_mod, torch_cuda, k, r, P):
    G = 97
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + k * 1000 + r * 10 + P)
    exp = oracle_mod.rs_encode(data, G, k, r, P)
    par = np.zeros(G * r * P, dtype=np.uint8)
    gpu_ctx.encode(data, k, r, P, par, num_groups=G)
    assert np.array_equal(par, exp)
    dd = _dev(torch_cuda, data)
    dp = torch_cuda.zeros(G * r * P, dtype=torch_cuda.uint8, device="cuda")
    gpu_ctx.encode_dev(dd, G, k, r, P, dp)
    gpu_ctx.synchronize()
    assert np.array_equal(dp.cpu().numpy(), exp)


@pytest.mark.parametrize("aligned", [True, False])
def test_rs_encode_gather_offsets(gpu_ctx, oracle_mod, aligned):
    k, r, P, G = 10, 3, 1200 if aligned else 1201, 23
    rng = np.random.default_rng(7)
    slab = oracle_mod.splitmix_bytes(G * k * P * 2 + 64, 99)
    slots = rng.permutation(G * k * 2)[:G * k]
    offs = (slots.astype(np.uint64) * P).astype(np.uint64)
    contig = np.concatenate([slab[int(o):int(o) + P] for o in offs])
    exp = oracle_mod.rs_encode(contig, G, k, r, P)
    par = np.zeros(G * r * P, dtype=np.uint8)
    gpu_ctx.encode(slab, k, r, P, par, num_groups=G, offsets=offs)
    assert np.array_equal(par, exp)


def _random_masks(rng, G, k, r, max_lost):
    masks = np.zeros(G, dtype=np.uint64)
    for g in range(G):
        ne = int(rng.integers(0, max_lost + 1))
        pos = rng.choice(k + r, size=min(ne, k + r), replace=False)
        masks[g] = np.uint64(sum(1 << int(p) for p in pos))
    return masks


def _poison(data, masks, G, k, P):
    d = data.copy().reshape(G, k, P)
    for g in range(G):
        for j in range(k):
            if (int(masks[g]) >> j) & 1:
                d[g, j, :] = 0xEE
    return d.reshape(-1)


@pytest.mark.parametrize("k,r,P", SHAPES + [(16, 16, 32), (32, 8, 48)])
def test_rs_decode_matches_oracle(gpu_ctx, oracle_mod, torch_cuda, k, r, P):
    """Dense codebook shapes and, for (30,20), (16,16), (32,8), the per-call sparse plan."""
    G = 211
    rng = np.random.default_rng(k * 131 + r * 7 + P)
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 77 + k + r + P)
    par = oracle_mod.rs_encode(data, G, k, r, P)
    masks = _random_masks(rng, G, k, r, r + 1)
    broken = _poison(data, masks, G, k, P)
    exp = broken.copy()
    bad_exp, st_exp = oracle_mod.rs_decode(exp, par, masks, G, k, r, P)
    got = broken.copy()
    st = np.zeros(G, dtype=np.uint8)
    bad = gpu_ctx.decode(got, par, masks, k, r, P, status_out=st)
    assert bad == bad_exp
    assert np.array_equal(st, st_exp)
    assert np.array_equal(got, exp)
    # device-resident API
    dd, dpar, dm = _dev(torch_cuda, broken), _dev(torch_cuda, par), _dev(torch_cuda, masks.view(np.int64))
    # 0xAA: every status byte must be written by the device (inline classify included)
    dst = torch_cuda.full((G,), 0xAA, dtype=torch_cuda.uint8, device="cuda")
    gpu_ctx.decode_dev(dd, dpar, dm, G, k, r, P, dst)
    gpu_ctx.synchronize()
    assert np.array_equal(dd.cpu().numpy(), exp)
    assert np.array_equal(dst.cpu().numpy(), st_exp)


def test_gf_golden_fixtures(gpu_ctx, oracle_mod, manifest, gf_golden):
    for c in manifest["cases"]:
        if not c["name"].startswith("rs_"):
            continue
        G, k, r, P = c["G"], c["k"], c["r"], c["P"]
        data = oracle_mod.splitmix_bytes(G * k * P, c["seed"])
        par = np.zeros(G * r * P, dtype=np.uint8)
        gpu_ctx.encode(data, k, r, P, par, num_groups=G)
        assert np.array_equal(par, gf_golden[c["name"] + "_parity"]), c["name"]
        masks = gf_golden[c["name"] + "_masks"]
        broken = _poison(data, masks, G, k, P)
        st = np.zeros(G, dtype=np.uint8)
        bad = gpu_ctx.decode(broken, par, masks, k, r, P, status_out=st)
        assert bad == c["unrecoverable"]
        assert np.array_equal(broken, gf_golden[c["name"] + "_decoded"]), c["name"]


def test_single_loss_is_reference_xor_recovery(gpu_ctx, oracle_mod):
    """1 lost data shard + parity row 0 alive == FECDecoder.recoverSingle (decoder.go:255-287)."""
    k, r, P, G = 10, 3, 1200, 50
    data = oracle_mod.splitmix_bytes(G * k * P, 4242)
    par = oracle_mod.rs_encode(data, G, k, r, P)
    rng = np.random.default_rng(3)
    lost = rng.integers(0, k, size=G)
    masks = np.array([1 << int(j) for j in lost], dtype=np.uint64)
    got = _poison(data, masks, G, k, P)
    assert gpu_ctx.decode(got, par, masks, k, r, P) == 0
    for g in range(G):
        pk = [None if j == lost[g] else data[(g * k + j) * P:(g * k + j + 1) * P] for j in range(k)]
        mid, rec = oracle_mod.go_recover_single(pk, par[g * r * P:g * r * P + P], P)
        assert mid == lost[g]
        assert np.array_equal(got[(g * k + mid) * P:(g * k + mid + 1) * P], rec)


@pytest.mark.parametrize("pinned,dma", [(True, False), (True, True), (False, False)])
def test_host_pipeline_multi_chunk(gpu_ctx, oracle_mod, torch_cuda, monkeypatch, pinned, dma):
    """Host-resident batches larger than one 64 MB pipeline chunk (5 chunks over 3 slots);
    page-locked buffers run zero-copy unless QUICFEC_SMALL_CALL_BYTES=0 forces the DMA path."""
    if dma:
        monkeypatch.setenv("QUICFEC_SMALL_CALL_BYTES", "0")
    k, r, P, G = 10, 3, 1200, 27_000
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 11)
    exp = oracle_mod.rs_encode(data, G, k, r, P, nthreads=8)
    if pinned:
        h_data = torch_cuda.from_numpy(data).pin_memory()
        h_par = torch_cuda.zeros(G * r * P, dtype=torch_cuda.uint8).pin_memory()
    else:
        h_data, h_par = data.copy(), np.zeros(G * r * P, dtype=np.uint8)
    gpu_ctx.encode(h_data, k, r, P, h_par, num_groups=G)
    got = h_par.numpy() if pinned else h_par
    assert np.array_equal(got, exp)
    rng = np.random.default_rng(12)
    masks = _random_masks(rng, G, k, r, r + 1)
    broken = _poison(data, masks, G, k, P)
    ref = broken.copy()
    bad_exp, st_exp = oracle_mod.rs_decode(ref, exp, masks, G, k, r, P, nthreads=8)
    if pinned:
        hb = torch_cuda.from_numpy(broken).pin_memory()
        st = torch_cuda.zeros(G, dtype=torch_cuda.uint8).pin_memory()
        bad = gpu_ctx.decode(hb, h_par, masks, k, r, P, status_out=st, num_groups=G)
        hb, st = hb.numpy(), st.numpy()
    else:
        hb, st = broken, np.zeros(G, dtype=np.uint8)
        bad = gpu_ctx.decode(hb, exp, masks, k, r, P, status_out=st)
    assert bad == bad_exp
    assert np.array_equal(st, st_exp)
    assert np.array_equal(hb, ref)


@pytest.mark.parametrize("k,r,P,pinned,dma", [(10, 3, 1200, True, True), (10, 3, 1200, True, False),
                                              (10, 3, 1200, False, False), (20, 5, 96, False, False),
                                              (10, 3, 100, True, True), (4, 2, 256, False, False)])
def test_host_decode_compacted_sparse_loss(gpu_ctx, oracle_mod, torch_cuda, monkeypatch, k, r, P, pinned, dma):
    """Host-resident decode under iid loss (satellite profile, network_profiles.go:78): at most
    half the groups need work, so only those cross PCIe (gathered, decoded, scattered back).
    Small pipeline chunks so the 3 slots rotate several times; some groups unrecoverable."""
    G = 6_000
    monkeypatch.setenv("QUICFEC_PIPE_CHUNK_BYTES", str(k * P * 97))
    monkeypatch.setenv("QUICFEC_SMALL_CALL_BYTES", "0" if dma else "1000000000000" if pinned else "")
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 21 + k + P)
    par = oracle_mod.rs_encode(data, G, k, r, P, nthreads=8)
    rng = np.random.default_rng(k * 7 + P)
    w = np.left_shift(np.uint64(1), np.arange(k + r, dtype=np.uint64))
    masks = ((rng.random((G, k + r)) < 0.02) * w).sum(axis=1, dtype=np.uint64)
    masks[rng.integers(0, G, size=9)] = np.uint64((1 << (r + 1)) - 1)   # r+1 data shards lost
    masks[5] = np.uint64(0)
    broken = _poison(data, masks, G, k, P)
    ref = broken.copy()
    bad_exp, st_exp = oracle_mod.rs_decode(ref, par, masks, G, k, r, P, nthreads=8)
    assert 0 < bad_exp and (st_exp == 0).sum() > 0
    if pinned:
        hb = torch_cuda.from_numpy(broken).pin_memory()
        hp = torch_cuda.from_numpy(par).pin_memory()
        st = np.zeros(G, dtype=np.uint8)
        bad = gpu_ctx.decode(hb, hp, masks, k, r, P, status_out=st, num_groups=G)
        got = hb.numpy()
    else:
        got, st = broken.copy(), np.zeros(G, dtype=np.uint8)
        bad = gpu_ctx.decode(got, par, masks, k, r, P, status_out=st)
    assert bad == bad_exp
    assert np.array_equal(st, st_exp)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_device_group_shards_host_batches(quicfec_mod, oracle_mod, torch_cuda, devices):
    """fec_group_*: a host batch split over shards (one context + host thread each); with
    one GPU, [0, 0, 0] runs three shards concurrently on it.  Bit-exact vs the oracle."""
    k, r, P, G = 10, 3, 1200, 3001
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 31)
    exp = oracle_mod.rs_encode(data, G, k, r, P, nthreads=8)
    rng = np.random.default_rng(31)
    masks = _random_masks(rng, G, k, r, r + 1)
    broken = _poison(data, masks, G, k, P)
    ref = broken.copy()
    bad_exp, st_exp = oracle_mod.rs_decode(ref, exp, masks, G, k, r, P, nthreads=8)
    with quicfec_mod.DeviceGroup(devices) as grp:
        assert len(grp) == (3 if devices else quicfec_mod.device_count())
        par = np.zeros(G * r * P, dtype=np.uint8)
        grp.encode(data, k, r, P, par)
        assert np.array_equal(par, exp)
        h_par = torch_cuda.from_numpy(par).pin_memory()         # page-locked parity
        st = np.zeros(G, dtype=np.uint8)
        bad = grp.decode(broken, h_par, masks, k, r, P, status_out=st)
        assert bad == bad_exp
        assert np.array_equal(st, st_exp)
        assert np.array_equal(broken, ref)
        dd = torch_cuda.from_numpy(data).cuda()                  # device buffers are refused
        with pytest.raises(quicfec_mod.FecError) as ei:
            grp.encode(dd, k, r, P, par, num_groups=G)
        assert ei.value.code == quicfec_mod.FEC_ERR_RANGE
    with pytest.raises(quicfec_mod.FecError):
        quicfec_mod.DeviceGroup([quicfec_mod.device_count()])    # ordinal out of range


def test_fill_random_matches_oracle(gpu_ctx, oracle_mod, torch_cuda):
    for n, off in ((4096, 0), (1000, 8), (777, 3)):
        d = torch_cuda.zeros(n + 16, dtype=torch_cuda.uint8, device="cuda")
        gpu_ctx.fill_random_dev(d, n, 0x1234, off)
        gpu_ctx.synchronize()
        assert np.array_equal(d.cpu().numpy()[:n], oracle_mod.splitmix_bytes(n, 0x1234, off))


def test_copy_dev(gpu_ctx, quicfec_mod, torch_cuda):
    src = torch_cuda.randint(0, 256, (1 << 20,), dtype=torch_cuda.uint8, device="cuda")
    dst = torch_cuda.zeros(src.numel() + 32, dtype=torch_cuda.uint8, device="cuda")
    gpu_ctx.copy_dev(src, dst, src.numel())
    gpu_ctx.synchronize()
    assert torch_cuda.equal(dst[:src.numel()], src) and int(dst[src.numel():].sum()) == 0
    with pytest.raises(quicfec_mod.FecError) as ei:
        gpu_ctx.copy_dev(src, dst, 100)
    assert ei.value.code == quicfec_mod.FEC_ERR_RANGE


def test_decode_prepare_sizes(gpu_ctx):
    assert gpu_ctx.decode_prepare(10, 3) > 0
    assert gpu_ctx.decode_prepare(20, 5) > 0
    assert gpu_ctx.decode_prepare(16, 16) == 0      # over the dense cap: sparse per-call plans
    import quicfec
    with pytest.raises(quicfec.FecError):
        gpu_ctx.decode_prepare(40, 30)


# ---------------- BASELINE.json full sizes (size-independent properties) ----------------

def _sample_check(torch, gpu_ctx, oracle_mod, d_data, d_par, G, k, r, P, n=48, seed=1):
    rng = np.random.default_rng(seed)
    gs = np.unique(np.concatenate([[0, G - 1], rng.integers(0, G, size=n)]))
    for g in gs:
        g = int(g)
        blk = d_data[g * k * P:(g + 1) * k * P].cpu().numpy()
        exp = oracle_mod.rs_encode(blk, 1, k, r, P)
        assert np.array_equal(d_par[g * r * P:(g + 1) * r * P].cpu().numpy(), exp), g


@pytest.mark.slow
def test_full_size_c2_c3_round_trip(gpu_ctx, oracle_mod, torch_cuda):
    torch = torch_cuda
    k, r, P, G = 10, 3, 1200, 1_000_000
    data = torch.empty(G * k * P, dtype=torch.uint8, device="cuda")
    par = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_random_dev(data, data.numel(), SEED + 2)
    gpu_ctx.encode_dev(data, G, k, r, P, par)
    gpu_ctx.synchronize()
    _sample_check(torch, gpu_ctx, oracle_mod, data, par, G, k, r, P)
    # C3: exactly 2 erasures per group, uniform over the 13 shards
    rng = np.random.default_rng(SEED + 3)
    keys = rng.random((G, k + r))
    pos = np.argsort(keys, axis=1)[:, :2]
    masks = (np.left_shift(np.uint64(1), pos.astype(np.uint64))).sum(axis=1, dtype=np.uint64)
    orig = data.clone()
    dm = torch.from_numpy(masks.view(np.int64)).cuda()
    lost = torch.zeros((G, k), dtype=torch.bool, device="cuda")
    bits = torch.arange(k, device="cuda", dtype=torch.int64)
    lost = ((dm.view(G, 1) >> bits.view(1, k)) & 1).bool()
    data.view(G, k, P)[lost] = 0xEE
    st = torch.zeros(G, dtype=torch.uint8, device="cuda")
    gpu_ctx.decode_dev(data, par, dm, G, k, r, P, st, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(st.sum().item()) == 0
    assert torch.equal(data, orig)


@pytest.mark.slow
def test_full_size_c4_shard_encode(gpu_ctx, oracle_mod, torch_cuda):
    torch = torch_cuda
    k, r, P, G = 20, 5, 1200, 1_000_000      # one GPU's shard of C4 (8M groups / 8)
    data = torch.empty(G * k * P, dtype=torch.uint8, device="cuda")
    par = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_random_dev(data, data.numel(), SEED + 4)
    gpu_ctx.encode_dev(data, G, k, r, P, par)
    gpu_ctx.synchronize()
    _sample_check(torch, gpu_ctx, oracle_mod, data, par, G, k, r, P, n=24)
    # erase r shards in a slice of groups and rebuild
    Gs = 50_000
    rng = np.random.default_rng(5)
    pos = np.argsort(rng.random((Gs, k + r)), axis=1)[:, :r]
    masks = (np.left_shift(np.uint64(1), pos.astype(np.uint64))).sum(axis=1, dtype=np.uint64)
    dm = torch.from_numpy(masks.view(np.int64)).cuda()
    sub = data[:Gs * k * P]
    orig = sub.clone()
    bits = torch.arange(k, device="cuda", dtype=torch.int64)
    lost = ((dm.view(Gs, 1) >> bits.view(1, k)) & 1).bool()
    sub.view(Gs, k, P)[lost] = 0x11
    gpu_ctx.decode_dev(sub, par[:Gs * r * P], dm, Gs, k, r, P, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(sub, orig)


# ---------------- any packet size, any packet address ----------------
#
# P >= 16 runs on the 16-byte-column kernels whatever P % 16 and the packet alignment are:
# the last column of a packet is shifted back to end at P (fec_kernels.hip header).  These
# cases cover every encode form (compile-time k, runtime-k loop, gathered offsets) and every
# decode form the library picks (fused with NT = 1..4 tail pieces, mask-addressed or not,
# the runtime-k wave kernel), with sizes around the 16-B, 256-B and 1 KiB boundaries.

ANY_P = [(10, 3, 1201), (10, 3, 1350), (10, 3, 1400), (10, 3, 1452), (10, 3, 1500), (10, 3, 1023),
         (10, 3, 1025), (10, 3, 2047), (10, 3, 3001), (10, 3, 17), (10, 3, 31), (20, 5, 1399),
         (20, 5, 1235), (10, 1, 1350), (4, 2, 250), (4, 2, 301), (7, 4, 1399), (12, 9, 70),
         (3, 1, 18), (16, 16, 45),
         # k=20 r=5 fused forms with LDS-staged tables: every (NM, NT) piece layout
         (20, 5, 300), (20, 5, 700), (20, 5, 1000), (20, 5, 1024), (20, 5, 1500), (20, 5, 1600),
         (20, 5, 1800)]


@pytest.mark.parametrize("k,r,P", ANY_P)
def test_any_packet_size_round_trip(gpu_ctx, oracle_mod, torch_cuda, k, r, P):
    torch = torch_cuda
    G = 67
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 901 + k * 7 + P)
    exp_par = oracle_mod.rs_encode(data, G, k, r, P)
    par = np.zeros(G * r * P, dtype=np.uint8)
    gpu_ctx.encode(data, k, r, P, par, num_groups=G)
    assert np.array_equal(par, exp_par)
    rng = np.random.default_rng(P * 31 + k)
    masks = _random_masks(rng, G, k, r, r + 1)
    broken = _poison(data, masks, G, k, P)
    exp = broken.copy()
    bad_exp, st_exp = oracle_mod.rs_decode(exp, exp_par, masks, G, k, r, P)
    got = broken.copy()
    st = np.zeros(G, dtype=np.uint8)
    assert gpu_ctx.decode(got, exp_par, masks, k, r, P, status_out=st) == bad_exp
    assert np.array_equal(st, st_exp)
    assert np.array_equal(got, exp)
    # Device views at odd byte addresses (packet bases misaligned for every dword / 16-B access).
    for shift_d, shift_p in [(1, 3), (5, 15), (8, 0)]:
        bd = torch.zeros(G * k * P + 32, dtype=torch.uint8, device="cuda")
        bp = torch.zeros(G * r * P + 32, dtype=torch.uint8, device="cuda")
        dd = bd[shift_d:shift_d + G * k * P]
        dp = bp[shift_p:shift_p + G * r * P]
        dd.copy_(torch.from_numpy(data))
        gpu_ctx.encode_dev(dd, G, k, r, P, dp)
        gpu_ctx.synchronize()
        assert np.array_equal(dp.cpu().numpy(), exp_par), (shift_d, shift_p)
        # guard bytes around the views untouched
        assert int(bp[:shift_p].sum().item()) == 0 and int(bp[shift_p + G * r * P:].sum().item()) == 0
        dd.copy_(torch.from_numpy(broken))
        dm = _dev(torch, masks.view(np.int64))
        dst = torch.full((G,), 0xAA, dtype=torch.uint8, device="cuda")  # every byte written
        gpu_ctx.decode_dev(dd, dp, dm, G, k, r, P, dst)
        gpu_ctx.synchronize()
        assert np.array_equal(dd.cpu().numpy(), exp), (shift_d, shift_p)
        assert np.array_equal(dst.cpu().numpy(), st_exp)
        assert int(bd[:shift_d].sum().item()) == 0 and int(bd[shift_d + G * k * P:].sum().item()) == 0


@pytest.mark.parametrize("P", [1201, 1350, 37])
def test_any_packet_size_gather_offsets_odd(gpu_ctx, oracle_mod, P):
    """u64 offsets at arbitrary (odd) byte positions of the slab."""
    k, r, G = 10, 3, 29
    rng = np.random.default_rng(P)
    slab = oracle_mod.splitmix_bytes(G * k * (P + 7) + 64, 1234 + P)
    offs = (np.arange(G * k, dtype=np.uint64) * np.uint64(P + 7) + np.uint64(3)).astype(np.uint64)
    offs = offs[rng.permutation(G * k)]
    contig = np.concatenate([slab[int(o):int(o) + P] for o in offs])
    exp = oracle_mod.rs_encode(contig, G, k, r, P)
    par = np.zeros(G * r * P, dtype=np.uint8)
    gpu_ctx.encode(slab, k, r, P, par, num_groups=G, offsets=offs)
    assert np.array_equal(par, exp)


# ---------------- small host-resident calls: zero-copy vs DMA ----------------
#
# Calls of at most QUICFEC_SMALL_CALL_BYTES (default 1 MiB) run the kernels directly on
# page-locked host memory (the caller's, or the context's staging); 0 forces the DMA paths.

@pytest.mark.parametrize("small", ["0", None])
@pytest.mark.parametrize("pinned", [True, False])
def test_small_calls_zero_copy_and_dma(gpu_ctx, quicfec_mod, oracle_mod, xor_golden, manifest, torch_cuda,
                                       monkeypatch, small, pinned):
    import ctypes
    if small is None:
        monkeypatch.delenv("QUICFEC_SMALL_CALL_BYTES", raising=False)
    else:
        monkeypatch.setenv("QUICFEC_SMALL_CALL_BYTES", small)
    torch = torch_cuda

    def host(a):
        return torch.from_numpy(np.ascontiguousarray(a)).pin_memory() if pinned else np.ascontiguousarray(a).copy()

    def npy(a):
        return a.numpy() if pinned else a

    # legacy fec_encode_batch: golden fixture, and scattered offsets into a larger slab
    c = next(c for c in manifest["cases"] if c["name"] == "batch_k10_p1200_g64")
    G, P = c["G"], c["P"]
    slab = host(oracle_mod.splitmix_bytes(G * 10 * P, c["seed"]))
    offs = (np.arange(G * 10, dtype=np.uint32) * P).astype(np.uint32)
    rep = host(np.zeros(G * P, dtype=np.uint8))
    assert gpu_ctx.encode_batch_legacy(slab, offs, G, P, rep) == 0
    assert np.array_equal(npy(rep), xor_golden["batch_k10_p1200_g64"])
    c = next(c for c in manifest["cases"] if c["name"] == "batch_scattered_p100_g16")
    slab = host(oracle_mod.splitmix_bytes(c["slab_bytes"], c["seed"]))
    rep = host(np.zeros(c["G"] * c["P"], dtype=np.uint8))
    assert gpu_ctx.encode_batch_legacy(slab, xor_golden["batch_scattered_p100_g16_offsets"], c["G"], c["P"], rep) == 0
    assert np.array_equal(npy(rep), xor_golden["batch_scattered_p100_g16"])
    # batch API, one group and a few, odd packet size
    for k, r, P, G in [(10, 3, 1200, 1), (10, 3, 1201, 7), (20, 5, 1200, 3), (4, 2, 256, 40)]:
        data = oracle_mod.splitmix_bytes(G * k * P, SEED + 5000 + G + P)
        exp = oracle_mod.rs_encode(data, G, k, r, P)
        hd, hp = host(data), host(np.zeros(G * r * P, dtype=np.uint8))
        gpu_ctx.encode(hd, k, r, P, hp, num_groups=G)
        assert np.array_equal(npy(hp), exp), (k, r, P, G)
        rng = np.random.default_rng(G + P)
        masks = _random_masks(rng, G, k, r, r + 1)
        masks[0] = np.uint64(1)  # at least one rebuilt group
        broken = _poison(data, masks, G, k, P)
        ref = broken.copy()
        bad_exp, st_exp = oracle_mod.rs_decode(ref, exp, masks, G, k, r, P)
        hb = host(broken)
        st = np.zeros(G, dtype=np.uint8)
        assert gpu_ctx.decode(hb, hp, masks, k, r, P, status_out=st, num_groups=G) == bad_exp
        assert np.array_equal(st, st_exp)
        assert np.array_equal(npy(hb), ref), (k, r, P, G)
    # xor_packets_* (context-free entry point): ten host packets
    pk = [oracle_mod.splitmix_bytes(1200, 77 + i) for i in range(10)]
    out = np.zeros(1200, dtype=np.uint8)
    quicfec_mod.xor_packets(pk, 1200, out)
    assert np.array_equal(out, oracle_mod.xor_packets(pk, 1200))


# ---------------- round-2 fixes ----------------

@pytest.mark.parametrize("n", [255, 256, 300, 1000])
def test_xor_packets_many_packets(quicfec_mod, oracle_mod, n):
    """xor_packets_* XOR any number of packets like xor_packets_scalar
    (fec_xor_simd.cpp:411-427): the XOR row needs no GF matrix, so n >= 256 works."""
    P = 1200
    pk = [oracle_mod.splitmix_bytes(P, 0xA000 + i) for i in range(n)]
    out = np.full(P, 0xCC, dtype=np.uint8)
    quicfec_mod.xor_packets(pk, P, out)
    assert quicfec_mod.last_error() == ""
    assert np.array_equal(out, oracle_mod.xor_packets(pk, P, avx2=False))


@pytest.mark.parametrize("k,r,P,erasures", [(20, 5, 1200, 5), (10, 3, 200, 2), (6, 4, 1000, 3)])
def test_concurrent_decodes_on_two_streams(gpu_ctx, oracle_mod, torch_cuda, k, r, P, erasures):
    """Two decodes in flight at once on two streams of one context, each with its own
    record-offset workspace (forms that classify first: record-addressed k=20 r=5, tiled
    P <= 256, runtime k).  Each must rebuild its own batch exactly."""
    torch = torch_cuda
    G = 4096
    batches = []
    for b in range(2):
        data = oracle_mod.splitmix_bytes(G * k * P, SEED + 77 + b)
        par = oracle_mod.rs_encode(data, G, k, r, P, nthreads=4)
        rng = np.random.default_rng(100 + b)
        pos = np.argsort(rng.random((G, k + r)), axis=1)[:, :erasures].astype(np.uint64)
        masks = np.left_shift(np.uint64(1), pos).sum(axis=1, dtype=np.uint64)
        lost = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
        broken = data.copy().reshape(G, k, P)
        broken[lost] = 0xEE
        batches.append((data, _dev(torch, broken.reshape(-1)), _dev(torch, par), _dev(torch, masks.view(np.int64))))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    sts = [torch.full((G,), 7, dtype=torch.uint8, device="cuda") for _ in range(2)]
    for rep in range(3):                        # several rounds, no host sync between streams
        for b in range(2):
            _, dd, dp, dm = batches[b]
            gpu_ctx.decode_dev(dd, dp, dm, G, k, r, P, sts[b], stream=streams[b].cuda_stream)
    torch.cuda.synchronize()
    for b in range(2):
        data, dd, _, _ = batches[b]
        assert int(sts[b].sum().item()) == 0
        assert np.array_equal(dd.cpu().numpy(), data), b


def test_ctx_last_error_set_on_failure(gpu_ctx, quicfec_mod):
    lib = quicfec_mod.load_library()
    buf = np.zeros(1200 * 4, dtype=np.uint8)
    rc = lib.fec_encode_batch_rs(gpu_ctx.handle, buf.ctypes.data, None, 1, 200, 100, 16, buf.ctypes.data)
    assert rc == quicfec_mod.FEC_ERR_RANGE
    assert "k=200 r=100" in gpu_ctx.last_error()
    # read from another thread: the context keeps the text
    import threading
    seen = []
    t = threading.Thread(target=lambda: seen.append(gpu_ctx.last_error()))
    t.start()
    t.join()
    assert "k=200 r=100" in seen[0]


@pytest.mark.parametrize("loss,P", [(0.01, 1200), (0.2, 1200), (0.01, 700), (0.05, 1400)])
def test_device_decode_scan_form(gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch, loss, P):
    """The mask-addressed decode with 8 groups per wave (DecodeLaunch::scan; host paths pick
    it for sparse loss, QUICFEC_DECODE_SCAN forces it here): statuses of every group and the
    rebuilt bytes equal the oracle's, with unrecoverable groups and a partial last wave."""
    gpu_ctx = gpu_ctx_hooks  # QUICFEC_DECODE_SCAN: a test-library switch
    monkeypatch.setenv("QUICFEC_DECODE_SCAN", "8")
    torch = torch_cuda
    k, r, G = 10, 3, 20_011
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 41 + P)
    par = oracle_mod.rs_encode(data, G, k, r, P, nthreads=8)
    rng = np.random.default_rng(int(loss * 1000) + P)
    w = np.left_shift(np.uint64(1), np.arange(k + r, dtype=np.uint64))
    masks = ((rng.random((G, k + r)) < loss) * w).sum(axis=1, dtype=np.uint64)
    masks[rng.integers(0, G, size=7)] = np.uint64(0xF)          # 4 data shards lost: unrecoverable
    broken = _poison(data, masks, G, k, P)
    ref = broken.copy()
    bad_exp, st_exp = oracle_mod.rs_decode(ref, par, masks, G, k, r, P, nthreads=8)
    dd, dp, dm = _dev(torch, broken), _dev(torch, par), _dev(torch, masks.view(np.int64))
    st = torch.full((G,), 0x55, dtype=torch.uint8, device="cuda")
    gpu_ctx.decode_dev(dd, dp, dm, G, k, r, P, st)
    gpu_ctx.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_exp)
    assert int((st_exp != 0).sum()) == bad_exp
    assert np.array_equal(dd.cpu().numpy(), ref)


RECOVER_SHAPES = [(10, 3, 1200), (10, 3, 700), (10, 3, 1400), (20, 5, 1200), (20, 5, 96), (4, 2, 256), (7, 4, 48),
                  (12, 9, 64), (10, 1, 1200), (5, 3, 33), (3, 2, 7), (30, 20, 32), (10, 3, 2500),
                  (10, 2, 1200), (10, 2, 700), (10, 1, 1400), (4, 2, 1200),
                  (10, 3, 256), (10, 3, 200), (10, 1, 128), (20, 5, 200), (4, 2, 100), (10, 3, 17), (10, 2, 256)]


@pytest.mark.parametrize("k,r,P", RECOVER_SHAPES)
def test_recover_compact_output(gpu_ctx, oracle_mod, torch_cuda, k, r, P):
    """fec_recover_batch_rs_dev: the m-th lost data shard of group g lands at
    rebuilt[(g*r + m)*P], bit-exact vs the oracle; data is not modified; slots past e and
    unrecoverable groups stay unwritten; statuses match."""
    torch = torch_cuda
    G = 1031
    rng = np.random.default_rng(k * 100 + r * 10 + P)
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 51 + k + P)
    par = oracle_mod.rs_encode(data, G, k, r, P, nthreads=8)
    masks = np.zeros(G, dtype=np.uint64)
    for g in range(G):
        for s in rng.permutation(k + r)[: rng.integers(0, r + 2)]:
            masks[g] |= np.uint64(1) << np.uint64(int(s))
    lost = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
    broken = data.copy().reshape(G, k, P)
    broken[lost] = 0xEE
    ref = broken.copy().reshape(-1)
    bad_exp, st_exp = oracle_mod.rs_decode(ref, par, masks, G, k, r, P, nthreads=8)
    exp = np.full((G, r, P), 0x5A, dtype=np.uint8)
    ref3 = ref.reshape(G, k, P)
    for g in np.nonzero(st_exp == 0)[0]:
        for m, j in enumerate(np.nonzero(lost[g])[0]):
            exp[g, m] = ref3[g, j]
    dd, dp, dm = _dev(torch, broken.reshape(-1)), _dev(torch, par), _dev(torch, masks.view(np.int64))
    out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
    st = torch.full((G,), 7, dtype=torch.uint8, device="cuda")
    gpu_ctx.recover_dev(dd, dp, dm, G, k, r, P, out, st)
    gpu_ctx.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_exp)
    assert np.array_equal(out.cpu().numpy().reshape(G, r, P), exp)
    assert np.array_equal(dd.cpu().numpy(), broken.reshape(-1))     # data untouched


@pytest.mark.parametrize("loss,P", [(0.01, 1200), (0.3, 1400)])
def test_recover_scan_form(gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch, loss, P):
    """fec_recover_batch_rs_dev in the 8-groups-per-wave form (sparse loss): compact rows
    and statuses equal the oracle's."""
    gpu_ctx = gpu_ctx_hooks  # QUICFEC_DECODE_SCAN: a test-library switch
    monkeypatch.setenv("QUICFEC_DECODE_SCAN", "8")
    torch = torch_cuda
    k, r, G = 10, 3, 10_007
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 61 + P)
    par = oracle_mod.rs_encode(data, G, k, r, P, nthreads=8)
    rng = np.random.default_rng(int(loss * 100) + P)
    w = np.left_shift(np.uint64(1), np.arange(k + r, dtype=np.uint64))
    masks = ((rng.random((G, k + r)) < loss) * w).sum(axis=1, dtype=np.uint64)
    lost = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
    _, st_exp = oracle_mod.rs_decode(_poison(data, masks, G, k, P), par, masks, G, k, r, P, nthreads=8)
    exp = np.full((G, r, P), 0x5A, dtype=np.uint8)
    d3 = data.reshape(G, k, P)
    for g in np.nonzero(st_exp == 0)[0]:
        for m, j in enumerate(np.nonzero(lost[g])[0]):
            exp[g, m] = d3[g, j]
    dd, dp, dm = _dev(torch, data), _dev(torch, par), _dev(torch, masks.view(np.int64))
    out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
    st = torch.full((G,), 7, dtype=torch.uint8, device="cuda")
    gpu_ctx.recover_dev(dd, dp, dm, G, k, r, P, out, st)
    gpu_ctx.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_exp)
    assert np.array_equal(out.cpu().numpy().reshape(G, r, P), exp)


@pytest.mark.parametrize("k,r", [(6, 3), (12, 4), (10, 2)])   # record-addressed, and one mask-addressed
def test_recover_back_to_back_on_one_stream(gpu_ctx, oracle_mod, torch_cuda, k, r):
    """Record-addressed decodes (classify + per-call record offsets) queued back to back on
    one stream with no synchronize in between, each with its own erasure pattern: every call
    must read its own record offsets.  (A per-call stream-ordered allocation of that
    workspace handed out memory a queued decode was still reading.)"""
    torch = torch_cuda
    G, P, calls = 1500, 1200, 12
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 71 + k + r)
    par = oracle_mod.rs_encode(data, G, k, r, P, nthreads=8)
    dd, dp = _dev(torch, data), _dev(torch, par)
    rng = np.random.default_rng(k + r)
    runs = []
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for c in range(calls):
            masks = np.zeros(G, dtype=np.uint64)
            for g in range(G):
                for s in rng.permutation(k + r)[: rng.integers(1, r + 1)]:
                    masks[g] |= np.uint64(1) << np.uint64(int(s))
            dm = _dev(torch, masks.view(np.int64))
            out = torch.zeros(G * r * P, dtype=torch.uint8, device="cuda")
            gpu_ctx.recover_dev(dd, dp, dm, G, k, r, P, out, None, stream=stream.cuda_stream)
            runs.append((masks, dm, out))
    stream.synchronize()
    d3 = data.reshape(G, k, P)
    for masks, _, out in runs:
        o3 = out.cpu().numpy().reshape(G, r, P)
        for g in range(0, G, 7):
            lost = [j for j in range(k) if (int(masks[g]) >> j) & 1]
            for m, j in enumerate(lost):
                assert np.array_equal(o3[g, m], d3[g, j]), (g, j)
