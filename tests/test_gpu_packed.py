"""fec_recover_batch_rs_dev_packed: the rebuilt packets of all groups back to back (the shape of
decoder.go's Recovered list, :29-34), group g's rows starting at row_start[g] = the rows rebuilt
for groups 0..g-1.  Bit-exact against the oracle, row starts against a host prefix sum, the
total, statuses, `data` untouched; one wave per group and the sparse-loss scan form; prefix
sums across many 1024-group scan blocks (both prefix forms), masks at an 8-B-aligned address;
unsupported shapes refused."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED5000


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def _case(oracle_mod, k, r, P, G, masks):
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + k * 31 + r * 7 + P)
    par = oracle_mod.rs_encode(data, G, k, r, P, nthreads=8)
    lost = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
    broken = data.copy().reshape(G, k, P)
    broken[lost] = 0xEE
    ref = broken.copy().reshape(-1)
    _, st_exp = oracle_mod.rs_decode(ref, par, masks, G, k, r, P, nthreads=8)
    ok = st_exp == 0
    rows = np.where(ok, lost.sum(axis=1), 0).astype(np.int64)
    start = np.concatenate([[0], np.cumsum(rows)[:-1]]).astype(np.uint32)
    exp = ref.reshape(G, k, P)[lost & ok[:, None]]          # (g, j ascending) order
    return broken.reshape(-1), par, st_exp, start, exp


def _run(gpu_ctx, torch, broken, par, masks, G, k, r, P):
    dd, dp, dm = _dev(torch, broken), _dev(torch, par), _dev(torch, masks.view(np.int64))
    out = torch.full((max(1, G * r) * P,), 0x5A, dtype=torch.uint8, device="cuda")
    rs = torch.full((max(1, G),), 0x7FFFFFFF, dtype=torch.int32, device="cuda")
    tot = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    st = torch.full((max(1, G),), 7, dtype=torch.uint8, device="cuda")
    gpu_ctx.recover_packed_dev(dd, dp, dm, G, k, r, P, out, rs, tot, st)
    gpu_ctx.synchronize()
    return dd, out, rs, tot, st


@pytest.mark.parametrize("k,r,P", [(10, 3, 1200), (10, 3, 700), (10, 3, 1400), (10, 3, 2000), (10, 3, 300),
                                   (10, 1, 1200), (10, 2, 1200), (10, 2, 700), (4, 2, 1200), (4, 2, 513)])
def test_packed_rows_match_oracle(gpu_ctx, oracle_mod, torch_cuda, k, r, P):
    G = 1031
    rng = np.random.default_rng(k * 1000 + r * 100 + P)
    masks = np.zeros(G, dtype=np.uint64)
    for g in range(G):
        for s in rng.permutation(k + r)[: rng.integers(0, r + 2)]:
            masks[g] |= np.uint64(1) << np.uint64(int(s))
    broken, par, st_exp, start, exp = _case(oracle_mod, k, r, P, G, masks)
    dd, out, rs, tot, st = _run(gpu_ctx, torch_cuda, broken, par, masks, G, k, r, P)
    n = len(exp)
    assert int(tot.item()) == n
    assert np.array_equal(rs.cpu().numpy().view(np.uint32), start)
    assert np.array_equal(st.cpu().numpy(), st_exp)
    o = out.cpu().numpy().reshape(G * r, P)
    assert np.array_equal(o[:n], exp)
    assert (o[n:] == 0x5A).all()                                   # nothing past the last row
    assert np.array_equal(dd.cpu().numpy(), broken)                # data untouched


@pytest.mark.parametrize("loss,G,scan,direct", [(0.01, 50_000, "8", None), (0.3, 20_011, "8", None),
                                                (0.05, 30_000, None, None), (0.05, 30_001, None, "4"),
                                                (0.3, 9_000, "8", "1")])
def test_packed_rows_sparse_and_many_blocks(gpu_ctx, gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch, loss, G,
                                            scan, direct):
    """iid loss (the scan form when QUICFEC_DECODE_SCAN=8), row starts across many prefix
    blocks of 1024 groups, in the two-launch form and (QUICFEC_ROWS_DIRECT_BLOCKS below the
    block count) the one with a separate scan of the block sums.  The switches are the test
    library's (gpu_ctx_hooks); unswitched cases run the product library."""
    ctx = gpu_ctx_hooks if (scan or direct) else gpu_ctx
    if scan:
        monkeypatch.setenv("QUICFEC_DECODE_SCAN", scan)
    if direct:
        monkeypatch.setenv("QUICFEC_ROWS_DIRECT_BLOCKS", direct)
    k, r, P = 10, 3, 1200
    rng = np.random.default_rng(int(loss * 1000) + G)
    w = np.left_shift(np.uint64(1), np.arange(k + r, dtype=np.uint64))
    masks = ((rng.random((G, k + r)) < loss) * w).sum(axis=1, dtype=np.uint64)
    broken, par, st_exp, start, exp = _case(oracle_mod, k, r, P, G, masks)
    dd, out, rs, tot, st = _run(ctx, torch_cuda, broken, par, masks, G, k, r, P)
    n = len(exp)
    assert int(tot.item()) == n
    assert np.array_equal(rs.cpu().numpy().view(np.uint32), start)
    assert np.array_equal(st.cpu().numpy(), st_exp)
    assert np.array_equal(out.cpu().numpy().reshape(G * r, P)[:n], exp)


def test_packed_refusals_and_empty(gpu_ctx, quicfec_mod, torch_cuda):
    torch = torch_cuda
    # shapes without a mask-addressed form: record-addressed k=20 r=5, tiled P <= 256, P > 2048
    for k, r, P in ((20, 5, 1200), (10, 3, 200), (10, 3, 3000), (6, 3, 1200)):
        G = 4
        d = torch.zeros(G * k * P, dtype=torch.uint8, device="cuda")
        p = torch.zeros(G * r * P, dtype=torch.uint8, device="cuda")
        m = torch.ones(G, dtype=torch.int64, device="cuda")
        out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
        rs = torch.full((G,), 0x3C3C3C3C, dtype=torch.int32, device="cuda")
        tot = torch.full((1,), -5, dtype=torch.int64, device="cuda")
        with pytest.raises(quicfec_mod.FecError) as ei:
            gpu_ctx.recover_packed_dev(d, p, m, G, k, r, P, out, rs, tot)
        assert ei.value.code == quicfec_mod.FEC_ERR_RANGE, (k, r, P)
        gpu_ctx.synchronize()
        # refused before anything ran: rebuilt rows, row starts and total untouched
        assert bool((out == 0x5A).all())
        assert bool((rs == 0x3C3C3C3C).all()) and int(tot.item()) == -5
    # no groups: the total is 0
    z = torch.zeros(16, dtype=torch.uint8, device="cuda")
    tot = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    gpu_ctx.recover_packed_dev(z, z, z, 0, 10, 3, 1200, z, z, tot)
    gpu_ctx.synchronize()
    assert int(tot.item()) == 0


def test_packed_masks_at_odd_word(gpu_ctx, oracle_mod, torch_cuda):
    """The prefix kernels read four masks per load: a mask array starting one u64 into an
    allocation (8-B aligned only) gives the same rows."""
    torch = torch_cuda
    k, r, P, G = 10, 3, 700, 5_003
    rng = np.random.default_rng(77)
    w = np.left_shift(np.uint64(1), np.arange(k + r, dtype=np.uint64))
    masks = ((rng.random((G, k + r)) < 0.1) * w).sum(axis=1, dtype=np.uint64)
    broken, par, st_exp, start, exp = _case(oracle_mod, k, r, P, G, masks)
    dd, dp = _dev(torch, broken), _dev(torch, par)
    dm_all = _dev(torch, np.concatenate([[np.uint64(0)], masks]).view(np.int64))
    dm = dm_all[1:]
    out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
    rs = torch.zeros(G, dtype=torch.int32, device="cuda")
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    gpu_ctx.recover_packed_dev(dd, dp, dm, G, k, r, P, out, rs, tot)
    gpu_ctx.synchronize()
    n = len(exp)
    assert int(tot.item()) == n
    assert np.array_equal(rs.cpu().numpy().view(np.uint32), start)
    assert np.array_equal(out.cpu().numpy().reshape(G * r, P)[:n], exp)


@pytest.mark.parametrize("api", ["packed", "packed_scan", "slots", "in_place"])
@pytest.mark.parametrize("k,r,P", [(10, 3, 1200), (10, 2, 700), (20, 5, 1200)])
def test_chunked_launches(gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch, api, k, r, P):
    """Launches split into chunks of QUICFEC_MAX_WAVE_BLOCKS workgroups (otherwise only past
    16.7M groups; a test-library switch): packed rows keep their global row starts in every
    chunk, and the forms that take no record offsets get none in later chunks."""
    gpu_ctx = gpu_ctx_hooks
    if k == 20 and api.startswith("packed"):
        pytest.skip("no packed form for the record-addressed shape")
    monkeypatch.setenv("QUICFEC_MAX_WAVE_BLOCKS", "7")
    if api == "packed_scan":
        monkeypatch.setenv("QUICFEC_DECODE_SCAN", "8")
    torch = torch_cuda
    G = 1_237
    rng = np.random.default_rng(k * 100 + r + P)
    masks = np.zeros(G, dtype=np.uint64)
    for g in range(G):
        for sh in rng.permutation(k + r)[: rng.integers(0, r + 2)]:
            masks[g] |= np.uint64(1) << np.uint64(int(sh))
    broken, par, st_exp, start, exp = _case(oracle_mod, k, r, P, G, masks)
    if api.startswith("packed"):
        dd, out, rs, tot, st = _run(gpu_ctx, torch, broken, par, masks, G, k, r, P)
        n = len(exp)
        assert int(tot.item()) == n
        assert np.array_equal(rs.cpu().numpy().view(np.uint32), start)
        o = out.cpu().numpy().reshape(G * r, P)
        assert np.array_equal(o[:n], exp)
        assert (o[n:] == 0x5A).all()
        assert np.array_equal(st.cpu().numpy(), st_exp)
        return
    dd, dp, dm = _dev(torch, broken), _dev(torch, par), _dev(torch, masks.view(np.int64))
    st = torch.full((G,), 7, dtype=torch.uint8, device="cuda")
    lost = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
    ok = st_exp == 0
    if api == "slots":
        out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
        gpu_ctx.recover_dev(dd, dp, dm, G, k, r, P, out, st)
        gpu_ctx.synchronize()
        o = out.cpu().numpy().reshape(G, r, P)
        ref = broken.copy().reshape(G, k, P)
        oracle_mod.rs_decode(ref.reshape(-1), par, masks, G, k, r, P, nthreads=8)
        for g in np.nonzero(ok & lost.any(axis=1))[0]:
            ids = np.nonzero(lost[g])[0]
            assert np.array_equal(o[g, :len(ids)], ref[g, ids]), g
    else:
        gpu_ctx.decode_dev(dd, dp, dm, G, k, r, P, st)
        gpu_ctx.synchronize()
        ref = broken.copy()
        oracle_mod.rs_decode(ref, par, masks, G, k, r, P, nthreads=8)
        assert np.array_equal(dd.cpu().numpy(), ref)
    assert np.array_equal(st.cpu().numpy(), st_exp)


@pytest.mark.slow
@pytest.mark.parametrize("profile", ["c3_two_erasures", "c5_satellite_iid"])
def test_full_size_packed_recover(gpu_ctx, oracle_mod, torch_cuda, profile):
    """The bench's decode API at BASELINE size (1M groups of k=10 r=3, 1200 B): C3 (2 erased
    shards per group) and C5 (iid loss 0.01 per shard, the scan form via the loss hint).  The
    whole packed list against the original packets, row starts against a host prefix sum,
    sampled groups against the oracle's decode (decoder.go:29-34's Recovered list shape)."""
    torch = torch_cuda
    k, r, P, G = 10, 3, 1200, 1_000_000
    data = torch.empty(G * k * P, dtype=torch.uint8, device="cuda")
    par = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_random_dev(data, data.numel(), SEED + 11)
    gpu_ctx.encode_dev(data, G, k, r, P, par)
    rng = np.random.default_rng(SEED + 12)
    if profile == "c3_two_erasures":
        pos = np.argsort(rng.random((G, k + r)), axis=1)[:, :2].astype(np.uint64)
        masks = np.left_shift(np.uint64(1), pos).sum(axis=1, dtype=np.uint64)
    else:
        w = np.left_shift(np.uint64(1), np.arange(k + r, dtype=np.uint64))
        masks = ((rng.random((G, k + r)) < 0.01) * w).sum(axis=1, dtype=np.uint64)
        gpu_ctx.decode_loss_hint(1.0 - 0.99 ** k)
    try:
        orig = data.clone()
        dm = torch.from_numpy(masks.view(np.int64)).cuda()
        bits = torch.arange(k, device="cuda", dtype=torch.int64)
        lost = ((dm.view(G, 1) >> bits.view(1, k)) & 1).bool()
        data.view(G, k, P)[lost] = 0xEE
        out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
        rs = torch.zeros(G, dtype=torch.int32, device="cuda")
        tot = torch.full((1,), -1, dtype=torch.int64, device="cuda")
        st = torch.full((G,), 7, dtype=torch.uint8, device="cuda")
        gpu_ctx.recover_packed_dev(data, par, dm, G, k, r, P, out, rs, tot, st)
        gpu_ctx.synchronize()
        lost_h = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
        plost = ((masks[:, None] >> np.arange(k, k + r, dtype=np.uint64)[None, :]) & np.uint64(1)).sum(axis=1)
        e = lost_h.sum(axis=1)
        ok = e <= r - plost
        rows = np.where(ok, e, 0)
        start = np.concatenate([[0], np.cumsum(rows)[:-1]]).astype(np.uint32)
        n = int(rows.sum())
        assert int(tot.item()) == n
        assert np.array_equal(rs.cpu().numpy().view(np.uint32), start)
        assert np.array_equal(st.cpu().numpy(), (~ok).astype(np.uint8))
        okd = torch.from_numpy(ok).cuda()
        want = orig.view(G, k, P)[lost & okd.view(G, 1)]         # (g, j ascending) order
        assert want.shape[0] == n
        assert torch.equal(out.view(-1, P)[:n], want)
        assert bool((out.view(-1, P)[n:] == 0x5A).all())
        # sampled groups through the oracle's own decode
        cand = np.nonzero(rows > 0)[0]
        for g in [int(x) for x in rng.choice(cand, size=min(48, len(cand)), replace=False)]:
            blk = data[g * k * P:(g + 1) * k * P].cpu().numpy().copy()
            pb = par[g * r * P:(g + 1) * r * P].cpu().numpy()
            oracle_mod.rs_decode(blk, pb, masks[g:g + 1].copy(), 1, k, r, P)
            ids = np.nonzero(lost_h[g])[0]
            got = out.view(-1, P)[int(start[g]):int(start[g]) + len(ids)].cpu().numpy()
            assert np.array_equal(got, blk.reshape(k, P)[ids]), g
        # the data stays as received (recover reads it only)
        assert bool((data.view(G, k, P)[lost] == 0xEE).all())
    finally:
        gpu_ctx.decode_loss_hint(-1.0)


def _iid_masks(rng, G, n, loss):
    w = np.left_shift(np.uint64(1), np.arange(n, dtype=np.uint64))
    return ((rng.random((G, n)) < loss) * w).sum(axis=1, dtype=np.uint64)


def _check_packed(gpu_ctx, torch, oracle_mod, k, r, P, G, masks, out_offset=0):
    broken, par, st_exp, start, exp = _case(oracle_mod, k, r, P, G, masks)
    dd, dp, dm = _dev(torch, broken), _dev(torch, par), _dev(torch, masks.view(np.int64))
    base = torch.full((max(1, G * r) * P + out_offset,), 0x5A, dtype=torch.uint8, device="cuda")
    out = base[out_offset:]
    rs = torch.full((max(1, G),), 0x7FFFFFFF, dtype=torch.int32, device="cuda")
    tot = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    st = torch.full((max(1, G),), 7, dtype=torch.uint8, device="cuda")
    gpu_ctx.recover_packed_dev(dd, dp, dm, G, k, r, P, out, rs, tot, st)
    gpu_ctx.synchronize()
    n = len(exp)
    assert int(tot.item()) == n
    assert np.array_equal(rs.cpu().numpy().view(np.uint32), start)
    assert np.array_equal(st.cpu().numpy(), st_exp)
    o = out.cpu().numpy().reshape(G * r, P)
    assert np.array_equal(o[:n], exp)
    assert (o[n:] == 0x5A).all()                                   # nothing past the last row
    assert (base[:out_offset].cpu().numpy() == 0x5A).all()        # nothing before the first
    assert np.array_equal(dd.cpu().numpy(), broken)                # data untouched


@pytest.mark.parametrize("k,r,P", [(10, 3, 1200), (10, 3, 700), (10, 3, 1400), (10, 3, 2000), (10, 3, 300),
                                   (10, 3, 1024), (10, 3, 1040), (10, 3, 1201), (10, 1, 1200), (10, 2, 1200),
                                   (10, 2, 700), (4, 2, 513), (4, 2, 1200)])
@pytest.mark.parametrize("stage", ["default", "0", "16384", "65536"])
def test_packed_runs_one_launch(gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch, k, r, P, stage):
    """The one-launch packed recover (recover_runs: decoupled look-back row starts, rows staged
    per workgroup in an LDS image and written as one run) on every mask-addressed piece layout,
    forced for mixed loss (QUICFEC_PACKED_RUNS=1), with the image off, small (most rows past it go
    straight to HBM), the default 48 KB and 64 KB (test-library switches); bit-exact against the
    oracle."""
    gpu_ctx = gpu_ctx_hooks
    monkeypatch.setenv("QUICFEC_PACKED_RUNS", "1")
    if stage != "default":
        monkeypatch.setenv("QUICFEC_RUNS_STAGE", stage)
    G = 3_001
    rng = np.random.default_rng(k * 1000 + r * 100 + P + len(stage))
    masks = np.zeros(G, dtype=np.uint64)
    for g in range(G):
        for s in rng.permutation(k + r)[: rng.integers(0, r + 2)]:
            masks[g] |= np.uint64(1) << np.uint64(int(s))
    _check_packed(gpu_ctx, torch_cuda, oracle_mod, k, r, P, G, masks)


@pytest.mark.parametrize("case", ["chunks", "odd_output", "sparse_hint", "tiny", "one_group_per_tile"])
def test_packed_runs_edges(gpu_ctx, gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch, case):
    """recover_runs edges: chunked launches (QUICFEC_MAX_WAVE_BLOCKS=2, each chunk's rows start
    after the previous chunk's total), an output at an odd address (no LDS image: rows straight
    to HBM), the library's own choice from the loss hint (the product library), calls of 1-7
    groups, and tiles where a single group rebuilds."""
    torch = torch_cuda
    if case != "sparse_hint":
        gpu_ctx = gpu_ctx_hooks  # QUICFEC_PACKED_RUNS / QUICFEC_MAX_WAVE_BLOCKS: test-library switches
    k, r, P = 10, 3, 1200
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    off = 0
    if case == "chunks":
        monkeypatch.setenv("QUICFEC_PACKED_RUNS", "1")
        monkeypatch.setenv("QUICFEC_MAX_WAVE_BLOCKS", "2")
        G = 5_555
        masks = _iid_masks(rng, G, k + r, 0.05)
    elif case == "odd_output":
        monkeypatch.setenv("QUICFEC_PACKED_RUNS", "1")
        G, off = 2_049, 5
        masks = _iid_masks(rng, G, k + r, 0.08)
    elif case == "sparse_hint":
        G = 20_000
        masks = _iid_masks(rng, G, k + r, 0.01)
        gpu_ctx.decode_loss_hint(1.0 - 0.99 ** k)
    elif case == "tiny":
        monkeypatch.setenv("QUICFEC_PACKED_RUNS", "1")
        for G in range(1, 8):
            masks = _iid_masks(rng, G, k + r, 0.3)
            _check_packed(gpu_ctx, torch, oracle_mod, k, r, P, G, masks)
        return
    else:
        monkeypatch.setenv("QUICFEC_PACKED_RUNS", "1")
        G = 4_096
        masks = np.zeros(G, dtype=np.uint64)
        masks[::700] = np.uint64(0b101)                                 # 2 lost data shards
    try:
        _check_packed(gpu_ctx, torch, oracle_mod, k, r, P, G, masks, out_offset=off)
    finally:
        gpu_ctx.decode_loss_hint(-1.0)


def test_packed_runs_back_to_back(gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch):
    """Several one-launch packed recovers queued on one stream without a synchronise between
    them, growing and shrinking: every launch takes fresh look-back epochs (words left by the
    earlier launches never match) and the workspace grows under queued work."""
    gpu_ctx = gpu_ctx_hooks
    monkeypatch.setenv("QUICFEC_PACKED_RUNS", "1")
    torch = torch_cuda
    k, r, P = 10, 3, 700
    rng = np.random.default_rng(4242)
    runs = []
    for G in (1_031, 60_000, 7, 60_000, 300):
        masks = _iid_masks(rng, G, k + r, 0.06)
        broken, par, st_exp, start, exp = _case(oracle_mod, k, r, P, G, masks)
        dd, dp, dm = _dev(torch, broken), _dev(torch, par), _dev(torch, masks.view(np.int64))
        out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
        rs = torch.zeros(G, dtype=torch.int32, device="cuda")
        tot = torch.full((1,), -1, dtype=torch.int64, device="cuda")
        gpu_ctx.recover_packed_dev(dd, dp, dm, G, k, r, P, out, rs, tot)
        runs.append((G, out, rs, tot, start, exp, dd, dp, dm))
    gpu_ctx.synchronize()
    for G, out, rs, tot, start, exp, *_ in runs:
        n = len(exp)
        assert int(tot.item()) == n, G
        assert np.array_equal(rs.cpu().numpy().view(np.uint32), start), G
        assert np.array_equal(out.cpu().numpy().reshape(G * r, P)[:n], exp), G


@pytest.mark.slow
@pytest.mark.parametrize("profile", ["c3_two_erasures", "c5_satellite_iid"])
def test_full_size_slot_recover(gpu_ctx, oracle_mod, torch_cuda, profile):
    """fec_recover_batch_rs_dev (rebuilt packets at (g*r + m)*P, the bench's C3 decode) at
    BASELINE size: every group's slots against the original packets, statuses against the
    masks, sampled groups against the oracle's decode."""
    torch = torch_cuda
    k, r, P, G = 10, 3, 1200, 1_000_000
    data = torch.empty(G * k * P, dtype=torch.uint8, device="cuda")
    par = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_random_dev(data, data.numel(), SEED + 21)
    gpu_ctx.encode_dev(data, G, k, r, P, par)
    rng = np.random.default_rng(SEED + 22)
    if profile == "c3_two_erasures":
        pos = np.argsort(rng.random((G, k + r)), axis=1)[:, :2].astype(np.uint64)
        masks = np.left_shift(np.uint64(1), pos).sum(axis=1, dtype=np.uint64)
    else:
        masks = _iid_masks(rng, G, k + r, 0.01)
        gpu_ctx.decode_loss_hint(1.0 - 0.99 ** k)
    try:
        orig = data.clone()
        dm = torch.from_numpy(masks.view(np.int64)).cuda()
        bits = torch.arange(k, device="cuda", dtype=torch.int64)
        lost = ((dm.view(G, 1) >> bits.view(1, k)) & 1).bool()
        data.view(G, k, P)[lost] = 0xEE
        out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
        st = torch.full((G,), 7, dtype=torch.uint8, device="cuda")
        gpu_ctx.recover_dev(data, par, dm, G, k, r, P, out, st)
        gpu_ctx.synchronize()
        lost_h = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
        plost = ((masks[:, None] >> np.arange(k, k + r, dtype=np.uint64)[None, :]) & np.uint64(1)).sum(axis=1)
        e = lost_h.sum(axis=1)
        ok = e <= r - plost
        assert np.array_equal(st.cpu().numpy(), (~ok).astype(np.uint8))
        okd = torch.from_numpy(ok).cuda()
        e_g = lost.sum(dim=1, keepdim=True)
        slots = torch.arange(r, device="cuda").view(1, r) < e_g
        got = out.view(G, r, P)[slots & okd.view(G, 1)]
        want = orig.view(G, k, P)[lost & okd.view(G, 1)]
        assert torch.equal(got, want)
        # slots past a group's rebuilt rows, and every slot of unrecoverable groups, untouched
        assert bool((out.view(G, r, P)[~(slots & okd.view(G, 1))] == 0x5A).all())
        cand = np.nonzero(ok & (e > 0))[0]
        for g in [int(x) for x in rng.choice(cand, size=min(48, len(cand)), replace=False)]:
            blk = data[g * k * P:(g + 1) * k * P].cpu().numpy().copy()
            pb = par[g * r * P:(g + 1) * r * P].cpu().numpy()
            oracle_mod.rs_decode(blk, pb, masks[g:g + 1].copy(), 1, k, r, P)
            ids = np.nonzero(lost_h[g])[0]
            assert np.array_equal(out.view(G, r, P)[g, :len(ids)].cpu().numpy(), blk.reshape(k, P)[ids]), g
    finally:
        gpu_ctx.decode_loss_hint(-1.0)
