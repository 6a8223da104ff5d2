"""Randomised shapes through every entry point, against the oracle: k, r, packet size, group
count, erasure patterns (up to r + 1 lost, so some groups are unrecoverable) and the API
(host pageable, host page-locked, device in place, device recover) drawn from a seeded
generator.  Each case is small, the whole sweep runs in seconds; it exists to catch the
interaction bugs that the per-shape parity tests do not pin (form selection, workspace and
staging reuse across calls of different shapes on one context)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# QUICFEC_FUZZ_SEED / QUICFEC_FUZZ_BLOCKS widen the sweep for a long run (the default is the
# committed 12 blocks of 10 cases)
SEED = int(os.environ.get("QUICFEC_FUZZ_SEED", str(0x5EED0F00)), 0)
BLOCKS = int(os.environ.get("QUICFEC_FUZZ_BLOCKS", "12"))
# the packed-recover sweep: 4 blocks of 8 calls by default, a third of QUICFEC_FUZZ_BLOCKS when wider
PACKED_BLOCKS = max(4, BLOCKS // 3)


def _case(rng):
    k = int(rng.integers(1, 21))
    r = int(rng.integers(1, min(8, 64 - k) + 1))
    P = int(rng.choice([int(rng.integers(1, 64)), int(rng.integers(64, 1600)), 1200, 256, 1024]))
    G = int(rng.integers(1, 400))
    api = str(rng.choice(["host", "pinned", "dev_inplace", "dev_recover"]))
    return k, r, P, G, api


def _masks(rng, G, k, r):
    m = np.zeros(G, dtype=np.uint64)
    for g in range(G):
        for s in rng.permutation(k + r)[: int(rng.integers(0, r + 2))]:
            m[g] |= np.uint64(1) << np.uint64(int(s))
    return m


@pytest.mark.parametrize("block", range(BLOCKS))
def test_random_shapes_all_apis(gpu_ctx, oracle_mod, torch_cuda, block):
    torch = torch_cuda
    rng = np.random.default_rng(SEED + block)
    for _ in range(10):   # one context, shapes and APIs interleaved
        k, r, P, G, api = _case(rng)
        data = oracle_mod.splitmix_bytes(G * k * P, int(rng.integers(0, 1 << 30)))
        par_exp = oracle_mod.rs_encode(data, G, k, r, P, nthreads=4)
        masks = _masks(rng, G, k, r)
        lost = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
        broken = data.copy().reshape(G, k, P)
        broken[lost] = 0xEE
        ref = broken.copy().reshape(-1)
        bad_exp, st_exp = oracle_mod.rs_decode(ref, par_exp, masks, G, k, r, P, nthreads=4)
        tag = (k, r, P, G, api)
        if api in ("host", "pinned"):
            if api == "pinned":
                d = torch.from_numpy(data).pin_memory()
                par = torch.zeros(G * r * P, dtype=torch.uint8).pin_memory()
                gpu_ctx.encode(d, k, r, P, par, num_groups=G)
                par_np = par.numpy()
                dd = torch.from_numpy(broken.reshape(-1)).pin_memory()
                st = torch.zeros(G, dtype=torch.uint8).pin_memory()
                bad = gpu_ctx.decode(dd, par, torch.from_numpy(masks.view(np.int64)), k, r, P, st, num_groups=G)
                got, st_np = dd.numpy(), st.numpy()
            else:
                par_np = np.zeros(G * r * P, dtype=np.uint8)
                gpu_ctx.encode(data, k, r, P, par_np, num_groups=G)
                got = broken.reshape(-1).copy()
                st_np = np.zeros(G, dtype=np.uint8)
                bad = gpu_ctx.decode(got, par_np, masks, k, r, P, st_np, num_groups=G)
            assert np.array_equal(par_np, par_exp), tag
            assert bad == bad_exp and np.array_equal(st_np, st_exp), tag
            assert np.array_equal(got, ref), tag
            continue
        dd = torch.from_numpy(broken.reshape(-1)).cuda()
        d_src = torch.from_numpy(data).cuda()
        dp = torch.zeros(G * r * P, dtype=torch.uint8, device="cuda")
        gpu_ctx.encode_dev(d_src, G, k, r, P, dp)
        dm = torch.from_numpy(masks.view(np.int64)).cuda()
        st = torch.full((G,), 7, dtype=torch.uint8, device="cuda")
        if api == "dev_inplace":
            gpu_ctx.decode_dev(dd, dp, dm, G, k, r, P, st)
            gpu_ctx.synchronize()
            assert np.array_equal(dd.cpu().numpy(), ref), tag
        else:
            out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
            gpu_ctx.recover_dev(dd, dp, dm, G, k, r, P, out, st)
            gpu_ctx.synchronize()
            o3 = out.cpu().numpy().reshape(G, r, P)
            ref3 = ref.reshape(G, k, P)
            for g in np.nonzero(st_exp == 0)[0]:
                for m, j in enumerate(np.nonzero(lost[g])[0]):
                    assert np.array_equal(o3[g, m], ref3[g, j]), tag + (int(g), int(j))
        assert np.array_equal(dp.cpu().numpy(), par_exp), tag
        assert np.array_equal(st.cpu().numpy(), st_exp), tag


@pytest.mark.parametrize("block", range(4))
def test_random_batchers(quicfec_mod, oracle_mod, block):
    """Both batchers with random shapes, slab sizes, deadlines, packet counts and lengths,
    and erasure patterns; results collected in random order (polls and blocking waits)."""
    rng = np.random.default_rng(SEED + 100 + block)
    for _ in range(3):
        k = int(rng.integers(1, 17))
        r = int(rng.integers(1, min(6, 64 - k) + 1))
        slot = int(rng.integers(1, 1601))
        mg = int(rng.integers(1, 40))
        dl = int(rng.choice([0, 50, 500]))
        slabs = int(rng.integers(2, 5))
        # every result stays collectable while fewer than 2 * slabs * max_groups newer groups
        # were encoded (include/fec_hip.h); the submissions stay within that
        n = min(int(rng.integers(1, 90)), 2 * 3 * mg, 2 * slabs * mg)
        with quicfec_mod.Batcher(k, r, slot_bytes=slot, max_groups=mg, deadline_us=dl, slabs=slabs) as b:
            subs = []
            for g in range(n):
                cnt = int(rng.integers(1, k + 1))
                pk = [oracle_mod.splitmix_bytes(int(rng.integers(1, slot + 1)), 99 * g + j + 7 * block) for j in range(cnt)]
                subs.append((b.submit(pk), pk))
            b.flush()
            for i in rng.permutation(len(subs)):
                t, pk = subs[i]
                rows = b.wait(int(t), timeout_us=5_000_000)
                L = max(len(p) for p in pk)
                P = (L + 15) // 16 * 16
                data = np.zeros(k * P, dtype=np.uint8)
                for j, p in enumerate(pk):
                    data[j * P:j * P + len(p)] = p
                par = oracle_mod.rs_encode(data, 1, k, r, P)
                assert all(np.array_equal(rows[m], par[m * P:m * P + L]) for m in range(r)), (k, r, slot, mg, dl)
        with quicfec_mod.DecodeBatcher(k, r, slot_bytes=slot, max_groups=mg, deadline_us=dl) as db:
            subs = []
            for g in range(n):
                L = int(rng.integers(1, slot + 1))
                P = (L + 15) // 16 * 16
                data = oracle_mod.splitmix_bytes(k * P, 1000 + g + 13 * block)
                par = oracle_mod.rs_encode(data, 1, k, r, P)
                shards = [data[j * P:j * P + L] for j in range(k)] + [par[m * P:m * P + L] for m in range(r)]
                lost = set(int(x) for x in rng.permutation(k + r)[: int(rng.integers(0, r + 2))])
                t = db.submit([None if s in lost else shards[s] for s in range(k + r)], L)
                subs.append((t, shards, lost))
            db.flush()
            for i in rng.permutation(len(subs)):
                t, shards, lost = subs[i]
                if len(lost) > r:
                    with pytest.raises(quicfec_mod.FecError) as ei:
                        db.wait(int(t), timeout_us=5_000_000)
                    assert ei.value.code == quicfec_mod.FEC_ERR_UNRECOVERABLE
                    continue
                ids, rows = db.wait(int(t), timeout_us=5_000_000)
                assert ids == sorted(s for s in lost if s < k)
                assert all(np.array_equal(row, shards[j]) for j, row in zip(ids, rows)), (k, r, slot, mg, dl)


@pytest.mark.parametrize("block", range(PACKED_BLOCKS))
def test_random_packed_recover(gpu_ctx_hooks, oracle_mod, torch_cuda, block):
    """The packed recover with random mask-addressed shapes, sizes and loss rates, through both
    of its forms chosen at random per call (the one-launch recover_runs and the prefix launches +
    decode_fused; QUICFEC_PACKED_RUNS is a test-library switch), one context, calls of different
    shapes interleaved: rows, row starts, total and statuses against the oracle."""
    gpu_ctx = gpu_ctx_hooks
    torch = torch_cuda
    rng = np.random.default_rng(SEED + 200 + block)
    shapes = [(10, 3), (10, 2), (10, 1), (4, 2)]
    saved = os.environ.get("QUICFEC_PACKED_RUNS")
    try:
        for _ in range(8):
            k, r = shapes[int(rng.integers(0, len(shapes)))]
            P = int(rng.choice([1200, int(rng.integers(257, 2048))]))
            G = int(rng.integers(1, 6000))
            loss = float(rng.choice([0.005, 0.02, 0.1, 0.3]))
            mode = str(rng.choice(["auto", "1", "0"]))
            if mode == "auto":
                os.environ.pop("QUICFEC_PACKED_RUNS", None)
            else:
                os.environ["QUICFEC_PACKED_RUNS"] = mode
            gpu_ctx.decode_loss_hint(1.0 - (1.0 - loss) ** k if rng.random() < 0.5 else -1.0)
            w = np.left_shift(np.uint64(1), np.arange(k + r, dtype=np.uint64))
            masks = ((rng.random((G, k + r)) < loss) * w).sum(axis=1, dtype=np.uint64)
            data = oracle_mod.splitmix_bytes(G * k * P, int(rng.integers(0, 1 << 30)))
            par = oracle_mod.rs_encode(data, G, k, r, P, nthreads=4)
            lost = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
            broken = data.copy().reshape(G, k, P)
            broken[lost] = 0xEE
            ref = broken.copy().reshape(-1)
            _, st_exp = oracle_mod.rs_decode(ref, par, masks, G, k, r, P, nthreads=4)
            ok = st_exp == 0
            rows = np.where(ok, lost.sum(axis=1), 0)
            start = np.concatenate([[0], np.cumsum(rows)[:-1]]).astype(np.uint32)
            exp = ref.reshape(G, k, P)[lost & ok[:, None]]
            dd = torch.from_numpy(broken.reshape(-1)).cuda()
            dp = torch.from_numpy(par).cuda()
            dm = torch.from_numpy(masks.view(np.int64)).cuda()
            out = torch.full((G * r * P,), 0x5A, dtype=torch.uint8, device="cuda")
            rs = torch.zeros(G, dtype=torch.int32, device="cuda")
            tot = torch.full((1,), -1, dtype=torch.int64, device="cuda")
            st = torch.full((G,), 7, dtype=torch.uint8, device="cuda")
            gpu_ctx.recover_packed_dev(dd, dp, dm, G, k, r, P, out, rs, tot, st)
            gpu_ctx.synchronize()
            tag = (k, r, P, G, loss, mode)
            n = len(exp)
            assert int(tot.item()) == n, tag
            assert np.array_equal(rs.cpu().numpy().view(np.uint32), start), tag
            assert np.array_equal(st.cpu().numpy(), st_exp), tag
            o = out.cpu().numpy().reshape(G * r, P)
            assert np.array_equal(o[:n], exp), tag
            assert (o[n:] == 0x5A).all(), tag
    finally:
        gpu_ctx.decode_loss_hint(-1.0)
        if saved is None:
            os.environ.pop("QUICFEC_PACKED_RUNS", None)
        else:
            os.environ["QUICFEC_PACKED_RUNS"] = saved
