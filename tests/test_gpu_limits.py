"""Edge shapes of the batch API on the GPU, against the oracle: the largest codes (k + r = 256
encode, k + r = 64 decode with up to r erasures), jumbo and 64 KiB packets, one group, empty
calls that must touch nothing, and shapes past the limits that must be refused with an error
code (never a partial write).  The reference's own limits: up to 256 packets per XOR
(fec_xor_simd.cpp:573 `packets[256]`), packets up to 1500 B on the wire (decoder.go:115-120)
but any packet_size through the C call (fec_xor_simd.h:68-75)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED4000


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


@pytest.mark.parametrize("k,r,P,G", [(255, 1, 64, 5), (1, 255, 64, 5), (200, 56, 48, 4), (128, 128, 40, 3),
                                     (10, 3, 9000, 9), (4, 2, 65535, 3), (10, 3, 1200, 1)])
def test_encode_extreme_shapes(gpu_ctx, oracle_mod, torch_cuda, k, r, P, G):
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + k * 1000 + r)
    exp = oracle_mod.rs_encode(data, G, k, r, P)
    par = np.full(G * r * P, 0x5A, dtype=np.uint8)
    gpu_ctx.encode(data, k, r, P, par, num_groups=G)
    assert np.array_equal(par, exp)
    dp = torch_cuda.full((G * r * P,), 0x5A, dtype=torch_cuda.uint8, device="cuda")
    gpu_ctx.encode_dev(_dev(torch_cuda, data), G, k, r, P, dp)
    gpu_ctx.synchronize()
    assert np.array_equal(dp.cpu().numpy(), exp)


def _masks_exact(rng, G, k, r, lost):
    """`lost` distinct shards lost in every group, at least one of them a data shard."""
    m = np.zeros(G, dtype=np.uint64)
    for g in range(G):
        while True:
            pos = rng.choice(k + r, size=lost, replace=False)
            if (pos < k).any():
                break
        m[g] = np.uint64(sum(1 << int(p) for p in pos))
    return m


@pytest.mark.parametrize("k,r,P,G,lost", [(48, 16, 100, 6, 16), (32, 32, 16, 4, 32), (63, 1, 64, 8, 1),
                                          (1, 63, 50, 8, 63), (10, 3, 9000, 7, 3), (4, 2, 65535, 3, 2),
                                          (20, 5, 1200, 1, 5)])
def test_decode_and_recover_extreme_shapes(gpu_ctx, oracle_mod, torch_cuda, k, r, P, G, lost):
    rng = np.random.default_rng(k * 7 + r)
    data = oracle_mod.splitmix_bytes(G * k * P, SEED + 5 + k + r)
    par = oracle_mod.rs_encode(data, G, k, r, P)
    masks = _masks_exact(rng, G, k, r, lost)
    broken = data.copy().reshape(G, k, P)
    for g in range(G):
        for j in range(k):
            if (int(masks[g]) >> j) & 1:
                broken[g, j] = 0xEE
    broken = broken.reshape(-1)
    got = broken.copy()
    st = np.full(G, 0xAA, dtype=np.uint8)
    assert gpu_ctx.decode(got, par, masks, k, r, P, status_out=st) == 0
    assert np.array_equal(got, data) and not st.any()
    # device-resident recover: group g's m-th lost data shard at (g*r + m)*P
    out = torch_cuda.full((G * r * P,), 0x5A, dtype=torch_cuda.uint8, device="cuda")
    dst = torch_cuda.full((G,), 0xAA, dtype=torch_cuda.uint8, device="cuda")
    gpu_ctx.recover_dev(_dev(torch_cuda, broken), _dev(torch_cuda, par), _dev(torch_cuda, masks.view(np.int64)),
                        G, k, r, P, out, dst)
    gpu_ctx.synchronize()
    assert not dst.cpu().numpy().any()
    o = out.cpu().numpy().reshape(G, r, P)
    d = data.reshape(G, k, P)
    for g in range(G):
        ids = [j for j in range(k) if (int(masks[g]) >> j) & 1]
        for m, j in enumerate(ids):
            assert np.array_equal(o[g, m], d[g, j]), (g, m, j)


def test_empty_calls_touch_nothing(gpu_ctx, quicfec_mod, torch_cuda):
    buf = np.full(64, 0x33, dtype=np.uint8)
    gpu_ctx.encode(buf, 4, 2, 16, buf, num_groups=0)
    assert gpu_ctx.decode(buf, buf, np.zeros(0, dtype=np.uint64), 4, 2, 16, num_groups=0) == 0
    d = torch_cuda.full((64,), 0x33, dtype=torch_cuda.uint8, device="cuda")
    gpu_ctx.encode_dev(d, 0, 4, 2, 16, d)
    gpu_ctx.decode_dev(d, d, d, 0, 4, 2, 16)
    gpu_ctx.recover_dev(d, d, d, 0, 4, 2, 16, d, None)
    gpu_ctx.synchronize()
    assert (buf == 0x33).all() and bool((d == 0x33).all())
    # the reference's legacy call: 0 groups or packet size 0 -> 0 (fec_xor_simd.cpp:568-570)
    off = np.zeros(10, dtype=np.uint32)
    assert gpu_ctx.encode_batch_legacy(buf, off, 0, 16, buf) == 0
    assert gpu_ctx.encode_batch_legacy(buf, off, 1, 0, buf) == 0
    assert (buf == 0x33).all()


@pytest.mark.parametrize("k,r,decode", [(200, 57, False), (0, 3, False), (10, 0, False), (60, 5, True), (0, 2, True)])
def test_shapes_past_the_limits_are_refused(gpu_ctx, quicfec_mod, k, r, decode):
    P, G = 16, 2
    data = np.full(G * max(k, 1) * P, 0x11, dtype=np.uint8)
    par = np.full(G * max(r, 1) * P, 0x22, dtype=np.uint8)
    with pytest.raises(quicfec_mod.FecError) as ei:
        if decode:
            gpu_ctx.decode(data, par, np.ones(G, dtype=np.uint64), k, r, P, num_groups=G)
        else:
            gpu_ctx.encode(data, k, r, P, par, num_groups=G)
    assert ei.value.code == quicfec_mod.FEC_ERR_RANGE
    assert (data == 0x11).all() and (par == 0x22).all()
    assert gpu_ctx.last_error()
