"""GPU tests of the bit-sliced encode (encode_bits, quic-test_amd/csrc/bitslice.hpp): the
code's coefficients compiled into XOR networks over bit planes.  It must write exactly the
bytes of the table form (encode_v16) and of the oracle's restatement (oracle/fec_oracle.c
rs_encode) for every packet size (P from 16 up, the last column shifted back), odd group
counts (a lane's second group past the end), tiles and multi-chunk launches.  Device-contiguous
packets only.  QUICFEC_ENCODE_BITS (a switch of the test library, libfec_hip_test.so, which
these tests load through gpu_ctx_hooks): 1 forces it for every instantiated shape, 0 the
tables; the product library takes it for r >= 4 (test_bits_is_the_default_for_c4)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [16, 24, 31, 32, 33, 48, 100, 1200, 1216, 1500, 4000, 9000]


def _dev(torch, arr):
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


def _encode(ctx, torch, data, G, k, r, P):
    dd = _dev(torch, data)
    dp = torch.full((G * r * P,), 0xA5, dtype=torch.uint8, device="cuda")
    ctx.encode_dev(dd, G, k, r, P, dp)
    ctx.synchronize()
    return dp.cpu().numpy()


@pytest.mark.parametrize("k,r", [(20, 5), (10, 3)])
@pytest.mark.parametrize("P", SIZES)
def test_bits_equals_oracle_and_tables(gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch, k, r, P):
    gpu_ctx = gpu_ctx_hooks
    G = 53
    data = oracle_mod.splitmix_bytes(G * k * P, 0xB175 + 131 * P + k)
    exp = oracle_mod.rs_encode(data, G, k, r, P)
    monkeypatch.setenv("QUICFEC_ENCODE_BITS", "1")
    bits = _encode(gpu_ctx, torch_cuda, data, G, k, r, P)
    monkeypatch.setenv("QUICFEC_ENCODE_BITS", "0")
    tabs = _encode(gpu_ctx, torch_cuda, data, G, k, r, P)
    assert np.array_equal(bits, exp.reshape(-1))
    assert np.array_equal(tabs, exp.reshape(-1))


@pytest.mark.parametrize("stage", ["0", "1"])
@pytest.mark.parametrize("tile", ["0", "1", "3"])
def test_bits_tiles_and_chunks(gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch, tile, stage):
    """Groups per workgroup (QUICFEC_ENCODE_TILE), rows staged or stored directly
    (QUICFEC_ENCODE_STAGE) and launches split into chunks of QUICFEC_MAX_WAVE_BLOCKS
    workgroups: every group's rows land at their global place."""
    gpu_ctx = gpu_ctx_hooks
    k, r, P, G = 20, 5, 1200, 1_001
    monkeypatch.setenv("QUICFEC_ENCODE_BITS", "1")
    monkeypatch.setenv("QUICFEC_ENCODE_STAGE", stage)
    if tile != "0":
        monkeypatch.setenv("QUICFEC_ENCODE_TILE", tile)
    monkeypatch.setenv("QUICFEC_MAX_WAVE_BLOCKS", "37")
    data = oracle_mod.splitmix_bytes(G * k * P, 0xC4C4 + int(tile) + 7 * int(stage))
    got = _encode(gpu_ctx, torch_cuda, data, G, k, r, P)
    assert np.array_equal(got, oracle_mod.rs_encode(data, G, k, r, P, nthreads=8).reshape(-1))


def test_bits_is_the_default_for_c4(gpu_ctx, oracle_mod, torch_cuda, monkeypatch):
    """Without the switch, k=20 r=5 runs the bit-sliced form (r >= 4) and k=10 r=3 the tables;
    both exact.  The round trip through the decoder closes the check at a size the oracle
    handles quickly."""
    monkeypatch.delenv("QUICFEC_ENCODE_BITS", raising=False)
    for k, r in ((20, 5), (10, 3)):
        G, P = 4_099, 1200
        data = oracle_mod.splitmix_bytes(G * k * P, 0xDEF0 + k)
        got = _encode(gpu_ctx, torch_cuda, data, G, k, r, P)
        assert np.array_equal(got, oracle_mod.rs_encode(data, G, k, r, P, nthreads=8).reshape(-1))


@pytest.mark.parametrize("form", ["tables", "bits"])
@pytest.mark.parametrize("k,r", [(10, 3), (20, 5)])
@pytest.mark.parametrize("P,G", [(1200, 1), (1200, 3), (1200, 4), (1200, 9), (1200, 1_001), (1024, 77), (64, 301),
                                 (1216, 50), (1500, 33), (1201, 21)])
def test_staged_rows_equal_oracle(gpu_ctx_hooks, oracle_mod, torch_cuda, monkeypatch, form, k, r, P, G):
    """QUICFEC_ENCODE_STAGE=1 (kStageRows): the workgroup's parity rows go
    through LDS and leave as one run of whole 16-B pieces.  Exact for partial last tiles (G not
    a multiple of the tile, a lane's second group past the end), small and large tiles, packet
    sizes that are not a multiple of 16 (the staged form then stands aside), and chunked
    launches, at an odd parity address; the bytes outside the parity are untouched (guard bytes)."""
    gpu_ctx = gpu_ctx_hooks
    monkeypatch.setenv("QUICFEC_ENCODE_STAGE", "1")
    monkeypatch.setenv("QUICFEC_ENCODE_BITS", "1" if form == "bits" else "0")
    monkeypatch.setenv("QUICFEC_MAX_WAVE_BLOCKS", "37")
    data = oracle_mod.splitmix_bytes(G * k * P, 0x57A6E + 7 * P + G + k)
    exp = oracle_mod.rs_encode(data, G, k, r, P, nthreads=8).reshape(-1)
    dd = _dev(torch_cuda, data)
    guard = 67  # an odd parity address: the staged run's 16-B stores are unaligned
    dp = torch_cuda.full((G * r * P + 2 * guard,), 0xA5, dtype=torch_cuda.uint8, device="cuda")
    gpu_ctx.encode_dev(dd, G, k, r, P, dp[guard:guard + G * r * P])
    gpu_ctx.synchronize()
    got = dp.cpu().numpy()
    assert np.array_equal(got[guard:guard + G * r * P], exp)
    assert (got[:guard] == 0xA5).all() and (got[guard + G * r * P:] == 0xA5).all()
