"""GPU tests of the bit-sliced encode (encode_bits, quic-test_amd/csrc/bitslice.hpp): the
code's coefficients compiled into XOR networks over bit planes.  It must write exactly the
bytes of the table form (encode_v16) and of the oracle's restatement (oracle/fec_oracle.c
rs_encode) for every packet size (P from 16 up, the last column shifted back), odd group
counts (a lane's second group past the end), tiles and multi-chunk launches.  Device-contiguous
packets only.  QUICFEC_ENCODE_BITS: 1 forces it for every instantiated shape, 0 the
tables; the default takes it for r >= 4."""
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
def test_bits_equals_oracle_and_tables(gpu_ctx, oracle_mod, torch_cuda, monkeypatch, k, r, P):
    G = 53
    data = oracle_mod.splitmix_bytes(G * k * P, 0xB175 + 131 * P + k)
    exp = oracle_mod.rs_encode(data, G, k, r, P)
    monkeypatch.setenv("QUICFEC_ENCODE_BITS", "1")
    bits = _encode(gpu_ctx, torch_cuda, data, G, k, r, P)
    monkeypatch.setenv("QUICFEC_ENCODE_BITS", "0")
    tabs = _encode(gpu_ctx, torch_cuda, data, G, k, r, P)
    assert np.array_equal(bits, exp.reshape(-1))
    assert np.array_equal(tabs, exp.reshape(-1))


@pytest.mark.parametrize("window", ["4", "8"])
@pytest.mark.parametrize("tile", ["0", "1", "3"])
def test_bits_tiles_and_chunks(gpu_ctx, oracle_mod, torch_cuda, monkeypatch, tile, window):
    """Groups per workgroup (QUICFEC_ENCODE_TILE), packets in flight per lane
    (QUICFEC_ENCODE_BITS_WINDOW) and launches split into chunks of QUICFEC_MAX_WAVE_BLOCKS
    workgroups: every group's rows land at their global place."""
    k, r, P, G = 20, 5, 1200, 1_001
    monkeypatch.setenv("QUICFEC_ENCODE_BITS", "1")
    monkeypatch.setenv("QUICFEC_ENCODE_BITS_WINDOW", window)
    if tile != "0":
        monkeypatch.setenv("QUICFEC_ENCODE_TILE", tile)
    monkeypatch.setenv("QUICFEC_MAX_WAVE_BLOCKS", "37")
    data = oracle_mod.splitmix_bytes(G * k * P, 0xC4C4 + int(tile))
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
