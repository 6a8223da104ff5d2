"""Pin the CPU restatement (oracle/) against the reference's own outputs.

Fixtures in tests/golden/ come from the reference library compiled from
/root/reference/internal/fec/fec_xor_simd.cpp (tests/golden/make_golden.py).  The
reference's Go tests hold no byte-level assertions, so besides the
fixtures the only known answer is the one implied by encoder_test.go:70-86.
"""
import json

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st


def _groups(data, G, k, P):
    return [[data[(g * k + j) * P:(g * k + j + 1) * P] for j in range(k)] for g in range(G)]


def test_input_generator_is_stable(oracle_mod, manifest):
    import hashlib
    for c in manifest["cases"]:
        if "seed" in c and "input_sha256" in c and c.get("layout") == "contiguous":
            data = oracle_mod.splitmix_bytes(c["G"] * c["k"] * c["P"], c["seed"])
            assert hashlib.sha256(data.tobytes()).hexdigest() == c["input_sha256"], c["name"]


@pytest.mark.parametrize("avx2", [True, False])
def test_xor_restatement_matches_reference(oracle_mod, manifest, xor_golden, avx2):
    n = 0
    for c in manifest["cases"]:
        if c["api"] != "xor_packets_avx2" or "seed" not in c or "G" not in c:
            continue
        data = oracle_mod.splitmix_bytes(c["G"] * c["k"] * c["P"], c["seed"])
        mine = np.concatenate([oracle_mod.xor_packets(pk, c["P"], avx2=avx2) for pk in _groups(data, c["G"], c["k"], c["P"])])
        assert np.array_equal(mine, xor_golden[c["name"]]), c["name"]
        n += 1
    assert n >= 12


def test_legacy_batch_matches_reference(oracle_mod, xor_golden, manifest):
    c = next(c for c in manifest["cases"] if c["name"] == "batch_k10_p1200_g64")
    slab = oracle_mod.splitmix_bytes(c["G"] * 10 * c["P"], c["seed"])
    offs = (np.arange(c["G"] * 10, dtype=np.uint32) * c["P"]).astype(np.uint32)
    for avx2 in (True, False):
        rc, out = oracle_mod.encode_batch_legacy(slab, offs, c["G"], c["P"], avx2=avx2)
        assert rc == 0 and np.array_equal(out, xor_golden[c["name"]])
    c = next(c for c in manifest["cases"] if c["name"] == "batch_scattered_p100_g16")
    slab = oracle_mod.splitmix_bytes(c["slab_bytes"], c["seed"])
    offs = xor_golden["batch_scattered_p100_g16_offsets"]
    rc, out = oracle_mod.encode_batch_legacy(slab, offs, c["G"], c["P"])
    assert rc == 0 and np.array_equal(out, xor_golden[c["name"]])


def test_legacy_return_codes_match_reference(oracle_mod, manifest):
    import ctypes
    codes = manifest["legacy_return_codes"]
    L = oracle_mod.lib()
    buf = np.zeros(64, dtype=np.uint8)
    off = np.zeros(10, dtype=np.uint32)
    rep = np.full(8, 0xAB, dtype=np.uint8)
    assert L.oracle_encode_batch_legacy(None, off.ctypes.data, 1, 8, rep.ctypes.data, 1) == codes["null_slab"]
    assert L.oracle_encode_batch_legacy(buf.ctypes.data, None, 1, 8, rep.ctypes.data, 1) == codes["null_offsets"]
    assert L.oracle_encode_batch_legacy(buf.ctypes.data, off.ctypes.data, 1, 8, None, 1) == codes["null_repair"]
    assert L.oracle_encode_batch_legacy(buf.ctypes.data, off.ctypes.data, 0, 8, rep.ctypes.data, 1) == codes["zero_groups"]
    assert L.oracle_encode_batch_legacy(buf.ctypes.data, off.ctypes.data, 1, 0, rep.ctypes.data, 1) == codes["zero_size"]
    assert (rep == 0xAB).all()
    del ctypes


def test_known_answer_encoder_test(oracle_mod, xor_golden):
    # encoder_test.go:70-86: packets i = 1200 x byte(i) -> repair 0^1^...^9 = 1
    pk = [np.full(1200, i, dtype=np.uint8) for i in range(10)]
    assert np.array_equal(oracle_mod.xor_packets(pk, 1200), xor_golden["kat_encoder_test"])
    red = oracle_mod.go_generate_redundancy(pk, group_id=0)
    assert red[:11].tolist() == [0xFE, 0xC0] + [0] * 8 + [10]
    assert (red[11:] == 1).all() and len(red) == 1211


def test_degenerate_xor_writes_nothing(oracle_mod):
    out = np.full(16, 0x5A, dtype=np.uint8)
    L = oracle_mod.lib()
    arr = (oracle_mod._vp * 1)()
    L.oracle_xor_avx2(arr, 0, 16, out.ctypes.data)
    L.oracle_xor_scalar(arr, 0, 16, out.ctypes.data)
    assert (out == 0x5A).all()


def test_go_redundancy_zero_pads_and_header(oracle_mod):
    # encoder.go:118-157: shorter packets are zero-padded to the longest
    pk = [np.arange(5, dtype=np.uint8), np.arange(9, dtype=np.uint8) * 3, np.full(2, 7, dtype=np.uint8)]
    red = oracle_mod.go_generate_redundancy(pk, group_id=0x0102030405060708)
    assert red[:11].tolist() == [0xFE, 0xC0, 8, 7, 6, 5, 4, 3, 2, 1, 3]
    exp = np.zeros(9, dtype=np.uint8)
    for p in pk:
        exp[:len(p)] ^= p
    assert np.array_equal(red[11:], exp)


def test_go_recover_single_matches_rs_decode(oracle_mod):
    k, P = 10, 1200
    data = oracle_mod.splitmix_bytes(k * P, 0xABC)
    pk = [data[j * P:(j + 1) * P] for j in range(k)]
    parity = oracle_mod.rs_encode(data, 1, k, 3, P)
    for lost in (0, 4, 9):
        have = [p if j != lost else None for j, p in enumerate(pk)]
        mid, out = oracle_mod.go_recover_single(have, parity[:P], P)
        assert mid == lost and np.array_equal(out, pk[lost])
        d2 = data.copy()
        d2[lost * P:(lost + 1) * P] = 0
        bad, st = oracle_mod.rs_decode(d2, parity, np.array([1 << lost], dtype=np.uint64), 1, k, 3, P)
        assert bad == 0 and np.array_equal(d2, data)


def test_parity_matrix_fixture(oracle_mod, golden_dir):
    mats = json.loads((golden_dir / "parity_matrices.json").read_text())
    for key, M in mats.items():
        k, r = map(int, key.split(","))
        assert np.array_equal(oracle_mod.parity_matrix(k, r), np.array(M, dtype=np.uint8)), key


def test_gf_fixtures(oracle_mod, manifest, gf_golden):
    for c in manifest["cases"]:
        if not c["name"].startswith("rs_"):
            continue
        G, k, r, P = c["G"], c["k"], c["r"], c["P"]
        data = oracle_mod.splitmix_bytes(G * k * P, c["seed"])
        par = oracle_mod.rs_encode(data, G, k, r, P)
        assert np.array_equal(par, gf_golden[c["name"] + "_parity"])
        masks = gf_golden[c["name"] + "_masks"]
        broken = data.copy().reshape(G, k, P)
        for g in range(G):
            for j in range(k):
                if (int(masks[g]) >> j) & 1:
                    broken[g, j, :] = 0xEE
        broken = broken.reshape(-1)
        bad, st = oracle_mod.rs_decode(broken, par, masks, G, k, r, P)
        assert np.array_equal(broken, gf_golden[c["name"] + "_decoded"])
        assert np.array_equal(st, gf_golden[c["name"] + "_status"])
        assert bad == c["unrecoverable"]
        # every recoverable group is restored exactly
        ok = st == 0
        assert np.array_equal(broken.reshape(G, -1)[ok], data.reshape(G, -1)[ok])


def test_gf_field_axioms(oracle_mod):
    rng = np.random.default_rng(1)
    for a, b, c in rng.integers(0, 256, size=(300, 3)):
        a, b, c = int(a), int(b), int(c)
        m = oracle_mod.gf_mul
        assert m(a, b) == m(b, a)
        assert m(a, m(b, c)) == m(m(a, b), c)
        assert m(a, b ^ c) == m(a, b) ^ m(a, c)
    for a in range(1, 256):
        assert oracle_mod.gf_mul(a, int(oracle_mod.lib().oracle_gf_inv(a))) == 1


@settings(max_examples=40, deadline=None)
@given(k=st.integers(1, 24), r=st.integers(1, 8), P=st.integers(1, 70), seed=st.integers(0, 2**32),
       data=st.data())
def test_mds_round_trip(oracle_mod, k, r, P, seed, data):
    if k + r > 64:
        return
    G = 3
    d = oracle_mod.splitmix_bytes(G * k * P, seed)
    par = oracle_mod.rs_encode(d, G, k, r, P)
    masks = np.zeros(G, dtype=np.uint64)
    for g in range(G):
        lost = data.draw(st.lists(st.integers(0, k + r - 1), max_size=r, unique=True))
        masks[g] = np.uint64(sum(1 << x for x in lost))
    broken = d.copy().reshape(G, k, P)
    for g in range(G):
        for j in range(k):
            if (int(masks[g]) >> j) & 1:
                broken[g, j] = 0x77
    broken = broken.reshape(-1)
    bad, st_ = oracle_mod.rs_decode(broken, par, masks, G, k, r, P)
    assert bad == 0 and np.array_equal(broken, d)


def test_gf_affine_matrices(oracle_mod):
    """oracle_gf_affine(c) applied as VGF2P8AFFINEQB does (output bit i = parity of matrix
    byte 7-i AND x) is multiplication by c."""
    xs = np.arange(256)
    for c in range(256):
        A = int(oracle_mod.lib().oracle_gf_affine(c))
        rows = [(A >> (8 * (7 - i))) & 0xFF for i in range(8)]
        for x in xs[:: 7 if c % 5 else 1]:
            y = sum((bin(rows[i] & int(x)).count("1") & 1) << i for i in range(8))
            assert y == oracle_mod.gf_mul(c, int(x)), (c, int(x))


@pytest.mark.parametrize("k,r,P,G", [(10, 3, 1200, 300), (20, 5, 1200, 60), (4, 2, 256, 200), (10, 3, 1201, 90),
                                     (7, 9, 33, 80), (30, 8, 100, 40), (10, 1, 1200, 50), (12, 12, 17, 40),
                                     (3, 2, 1, 20)])
def test_fast_comparator_equals_restatement(oracle_mod, k, r, P, G):
    """The bench's CPU comparator (GFNI form) produces the restatement's bytes, statuses and
    unrecoverable counts (tails, every parity-row pass, unrecoverable groups)."""
    rng = np.random.default_rng(k * 1000 + r * 10 + P)
    data = oracle_mod.splitmix_bytes(G * k * P, 0x5EED + k + r)
    par = oracle_mod.rs_encode(data, G, k, r, P)
    assert np.array_equal(oracle_mod.rs_encode_fast(data, G, k, r, P, nthreads=3), par)
    masks = np.zeros(G, dtype=np.uint64)
    for g in range(G):
        for s in rng.permutation(k + r)[: rng.integers(0, r + 2)]:
            masks[g] |= np.uint64(1) << np.uint64(int(s))
    lost = ((masks[:, None] >> np.arange(k, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
    a = data.copy().reshape(G, k, P)
    a[lost] = 0xEE
    b = a.copy()
    bad_a, st_a = oracle_mod.rs_decode(a.reshape(-1), par, masks, G, k, r, P)
    bad_b, st_b = oracle_mod.rs_decode_fast(b.reshape(-1), par, masks, G, k, r, P, nthreads=2)
    assert bad_a == bad_b and np.array_equal(st_a, st_b) and np.array_equal(a, b)
