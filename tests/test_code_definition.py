"""The GF(2^8) code restated a second time, from its written definition only (SURVEY.md §8(a)
"Code definition for r > 1"), in plain Python: carry-less multiplication
modulo 0x11D (no tables), inverses as a^254, the normalised Cauchy matrix built from the
formula, and erasure decoding by Gauss-Jordan elimination over the generator's rows.  None
of it shares code with oracle/fec_oracle.c or quic-test_amd/csrc/gf256.hpp, so these checks
pin the committed matrices, the C restatement's encode and decode (and through the GPU
parity tests, the kernels) to the definition rather than to one implementation of it.
Rows 1..r-1 remain "parity unpinned by the reference" (the reference is XOR-only); row 0 is
the reference XOR (fec_xor_simd.cpp:411-427)."""
import itertools
import json

import numpy as np
import pytest


def gf_mul(a: int, b: int) -> int:
    """Shift-and-add multiplication in GF(2^8) with the polynomial x^8+x^4+x^3+x^2+1."""
    p = 0
    while b:
        if b & 1:
            p ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
    return p


def gf_inv(a: int) -> int:
    assert a != 0
    r, x, e = 1, a, 254          # a^(2^8 - 2)
    while e:
        if e & 1:
            r = gf_mul(r, x)
        x = gf_mul(x, x)
        e >>= 1
    return r


def cauchy_parity(k: int, r: int):
    """r x k: C_ij = 1 / (x_i ^ y_j), x_i = i, y_j = r + j; columns scaled so row 0 is all
    ones, then rows i >= 1 scaled so column 0 is all ones."""
    C = [[gf_inv(i ^ (r + j)) for j in range(k)] for i in range(r)]
    for j in range(k):
        s = gf_inv(C[0][j])
        for i in range(r):
            C[i][j] = gf_mul(C[i][j], s)
    for i in range(1, r):
        s = gf_inv(C[i][0])
        C[i] = [gf_mul(c, s) for c in C[i]]
    return C


def solve(A, B):
    """X with A X = B over GF(2^8) (A square, non-singular), Gauss-Jordan; rows are lists."""
    n = len(A)
    M = [list(A[i]) + list(B[i]) for i in range(n)]
    for c in range(n):
        piv = next(i for i in range(c, n) if M[i][c])
        M[c], M[piv] = M[piv], M[c]
        inv = gf_inv(M[c][c])
        M[c] = [gf_mul(v, inv) for v in M[c]]
        for i in range(n):
            if i != c and M[i][c]:
                f = M[i][c]
                M[i] = [v ^ gf_mul(f, w) for v, w in zip(M[i], M[c])]
    return [row[n:] for row in M]


def det_nonzero(A) -> bool:
    n = len(A)
    M = [list(r) for r in A]
    for c in range(n):
        piv = next((i for i in range(c, n) if M[i][c]), None)
        if piv is None:
            return False
        M[c], M[piv] = M[piv], M[c]
        inv = gf_inv(M[c][c])
        for i in range(c + 1, n):
            if M[i][c]:
                f = gf_mul(M[i][c], inv)
                M[i] = [v ^ gf_mul(f, w) for v, w in zip(M[i], M[c])]
    return True


def test_field_is_the_0x11d_field():
    # 2 generates the multiplicative group (the code's generator) and x^8 = x^4+x^3+x^2+1
    seen, x = set(), 1
    for _ in range(255):
        seen.add(x)
        x = gf_mul(x, 2)
    assert len(seen) == 255 and x == 1
    assert gf_mul(0x80, 2) == 0x1D


def test_committed_matrices_follow_the_definition(golden_dir, oracle_mod):
    mats = json.loads((golden_dir / "parity_matrices.json").read_text())
    assert mats
    for key, M in mats.items():
        k, r = map(int, key.split(","))
        exp = cauchy_parity(k, r)
        assert np.array_equal(np.array(M, dtype=np.uint8), np.array(exp, dtype=np.uint8)), key
    for k, r in ((10, 3), (20, 5), (1, 255), (200, 56)):       # also the oracle's own builder
        assert np.array_equal(oracle_mod.parity_matrix(k, r), np.array(cauchy_parity(k, r), dtype=np.uint8))


@pytest.mark.parametrize("k,r", [(4, 2), (10, 3), (6, 4)])
def test_every_square_submatrix_is_nonsingular(k, r):
    """MDS: any e <= r lost data shards are recoverable from any e surviving parity rows."""
    C = cauchy_parity(k, r)
    assert all(v == 1 for v in C[0]) and all(C[i][0] == 1 for i in range(r))
    for e in range(1, r + 1):
        for rows in itertools.combinations(range(r), e):
            for cols in itertools.combinations(range(k), e):
                assert det_nonzero([[C[i][j] for j in cols] for i in rows]), (rows, cols)


@pytest.mark.parametrize("k,r,P,seed", [(10, 3, 24, 1), (4, 2, 16, 2), (20, 5, 8, 3), (6, 4, 5, 4)])
def test_oracle_encode_and_decode_follow_the_definition(oracle_mod, k, r, P, seed):
    """Parity = C x data byte-wise; every recoverable erasure pattern tried on a small group
    is rebuilt by the oracle exactly as Gauss-Jordan over the generator rows rebuilds it."""
    C = cauchy_parity(k, r)
    data = oracle_mod.splitmix_bytes(k * P, 0x5EED7000 + seed)
    d = data.reshape(k, P).tolist()
    par = [[0] * P for _ in range(r)]
    for i in range(r):
        for j in range(k):
            for b in range(P):
                par[i][b] ^= gf_mul(C[i][j], d[j][b])
    assert np.array_equal(oracle_mod.rs_encode(data, 1, k, r, P), np.array(par, dtype=np.uint8).reshape(-1))
    assert par[0] == [int(x) for x in np.bitwise_xor.reduce(data.reshape(k, P), axis=0)]   # row 0 = XOR
    rng = np.random.default_rng(seed)
    G = [[int(i == j) for j in range(k)] for i in range(k)] + C          # generator [I_k ; C]
    shards = d + par
    for _ in range(12):
        lost = sorted(int(x) for x in rng.choice(k + r, size=int(rng.integers(1, r + 1)), replace=False))
        alive = [s for s in range(k + r) if s not in lost]
        rows = alive[:k]                                                  # any k survivors
        X = solve([G[s] for s in rows], [shards[s] for s in rows])        # the data, rebuilt
        assert X == d
        broken = data.copy().reshape(k, P)
        for s in lost:
            if s < k:
                broken[s] = 0xEE
        mask = np.array([sum(1 << s for s in lost)], dtype=np.uint64)
        out = broken.reshape(-1).copy()
        bad, st = oracle_mod.rs_decode(out, np.array(par, dtype=np.uint8).reshape(-1), mask, 1, k, r, P)
        assert bad == 0 and st[0] == 0
        assert np.array_equal(out.reshape(k, P), np.array(X, dtype=np.uint8)), lost
