#!/usr/bin/env python3
"""Generate the committed golden fixtures for the FEC parity tests.

Run in the build container, where /root/reference exists:

    make -C oracle            # builds oracle/liboracle.so and oracle/_ref/libfec_ref.so
    python tests/golden/make_golden.py

Outputs (data only — inputs are regenerated from seeds; their SHA-256 is recorded so a
drifting generator is caught):

  xor_ref.npz            parity row 0 / XOR outputs of the REFERENCE library
                         (oracle/_ref/libfec_ref.so = /root/reference/internal/fec/
                         fec_xor_simd.cpp compiled in place; xor_packets_avx2,
                         xor_packets_scalar, fec_encode_batch).  Pins row 0.
  gf_restatement.npz     GF(2^8) rows 1..r-1 and multi-erasure decode outputs of this
                         repo's CPU restatement (oracle/fec_oracle.c).  The reference has
                         no GF code: these are "parity unpinned by the reference" and only
                         freeze the code definition.
  parity_matrices.json   the r x k parity matrices of the code definition.
  manifest.json          case list, seeds, shapes, SHA-256 of inputs and outputs.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO / "oracle"))
import oracle  # noqa: E402

_vp, _sz = ctypes.c_void_p, ctypes.c_size_t

SEED_BASE = 0x5EED0000


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ref_xor(ref, pkts, P, fn="xor_packets_avx2", prefill=0):
    out = np.full(P, prefill, dtype=np.uint8)
    arr = (_vp * max(1, len(pkts)))(*[p.ctypes.data for p in pkts])
    getattr(ref, fn)(arr, len(pkts), P, out.ctypes.data)
    return out


def main() -> int:
    ref = oracle.ref_lib()
    if ref is None:
        print("oracle/_ref/libfec_ref.so missing: run `make -C oracle` where /root/reference exists")
        return 1
    manifest = {"generator": "tests/golden/make_golden.py", "cases": []}
    xor_out = {}

    # 1. fec_encode_batch: k=10, P=1200, 64 groups, contiguous offsets
    seed = SEED_BASE + 0x101
    G, k, P = 64, 10, 1200
    slab = oracle.splitmix_bytes(G * k * P, seed)
    offs = (np.arange(G * k, dtype=np.uint32) * P).astype(np.uint32)
    rep = np.zeros(G * P, dtype=np.uint8)
    ctx = ref.fec_encoder_new(0.10, 1024)
    rc = ref.fec_encode_batch(ctx, slab.ctypes.data, offs.ctypes.data, G, P, rep.ctypes.data)
    assert rc == 0
    xor_out["batch_k10_p1200_g64"] = rep
    manifest["cases"].append({"name": "batch_k10_p1200_g64", "api": "fec_encode_batch", "seed": seed,
                              "G": G, "k": k, "P": P, "layout": "contiguous", "input_sha256": sha(slab),
                              "output_sha256": sha(rep)})

    # 2. fec_encode_batch with scattered, unaligned offsets inside a larger slab
    seed = SEED_BASE + 0x102
    G, P = 16, 100
    slab = oracle.splitmix_bytes(64 * 1024, seed)
    rng = np.random.default_rng(seed)
    offs = rng.integers(0, 64 * 1024 - P, size=G * 10, dtype=np.uint64).astype(np.uint32)
    rep = np.zeros(G * P, dtype=np.uint8)
    assert ref.fec_encode_batch(ctx, slab.ctypes.data, offs.ctypes.data, G, P, rep.ctypes.data) == 0
    xor_out["batch_scattered_p100_g16"] = rep
    xor_out["batch_scattered_p100_g16_offsets"] = offs
    manifest["cases"].append({"name": "batch_scattered_p100_g16", "api": "fec_encode_batch", "seed": seed,
                              "G": G, "k": 10, "P": P, "slab_bytes": 64 * 1024, "offsets": "stored",
                              "input_sha256": sha(slab), "output_sha256": sha(rep)})

    # 3. fec_encode_batch argument edge cases (return codes; repair must stay untouched)
    rep = np.full(8, 0xAB, dtype=np.uint8)
    one = np.zeros(10, dtype=np.uint32)
    codes = {
        "null_ctx": ref.fec_encode_batch(None, slab.ctypes.data, one.ctypes.data, 1, 8, rep.ctypes.data),
        "null_slab": ref.fec_encode_batch(ctx, None, one.ctypes.data, 1, 8, rep.ctypes.data),
        "null_offsets": ref.fec_encode_batch(ctx, slab.ctypes.data, None, 1, 8, rep.ctypes.data),
        "null_repair": ref.fec_encode_batch(ctx, slab.ctypes.data, one.ctypes.data, 1, 8, None),
        "zero_groups": ref.fec_encode_batch(ctx, slab.ctypes.data, one.ctypes.data, 0, 8, rep.ctypes.data),
        "zero_size": ref.fec_encode_batch(ctx, slab.ctypes.data, one.ctypes.data, 1, 0, rep.ctypes.data),
    }
    assert (rep == 0xAB).all()
    manifest["legacy_return_codes"] = codes
    ref.fec_encoder_free(ctx)

    # 4. xor_packets_avx2 with k != 10 (only reachable per group): k=4 P=256 x16, k=20 P=1200 x8
    for (k, P, G, tag) in ((4, 256, 16, 0x103), (20, 1200, 8, 0x104)):
        seed = SEED_BASE + tag
        data = oracle.splitmix_bytes(G * k * P, seed)
        reps = []
        for g in range(G):
            pk = [data[(g * k + j) * P:(g * k + j + 1) * P] for j in range(k)]
            a = ref_xor(ref, pk, P, "xor_packets_avx2")
            b = ref_xor(ref, pk, P, "xor_packets_scalar")
            assert (a == b).all()
            reps.append(a)
        rep = np.concatenate(reps)
        name = f"xor_k{k}_p{P}_g{G}"
        xor_out[name] = rep
        manifest["cases"].append({"name": name, "api": "xor_packets_avx2", "seed": seed, "G": G, "k": k, "P": P,
                                  "layout": "contiguous", "input_sha256": sha(data), "output_sha256": sha(rep)})

    # 5. tail sizes around the 16/32/128-byte vector steps of the AVX2 loop
    tails = [1, 15, 16, 31, 33, 127, 129, 1234, 1500, 9000]
    for P in tails:
        seed = SEED_BASE + 0x200 + P
        k, G = 10, 2
        data = oracle.splitmix_bytes(G * k * P, seed)
        reps = []
        for g in range(G):
            pk = [data[(g * k + j) * P:(g * k + j + 1) * P] for j in range(k)]
            a = ref_xor(ref, pk, P, "xor_packets_avx2")
            assert (a == ref_xor(ref, pk, P, "xor_packets_scalar")).all()
            reps.append(a)
        rep = np.concatenate(reps)
        name = f"tail_p{P}"
        xor_out[name] = rep
        manifest["cases"].append({"name": name, "api": "xor_packets_avx2", "seed": seed, "G": G, "k": k, "P": P,
                                  "layout": "contiguous", "input_sha256": sha(data), "output_sha256": sha(rep)})

    # 6. known-answer test implied by encoder_test.go:70-86 (packet i = 1200 x byte(i))
    pk = [np.full(1200, i, dtype=np.uint8) for i in range(10)]
    kat = ref_xor(ref, pk, 1200)
    assert (kat == 1).all()
    xor_out["kat_encoder_test"] = kat
    manifest["cases"].append({"name": "kat_encoder_test", "api": "xor_packets_avx2", "k": 10, "P": 1200,
                              "input": "packet i = 1200 x byte(i), i < 10", "output_sha256": sha(kat)})

    # 7. degenerate calls: n=0 or size=0 write nothing; n=1 copies
    pre = ref_xor(ref, [], 16, prefill=0x5A)
    assert (pre == 0x5A).all()
    one_pkt = oracle.splitmix_bytes(77, SEED_BASE + 0x105)
    xor_out["single_packet_p77"] = ref_xor(ref, [one_pkt], 77)
    assert (xor_out["single_packet_p77"] == one_pkt).all()
    manifest["cases"].append({"name": "single_packet_p77", "api": "xor_packets_avx2", "seed": SEED_BASE + 0x105,
                              "k": 1, "P": 77, "output_sha256": sha(xor_out["single_packet_p77"])})

    # Cross-check the restatement against the reference on every case before saving.
    for c in manifest["cases"]:
        if c["name"].startswith(("xor_", "tail_")):
            data = oracle.splitmix_bytes(c["G"] * c["k"] * c["P"], c["seed"])
            mine = np.concatenate([oracle.xor_packets([data[(g * c["k"] + j) * c["P"]:(g * c["k"] + j + 1) * c["P"]]
                                                       for j in range(c["k"])], c["P"]) for g in range(c["G"])])
            assert (mine == xor_out[c["name"]]).all(), c["name"]
    np.savez_compressed(HERE / "xor_ref.npz", **xor_out)

    # ---- GF restatement fixtures (parity unpinned by the reference) ----
    mats = {}
    for (k, r) in ((1, 1), (4, 2), (10, 1), (10, 3), (20, 5), (8, 8), (32, 32)):
        M = oracle.parity_matrix(k, r)
        assert (M[0] == 1).all() and (M[:, 0] == 1).all()
        mats[f"{k},{r}"] = M.tolist()
    (HERE / "parity_matrices.json").write_text(json.dumps(mats, indent=0))

    gf_out = {}
    for (k, r, P, G, tag) in ((4, 2, 256, 16, 0x301), (10, 3, 1200, 16, 0x302), (20, 5, 1200, 4, 0x303),
                              (10, 3, 100, 8, 0x304)):
        seed = SEED_BASE + tag
        data = oracle.splitmix_bytes(G * k * P, seed)
        par = oracle.rs_encode(data, G, k, r, P)
        # row 0 must be the reference XOR
        rows0 = par.reshape(G, r, P)[:, 0, :].reshape(-1)
        xr = np.concatenate([ref_xor(ref, [data[(g * k + j) * P:(g * k + j + 1) * P] for j in range(k)], P)
                             for g in range(G)])
        assert (rows0 == xr).all()
        name = f"rs_k{k}_r{r}_p{P}_g{G}"
        gf_out[name + "_parity"] = par
        # erasure masks: seeded, 0..r+1 erasures per group (some unrecoverable)
        rng = np.random.default_rng(seed)
        masks = np.zeros(G, dtype=np.uint64)
        for g in range(G):
            ne = int(rng.integers(0, r + 2))
            pos = rng.choice(k + r, size=min(ne, k + r), replace=False)
            masks[g] = np.uint64(sum(1 << int(p) for p in pos))
        broken = data.copy().reshape(G, k, P)
        for g in range(G):
            for j in range(k):
                if (int(masks[g]) >> j) & 1:
                    broken[g, j, :] = 0xEE
        broken = broken.reshape(-1)
        bad, st = oracle.rs_decode(broken, par, masks, G, k, r, P)
        gf_out[name + "_masks"] = masks
        gf_out[name + "_decoded"] = broken
        gf_out[name + "_status"] = st
        manifest["cases"].append({"name": name, "api": "rs_encode/rs_decode (restatement)", "seed": seed,
                                  "G": G, "k": k, "r": r, "P": P, "input_sha256": sha(data),
                                  "parity_sha256": sha(par), "decoded_sha256": sha(broken),
                                  "unrecoverable": bad, "pinned": "unpinned by reference (GF rows)"})
    np.savez_compressed(HERE / "gf_restatement.npz", **gf_out)
    (HERE / "manifest.json").write_text(json.dumps(manifest, indent=1))
    print(f"wrote {len(xor_out)} XOR fixtures, {len(gf_out)} GF arrays, {len(mats)} matrices")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
