#!/usr/bin/env python3
"""C1 leg of the campaign (BASELINE.json configs[0]): FEC encode k=4 r=2, 256 B packets, 1k
groups on the host CPU "via internal/fec AVX2 path" -- plumbing, no GPU needed.

Runs the reference's own AVX2 path: oracle/_ref/libfec_ref.so, the reference's
internal/fec/fec_xor_simd.cpp compiled by oracle/Makefile, `xor_packets_avx2` (fec_xor_simd.cpp:
74-204) once per group over its k=4 packets (fec_encode_batch is fixed at 10 packets per group,
:580, so it cannot take k=4).  Byte-compares its repair rows with this repo's AVX2 restatement
(oracle.xor_packets) and with row 0 of the GF(2^8) restatement (oracle.rs_encode), and -- when
a GPU is usable -- with row 0 of libfec_hip.so's encode (rows 1..r-1 against the restatement).
Prints one JSON object.  Test infrastructure and measurement only: nothing here is the product.
"""
from __future__ import annotations

import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "quic-test_amd"))

import oracle  # noqa: E402

K, R, P, G = 4, 2, 256, 1024
SEED = 0x5EED0001


def _timed(fn, min_seconds: float = 0.5):
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            return dt / reps


def main(gpu: bool = True) -> dict:
    data = oracle.splitmix_bytes(G * K * P, SEED)
    pk = data.reshape(G, K, P)
    out = {"config": "C1", "k": K, "r": R, "P": P, "groups": G}
    # the restatements
    xr = np.concatenate([oracle.xor_packets(list(pk[g]), P) for g in range(G)])
    par = oracle.rs_encode(data, G, K, R, P)
    row0 = par.reshape(G, R, P)[:, 0, :].reshape(-1)
    out["restatement_row0_equals_xor"] = bool(np.array_equal(row0, xr))
    t = _timed(lambda: oracle.rs_encode(data, G, K, R, P))
    out["restatement_rs_encode_GiBps"] = round(G * K * P / t / 2**30, 3)
    # the reference's AVX2 path, as compiled from /root/reference
    ref = oracle.ref_lib()
    out["reference_lib_present"] = ref is not None
    expect_row0 = xr  # the reference's own rows when its library is here (equal to xr, checked)
    if ref is not None:
        rep = np.zeros(G * P, dtype=np.uint8)
        fn = ctypes.cast(ref.xor_packets_avx2, ctypes.c_void_p).value
        L = oracle.lib()

        def ref_all():  # the reference's function once per group, driven from C (oracle_xor_groups)
            L.oracle_xor_groups(fn, data.ctypes.data, G, K, P, rep.ctypes.data)

        ref_all()
        out["reference_xor_avx2_equals_restatement"] = bool(np.array_equal(rep, xr))
        expect_row0 = rep.copy()
        t = _timed(ref_all)
        out["reference_xor_avx2_GiBps"] = round(G * K * P / t / 2**30, 3)
        out["reference_xor_avx2_us_per_group"] = round(t / G * 1e6, 3)
        out["reference_note"] = ("oracle/_ref/libfec_ref.so (reference internal/fec/fec_xor_simd.cpp built by "
                                 "oracle/Makefile), xor_packets_avx2 called once per group by a C loop "
                                 "(oracle_xor_groups), 1 thread")
    if gpu:
        try:
            import torch
            has_gpu = torch.cuda.is_available()
        except ImportError:
            has_gpu = False
        out["gpu_present"] = has_gpu
        if has_gpu:
            import quicfec
            with quicfec.Context(device=0) as ctx:
                gp = np.zeros(G * R * P, dtype=np.uint8)
                ctx.encode(data, K, R, P, gp, num_groups=G)
                out["gpu_row0_equals_reference"] = bool(np.array_equal(gp.reshape(G, R, P)[:, 0, :].reshape(-1), expect_row0))
                out["gpu_rows_equal_restatement"] = bool(np.array_equal(gp, par))
    return out


if __name__ == "__main__":
    res = main(gpu="--no-gpu" not in sys.argv)
    print(json.dumps(res), flush=True)
    ok = res["restatement_row0_equals_xor"] and res.get("reference_xor_avx2_equals_restatement", True) \
        and res.get("gpu_row0_equals_reference", True) and res.get("gpu_rows_equal_restatement", True)
    sys.exit(0 if ok else 1)
