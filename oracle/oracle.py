"""ctypes wrapper of the CPU checker (oracle/liboracle.so) and of the reference library
compiled from /root/reference (oracle/_ref/libfec_ref.so).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; never by the product path (quic-test_amd/).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path
from typing import Optional, Sequence

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
ORACLE_LIB = ORACLE_DIR / "liboracle.so"
REF_LIB = ORACLE_DIR / "_ref" / "libfec_ref.so"

_vp, _u32, _u64, _int, _sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t
_lib: Optional[ctypes.CDLL] = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR), "liboracle.so"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not ORACLE_LIB.exists():
            build()
        L = ctypes.CDLL(str(ORACLE_LIB))
        sig = {
            "oracle_fill_splitmix": (None, [_vp, _u64, _u64, _u64]),
            "oracle_xor_scalar": (None, [ctypes.POINTER(_vp), _sz, _sz, _vp]),
            "oracle_xor_avx2": (None, [ctypes.POINTER(_vp), _sz, _sz, _vp]),
            "oracle_encode_batch_legacy": (_int, [_vp, _vp, _u32, _u32, _vp, _int]),
            "oracle_xor_encode_contig": (None, [_vp, _u64, _u32, _u32, _vp, _int]),
            "oracle_xor_groups": (None, [_vp, _vp, _u64, _u32, _u32, _vp]),
            "oracle_gf_mul": (ctypes.c_uint8, [ctypes.c_uint8, ctypes.c_uint8]),
            "oracle_gf_inv": (ctypes.c_uint8, [ctypes.c_uint8]),
            "oracle_parity_matrix": (_int, [_u32, _u32, _vp]),
            "oracle_rs_encode": (_int, [_vp, _u64, _u32, _u32, _u32, _vp, _int]),
            "oracle_rs_decode": (ctypes.c_int64, [_vp, _vp, _vp, _u64, _u32, _u32, _u32, _vp, _int]),
            "oracle_fast_isa": (_int, []),
            "oracle_gf_affine": (_u64, [ctypes.c_uint8]),
            "oracle_rs_encode_fast": (_int, [_vp, _u64, _u32, _u32, _u32, _vp, _int]),
            "oracle_rs_decode_fast": (ctypes.c_int64, [_vp, _vp, _vp, _u64, _u32, _u32, _u32, _vp, _int]),
            "oracle_go_generate_redundancy": (ctypes.c_int64, [ctypes.POINTER(_vp), ctypes.POINTER(_sz), _sz, _u64, _vp, _sz]),
            "oracle_go_recover_single": (ctypes.c_int64, [ctypes.POINTER(_vp), ctypes.POINTER(_sz), _vp, _sz, _vp, _sz, _sz, _vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def splitmix_bytes(nbytes: int, seed: int, byte_offset: int = 0) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    lib().oracle_fill_splitmix(out.ctypes.data, nbytes, seed, byte_offset)
    return out


def _ptrs(pkts: Sequence[np.ndarray]):
    return (_vp * max(1, len(pkts)))(*[p.ctypes.data for p in pkts])


def xor_packets(pkts: Sequence[np.ndarray], packet_size: int, avx2: bool = True) -> np.ndarray:
    out = np.zeros(packet_size, dtype=np.uint8)
    f = lib().oracle_xor_avx2 if avx2 else lib().oracle_xor_scalar
    f(_ptrs(pkts), len(pkts), packet_size, out.ctypes.data)
    return out


def encode_batch_legacy(slab: np.ndarray, offsets: np.ndarray, num_groups: int, packet_size: int,
                        avx2: bool = True):
    out = np.zeros(num_groups * packet_size, dtype=np.uint8)
    rc = lib().oracle_encode_batch_legacy(slab.ctypes.data, offsets.ctypes.data, num_groups, packet_size,
                                          out.ctypes.data, int(avx2))
    return rc, out


def parity_matrix(k: int, r: int) -> np.ndarray:
    M = np.zeros((r, k), dtype=np.uint8)
    assert lib().oracle_parity_matrix(k, r, M.ctypes.data) == 0
    return M


def gf_mul(a: int, b: int) -> int:
    return int(lib().oracle_gf_mul(a, b))


def rs_encode(data: np.ndarray, G: int, k: int, r: int, P: int, nthreads: int = 1) -> np.ndarray:
    par = np.zeros(G * r * P, dtype=np.uint8)
    assert lib().oracle_rs_encode(data.ctypes.data, G, k, r, P, par.ctypes.data, nthreads) == 0
    return par


def xor_encode_contig(data: np.ndarray, G: int, k: int, P: int, nthreads: int = 1) -> np.ndarray:
    out = np.zeros(G * P, dtype=np.uint8)
    lib().oracle_xor_encode_contig(data.ctypes.data, G, k, P, out.ctypes.data, nthreads)
    return out


def rs_decode(data: np.ndarray, parity: np.ndarray, masks: np.ndarray, G: int, k: int, r: int, P: int,
              nthreads: int = 1):
    """In place on `data`.  Returns (unrecoverable_count, status)."""
    st = np.zeros(G, dtype=np.uint8)
    bad = lib().oracle_rs_decode(data.ctypes.data, parity.ctypes.data, masks.ctypes.data, G, k, r, P,
                                 st.ctypes.data, nthreads)
    assert bad >= 0
    return int(bad), st


def fast_isa() -> int:
    """2 = AVX-512 + GFNI, 1 = AVX2 + GFNI, 0 = table fallback (oracle_rs_*_fast)."""
    return int(lib().oracle_fast_isa())


def rs_encode_fast(data: np.ndarray, G: int, k: int, r: int, P: int, nthreads: int = 1) -> np.ndarray:
    """The GFNI comparator (bench.py cpu_baseline); same bytes as rs_encode."""
    par = np.zeros(G * r * P, dtype=np.uint8)
    assert lib().oracle_rs_encode_fast(data.ctypes.data, G, k, r, P, par.ctypes.data, nthreads) == 0
    return par


def rs_decode_fast(data: np.ndarray, parity: np.ndarray, masks: np.ndarray, G: int, k: int, r: int, P: int,
                   nthreads: int = 1):
    """The GFNI comparator of rs_decode (in place).  Returns (unrecoverable_count, status)."""
    st = np.zeros(G, dtype=np.uint8)
    bad = lib().oracle_rs_decode_fast(data.ctypes.data, parity.ctypes.data, masks.ctypes.data, G, k, r, P,
                                      st.ctypes.data, nthreads)
    assert bad >= 0
    return int(bad), st


def go_generate_redundancy(pkts: Sequence[np.ndarray], group_id: int) -> np.ndarray:
    lens = (_sz * max(1, len(pkts)))(*[len(p) for p in pkts])
    cap = 11 + max([len(p) for p in pkts] + [0])
    out = np.zeros(cap, dtype=np.uint8)
    n = lib().oracle_go_generate_redundancy(_ptrs(pkts), lens, len(pkts), group_id, out.ctypes.data, cap)
    if n < 0:
        raise ValueError(f"generateRedundancy error {n}")
    return out[:n]


def go_recover_single(pkts: Sequence[Optional[np.ndarray]], parity_payload: np.ndarray, symbol_len: int):
    n = len(pkts)
    present = np.array([p is not None for p in pkts], dtype=np.uint8)
    dummy = np.zeros(1, dtype=np.uint8)
    arrs = [p if p is not None else dummy for p in pkts]
    lens = (_sz * max(1, n))(*[len(p) if p is not None else 0 for p in pkts])
    out = np.zeros(symbol_len, dtype=np.uint8)
    mid = lib().oracle_go_recover_single(_ptrs(arrs), lens, present.ctypes.data, n, parity_payload.ctypes.data,
                                         len(parity_payload), symbol_len, out.ctypes.data)
    return int(mid), out


# ---- the reference itself: oracle/_ref/libfec_ref.so, compiled from /root/reference in the
# build container and carried to the GPU box with the tree (git-ignored, not gpurun-ignored);
# loaded only by the oracle tests and bench.py's cpu_baseline leg ----
def ref_lib() -> Optional[ctypes.CDLL]:
    if not REF_LIB.exists():
        return None
    L = ctypes.CDLL(str(REF_LIB))
    for name in ("xor_packets_scalar", "xor_packets_avx2"):
        f = getattr(L, name)
        f.restype = None
        f.argtypes = [ctypes.POINTER(_vp), _sz, _sz, _vp]
    L.fec_encoder_new.restype = _vp
    L.fec_encoder_new.argtypes = [ctypes.c_double, _u32]
    L.fec_encoder_free.argtypes = [_vp]
    L.fec_encode_batch.restype = _int
    L.fec_encode_batch.argtypes = [_vp, _vp, _vp, _u32, _u32, _vp]
    return L
