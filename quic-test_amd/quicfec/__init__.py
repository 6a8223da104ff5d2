"""quicfec — Python binding of libfec_hip.so (the MI355X FEC engine) over its C-ABI.

This is the host-side mirror the tests and ``bench.py`` drive.  It binds exactly the
symbols declared in ``include/fec_xor_simd.h`` (the reference cgo surface,
internal/fec/fec_xor_simd.h:22-137) and ``include/fec_hip.h`` (batch GF(2^8) API).

There is no fallback: if ``libfec_hip.so`` is missing, :func:`load_library` raises, and
if no GPU is usable, :class:`Context` raises :class:`FecError` (the C library returns
NULL from ``fec_encoder_new``, which is what lets the Go hybrid encoder fall back to Go,
encoder_hybrid.go:44-52).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent          # quic-test_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_PATH = PKG_ROOT / "lib" / "libfec_hip.so"
# The same library with the test and tuning switches live (csrc/fec_knobs.hpp): only tests that
# force a kernel form, a size or a fault load it (tests/conftest.py gpu_ctx_hooks).
TEST_LIB_PATH = PKG_ROOT / "lib" / "libfec_hip_test.so"
INCLUDE_DIR = REPO_ROOT / "include"

FEC_OK = 0
FEC_ERR_NULL = -1
FEC_ERR_HIP = -2
FEC_ERR_RANGE = -3
FEC_ERR_NODEV = -4
FEC_ERR_NOMEM = -5
FEC_ERR_AGAIN = -6
FEC_ERR_UNRECOVERABLE = -7

# Every function the headers declare (tests check the library exports all of them).
REFERENCE_SYMBOLS = (
    "fec_encoder_new", "fec_alloc_slab", "fec_alloc_slab_numa", "fec_alloc_repair_buffer",
    "fec_free_repair_buffer", "fec_encode_batch", "fec_encoder_free", "fec_free_slab",
    "fec_select_xor_impl", "xor_packets_scalar", "xor_packets_avx2", "xor_packets_avx512",
    "xor_packets_neon",
)
HIP_SYMBOLS = (
    "fec_hip_device_count", "fec_hip_last_error", "fec_ctx_last_error", "fec_encoder_new_device", "fec_encoder_device",
    "fec_hip_version", "fec_parity_matrix", "fec_encode_batch_rs", "fec_decode_batch_rs",
    "fec_encode_batch_rs_dev", "fec_decode_batch_rs_dev", "fec_recover_batch_rs_dev", "fec_decode_prepare",
    "fec_fill_random_dev", "fec_copy_dev", "fec_synchronize", "fec_decode_loss_hint",
    "fec_group_new", "fec_group_free", "fec_group_size", "fec_group_context",
    "fec_group_encode_batch_rs", "fec_group_decode_batch_rs",
    "fec_batcher_new", "fec_batcher_free", "fec_batcher_submit", "fec_batcher_submit_packets",
    "fec_batcher_wait", "fec_batcher_flush", "fec_batcher_stats", "fec_batcher_last_error",
    "fec_batcher_new_decoder", "fec_batcher_submit_shards", "fec_batcher_wait_rebuilt",
    "fec_batcher_new_multi", "fec_batcher_new_decoder_multi", "fec_batcher_devices",
    "fec_recover_batch_rs_dev_packed", "fec_coalesce_stats", "fec_coalesce_stats_sized",
)


class FecError(RuntimeError):
    def __init__(self, what: str, code: int, detail: str = ""):
        super().__init__(f"{what} failed with code {code}" + (f": {detail}" if detail else ""))
        self.code = code


_lib: Optional[ctypes.CDLL] = None
_test_lib: Optional[ctypes.CDLL] = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p
_u32, _u64, _int, _dbl, _sz = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_double, ctypes.c_size_t
XOR_IMPL_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(_vp), _sz, _sz, _vp)


def load_library(path: Optional[os.PathLike] = None) -> ctypes.CDLL:
    """Load libfec_hip.so (built by ``__graft_entry__.build()``); raise if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("QUICFEC_LIB", LIB_PATH))
    # One HIP runtime per process: torch ships its own libamdhip64.so.7.  If torch is
    # importable, load it first so libfec_hip.so binds to the same (already loaded)
    # runtime by SONAME instead of pulling /opt/rocm's copy next to it.
    if os.environ.get("QUICFEC_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not p.exists():
        raise FileNotFoundError(
            f"libfec_hip.so not found at {p}; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(str(p))
    sig = {
        "fec_encoder_new": (_vp, [_dbl, _u32]),
        "fec_encoder_new_device": (_vp, [_dbl, _u32, _int]),
        "fec_encoder_free": (None, [_vp]),
        "fec_encoder_device": (_int, [_vp]),
        "fec_alloc_slab": (_vp, [_sz]),
        "fec_alloc_slab_numa": (_vp, [_sz, _int]),
        "fec_alloc_repair_buffer": (_vp, [_sz]),
        "fec_free_slab": (None, [_vp]),
        "fec_free_repair_buffer": (None, [_vp]),
        "fec_encode_batch": (_int, [_vp, _vp, _vp, _u32, _u32, _vp]),
        "fec_select_xor_impl": (_vp, []),
        "xor_packets_scalar": (None, [ctypes.POINTER(_vp), _sz, _sz, _vp]),
        "xor_packets_avx2": (None, [ctypes.POINTER(_vp), _sz, _sz, _vp]),
        "xor_packets_avx512": (None, [ctypes.POINTER(_vp), _sz, _sz, _vp]),
        "xor_packets_neon": (None, [ctypes.POINTER(_vp), _sz, _sz, _vp]),
        "fec_hip_device_count": (_int, []),
        "fec_hip_last_error": (ctypes.c_char_p, []),
        "fec_hip_version": (ctypes.c_char_p, []),
        "fec_ctx_last_error": (_sz, [_vp, ctypes.c_char_p, _sz]),
        "fec_parity_matrix": (_int, [_u32, _u32, _vp]),
        "fec_encode_batch_rs": (_int, [_vp, _vp, _vp, _u64, _u32, _u32, _u32, _vp]),
        "fec_decode_batch_rs": (_int, [_vp, _vp, _vp, _vp, _u64, _u32, _u32, _u32, _vp, _vp]),
        "fec_encode_batch_rs_dev": (_int, [_vp, _vp, _u64, _u32, _u32, _u32, _vp, _vp]),
        "fec_decode_batch_rs_dev": (_int, [_vp, _vp, _vp, _vp, _u64, _u32, _u32, _u32, _vp, _vp]),
        "fec_recover_batch_rs_dev": (_int, [_vp, _vp, _vp, _vp, _u64, _u32, _u32, _u32, _vp, _vp, _vp]),
        "fec_decode_prepare": (_int, [_vp, _u32, _u32, ctypes.POINTER(_u64)]),
        "fec_fill_random_dev": (_int, [_vp, _vp, _u64, _u64, _u64, _vp]),
        "fec_copy_dev": (_int, [_vp, _vp, _vp, _u64, _vp]),
        "fec_synchronize": (_int, [_vp]),
        "fec_decode_loss_hint": (_int, [_vp, _dbl]),
        "fec_group_new": (_vp, [ctypes.POINTER(_int), _int]),
        "fec_group_free": (None, [_vp]),
        "fec_group_size": (_int, [_vp]),
        "fec_group_context": (_vp, [_vp, _int]),
        "fec_group_encode_batch_rs": (_int, [_vp, _vp, _u64, _u32, _u32, _u32, _vp]),
        "fec_group_decode_batch_rs": (_int, [_vp, _vp, _vp, _vp, _u64, _u32, _u32, _u32, _vp, _vp]),
        "fec_batcher_new": (_vp, [_int, _u32, _u32, _u32, _u32, _u32, _u32]),
        "fec_batcher_free": (None, [_vp]),
        "fec_batcher_submit": (ctypes.c_int64, [_vp, _vp, _vp, _u32]),
        "fec_batcher_submit_packets": (ctypes.c_int64, [_vp, ctypes.POINTER(_vp), _vp, _u32]),
        "fec_batcher_wait": (_int, [_vp, ctypes.c_int64, _vp, _u32, ctypes.c_int64]),
        "fec_batcher_flush": (_int, [_vp]),
        "fec_batcher_stats": (_int, [_vp, _vp]),
        "fec_batcher_last_error": (ctypes.c_char_p, []),
        "fec_batcher_new_decoder": (_vp, [_int, _u32, _u32, _u32, _u32, _u32, _u32]),
        "fec_batcher_submit_shards": (ctypes.c_int64, [_vp, ctypes.POINTER(_vp), _u32]),
        "fec_batcher_wait_rebuilt": (_int, [_vp, ctypes.c_int64, _vp, _u32, _vp, ctypes.c_int64]),
        "fec_batcher_new_multi": (_vp, [_vp, _int, _u32, _u32, _u32, _u32, _u32, _u32]),
        "fec_batcher_new_decoder_multi": (_vp, [_vp, _int, _u32, _u32, _u32, _u32, _u32, _u32]),
        "fec_batcher_devices": (_int, [_vp]),
        "fec_coalesce_stats": (_int, [_vp, _int]),
        "fec_coalesce_stats_sized": (_int, [_vp, _sz, _int]),
        "fec_recover_batch_rs_dev_packed": (_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, _u32, _u32, _u32, _vp, _vp,
                                                   _vp, _vp, _vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def load_test_library() -> ctypes.CDLL:
    """libfec_hip_test.so (tests only): the product's objects with the test switches live."""
    global _test_lib
    if _test_lib is None:
        _test_lib = load_library(TEST_LIB_PATH)
    return _test_lib


def last_error(lib: Optional[ctypes.CDLL] = None) -> str:
    return ((lib or load_library()).fec_hip_last_error() or b"").decode(errors="replace")


def device_count() -> int:
    return int(load_library().fec_hip_device_count())


def parity_matrix(k: int, r: int) -> np.ndarray:
    out = np.zeros((r, k), dtype=np.uint8)
    rc = load_library().fec_parity_matrix(k, r, out.ctypes.data)
    if rc != FEC_OK:
        raise FecError("fec_parity_matrix", rc)
    return out


def _ptr(a) -> int:
    """Address of a numpy array or torch tensor (device or host)."""
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        if hasattr(a, "is_contiguous") and not a.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return a.data_ptr()
    if isinstance(a, int):
        return a
    raise TypeError(f"unsupported buffer type {type(a)!r}")


def _check(rc: int, what: str, lib: Optional[ctypes.CDLL] = None) -> None:
    if rc != FEC_OK:
        raise FecError(what, rc, last_error(lib))


class Context:
    """An FECEncoderCtx (one per stream of work / per GPU)."""

    def __init__(self, device: Optional[int] = None, redundancy: float = 0.10, max_groups: int = 1024,
                 lib: Optional[ctypes.CDLL] = None):
        """lib: the loaded library to bind (default libfec_hip.so; tests pass load_test_library())."""
        self.lib = lib or load_library()
        if device is None:
            h = self.lib.fec_encoder_new(redundancy, max_groups)
        else:
            h = self.lib.fec_encoder_new_device(redundancy, max_groups, device)
        if not h:
            raise FecError("fec_encoder_new", FEC_ERR_NODEV, last_error(self.lib))
        self.handle = h

    def last_error(self) -> str:
        """Message of the last failing call on this context, from any thread."""
        n = int(self.lib.fec_ctx_last_error(self.handle, None, 0))
        buf = ctypes.create_string_buffer(n + 1)
        self.lib.fec_ctx_last_error(self.handle, buf, n + 1)
        return buf.value.decode(errors="replace")

    @property
    def device(self) -> int:
        return int(self.lib.fec_encoder_device(self.handle))

    def close(self) -> None:
        if getattr(self, "handle", None):
            self.lib.fec_encoder_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- reference ABI ----
    def encode_batch_legacy(self, slab, offsets, num_groups: int, packet_size: int, repair_out) -> int:
        """fec_encode_batch (k fixed to 10).  Returns the C return code."""
        return int(self.lib.fec_encode_batch(self.handle, _ptr(slab) if slab is not None else None,
                                             _ptr(offsets) if offsets is not None else None,
                                             num_groups, packet_size,
                                             _ptr(repair_out) if repair_out is not None else None))

    # ---- batch GF(2^8) API, host or device buffers ----
    def encode(self, data, k: int, r: int, packet_size: int, parity_out, num_groups: Optional[int] = None,
               offsets=None) -> None:
        G = num_groups if num_groups is not None else _nbytes(data) // (k * packet_size)
        rc = self.lib.fec_encode_batch_rs(self.handle, _ptr(data), _ptr(offsets) if offsets is not None else None,
                                          G, k, r, packet_size, _ptr(parity_out))
        _check(rc, "fec_encode_batch_rs", self.lib)

    def decode(self, data, parity, masks, k: int, r: int, packet_size: int, status_out=None,
               num_groups: Optional[int] = None) -> int:
        G = num_groups if num_groups is not None else _nbytes(masks) // 8
        bad = ctypes.c_uint64(0)
        rc = self.lib.fec_decode_batch_rs(self.handle, _ptr(data), _ptr(parity), _ptr(masks), G, k, r,
                                          packet_size, _ptr(status_out) if status_out is not None else None,
                                          ctypes.byref(bad))
        _check(rc, "fec_decode_batch_rs", self.lib)
        return int(bad.value)

    # ---- device-resident API ----
    def encode_dev(self, d_data, num_groups: int, k: int, r: int, packet_size: int, d_parity,
                   stream: Optional[int] = None) -> None:
        rc = self.lib.fec_encode_batch_rs_dev(self.handle, _ptr(d_data), num_groups, k, r, packet_size,
                                              _ptr(d_parity), stream)
        _check(rc, "fec_encode_batch_rs_dev", self.lib)

    def decode_dev(self, d_data, d_parity, d_masks, num_groups: int, k: int, r: int, packet_size: int,
                   d_status=None, stream: Optional[int] = None) -> None:
        rc = self.lib.fec_decode_batch_rs_dev(self.handle, _ptr(d_data), _ptr(d_parity), _ptr(d_masks),
                                              num_groups, k, r, packet_size,
                                              _ptr(d_status) if d_status is not None else None, stream)
        _check(rc, "fec_decode_batch_rs_dev", self.lib)

    def recover_dev(self, d_data, d_parity, d_masks, num_groups: int, k: int, r: int, packet_size: int,
                    d_rebuilt, d_status=None, stream: Optional[int] = None) -> None:
        """Rebuilt shards of group g at d_rebuilt[(g*r + m)*P:...], m over the lost data shards
        in ascending order; d_data is not modified."""
        rc = self.lib.fec_recover_batch_rs_dev(self.handle, _ptr(d_data), _ptr(d_parity), _ptr(d_masks),
                                               num_groups, k, r, packet_size, _ptr(d_rebuilt),
                                               _ptr(d_status) if d_status is not None else None, stream)
        _check(rc, "fec_recover_batch_rs_dev", self.lib)

    def recover_packed_dev(self, d_data, d_parity, d_masks, num_groups: int, k: int, r: int, packet_size: int,
                           d_rebuilt, d_row_start, d_total=None, d_status=None, stream: Optional[int] = None) -> None:
        """Rebuilt shards of all groups back to back: group g's m-th lost data shard at row
        d_row_start[g] + m of d_rebuilt (u32 row starts written by the call); d_total (one u64,
        nullable) = all rows.  Mask-addressed shapes only."""
        rc = self.lib.fec_recover_batch_rs_dev_packed(self.handle, _ptr(d_data), _ptr(d_parity), _ptr(d_masks),
                                                      num_groups, k, r, packet_size, _ptr(d_rebuilt),
                                                      _ptr(d_row_start),
                                                      _ptr(d_total) if d_total is not None else None,
                                                      _ptr(d_status) if d_status is not None else None, stream)
        _check(rc, "fec_recover_batch_rs_dev_packed", self.lib)

    def decode_prepare(self, k: int, r: int) -> int:
        n = ctypes.c_uint64(0)
        _check(self.lib.fec_decode_prepare(self.handle, k, r, ctypes.byref(n)), "fec_decode_prepare", self.lib)
        return int(n.value)

    def copy_dev(self, d_src, d_dst, nbytes: int, stream=None) -> None:
        """d_dst <- d_src (box HBM copy calibration; nbytes a multiple of 16)."""
        _check(self.lib.fec_copy_dev(self.handle, _ptr(d_src), _ptr(d_dst), nbytes, stream),
               "fec_copy_dev", self.lib)

    def fill_random_dev(self, d_dst, nbytes: int, seed: int, byte_offset: int = 0,
                        stream: Optional[int] = None) -> None:
        _check(self.lib.fec_fill_random_dev(self.handle, _ptr(d_dst), nbytes, seed, byte_offset, stream),
               "fec_fill_random_dev", self.lib)

    def decode_loss_hint(self, share: float) -> None:
        """Expected share of groups with lost data in device-resident decodes (< 0: unknown)."""
        _check(self.lib.fec_decode_loss_hint(self.handle, share), "fec_decode_loss_hint", self.lib)

    def synchronize(self) -> None:
        _check(self.lib.fec_synchronize(self.handle), "fec_synchronize", self.lib)


class DeviceGroup:
    """An FECDeviceGroup: host batches sharded over several GPUs (one context and host
    thread per shard, contiguous group ranges, no data moved between devices)."""

    def __init__(self, devices=None):
        self.lib = load_library()
        if devices is None:
            h = self.lib.fec_group_new(None, 0)
        else:
            arr = (_int * max(1, len(devices)))(*devices)
            h = self.lib.fec_group_new(arr, len(devices))
        if not h:
            raise FecError("fec_group_new", FEC_ERR_NODEV, last_error())
        self.handle = h

    def __len__(self) -> int:
        return int(self.lib.fec_group_size(self.handle))

    def close(self) -> None:
        if getattr(self, "handle", None):
            self.lib.fec_group_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def encode(self, data, k: int, r: int, packet_size: int, parity_out, num_groups: Optional[int] = None) -> None:
        G = num_groups if num_groups is not None else _nbytes(data) // (k * packet_size)
        _check(self.lib.fec_group_encode_batch_rs(self.handle, _ptr(data), G, k, r, packet_size, _ptr(parity_out)),
               "fec_group_encode_batch_rs")

    def decode(self, data, parity, masks, k: int, r: int, packet_size: int, status_out=None,
               num_groups: Optional[int] = None) -> int:
        G = num_groups if num_groups is not None else _nbytes(masks) // 8
        bad = ctypes.c_uint64(0)
        rc = self.lib.fec_group_decode_batch_rs(self.handle, _ptr(data), _ptr(parity), _ptr(masks), G, k, r,
                                                packet_size, _ptr(status_out) if status_out is not None else None,
                                                ctypes.byref(bad))
        _check(rc, "fec_group_decode_batch_rs")
        return int(bad.value)


class Batcher:
    """An FECBatcher: one batch for the groups of many streams, encoded when max_groups are
    pending or deadline_us after the oldest pending group (include/fec_hip.h)."""

    STATS = ("groups", "batches", "full_flushes", "deadline_flushes", "max_batch", "expired")

    def __init__(self, k: int, r: int, slot_bytes: int = 1500, max_groups: int = 4096, deadline_us: int = 1000,
                 device: int = -1, slabs: int = 3, devices=None):
        """devices: a list of GPU ordinals (repeats allowed) for one batcher per device behind
        this handle (fec_batcher_new_multi); None: the single `device`."""
        self.lib = load_library()
        self.k, self.r, self.slot = k, r, slot_bytes
        self.handle = self._create(False, device, devices, k, r, slot_bytes, max_groups, deadline_us, slabs)

    def _create(self, decoder, device, devices, *shape):
        if devices is None:
            fn = "fec_batcher_new_decoder" if decoder else "fec_batcher_new"
            h = getattr(self.lib, fn)(device, *shape)
        else:
            fn = "fec_batcher_new_decoder_multi" if decoder else "fec_batcher_new_multi"
            devs = np.ascontiguousarray(devices, dtype=np.int32)
            h = getattr(self.lib, fn)(devs.ctypes.data if devs.size else None, int(devs.size), *shape)
        if not h:
            raise FecError(fn, FEC_ERR_NODEV, self.last_error())
        return h

    def devices(self) -> int:
        """GPUs behind this handle."""
        return int(self.lib.fec_batcher_devices(self.handle))

    def last_error(self) -> str:
        return (self.lib.fec_batcher_last_error() or b"").decode(errors="replace")

    def submit(self, packets) -> int:
        """One group (1..k packets, any lengths <= slot); returns its ticket."""
        n = len(packets)
        lens = np.array([len(p) for p in packets], dtype=np.uint32)
        ptrs = (_vp * max(1, n))(*[_ptr(p) for p in packets])
        t = int(self.lib.fec_batcher_submit_packets(self.handle, ptrs, lens.ctypes.data, n))
        if t < 0:
            raise FecError("fec_batcher_submit_packets", t, self.last_error())
        return t

    def submit_packed(self, packed: np.ndarray, lens) -> int:
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        t = int(self.lib.fec_batcher_submit(self.handle, _ptr(packed), lens.ctypes.data, len(lens)))
        if t < 0:
            raise FecError("fec_batcher_submit", t, self.last_error())
        return t

    def wait(self, ticket: int, timeout_us: int = -1):
        """The group's r repair payloads (a list of arrays), or None when not ready in time."""
        out = np.zeros(self.r * self.slot, dtype=np.uint8)
        n = int(self.lib.fec_batcher_wait(self.handle, ticket, out.ctypes.data, self.slot, timeout_us))
        if n == FEC_ERR_AGAIN:
            return None
        if n < 0:
            raise FecError("fec_batcher_wait", n, self.last_error())
        return [out[i * self.slot:i * self.slot + n].copy() for i in range(self.r)]

    def flush(self) -> None:
        _check(self.lib.fec_batcher_flush(self.handle), "fec_batcher_flush")

    def stats(self) -> dict:
        st = np.zeros(len(self.STATS), dtype=np.uint64)
        _check(self.lib.fec_batcher_stats(self.handle, st.ctypes.data), "fec_batcher_stats")
        return dict(zip(self.STATS, (int(x) for x in st)))

    def close(self) -> None:
        if getattr(self, "handle", None):
            self.lib.fec_batcher_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class DecodeBatcher(Batcher):
    """A decoder FECBatcher: the groups of many connections recovered in one launch
    (fec_batcher_new_decoder, include/fec_hip.h)."""

    def __init__(self, k: int, r: int, slot_bytes: int = 1500, max_groups: int = 4096, deadline_us: int = 1000,
                 device: int = -1, slabs: int = 3, devices=None):
        self.lib = load_library()
        self.k, self.r, self.slot = k, r, slot_bytes
        self.handle = self._create(True, device, devices, k, r, slot_bytes, max_groups, deadline_us, slabs)
        self._lens = {}

    def submit(self, shards, length: int) -> int:
        """k + r shards (data, then parity rows; None = lost), each at most `length` bytes."""
        if len(shards) != self.k + self.r:
            raise ValueError(f"expected {self.k + self.r} shards")
        keep = [np.ascontiguousarray(x, dtype=np.uint8) if x is not None else None for x in shards]
        for x in keep:
            if x is not None and x.nbytes < length:
                raise ValueError("shard shorter than the symbol length")
        ptrs = (_vp * len(keep))(*[(x.ctypes.data if x is not None else None) for x in keep])
        t = int(self.lib.fec_batcher_submit_shards(self.handle, ptrs, length))
        if t < 0:
            raise FecError("fec_batcher_submit_shards", t, self.last_error())
        self._lens[t] = length
        return t

    def wait(self, ticket: int, timeout_us: int = -1):
        """(lost data shard ids, their rebuilt bytes), or None when not ready in time; raises
        FecError(FEC_ERR_UNRECOVERABLE) when too many shards were lost."""
        out = np.zeros(self.r * self.slot, dtype=np.uint8)
        mask = np.zeros(1, dtype=np.uint64)
        n = int(self.lib.fec_batcher_wait_rebuilt(self.handle, ticket, out.ctypes.data, self.slot, mask.ctypes.data,
                                                  timeout_us))
        if n == FEC_ERR_AGAIN:
            return None
        length = getattr(self, "_lens", {}).pop(ticket, self.slot)
        if n < 0:
            raise FecError("fec_batcher_wait_rebuilt", n, self.last_error())
        m = int(mask[0])
        lost = [j for j in range(self.k) if (m >> j) & 1]
        assert len(lost) == n
        return lost, [out[i * self.slot:i * self.slot + length].copy() for i in range(n)]


def _nbytes(a) -> int:
    if isinstance(a, np.ndarray):
        return a.nbytes
    if hasattr(a, "numel"):
        return a.numel() * a.element_size()
    raise TypeError("pass num_groups explicitly for raw pointers")


def xor_packets(packets, packet_size: int, repair, variant: str = "avx2") -> None:
    """Call one of the ABI-compat xor_packets_* entry points (GPU-backed)."""
    lib = load_library()
    arr = (_vp * max(1, len(packets)))(*[_ptr(p) for p in packets])
    getattr(lib, f"xor_packets_{variant}")(arr, len(packets), packet_size, _ptr(repair))


COALESCE_STATS = ("calls", "groups", "batches", "max_batch", "max_calls", "close_ns", "launch_ns", "done_ns", "resident_calls", "resident_launches",
                  "resident_pre_ns", "resident_wait_ns", "resident_post_ns", "resident_inline", "resident_vram",
                  "resident_bad_slots", "resident_scrubs", "resident_servers")


def coalesce_stats(reset: bool = False) -> dict:
    """Process-wide totals of the legacy-call coalescer (fec_coalesce_stats)."""
    lib = load_library()
    st = np.zeros(len(COALESCE_STATS), dtype=np.uint64)
    _check(lib.fec_coalesce_stats_sized(st.ctypes.data, st.nbytes, 1 if reset else 0), "fec_coalesce_stats_sized")
    return dict(zip(COALESCE_STATS, (int(x) for x in st)))
