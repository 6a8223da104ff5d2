#!/usr/bin/env python3
"""Probe: is the C3 recover's placement sensitivity the distance between its
parity rows and its rebuilt rows?

The slot-row recover (fec_recover_batch_rs_dev) reads group g's parity rows at parity + g*3*P and
writes its rebuilt rows at rebuilt + g*3*P: the same stride, so the two streams stay a constant
distance D = rebuilt - parity apart for the whole launch (the data stream, 10*P per group, does
not).  If D decides which HBM channels / banks the concurrent reads and writes meet in, the rate
must move with D.  Here parity and rebuilt live in ONE allocation (physically contiguous when
hipExtMallocWithFlags(hipDeviceMallocContiguous) gives one, so D is a physical distance too), and
the recover is timed with the rebuilt rows at D = span + delta for a sweep of delta.  One JSON line
per point; the sweep runs twice (second time reversed).

    python scripts/probe_recover_delta.py [--alloc contiguous|torch] [--reps 5]
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "quic-test_amd"))

import bench  # noqa: E402  (erasure_masks)

MB = 1 << 20
DELTAS = [0, 4096, 65536, 256 * 1024, 1 * MB, 2 * MB, 3 * MB, 4 * MB, 6 * MB, 8 * MB, 12 * MB, 16 * MB, 24 * MB,
          32 * MB, 48 * MB, 64 * MB, 96 * MB, 128 * MB, 192 * MB, 256 * MB]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--alloc", default="contiguous")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--groups", type=int, default=1_000_000)
    args = ap.parse_args()
    import numpy as np
    import torch
    import quicfec

    G, k, r, P = args.groups, 10, 3, 1200
    ctx = quicfec.Context(device=0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    data = torch.empty(G * k * P, dtype=torch.uint8, device="cuda")
    ctx.fill_random_dev(data, data.numel(), 0x5EED0002, stream=sp)
    span = (G * r * P + 2 * MB - 1) // (2 * MB) * (2 * MB)
    total = 2 * span + max(DELTAS) + 2 * MB
    hip_path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    hip = ctypes.CDLL(hip_path)
    base, keep = None, None
    if args.alloc == "contiguous":
        pp = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(pp), ctypes.c_size_t(total), ctypes.c_uint(0x4))
        if rc == 0:
            base = pp.value
        else:
            print(json.dumps({"alloc": "contiguous", "error": rc, "fallback": "torch"}), flush=True)
    if base is None:
        keep = torch.empty(total, dtype=torch.uint8, device="cuda")
        base = keep.data_ptr()
    parity = base
    ctx.encode_dev(data, G, k, r, P, parity, stream=sp)
    masks = torch.from_numpy(bench.erasure_masks(G, k + r, 2, 0x5EED0003).view(np.int64)).to("cuda")
    ctx.decode_prepare(k, r)
    torch.cuda.synchronize()

    def timed(rb):
        ctx.recover_dev(data, parity, masks, G, k, r, P, rb, None, stream=sp)  # warm
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(args.reps):
            ctx.recover_dev(data, parity, masks, G, k, r, P, rb, None, stream=sp)
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / args.reps

    for sweep in range(2):
        for d in (DELTAS if sweep == 0 else DELTAS[::-1]):
            rb = base + span + d
            ms = timed(rb)
            print(json.dumps({"alloc": args.alloc, "sweep": sweep, "delta": d, "D": span + d, "ms": round(ms, 4),
                              "parity": hex(parity), "rebuilt": hex(rb), "data": hex(data.data_ptr())}), flush=True)
    # one reference point: the rebuilt rows in a buffer of their own
    rb2 = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
    print(json.dumps({"alloc": "separate_torch", "ms": round(timed(rb2.data_ptr()), 4), "rebuilt": hex(rb2.data_ptr())}),
          flush=True)
    torch.cuda.synchronize()
    if keep is None:
        hip.hipFree(ctypes.c_void_p(base))
    ctx.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
