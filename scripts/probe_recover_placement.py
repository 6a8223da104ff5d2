#!/usr/bin/env python3
"""Probe: does the C3 recover's time depend on where its buffers sit in HBM?

One process: data (1M groups of k=10 x 1200 B) and parity are made once; the slot-row recover
(fec_recover_batch_rs_dev) is then timed into several freshly allocated rebuilt buffers, with
a fresh copy of the data, and with fresh parity, each 10 times on one stream (HIP events).  If
the time moves between allocations inside one process, placement decides it; if it stays put
here but differs between processes or boxes, it does not.  One JSON line per measurement.

    python scripts/probe_recover_placement.py [--trials 4]
"""
import argparse
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "quic-test_amd"))

import bench  # noqa: E402  (erasure_masks)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--block-orders", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch
    import quicfec

    G, k, r, P = 1_000_000, 10, 3, 1200
    ctx = quicfec.Context(device=0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    data = torch.empty(G * k * P, dtype=torch.uint8, device="cuda")
    parity = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
    ctx.fill_random_dev(data, data.numel(), 0x5EED0002, stream=sp)
    ctx.encode_dev(data, G, k, r, P, parity, stream=sp)
    masks = torch.from_numpy(bench.erasure_masks(G, k + r, 2, 0x5EED0003).view(np.int64)).to("cuda")
    ctx.decode_prepare(k, r)
    row_start = torch.empty(G, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()

    def timed(d, p, rb):
        ctx.recover_dev(d, p, masks, G, k, r, P, rb, None, stream=sp)  # warm
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(args.reps):
            ctx.recover_dev(d, p, masks, G, k, r, P, rb, None, stream=sp)
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / args.reps

    def out(kind, ms, **addrs):
        print(json.dumps({"kind": kind, "ms": round(ms, 4), **{n: hex(t.data_ptr()) for n, t in addrs.items()}}),
              flush=True)

    def timed_fn(fn):
        fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(args.reps):
            fn()
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / args.reps

    rbs = []
    for t in range(args.trials):
        rb = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
        rbs.append(rb)
        out("rebuilt", timed(data, parity, rb), data=data, parity=parity, rebuilt=rb)
        # the packed rows (no gaps between groups' rows) into the same buffer
        out("packed", timed_fn(lambda: ctx.recover_packed_dev(data, parity, masks, G, k, r, P, rb, row_start,
                                                              None, None, stream=sp)), rebuilt=rb)
        if args.block_orders:
            for swz in ("0", "2", "3"):   # QUICFEC_DECODE_SWIZZLE is read at every launch
                os.environ["QUICFEC_DECODE_SWIZZLE"] = swz
                out(f"rebuilt_swz{swz}", timed(data, parity, rb), rebuilt=rb)
            os.environ.pop("QUICFEC_DECODE_SWIZZLE", None)
        # the same buffer under a pure write (fill) and a copy from parity (read one, write one)
        out("fill_rebuilt", timed_fn(lambda: ctx.fill_random_dev(rb, rb.numel(), 7, stream=sp)), rebuilt=rb)
        out("copy_parity_to_rebuilt", timed_fn(lambda: ctx.copy_dev(parity, rb, rb.numel(), stream=sp)), rebuilt=rb)
    # rebuilt buffers straight from the HIP runtime torch loaded: plain hipMalloc and
    # hipExtMallocWithFlags(hipDeviceMallocContiguous = 0x4), physically contiguous
    import ctypes
    hip_path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    hip = ctypes.CDLL(hip_path)
    raw = []
    for kind, flags in (("hipMalloc", None), ("contiguous", 0x4), ("hipMalloc", None), ("contiguous", 0x4)):
        pp = ctypes.c_void_p()
        nb = ctypes.c_size_t(G * r * P)
        rc = hip.hipMalloc(ctypes.byref(pp), nb) if flags is None else \
            hip.hipExtMallocWithFlags(ctypes.byref(pp), nb, ctypes.c_uint(flags))
        if rc != 0:
            print(json.dumps({"kind": kind, "error": rc}), flush=True)
            continue
        raw.append(pp.value)
        out(f"raw_{kind}", timed(data, parity, pp.value), rebuilt=torch.empty(0))
        print(json.dumps({"kind": f"raw_{kind}_addr", "rebuilt": hex(pp.value)}), flush=True)
    torch.cuda.synchronize()
    for pv in raw:
        hip.hipFree(ctypes.c_void_p(pv))
    for t in range(2):
        d2 = data.clone()
        out("data_copy", timed(d2, parity, rbs[0]), data=d2, parity=parity, rebuilt=rbs[0])
        del d2
    p2 = parity.clone()
    out("parity_copy", timed(data, p2, rbs[0]), data=data, parity=p2, rebuilt=rbs[0])
    out("again", timed(data, parity, rbs[0]), data=data, parity=parity, rebuilt=rbs[0])
    ctx.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
