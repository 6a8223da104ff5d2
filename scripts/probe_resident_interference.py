#!/usr/bin/env python3
"""Probe: does the resident legacy encoder (a persistent one-workgroup kernel, fec_coalesce.cpp)
delay other work the same process launches on its own streams while it is alive?

A background thread keeps the resident encoder busy with the reference's call pattern (one
group per fec_encode_batch call from a page-locked slab) for the measuring window; the main
thread meanwhile launches a small device-resident encode (1,000 groups of k=10 r=3) on each of
eight torch streams in turn and times launch -> completion on the host.  The same loop runs
again with the background idle (after the resident instance has left).  One JSON line each.
"""
import ctypes
import json
import sys
import threading
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "quic-test_amd"))


def main() -> int:
    import numpy as np
    import torch
    import quicfec

    lib = quicfec.load_library()
    ctx = quicfec.Context(device=0)
    bg = quicfec.Context(device=0)
    G, k, r, P = 1000, 10, 3, 1200
    data = torch.randint(0, 256, (G * k * P,), dtype=torch.uint8, device="cuda")
    par = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(8)]
    slab = lib.fec_alloc_slab(10 * P)
    rep = lib.fec_alloc_repair_buffer(P)
    offs = (np.arange(10, dtype=np.uint32) * P).astype(np.uint32)
    stop = threading.Event()
    calls = [0]

    def background():
        while not stop.is_set():
            assert lib.fec_encode_batch(bg.handle, slab, offs.ctypes.data, 1, P, rep) == 0
            calls[0] += 1

    def window(label: str, seconds: float = 1.0):
        lat = []
        t_end = time.perf_counter() + seconds
        i = 0
        while time.perf_counter() < t_end:
            s = streams[i % len(streams)]
            t0 = time.perf_counter()
            ctx.encode_dev(data, G, k, r, P, par, stream=s.cuda_stream)
            s.synchronize()
            lat.append((time.perf_counter() - t0) * 1e6)
            i += 1
            time.sleep(0.002)
        lat.sort()
        print(json.dumps({"window": label, "launches": len(lat), "p50_us": round(lat[len(lat) // 2], 1),
                          "p99_us": round(lat[int(len(lat) * 0.99)], 1), "max_us": round(lat[-1], 1),
                          "background_calls": calls[0]}), flush=True)

    # the null stream too: a blocking stream the runtime orders against every blocking stream
    def null_window(label):
        lat = []
        for _ in range(100):
            t0 = time.perf_counter()
            ctx.encode_dev(data, G, k, r, P, par, stream=0)
            ctx.synchronize()
            lat.append((time.perf_counter() - t0) * 1e6)
            time.sleep(0.002)
        lat.sort()
        print(json.dumps({"window": label + ", null stream", "p50_us": round(lat[50], 1), "max_us": round(lat[-1], 1)}),
              flush=True)

    window("warm, resident idle")
    th = threading.Thread(target=background)
    th.start()
    time.sleep(0.05)
    c0 = calls[0]
    window("resident serving legacy calls")
    null_window("resident serving legacy calls")
    stop.set()
    th.join()
    print(json.dumps({"background_calls_per_s": round((calls[0] - c0) / 1.0)}), flush=True)
    time.sleep(0.1)  # the instance leaves after its idle bound
    window("after, resident idle")
    lib.fec_free_slab(slab)
    lib.fec_free_repair_buffer(rep)
    bg.close()
    ctx.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
