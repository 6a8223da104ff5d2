"""Workgroup shape of the staged encodes (groups per workgroup x workgroups per CU), swept in one
process with interleaved rounds: QUICFEC_ENCODE_TILE / QUICFEC_ENCODE_BLOCKS / QUICFEC_ENCODE_WAVES
are read at every launch.  The tile and occupancy were tuned before the parity rows were staged
through LDS (4 groups x 2 workgroups for k=10 r=3); a workgroup's store burst is now
its whole tile * R * P window, so the best shape may have moved.  Every shape's parity must equal
the default's.  One JSON line per (config, shape).

  python scripts/sweep_encode_tiles.py [--rounds 3] [--reps 10] [--configs c2,c4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "quic-test_amd"))
import quicfec  # noqa: E402

CONFIGS = {"c2": (10, 3, 1200, 1_000_000), "c4": (20, 5, 1200, 1_000_000),
           "c2pol": (10, 3, 1200, 1_000_000), "c4pol": (20, 5, 1200, 1_000_000)}
# (tile, env var for occupancy, value); None = the library's default
SHAPES = {
    "c2pol": [(None, None, None), (None, "QUICFEC_ENCODE_MEMPOL", 1), (None, "QUICFEC_ENCODE_MEMPOL", 2),
              (None, "QUICFEC_ENCODE_MEMPOL", 3)],
    "c4pol": [(None, None, None), (None, "QUICFEC_ENCODE_MEMPOL", 1), (None, "QUICFEC_ENCODE_MEMPOL", 2),
              (None, "QUICFEC_ENCODE_MEMPOL", 3)],
    "c2": [(None, None, None), (4, "QUICFEC_ENCODE_BLOCKS", 2), (4, "QUICFEC_ENCODE_BLOCKS", 3), (5, "QUICFEC_ENCODE_BLOCKS", 2),
           (6, "QUICFEC_ENCODE_BLOCKS", 2), (6, "QUICFEC_ENCODE_BLOCKS", 1), (3, "QUICFEC_ENCODE_BLOCKS", 3),
           (2, "QUICFEC_ENCODE_BLOCKS", 4), (3, "QUICFEC_ENCODE_BLOCKS", 2)],
    "c4": [(None, None, None), (2, "QUICFEC_ENCODE_WAVES", 0), (3, "QUICFEC_ENCODE_WAVES", 0), (5, "QUICFEC_ENCODE_WAVES", 0),
           (6, "QUICFEC_ENCODE_WAVES", 0), (4, "QUICFEC_ENCODE_WAVES", 10), (4, "QUICFEC_ENCODE_WAVES", 15),
           (4, "QUICFEC_ENCODE_WAVES", 8), (4, "QUICFEC_ENCODE_WAVES", 12), (5, "QUICFEC_ENCODE_WAVES", 10),
           (3, "QUICFEC_ENCODE_WAVES", 9), (5, "QUICFEC_ENCODE_WAVES", 12)],
}
KNOBS = ("QUICFEC_ENCODE_TILE", "QUICFEC_ENCODE_BLOCKS", "QUICFEC_ENCODE_WAVES", "QUICFEC_ENCODE_MEMPOL")


def set_shape(shape) -> str:
    for k in KNOBS:
        os.environ.pop(k, None)
    tile, var, val = shape
    if var is None:
        return "default"
    if tile is not None:
        os.environ["QUICFEC_ENCODE_TILE"] = str(tile)
    os.environ[var] = str(val)
    return (f"tile {tile} " if tile is not None else "") + f"{var.split('_')[-1].lower()} {val}"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--configs", default="c2,c4")
    args = ap.parse_args()
    stream = torch.cuda.Stream()
    with quicfec.Context(device=0) as ctx, torch.cuda.stream(stream):
        for name in args.configs.split(","):
            k, r, P, G = CONFIGS[name]
            data = torch.empty(G * k * P, dtype=torch.uint8, device="cuda")
            ctx.fill_random_dev(data, data.numel(), 0x5EED0000 + k, stream=stream.cuda_stream)
            ref = torch.empty(G * r * P, dtype=torch.uint8, device="cuda")
            par = torch.empty_like(ref)
            set_shape((None, None, None))
            ctx.encode_dev(data, G, k, r, P, ref, stream=stream.cuda_stream)
            ms = {i: [] for i in range(len(SHAPES[name]))}
            same = {i: True for i in ms}
            for rd in range(args.rounds):
                order = list(ms) if rd % 2 == 0 else list(ms)[::-1]
                for i in order:
                    set_shape(SHAPES[name][i])
                    par.fill_(0)
                    ctx.encode_dev(data, G, k, r, P, par, stream=stream.cuda_stream)
                    stream.synchronize()
                    same[i] = same[i] and bool(torch.equal(par, ref))
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.reps):
                        ctx.encode_dev(data, G, k, r, P, par, stream=stream.cuda_stream)
                    e1.record(stream)
                    e1.synchronize()
                    ms[i].append(e0.elapsed_time(e1) / args.reps)
            for i, v in ms.items():
                med = sorted(v)[len(v) // 2]
                print(json.dumps({"config": name, "shape": set_shape(SHAPES[name][i]), "identical": same[i],
                                  "ms": [round(x, 4) for x in v], "median_ms": round(med, 4),
                                  "TBps": round(G * (k + r) * P / med / 1e9, 3)}), flush=True)
            set_shape((None, None, None))
            del data, ref, par
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
