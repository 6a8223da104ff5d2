"""A/B of the encodes' LDS-staged parity rows (kStageRows, QUICFEC_ENCODE_STAGE) in one process.

For C2 (k=10 r=3, encode_v16) and C4 (k=20 r=5, encode_bits), 1M groups of 1200 B each: the same
device-resident data encoded with staging off and on, alternating over rounds on one stream, each
round `reps` back-to-back launches timed by HIP events on that stream.  The two parity buffers
must be byte-identical (the staged form changes where bytes are stored from, never their value).
Prints one JSON line per config.  VERDICT r04 item 3.

  python scripts/ab_stage_rows.py [--rounds 6] [--reps 10] [--configs c2,c4]
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

CONFIGS = {"c2": (10, 3, 1200, 1 << 20), "c4": (20, 5, 1200, 1 << 20), "k10r1": (10, 1, 1200, 1 << 20),
           "k10r2": (10, 2, 1200, 1 << 20), "k4r2": (4, 2, 1200, 1 << 20)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--configs", default="c2,c4")
    args = ap.parse_args()
    stream = torch.cuda.Stream()
    with quicfec.Context(device=0) as ctx, torch.cuda.stream(stream):
        for name in args.configs.split(","):
            k, r, P, G = CONFIGS[name]
            data = torch.empty(G * k * P, dtype=torch.uint8, device="cuda")
            ctx.fill_random_dev(data, data.numel(), 0x5EED0000 + k, stream=stream.cuda_stream)
            par = {m: torch.empty(G * r * P, dtype=torch.uint8, device="cuda") for m in (0, 1)}
            for m in (0, 1):
                os.environ["QUICFEC_ENCODE_STAGE"] = str(m)
                ctx.encode_dev(data, G, k, r, P, par[m], stream=stream.cuda_stream)
            stream.synchronize()
            same = bool(torch.equal(par[0], par[1]))
            ms = {0: [], 1: []}
            for rd in range(args.rounds):
                for m in ((0, 1) if rd % 2 == 0 else (1, 0)):
                    os.environ["QUICFEC_ENCODE_STAGE"] = str(m)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.reps):
                        ctx.encode_dev(data, G, k, r, P, par[m], stream=stream.cuda_stream)
                    e1.record(stream)
                    e1.synchronize()
                    ms[m].append(e0.elapsed_time(e1) / args.reps)
            alg = G * (k + r) * P
            best = {m: min(v) for m, v in ms.items()}
            med = {m: sorted(v)[len(v) // 2] for m, v in ms.items()}
            print(json.dumps({"config": name, "k": k, "r": r, "P": P, "groups": G, "identical": same,
                              "ms_off": [round(x, 4) for x in ms[0]], "ms_on": [round(x, 4) for x in ms[1]],
                              "median_off": round(med[0], 4), "median_on": round(med[1], 4),
                              "TBps_off": round(alg / med[0] / 1e9, 3), "TBps_on": round(alg / med[1] / 1e9, 3),
                              "on_vs_off": round(med[1] / med[0], 4)}), flush=True)
            del data, par
            torch.cuda.empty_cache()
    os.environ.pop("QUICFEC_ENCODE_STAGE", None)


if __name__ == "__main__":
    main()
