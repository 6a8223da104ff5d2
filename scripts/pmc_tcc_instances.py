#!/usr/bin/env python3
"""Per-TCC-channel counters for rocprofv3.

rocprofv3's CSV sums a counter over its dimensions (16 TCC instances x 8 XCDs on gfx950) within a
dispatch.  This writes a counter definition file -- the installed counter_defs.yaml plus derived
counters <BASE>_I<n> = reduce(select(<BASE>, [DIMENSION_INSTANCE=[n]]), sum): instance n summed over
the XCDs -- for rocprofv3 to load through ROCPROFILER_METRICS_PATH, and summarises a run's CSV per
dispatch.

    python scripts/pmc_tcc_instances.py defs <out_dir> BASE [BASE ...]
        -> <out_dir>/counter_defs.yaml; prints the passes: 4 instances of one base per line
    python scripts/pmc_tcc_instances.py summary <counter_collection.csv> [--kernel decode_fused]
        -> one JSON line per dispatch of the kernel: duration and per-instance values per base
"""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

DEFAULTS = Path("/opt/rocm/share/rocprofiler-sdk/counter_defs.yaml")
INSTANCES = 16


def defs(out_dir: str, bases: list[str]) -> None:
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    text = DEFAULTS.read_text().rstrip("\n") + "\n"
    for b in bases:
        for i in range(INSTANCES):
            text += (f"  - name: {b}_I{i}\n"
                     f"    description: {b} of TCC instance {i}, summed over XCDs.\n"
                     f"    properties: []\n"
                     f"    definitions:\n"
                     f"    - architectures:\n"
                     f"      - gfx950\n"
                     f"      expression: reduce(select({b},[DIMENSION_INSTANCE=[{i}]]),sum)\n")
    (out / "counter_defs.yaml").write_text(text)
    # one pass per line: at most 4 TCC counters a pass (the per-block limit), so 4 instances
    for b in bases:
        for i0 in range(0, INSTANCES, 4):
            print(" ".join(f"{b}_I{i}" for i in range(i0, i0 + 4)))


def summary(path: str, kernel: str) -> None:
    per = defaultdict(lambda: {"values": {}})
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"]:
            continue
        d = per[int(r["Dispatch_Id"])]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d["kernel"] = r["Kernel_Name"][r["Kernel_Name"].find(kernel):][:60]
        d["values"][r["Counter_Name"]] = float(r["Counter_Value"])
    for did in sorted(per):
        d = per[did]
        bases = defaultdict(lambda: [0.0] * INSTANCES)
        for name, v in d["values"].items():
            m = re.fullmatch(r"(.+)_I(\d+)", name)
            if m:
                bases[m.group(1)][int(m.group(2))] = v
        other = {n: v for n, v in d["values"].items() if not re.fullmatch(r"(.+)_I(\d+)", n)}
        print(json.dumps({"dispatch": did, "kernel": d["kernel"], "ms": round(d["ns"] / 1e6, 4),
                          **{b: v for b, v in bases.items()}, **other}))


if __name__ == "__main__":
    if sys.argv[1] == "defs":
        defs(sys.argv[2], sys.argv[3:])
    else:
        kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "decode_fused"
        summary(sys.argv[2], kern)
