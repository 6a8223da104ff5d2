#!/usr/bin/env python3
"""Per-kernel medians of any rocprofv3 --pmc counters.

    python scripts/pmc_generic.py <out.json> <dir> [<dir> ...]

Reads every *counter_collection.csv under the given pass directories and writes, per kernel
(name truncated), the median over its dispatches of each counter (summed over the dimensions
rocprofv3 reports, e.g. XCDs / shader engines, within one dispatch).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def main():
    out = Path(sys.argv[1])
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> value
    for d in sys.argv[2:]:
        for f in Path(d).rglob("*counter_collection.csv"):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")[:120]
                    disp = row.get("Dispatch_Id") or row.get("Correlation_Id") or "0"
                    per[name][row["Counter_Name"]][(str(f), disp)] += float(row["Counter_Value"])
    res = {}
    for name, counters in per.items():
        e = {}
        for c, vals in counters.items():
            v = sorted(vals.values())
            e[c] = {"median": v[len(v) // 2], "dispatches": len(v)}
        res[name] = e
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
