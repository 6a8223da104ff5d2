#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

    python scripts/pmc_summary.py <fetch_dir> <write_dir> <config> [out.json] [--tag NAME]

--tag NAME: the run timed one decode API only (bench.py --decode-api X --no-other-api), so its
recover kernel is stored as "recover_NAME" (packed / slots) and merged into an existing out.json
of the same build and workload, which then holds one entry per API.

The profiled bench's own JSON line (<fetch_dir>.json, as scripts/gpu_pmc.sh writes it) names the
workload the counters were taken on; it is recorded as "workload" (bench.py workload_of_line),
and bench.py uses the bytes only for a run of that exact workload (and library build).

Corrections (MI355X_MICROARCH.md §HBM and cdna_hip_programming.md §7):
  * FETCH_SIZE / WRITE_SIZE are in KiB;
  * on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide coalesced streaming
    read (16 B/lane global loads), so it is doubled;
  * WRITE_SIZE reads the bytes exactly for 16-B-per-lane streaming stores.
The kernels of this library only issue 16-B-per-lane streaming loads/stores on the hot
path, so both corrections apply as stated.
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def collect(d: Path, counter: str):
    vals = defaultdict(list)
    for f in d.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                vals[name].append(float(row["Counter_Value"]))
    return vals


K_COMPACT_OUT = 1024  # fec_kernels.hip kCompactOut: the recover (rebuilt packets back to back) forms


def short(name: str) -> str:
    """Summary key of a kernel: encode, recover (decode forms with kCompactOut in their
    policy template argument, and recover_runs), decode (in place), or the kernel's own name."""
    if "encode_v16" in name or "encode_bits" in name:
        return "encode"
    if "recover_runs" in name:  # the one-launch packed recover (always the recover layout)
        return "recover"
    for key in ("decode_fused", "decode_wave", "decode_v16", "decode_tiled"):
        if key in name:
            args = name.split(key + "<", 1)[1].split(">", 1)[0].split(",")
            pol = int(args[2]) if len(args) > 2 and args[2].strip().isdigit() else 0
            return "recover" if pol & K_COMPACT_OUT else "decode"
    for key in ("classify", "fill_words", "copy_words", "encode_bytes", "decode_bytes"):
        if key in name:
            return key
    return name[:40]


def bench_workload(fdir: Path):
    """The workload of the profiled bench run: its JSON line in <fdir>.json (last line that parses)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", Path(__file__).resolve().parents[1] / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    p = Path(str(fdir) + ".json")
    if not p.exists():
        return None
    line = None
    for ln in p.read_text().splitlines():
        try:
            d = json.loads(ln)
        except ValueError:
            continue
        if isinstance(d, dict) and "config" in d:
            line = d
    return bench.workload_of_line(line) if line else None


def main():
    argv = sys.argv[1:]
    tag = None
    if "--tag" in argv:
        i = argv.index("--tag")
        tag = argv[i + 1]
        del argv[i:i + 2]
    fdir, wdir, config = Path(argv[0]), Path(argv[1]), argv[2]
    out = Path(argv[3]) if len(argv) > 3 else Path(__file__).resolve().parents[1] / "profiles" / f"pmc_{config}.json"
    fetch = collect(fdir, "FETCH_SIZE")
    write = collect(wdir, "WRITE_SIZE")
    import hashlib
    lib = Path(__file__).resolve().parents[1] / "quic-test_amd" / "lib" / "libfec_hip.so"
    res = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes)",
           "correction": "FETCH_SIZE x2 (gfx950 wide-stream read), KiB -> bytes",
           # bench.py uses these bytes only while the loaded library is this build
           "lib_sha256": hashlib.sha256(lib.read_bytes()).hexdigest(),
           # ... and on this workload only
           "workload": bench_workload(fdir)}
    if tag and out.exists():
        prev = json.loads(out.read_text())
        if prev.get("lib_sha256") == res["lib_sha256"] and prev.get("workload") == res["workload"]:
            res = {**prev, **res}
    for name in set(fetch) | set(write):
        s = short(name)
        if tag and s == "recover":
            s = f"recover_{tag}"
        f = fetch.get(name, [])
        w = write.get(name, [])
        fk = sorted(f)[len(f) // 2] if f else None
        wk = sorted(w)[len(w) // 2] if w else None
        entry = {"kernel": name[:160], "dispatches": max(len(f), len(w)),
                 "fetch_size_kib_median": fk, "write_size_kib_median": wk}
        if fk is not None and wk is not None:
            entry["hbm_read_bytes_per_launch"] = int(fk * 1024 * 2)
            entry["hbm_write_bytes_per_launch"] = int(wk * 1024)
            entry["hbm_bytes_per_launch"] = entry["hbm_read_bytes_per_launch"] + entry["hbm_write_bytes_per_launch"]
        res[s] = entry
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
