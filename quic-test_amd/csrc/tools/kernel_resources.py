#!/usr/bin/env python3
"""Print VGPR/SGPR/spill/LDS per kernel from the amdgcn metadata of an assembly file
(make -C quic-test_amd/csrc asm).  Usage: kernel_resources.py [file.s] [name-filter]"""
import re
import subprocess
import sys
from pathlib import Path

path = Path(sys.argv[1]) if len(sys.argv) > 1 else Path(__file__).resolve().parents[2] / "lib/asm/fec_kernels.s"
filt = sys.argv[2] if len(sys.argv) > 2 else ""
text = path.read_text()
meta = text[text.find("amdhsa.kernels:"):]
rows = []
for blk in meta.split("\n  - ")[1:]:
    def f(key):
        m = re.search(r"\.%s:\s+(\S+)" % key, blk)
        return m.group(1) if m else "?"
    name = f("name")
    try:
        name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    except OSError:
        pass
    name = name.replace("qfec::(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    if filt in name:
        rows.append((name, f("vgpr_count"), f("sgpr_count"), f("vgpr_spill_count"), f("sgpr_spill_count"),
                     f("group_segment_fixed_size")))
print(f"{'kernel':60s} {'vgpr':>5s} {'sgpr':>5s} {'vspill':>6s} {'sspill':>6s} {'lds':>6s}")
for r in rows:
    print(f"{r[0][:60]:60s} {r[1]:>5s} {r[2]:>5s} {r[3]:>6s} {r[4]:>6s} {r[5]:>6s}")
