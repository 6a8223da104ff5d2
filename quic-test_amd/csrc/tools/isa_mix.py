#!/usr/bin/env python3
"""Instruction mix of kernels in the gfx950 assembly (make -C quic-test_amd/csrc asm).
Usage: isa_mix.py <name-substring> [file.s]   (static counts over the function body)"""
import re
import sys
from collections import Counter
from pathlib import Path

pat = sys.argv[1]
path = Path(sys.argv[2]) if len(sys.argv) > 2 else Path(__file__).resolve().parents[2] / "lib/asm/fec_kernels.s"
text = path.read_text()
for m in re.finditer(r"^(_Z\S*%s\S*):" % re.escape(pat), text, re.M):
    name = m.group(1)
    end = text.find(".Lfunc_end", m.end())
    body = text[m.end():end]
    ops = Counter(re.findall(r"^\s+([sv]_\w+|global_\w+|ds_\w+|buffer_\w+)", body, re.M))
    valu = sum(n for o, n in ops.items() if o.startswith("v_"))
    salu = sum(n for o, n in ops.items() if o.startswith("s_"))
    print(f"{name[:110]}\n  VALU {valu}  SALU {salu}")
    print("  " + ", ".join(f"{o} {n}" for o, n in ops.most_common(16)))
