"""The PMC summary's kernel keys (scripts/pmc_summary.py): bench.py reads roofline.traffic from
profiles/pmc_<config>.json under these keys, so every shipped encode and decode form must map to
one (a new kernel that maps to its own truncated name silently gives traffic: null)."""
import importlib.util
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def _mod():
    spec = importlib.util.spec_from_file_location("pmc_summary", REPO / "scripts" / "pmc_summary.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_kernel_keys():
    short = _mod().short
    ns = "void qfec::(anonymous namespace)::"
    assert short(ns + "encode_v16<10, 3, 0, true, 4098>(unsigned char const*, ...)") == "encode"
    assert short(ns + "encode_bits<20, 5, 4, 2>(unsigned char const*, unsigned char*, ...)") == "encode"
    assert short(ns + "decode_fused<10, 3, 1027, 1, 1, true, true, 0>(unsigned char const*, ...)") == "recover"
    assert short(ns + "decode_fused<10, 3, 3, 1, 1, true, true, 0>(unsigned char const*, ...)") == "decode"
    assert short("qfec::(anonymous namespace)::classify(unsigned long const*, ...)") == "classify"


def test_committed_pmc_files_have_the_bench_keys():
    import json
    for cfg, keys in (("c2c3", ("encode", "recover_slots", "recover_packed")), ("c5", ("encode", "recover_slots")),
                      ("c4", ("encode",)), ("c4d", ("encode", "recover_slots", "decode"))):
        d = json.loads((REPO / "profiles" / f"pmc_{cfg}.json").read_text())
        for k in keys:
            assert d[k]["hbm_bytes_per_launch"] > 0, (cfg, k)
