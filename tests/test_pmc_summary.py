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
    assert short(ns + "recover_runs<10, 3, 1, 1, 3, 4, 256>(unsigned char const*, ...)") == "recover"


def test_committed_pmc_files_have_the_bench_keys():
    import json
    for cfg, keys in (("c2c3", ("encode", "recover_slots", "recover_packed")), ("c5", ("encode", "recover_slots")),
                      ("c4", ("encode",)), ("c4d", ("encode", "recover_slots", "decode"))):
        d = json.loads((REPO / "profiles" / f"pmc_{cfg}.json").read_text())
        for k in keys:
            assert d[k]["hbm_bytes_per_launch"] > 0, (cfg, k)


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _pmc_file(tmp_path, workload, sha="abc123"):
    import json
    p = tmp_path / "pmc_c2c3.json"
    p.write_text(json.dumps({"lib_sha256": sha, "workload": workload,
                             "encode": {"hbm_bytes_per_launch": 15_765_477_376}}))
    return p


def test_traffic_only_for_the_exact_workload(tmp_path):
    """roofline.traffic comes from a PMC file only when build AND workload match: a --shape or a
    --groups override (or another loss model) gets null, with the mismatch named."""
    b = _bench()
    base = dict(b.CONFIGS["c2c3"])
    wl = b.workload_key(base, base["groups"])
    p = _pmc_file(tmp_path, wl)
    pmc, note = b.load_pmc_traffic("c2c3", wl, path=p, sha="abc123")
    assert pmc is not None and "same workload" in note
    # --shape 10,1,1200 (the k=10 r=1 leg): r differs
    shaped = dict(base, r=1)
    pmc, note = b.load_pmc_traffic("c2c3", b.workload_key(shaped, base["groups"]), path=p, sha="abc123")
    assert pmc is None and "r=3 there vs 1 here" in note
    # --groups 500000 (the --gpus 2 rehearsals)
    pmc, note = b.load_pmc_traffic("c2c3", b.workload_key(base, 500_000), path=p, sha="abc123")
    assert pmc is None and "groups=1000000 there vs 500000 here" in note
    # --loss 0.05
    pmc, note = b.load_pmc_traffic("c2c3", b.workload_key(dict(base, loss=0.05), base["groups"]), path=p, sha="abc123")
    assert pmc is None and "loss" in note
    # another build
    pmc, note = b.load_pmc_traffic("c2c3", wl, path=p, sha="other")
    assert pmc is None and "another build" in note
    # files from before the workload was recorded are never used
    p2 = _pmc_file(tmp_path, None)
    pmc, note = b.load_pmc_traffic("c2c3", wl, path=p2, sha="abc123")
    assert pmc is None and "no workload" in note


def test_summary_records_the_profiled_workload(tmp_path):
    """pmc_summary takes the workload from the profiled bench's own JSON line, in the form
    bench.py compares against."""
    import json
    b = _bench()
    fdir = tmp_path / "pmc_c5_packed_FETCH_SIZE"
    fdir.mkdir()
    line = {"metric": "x", "config": {"k": 10, "r": 3, "packet_bytes": 1200, "groups_per_gpu": 1000000,
                                      "erasures_per_group": None, "iid_loss": 0.01}}
    (tmp_path / "pmc_c5_packed_FETCH_SIZE.json").write_text("noise\n" + json.dumps(line) + "\n")
    wl = _mod().bench_workload(fdir)
    assert wl == b.workload_key(b.CONFIGS["c5"], 1_000_000)
