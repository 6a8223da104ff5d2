"""scripts/run_fec_tests.sh: the reference's QUIC FEC campaign loop (scripts/run_fec_tests.sh:
44-139 of the reference) with the flag fix -- FEC runs pass `--enable-fec --fec-rate=<r>`
(main.go:46-50), never the bool `--fec=<rate>` -- checked by syntax and a dry run (CPU)."""
import subprocess
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
SCRIPT = REPO / "scripts" / "run_fec_tests.sh"


def test_campaign_script_syntax():
    subprocess.run(["bash", "-n", str(SCRIPT)], check=True)


def test_campaign_dry_run_commands():
    out = subprocess.run(["bash", str(SCRIPT), "--dry-run", "--duration", "5s"], capture_output=True, text=True,
                         check=True, timeout=60).stdout.splitlines()
    assert len(out) == 16                                    # 2 profiles x 2 loads x 4 FEC levels
    assert all(ln.startswith("./bin/quic-test --mode=test ") for ln in out)
    assert not any("--fec=" in ln for ln in out)             # the reference's broken flag
    fec = [ln for ln in out if "--enable-fec" in ln]
    assert len(fec) == 12
    rates = sorted({ln.split("--fec-rate=")[1].split()[0] for ln in fec})
    assert rates == ["0.05", "0.10", "0.20"]
    base = [ln for ln in out if "--enable-fec" not in ln]
    assert len(base) == 4 and not any("--fec-rate" in ln for ln in base)
    mobile = [ln for ln in out if "--emulate-loss=0.05" in ln]
    assert len(mobile) == 8 and all("--emulate-latency=50ms" in ln for ln in mobile)
    assert sum("--connections=16 --streams=2" in ln for ln in out) == 8
    assert len({ln.split("--addr=")[1].split()[0] for ln in out}) == 16  # one port per run
    assert all("--duration=5s" in ln for ln in out)


def test_campaign_quic_leg_skips_without_binary(tmp_path):
    r = subprocess.run(["bash", str(SCRIPT), "--quic-only", "--out", str(tmp_path)], capture_output=True,
                       text=True, timeout=60, env={"PATH": "/usr/bin:/bin", "QUIC_TEST_BIN": str(tmp_path / "none")})
    assert r.returncode == 0 and "skipped" in r.stderr


def test_c1_leg_runs_reference_avx2_path():
    """C1 (BASELINE configs[0]): the reference's xor_packets_avx2 from oracle/_ref (when built
    here) byte-equal to the restatement; GPU part off on this CPU container."""
    import json
    import sys
    r = subprocess.run([sys.executable, str(REPO / "scripts" / "c1_leg.py"), "--no-gpu"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["config"] == "C1" and (out["k"], out["r"], out["P"], out["groups"]) == (4, 2, 256, 1024)
    assert out["restatement_row0_equals_xor"]
    if out["reference_lib_present"]:
        assert out["reference_xor_avx2_equals_restatement"] and out["reference_xor_avx2_GiBps"] > 0
