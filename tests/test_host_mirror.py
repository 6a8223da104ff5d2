"""The C++ mirror of the reference's Go FEC API (quic-test_amd/host) and its test program,
which restates internal/fec/encoder_test.go with byte-level checks (tests/csrc/)."""
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
LIB = REPO / "quic-test_amd" / "lib"


def _build(tmp_path: Path) -> Path:
    exe = tmp_path / "host_mirror_test"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-I", str(REPO / "include"), "-I", str(REPO / "quic-test_amd" / "host"),
                    str(REPO / "tests" / "csrc" / "host_mirror_test.cpp"), "-L", str(LIB), "-lquicfec_host", "-lfec_hip",
                    str(REPO / "oracle" / "liboracle.so"), f"-Wl,-rpath,{LIB}", f"-Wl,-rpath,{REPO / 'oracle'}",
                    "-lpthread", "-o", str(exe)], check=True)
    return exe


def test_host_mirror_builds(tmp_path, oracle_mod, quicfec_mod):
    assert (LIB / "libquicfec_host.so").exists()
    assert _build(tmp_path).exists()


@pytest.mark.gpu
def test_host_mirror_encoder_test_go(tmp_path, oracle_mod, quicfec_mod):
    exe = _build(tmp_path)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0 and out.stdout.strip().startswith("PASS"), out.stdout + out.stderr


@pytest.mark.gpu
def test_contexts_share_no_staging(tmp_path, quicfec_mod):
    """16 threads, one context each, the reference's one-group fec_encode_batch calls on their
    own page-locked slabs with shuffled offsets and random sizes: every repair equals the CPU XOR
    (tests/csrc/ctx_isolation_test.cpp)."""
    exe = tmp_path / "ctx_isolation_test"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-I", str(REPO / "include"),
                    str(REPO / "tests" / "csrc" / "ctx_isolation_test.cpp"), "-L", str(LIB), "-lfec_hip",
                    f"-Wl,-rpath,{LIB}", "-lpthread", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "16", "1500"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().startswith("PASS"), out.stdout + out.stderr
