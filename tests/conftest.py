import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "quic-test_amd", REPO / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfec_hip.so on the device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def xor_golden():
    import numpy as np
    return np.load(GOLDEN / "xor_ref.npz", allow_pickle=False)


@pytest.fixture(scope="session")
def gf_golden():
    import numpy as np
    return np.load(GOLDEN / "gf_restatement.npz", allow_pickle=False)


@pytest.fixture(scope="session")
def manifest():
    import json
    return json.loads((GOLDEN / "manifest.json").read_text())


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def quicfec_mod():
    import quicfec
    quicfec.load_library()
    return quicfec


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.fixture(scope="session")
def gpu_ctx(quicfec_mod):
    ctx = quicfec_mod.Context(device=0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def quicfec_hooks(quicfec_mod):
    """libfec_hip_test.so: the product library's objects with the test and tuning switches live
    (quic-test_amd/csrc/fec_knobs.hpp).  Only tests that force a kernel form, a size or a fault
    use it; every other GPU test runs libfec_hip.so, which ignores those switches."""
    return quicfec_mod.load_test_library()


@pytest.fixture(scope="session")
def gpu_ctx_hooks(quicfec_mod, quicfec_hooks):
    ctx = quicfec_mod.Context(device=0, lib=quicfec_hooks)
    yield ctx
    ctx.close()
