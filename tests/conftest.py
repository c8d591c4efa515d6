import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sgxv2-analytical-query-processing-benchmarks_amd")
for p in (os.path.join(PKG, "python"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu on an MI355X)")
    config.addinivalue_line("markers", "slow: full-size cases")
    # build the in-tree library and oracle if a fresh checkout lacks them
    if not os.path.exists(os.path.join(PKG, "libsgxamd.so")):
        subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


@pytest.fixture(scope="session")
def sgx():
    import sgxamd

    return sgxamd


@pytest.fixture(scope="session")
def orc():
    import oracle

    return oracle


@pytest.fixture(scope="session")
def gpu(sgx):
    """Skip-free GPU guard: on the GPU box a missing device is a failure, not a skip."""
    n = sgx.device_count()
    assert n > 0, "no gfx950 device visible: -m gpu tests must run on an MI355X"
    import torch

    assert torch.cuda.is_available()
    return torch.device("cuda:0")
