import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_mod():
    """The CPU oracle (test infrastructure), built on first use."""
    from oracle import oracle as O
    if not os.path.exists(O.LIB):
        O.build()
    return O


@pytest.fixture(scope="session")
def native_lib_path():
    from mobileraytracer_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "mobileraytracer_amd", "csrc")], check=True)
    return _native.LIB_PATH


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
