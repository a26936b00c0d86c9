import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def native_built():
    from parallel_heat_amd import _native
    _native.lib()  # builds with `make` if missing
    yield


@pytest.fixture
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def exp_kernels():
    """The experiment kernels (libheat_exp.so, `make exp`): the test files that
    cover the measured-slower TB builds (packed, float2, mixed shifts,
    chained passes) load them; the product library does not carry them."""
    from parallel_heat_amd import _native
    yield _native.load_exp()
    # Unregistered again: the product-path tests of later modules must not
    # lean on them (an odd-depth tile pass did, until round 6).
    _native.unload_exp()
