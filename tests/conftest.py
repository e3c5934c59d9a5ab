import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm MI355X GPU (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def core():
    from nodexa_chain_core_amd import _build

    _build.build_core()
    from nodexa_chain_core_amd import _core

    return _core


@pytest.fixture(scope="session")
def ctx0(core):
    return core.get_epoch_context(0)


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a ROCm GPU")
    from nodexa_chain_core_amd import _build

    _build.build_all()
    from nodexa_chain_core_amd.ops import runtime

    runtime.hip()
    return torch.device("cuda", 0)
