import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def lib():
    # PyTorch ships its own HIP runtime; when both are in one process, torch's
    # must initialize the GPU before this library's (tests hand torch device
    # buffers to the C-ABI).  torch only provides device memory here.
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    from minbft_amd import build, _lib
    build.build()
    return _lib.load()


@pytest.fixture(scope="session")
def gpu_auth(lib):
    from minbft_amd.authenticator import Authenticator
    a = Authenticator(0)
    yield a
    a.close()
