import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun; excluded from CPU CI)")
    config.addinivalue_line("markers", "slow: multi-process / long-running")


@pytest.fixture(scope="session")
def C():
    import parameter_server_distributed_amd as psd

    return psd.native()


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible (these must run on the MI355X box)")
    return torch.device("cuda", 0)
