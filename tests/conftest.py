import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu_lib():
    """The in-tree HIP library; GPU tests fail (not skip) when it is missing."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    from pyconsensus_amd import _lib

    return _lib.lib()
