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


_HEARTBEAT = {"test": None}


def pytest_runtest_logstart(nodeid, location):
    _HEARTBEAT["test"] = nodeid


def pytest_sessionstart(session):
    """On the GPU box (GRAFT_REPO_ROOT set): a heartbeat file under gpurun_out/ names the
    running test every 20 s, so a long parity case (the 1M-row restatement takes minutes)
    shows progress while pytest's own output waits for the test to end."""
    if not os.environ.get("GRAFT_REPO_ROOT"):
        return
    import threading
    import time

    path = os.path.join(ROOT, "gpurun_out", "pytest_heartbeat.log")

    def beat():
        t0 = time.time()
        while True:
            try:
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "a") as f:
                    f.write("%7.1f s  %s\n" % (time.time() - t0, _HEARTBEAT["test"]))
            except OSError:
                return
            time.sleep(20)

    threading.Thread(target=beat, daemon=True).start()
