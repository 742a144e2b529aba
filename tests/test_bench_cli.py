"""bench.py's launcher contract on the CPU: ``--gpus N`` without a launcher starts the
driver's own N-rank command as a child job; a WORLD_SIZE that disagrees with ``--gpus``
is refused before anything touches the GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(args, env_extra, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "1"], {"WORLD_SIZE": "2"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr
    r = _run(["--gpus", "4"], {"WORLD_SIZE": "2"})
    assert r.returncode == 2


def test_gpus_zero_refused():
    assert _run(["--gpus", "0"], {}).returncode == 2


def test_self_launch_command(monkeypatch):
    import bench

    seen = {}

    class FakeProc:
        pid = 12345

        def __init__(self, cmd, env):
            seen["cmd"], seen["env"] = cmd, env

        def wait(self, timeout=None):
            return 7

        def send_signal(self, s):  # pragma: no cover
            pass

    import signal

    old = signal.getsignal(signal.SIGTERM)
    monkeypatch.setattr(subprocess, "Popen", FakeProc)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "5"])
    try:
        assert bench.launch_ranks(4) == 7  # the child job's status is the parent's
    finally:
        signal.signal(signal.SIGTERM, old)
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "5"]
    assert cmd[-5].endswith("bench.py")
    assert bench.LAUNCHER_ENV in seen["env"]


@pytest.mark.timeout(300)
def test_self_launch_reaches_ranks():
    """The real child job: 2 ranks start and each fails on the GPU-less host (no CUDA device),
    so the parent returns non-zero -- it does not fall back to a 1-rank run."""
    import torch

    if torch.cuda.is_available():  # pragma: no cover - a GPU box runs the real thing
        pytest.skip("CPU-only check")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--c5-steps", "0", "--no-c4", "--no-cpu-baseline"],
             {"PCX_DIST_BACKEND": "gloo"}, timeout=280)
    assert r.returncode != 0
    assert '"n_gpus": 1' not in r.stdout
