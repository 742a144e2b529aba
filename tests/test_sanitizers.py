"""SURVEY.md 5 (race / failure detection): libpcx's host concurrency under sanitizers, on the CPU.

The threaded host layer -- the virtual-rank group exchange and its abort (pcx_comm.cpp,
pcx_create_grouped / pcx_create_devices), the RCCL handle's abort-once (pcx_comm.cpp RcclComm),
the per-device worker release (pcx_api.cpp run_devices) and the round scheduler's ENOMEM
hand-back (pcx_rounds.cpp) -- lives in csrc/pcx_sync.h, plain C++17 with no HIP or RCCL.
tests/c/host_selftest.cpp drives it through the self-tests of csrc/pcx_selftest.cpp (the same
sources libpcx is built from) and is compiled here with g++ under ThreadSanitizer and under
AddressSanitizer + UBSan; any report fails the test (halt_on_error).  GPU sanitizers are not
available on the pool: the device side is covered by the -m gpu parity tests instead.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pyconsensus_amd", "csrc")
SRC = [os.path.join(ROOT, "tests", "c", "host_selftest.cpp"), os.path.join(CSRC, "pcx_selftest.cpp")]


def _build_and_run(tmp_path, flags, env_name, env_val):
    exe = str(tmp_path / "host_selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", *flags, "-I", CSRC,
           "-I", os.path.join(ROOT, "include"), *SRC, "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=240)
    env = dict(os.environ, **{env_name: env_val})
    r = subprocess.run([exe, "2"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert "PASSED" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]  # UBSan


@pytest.mark.timeout(900)
def test_host_layer_thread_sanitizer(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], "TSAN_OPTIONS", "halt_on_error=1:second_deadlock_stack=1")


@pytest.mark.timeout(900)
def test_host_layer_address_ub_sanitizer(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "ASAN_OPTIONS",
                   "halt_on_error=1:detect_leaks=1")


def test_selftests_in_libpcx():
    """The same self-tests as exported by the shipped libpcx.so (the library's own build)."""
    import ctypes as C

    from pyconsensus_amd import _lib

    h = _lib.lib()
    assert h.pcx_selftest_abort_slow_holder(4, 3) == 0
    assert h.pcx_selftest_abort_slow_holder(0, 1) == -1
    for world, fr, fs in [(1, -1, -1), (2, 0, 0), (2, 1, 3), (4, 2, 1), (8, 7, 4)]:
        assert h.pcx_selftest_group_abort(world, 5, fr, fs) == 0, (world, fr, fs)
    assert h.pcx_selftest_group_abort(2, 5, 2, 0) == -1
    for slots, T, fail in [(3, 16, -1), (1, 1, -1), (2, 8, 4)]:
        assert h.pcx_selftest_chunked_copy(C.c_int64(5_000_011), C.c_int64(1 << 18), slots, T, C.c_int64(fail)) == 0
    for K, enw, fail in [(1, -1, -1), (4, 0, -1), (4, 3, -1), (16, 2, 9), (1, 0, -1)]:
        assert h.pcx_selftest_rounds_sched(K, C.c_int64(200), enw, C.c_int64(fail)) == 0, (K, enw, fail)
