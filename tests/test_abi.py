"""CPU-side checks of the C-ABI boundary: libpcx.so loads, exports every function
declared in include/pcx.h, and the ctypes mirror matches the header."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pcx.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pcx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("pcx_create", "pcx_destroy", "pcx_set_stream", "pcx_last_error",
                 "pcx_consensus_batched_f64", "pcx_abi_version", "pcx_consensus_f64", "pcx_create_rank",
                 "pcx_comm_unique_id", "pcx_interpolate_f64", "pcx_wpca_f64", "pcx_lie_detector_f64",
                 "pcx_nonconformity_f64", "pcx_create_devices"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from pyconsensus_amd import _lib

    h = _lib.lib()
    missing = [n for n in declared_functions() if not hasattr(h, n)]
    assert not missing, missing
    from pyconsensus_amd import _abi
    assert h.pcx_abi_version() == _abi.ABI_VERSION


def test_struct_layout_matches_header():
    """Field order/count of the ctypes mirrors equals the C structs in pcx.h."""
    from pyconsensus_amd import _abi

    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    def fields(struct):
        body = re.search(r"typedef struct \{([^{}]*)\}\s*%s;" % struct, src, re.S).group(1)
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            # "double *a, *b" / "int (*f)(...)" / "int64_t n"
            fp = re.match(r".*\(\s*\*\s*([a-z_0-9]+)\s*\)\s*\(", decl, re.S)
            if fp:
                names.append(fp.group(1))
                continue
            first, *rest = decl.split(",")
            names.append(re.findall(r"([a-z_0-9]+)\s*(?:\[[^\]]*\])?$", first.strip())[0])
            names += [re.sub(r"[*\s]", "", r) for r in rest]
        return names
    assert [f for f, _ in _abi.Batch._fields_] == fields("pcx_batch")
    assert [f for f, _ in _abi.BatchResult._fields_] == fields("pcx_batch_result")
    assert [f for f, _ in _abi.Problem._fields_] == fields("pcx_problem")
    assert [f for f, _ in _abi.Result._fields_] == fields("pcx_result")
    assert [f for f, _ in _abi.CommOps._fields_] == fields("pcx_comm_ops")


def test_struct_sizes_and_offsets_match_c():
    """Byte layout of pcx_problem / pcx_result / pcx_batch as the C compiler lays them out
    (a C probe compiled here with gcc against include/pcx.h) equals the ctypes mirrors."""
    import subprocess
    import tempfile

    from pyconsensus_amd import _abi

    structs = {"pcx_problem": _abi.Problem, "pcx_result": _abi.Result, "pcx_batch": _abi.Batch,
               "pcx_batch_result": _abi.BatchResult, "pcx_comm_ops": _abi.CommOps, "pcx_comm_id": _abi.CommId}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "pcx.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append('printf("%s size %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "probe.c")
        open(src, "w").write("\n".join(lines))
        exe = os.path.join(d, "probe")
        subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), src, "-o", exe])
        out = dict(l.rsplit(" ", 1) for l in subprocess.check_output([exe]).decode().splitlines())
    for cname, py in structs.items():
        assert int(out["%s size" % cname]) == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(out["%s.%s" % (cname, f)]) == getattr(py, f).offset, (cname, f)


def test_errors_without_gpu_are_loud():
    """No GPU here: creating a context must fail with a message (never a silent CPU path)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pyconsensus_amd import _lib

    assert not _lib.lib().pcx_create(0)
    assert b"no HIP device" in _lib.lib().pcx_last_error()
    from pyconsensus_amd.batched import consensus_batched
    with pytest.raises(_lib.PcxError):
        consensus_batched([[[1.0, 2.0]]])
    assert not _lib.lib().pcx_create_grouped(0, None, 0)
    import ctypes as C
    ids = (C.c_int * 2)(0, 1)
    assert not _lib.lib().pcx_create_devices(2, ids)  # the multi-device context needs the GPUs too
    assert b"no HIP device" in _lib.lib().pcx_last_error()
    assert not _lib.lib().pcx_create_devices(0, ids)
    from pyconsensus_amd import Oracle
    with pytest.raises(_lib.PcxError):
        Oracle(reports=[[1.0, 2.0]] * 100).consensus()  # the matrix path raises too (no CPU fallback)


def test_stage_names():
    from pyconsensus_amd import _abi, _lib

    names = [_lib.lib().pcx_stage_name(k).decode() for k in range(_abi.NSTAGES)]
    assert names[1] == "REPUTATION" and "SEL_HIST" in names and "HARD_WALK" in names


def test_comm_abort_once_selftest():
    """The RCCL abort path's exactly-once semantics (pcx_comm.cpp AbortOnce) without RCCL:
    threads exchanging on a fake handle while others abort it -- one free, no use of a freed
    handle, no successful exchange after an abort returned."""
    from pyconsensus_amd import _lib

    h = _lib.lib()
    for users, aborters in ((1, 1), (4, 1), (8, 8), (2, 16)):
        assert h.pcx_selftest_abort_once(users, aborters, 20000) == 0, (users, aborters)
    assert h.pcx_selftest_abort_once(0, 1, 10) == -1


def test_rccl_version_compatible():
    """The librccl this process resolves has the major version of the headers libpcx was built
    against and is >= 2.18, so RCCL contexts are not refused (pcx_rccl_version)."""
    import ctypes as C

    from pyconsensus_amd import _lib

    rt, ct = C.c_int(0), C.c_int(0)
    v = _lib.lib().pcx_rccl_version(C.byref(rt), C.byref(ct))
    assert v == rt.value and ct.value >= 21800
    major = lambda x: x // 10000 if x >= 10000 else x // 1000
    assert major(rt.value) == major(ct.value) and rt.value >= 21800, (rt.value, ct.value)
