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
                 "pcx_consensus_batched_f64", "pcx_abi_version"):
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
        return re.findall(r"\*?\s*\b([a-z_0-9]+)\s*;", body)
    assert [f for f, _ in _abi.Batch._fields_] == fields("pcx_batch")
    assert [f for f, _ in _abi.BatchResult._fields_] == fields("pcx_batch_result")


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
