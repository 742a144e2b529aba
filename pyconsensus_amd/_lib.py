"""ctypes binding of libpcx.so (include/pcx.h).

The library is built in-tree (``pyconsensus_amd/libpcx.so``, see csrc/Makefile)
and is the ONLY compute path of this package: if it cannot be loaded, or no GPU is
visible, every entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
# PCX_LIB: load another build of the same ABI (A/B performance runs, tools/ab_build.sh)
LIB_PATH = os.environ.get("PCX_LIB") or os.path.join(HERE, "libpcx.so")

_lock = threading.Lock()
_lib = None


class PcxError(RuntimeError):
    """An error reported by libpcx (the message is pcx_last_error())."""


def _declare(lib):
    lib.pcx_abi_version.restype = C.c_int
    lib.pcx_last_error.restype = C.c_char_p
    lib.pcx_create.argtypes = [C.c_int]
    lib.pcx_create.restype = C.c_void_p
    lib.pcx_destroy.argtypes = [C.c_void_p]
    lib.pcx_destroy.restype = None
    lib.pcx_set_stream.argtypes = [C.c_void_p, C.c_void_p]
    lib.pcx_set_stream.restype = C.c_int
    lib.pcx_synchronize.argtypes = [C.c_void_p]
    lib.pcx_synchronize.restype = C.c_int
    lib.pcx_consensus_batched_f64.argtypes = [C.c_void_p, C.POINTER(_abi.Batch), C.POINTER(_abi.BatchResult)]
    lib.pcx_consensus_batched_f64.restype = C.c_int
    vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
    for name, res, args in [
        ("pcx_comm_unique_id", i32, [C.POINTER(_abi.CommId)]),
        ("pcx_create_rank", vp, [i32, i32, i32, C.POINTER(_abi.CommId)]),
        ("pcx_group_create", vp, [i32]),
        ("pcx_group_destroy", None, [vp]),
        ("pcx_create_grouped", vp, [i32, vp, i32]),
        ("pcx_create_custom", vp, [i32, i32, i32, C.POINTER(_abi.CommOps)]),
        ("pcx_create_devices", vp, [i32, C.POINTER(C.c_int)]),
        ("pcx_ctx_world", i32, [vp]),
        ("pcx_ctx_rank", i32, [vp]),
        ("pcx_ctx_usable", i32, [vp]),
        ("pcx_release_workspace", i32, [vp]),
        ("pcx_consensus_f64", i32, [vp, C.POINTER(_abi.Problem), C.POINTER(_abi.Result)]),
        ("pcx_interpolate_f64", i32, [vp, C.POINTER(_abi.Problem), C.POINTER(_abi.Result)]),
        ("pcx_wpca_f64", i32, [vp, C.POINTER(_abi.Problem), C.POINTER(_abi.Result)]),
        ("pcx_lie_detector_f64", i32, [vp, C.POINTER(_abi.Problem), C.POINTER(_abi.Result)]),
        ("pcx_nonconformity_f64", i32, [vp, C.POINTER(_abi.Problem), vp, i32, vp, C.POINTER(_abi.Result)]),
        ("pcx_profile_enable", i32, [vp, i32]),
        ("pcx_profile_read", i32, [vp, C.POINTER(C.c_double)]),
        ("pcx_stage_name", C.c_char_p, [i32]),
        ("pcx_ctx_progress", i32, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        ("pcx_seqsum_const", C.c_double, [C.c_double, i64]),
        ("pcx_seqsum_first_above", i64, [C.c_double, C.c_double, i64]),
        ("pcx_mixed_digits", i32, []),
        ("pcx_rccl_version", i32, [C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        ("pcx_selftest_abort_once", i32, [i32, i32, i32]),
        ("pcx_selftest_abort_slow_holder", i32, [i32, i32]),
        ("pcx_selftest_group_abort", i32, [i32, i32, i32, i32]),
        ("pcx_selftest_rounds_sched", i32, [i32, i64, i32, i64]),
        ("pcx_selftest_chunked_copy", i32, [i64, i64, i32, i32, i64]),
        ("pcx_test_inject_enomem", i32, [vp, i32]),
    ]:
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def lib():
    """Load (once) and return the ctypes handle of libpcx.so; raise if missing."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise PcxError("libpcx.so is not built (%s); run `make -C pyconsensus_amd/csrc` "
                               "or __graft_entry__.build()" % LIB_PATH)
            h = C.CDLL(LIB_PATH)
            _declare(h)
            v = h.pcx_abi_version()
            if v != _abi.ABI_VERSION:
                raise PcxError("libpcx ABI version %d, expected %d" % (v, _abi.ABI_VERSION))
            _lib = h
    return _lib


PCX_ECOMM = -4  # include/pcx.h enum pcx_status


def check(rc):
    if rc != 0:
        raise PcxError("libpcx error %d: %s" % (rc, lib().pcx_last_error().decode(errors="replace")))


_ctx = {}


def context(device_index):
    """The per-(thread, device) pcx_ctx handle."""
    key = (threading.get_ident(), int(device_index))
    h = _ctx.get(key)
    if h is None:
        h = lib().pcx_create(int(device_index))
        if not h:
            raise PcxError("pcx_create(%d) failed: %s" % (device_index, lib().pcx_last_error().decode()))
        _ctx[key] = h
    return h


def devices_context(device_ids):
    """The per-thread multi-device pcx_ctx (pcx_create_devices) of ``device_ids``: the
    single-matrix calls on it shard the rows over those GPUs inside libpcx."""
    ids = tuple(int(d) for d in device_ids)
    key = (threading.get_ident(), ids)
    h = _ctx.get(key)
    if h is None:
        arr = (C.c_int * len(ids))(*ids)
        h = new_context(lib().pcx_create_devices(len(ids), arr), "pcx_create_devices(%s)" % (ids,))
        _ctx[key] = h
    return h


def drop_devices_context(device_ids):
    """Destroy and forget this thread's cached multi-device context of ``device_ids`` (after
    PCX_ECOMM its RCCL communicators are aborted; the next call creates a fresh one)."""
    key = (threading.get_ident(), tuple(int(d) for d in device_ids))
    h = _ctx.pop(key, None)
    if h is not None:
        lib().pcx_destroy(h)


def bind_stream(device_index, stream_handle, ctx=None):
    h = context(device_index) if ctx is None else ctx
    check(lib().pcx_set_stream(h, C.c_void_p(stream_handle)))
    return h


def new_context(ptr, what):
    """Check a pcx_create* result (NULL = error with pcx_last_error())."""
    if not ptr:
        raise PcxError("%s failed: %s" % (what, lib().pcx_last_error().decode(errors="replace")))
    return ptr
