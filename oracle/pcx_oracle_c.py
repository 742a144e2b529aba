"""ctypes front-end of the C oracle (oracle/lib/libpcx_oracle.so).

TEST INFRASTRUCTURE -- used only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Same structs as the product ABI (include/pcx.h), host memory.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from pyconsensus_amd._abi import BATCH_OUTPUTS, Batch, BatchResult, out_shape, ALGORITHMS
from pyconsensus_amd.batched import clusterfeck_threshold

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "libpcx_oracle.so")
LIB256 = os.path.join(HERE, "lib", "libpcx_oracle256.so")  # NMAX = 256: rounds above 64 reporters
_lib = None
_lib256 = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib(large=False):
    global _lib, _lib256
    if (_lib256 if large else _lib) is None:
        path = LIB256 if large else LIB
        if not os.path.exists(path):
            build()
        h = C.CDLL(path)
        h.pcxo_consensus_batched_f64.argtypes = [C.POINTER(Batch), C.POINTER(BatchResult), C.c_int]
        h.pcxo_consensus_batched_f64.restype = C.c_int
        if large:
            _lib256 = h
        else:
            _lib = h
    return _lib256 if large else _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def batched(reports, scaled=None, lo=None, hi=None, reputation=None, catch_tolerance=0.1,
            alpha=0.1, int_dtype=False, algorithm="PCA", threads=1, want=None, max_components=5,
            variance_threshold=0.9, aux_scores=None, hierarchy_threshold=0.5, kmeans_init=None,
            cluster_threshold=None):
    """Run B rounds; returns {name: array} for every output in ``want`` (default: all)."""
    R = np.ascontiguousarray(reports, dtype=np.float64)
    B, N, E = R.shape
    shared = scaled is not None and np.ndim(scaled) == 1
    keep = []
    def cont(a, dt):
        if a is None:
            return None
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a
    sc = cont(scaled, np.uint8)
    lo_ = cont(lo, np.float64)
    hi_ = cont(hi, np.float64)
    rp = cont(reputation, np.float64)
    ax = cont(aux_scores, np.float64)
    ki = cont(kmeans_init, np.int32)
    k = restarts = 0
    if ki is not None:
        restarts, k = ki.shape[1], ki.shape[2]
    cthr = clusterfeck_threshold(E) if cluster_threshold is None else float(cluster_threshold)
    inp = Batch(B, N, E, _ptr(R), _ptr(rp), _ptr(sc), _ptr(lo_), _ptr(hi_), int(shared), int(bool(int_dtype)),
                float(catch_tolerance), float(alpha), ALGORITHMS[algorithm], int(min(max_components, E)),
                float(variance_threshold), _ptr(ax), float(hierarchy_threshold), cthr, k, restarts, _ptr(ki))
    outs = {}
    res = BatchResult()
    for name, kind, dt in BATCH_OUTPUTS:
        if want is not None and name not in want:
            continue
        a = np.empty(out_shape(kind, B, N, E), dtype=dt)
        outs[name] = a
        setattr(res, name, a.ctypes.data)
    rc = lib(large=N > 64).pcxo_consensus_batched_f64(C.byref(inp), C.byref(res), int(threads))
    if rc != 0:
        raise ValueError("oracle rejected the batch (rc=%d)" % rc)
    return outs
