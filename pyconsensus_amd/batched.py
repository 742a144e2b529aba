"""Batched Monte Carlo regime: B independent oracle rounds in one launch.

Each round is exactly ``Oracle(reports[b], event_bounds_b, reputation[b]).consensus()``
(pyconsensus/__init__.py:102-611) and runs in one wavefront of
``batched_round_kernel`` (csrc/pcx_batched.hip).  This is the regime of
Simulator.jl-style Monte Carlo drivers (README.rst:52-56), which loop consensus()
over many small random rounds.
"""
from __future__ import annotations

import ctypes as C

from . import _abi, _device, _lib

MAX_REPORTERS = 64
MAX_EVENTS = 32


def consensus_batched(reports, reputation=None, scaled=None, lo=None, hi=None,
                      catch_tolerance=0.1, alpha=0.1, int_dtype=False, algorithm="PCA",
                      outputs=None, device=None, filled=False, original=False,
                      max_components=5, variance_threshold=0.9, aux_scores=None):
    """Run B rounds of N x E reports on the GPU.

    reports:    (B, N, E) float64, NaN = missing (0.0 is missing too, as in the reference)
    reputation: (B, N) raw weights or None (uniform)
    scaled/lo/hi: event bounds, (B, E) or (E,) shared by every round; None = all binary
    outputs:    iterable of result names to produce (default: all vector/scalar outputs)
    algorithm:  "PCA" (default), "absolute", "big-five", "fixed-variance", "cokurtosis"
                (__init__.py:368-457); max_components is capped at E like Oracle (:134-137);
                aux_scores (B, N) are aux["cokurt"] of each round

    Returns a dict of torch tensors on the device, named like the ABI fields
    (``smooth_rep``, ``outcomes_final``, ...).  Asynchronous on torch's current stream.
    """
    t = _device.require_gpu()
    dev = t.device(device) if device is not None else t.device("cuda", t.cuda.current_device())
    R = _device.as_device(reports, t.float64, dev)
    if R.dim() != 3:
        raise ValueError("reports must be (B, N, E)")
    B, N, E = R.shape
    if not (1 <= N <= MAX_REPORTERS and 1 <= E <= MAX_EVENTS):
        raise ValueError("batched rounds need 1 <= N <= %d and 1 <= E <= %d (got %d x %d)"
                         % (MAX_REPORTERS, MAX_EVENTS, N, E))
    rep = _device.as_device(reputation, t.float64, dev)
    if rep is not None and tuple(rep.shape) != (B, N):
        raise ValueError("reputation must be (B, N)")
    shared = 0
    sc = lo_ = hi_ = None
    if scaled is not None:
        sc = _device.as_device(scaled, t.uint8, dev)
        lo_ = _device.as_device(lo, t.float64, dev)
        hi_ = _device.as_device(hi, t.float64, dev)
        shared = int(sc.dim() == 1)
        want = (E,) if shared else (B, E)
        for a in (sc, lo_, hi_):
            if tuple(a.shape) != want:
                raise ValueError("scaled/lo/hi must all be %s" % (want,))
    alg = _abi.ALGORITHMS.get(algorithm)
    if alg is None:
        raise NotImplementedError("algorithm %r is not on the GPU path" % (algorithm,))
    aux = None
    if alg == _abi.ALG_COKURTOSIS:
        if aux_scores is None:
            raise ValueError("cokurtosis needs aux_scores (aux['cokurt'] of every round)")
        aux = _device.as_device(aux_scores, t.float64, dev)
        if tuple(aux.shape) != (B, N):
            raise ValueError("aux_scores must be (B, N)")
    mc = int(max_components) if E >= int(max_components) else E  # __init__.py:134-137
    inp = _abi.Batch(B, N, E, _device.ptr(R), _device.ptr(rep), _device.ptr(sc), _device.ptr(lo_),
                     _device.ptr(hi_), shared, int(bool(int_dtype)), float(catch_tolerance),
                     float(alpha), alg, mc, float(variance_threshold), _device.ptr(aux))
    res = _abi.BatchResult()
    outs = {}
    for name, kind, dt in _abi.BATCH_OUTPUTS:
        if name == "filled" and not filled or name == "original" and not original:
            continue
        if outputs is not None and name not in outputs and name not in ("filled", "original"):
            continue
        tdt = t.float64 if dt == "f8" else t.int32
        x = t.empty(_abi.out_shape(kind, B, N, E), dtype=tdt, device=dev)
        outs[name] = x
        setattr(res, name, x.data_ptr())
    h = _lib.bind_stream(dev.index, _device.current_stream_handle(dev))
    _lib.check(_lib.lib().pcx_consensus_batched_f64(h, C.byref(inp), C.byref(res)))
    outs["_inputs"] = (R, rep, sc, lo_, hi_, aux)  # keep inputs alive until the caller syncs
    return outs
