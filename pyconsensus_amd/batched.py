"""Batched Monte Carlo regime: B independent oracle rounds in one launch.

Each round is exactly ``Oracle(reports[b], event_bounds_b, reputation[b]).consensus()``
(pyconsensus/__init__.py:102-611).  This is the regime of Simulator.jl-style Monte
Carlo drivers (README.rst:52-56), which loop consensus() over many random rounds.
Rounds of at most 64 reporters x 32 events run in one wavefront each of
``batched_round_kernel`` (csrc/pcx_batched.hip); larger rounds run as single-matrix
consensuses, many in flight on a pool of worker streams (csrc/pcx_rounds.cpp).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi, _device, _lib

MAX_REPORTERS = 64  # one wavefront per round up to here (and MAX_EVENTS)
MAX_EVENTS = 32


def kmeans_k(N):
    """Code-book size of the reference's k-means, int(ceil(sqrt(N))) (__init__.py:396)."""
    return int(np.ceil(np.sqrt(N)))


def kmeans_draws(B, N, restarts=_abi.KMEANS_RESTARTS, random_state=None):
    """Initial code-book rows of B k-means rounds, [B][restarts][k] int32.

    scipy.cluster.vq.kmeans(obs, k) (seed=None, __init__.py:397) draws each restart's
    code book as ``rng.choice(N, size=k, replace=False)`` on numpy's global RandomState;
    these are the same draws in the same order (round after round), so a batch consumes
    the global stream exactly as B sequential reference consensus() calls would."""
    rs = np.random.mtrand._rand if random_state is None else random_state
    k = kmeans_k(N)
    out = np.empty((B, restarts, k), dtype=np.int32)
    for b in range(B):
        for r in range(restarts):
            out[b, r] = rs.choice(N, size=k, replace=False)
    return out


def clusterfeck_threshold(E):
    """The reference's default leader-clustering cut (__init__.py:187-190, 210-213)."""
    t = np.log10(E) / 1.77
    return 0.3 if t == 0 else float(t)


def consensus_batched(reports, reputation=None, scaled=None, lo=None, hi=None,
                      catch_tolerance=0.1, alpha=0.1, int_dtype=False, algorithm="PCA",
                      outputs=None, device=None, filled=False, original=False,
                      max_components=5, variance_threshold=0.9, aux_scores=None,
                      hierarchy_threshold=0.5, kmeans_init=None, cluster_threshold=None, packed=False):
    """Run B rounds of N x E reports on the GPU.

    reports:    (B, N, E) float64, NaN = missing (0.0 is missing too, as in the reference)
    reputation: (B, N) raw weights or None (uniform)
    scaled/lo/hi: event bounds, (B, E) or (E,) shared by every round; None = all binary
    outputs:    iterable of result names to produce (default: all vector/scalar outputs)
    algorithm:  "PCA" (default), "absolute", "big-five", "fixed-variance", "cokurtosis"
                (__init__.py:368-457), "k-means", "hierarchical", "clusterfeck" (:392-428);
                max_components is capped at E like Oracle (:134-137); aux_scores (B, N)
                are aux["cokurt"] of each round
    kmeans_init: (B, restarts, k) initial code-book rows (default: :func:`kmeans_draws`
                on numpy's global RandomState, as the reference's scipy call draws them)
    cluster_threshold: clusterfeck's cut (default: the reference's log10(E)/1.77 rule)
    packed:     numpy inputs travel to the device in ONE copy and every output is a view of ONE
                device buffer (``out["_packed"]``; :func:`unpack_round` brings it back in one
                copy) -- the drop-in's per-call path, where each separate small copy costs ~10 us

    Returns a dict of torch tensors on the device, named like the ABI fields
    (``smooth_rep``, ``outcomes_final``, ...).  Three regimes:
    rounds up to 64 x 32 (one wave per round) and up to 256 x 64 (one workgroup per round,
    any non-clustering algorithm) are ONE kernel launch, asynchronous on torch's current
    stream -- synchronise before reading the outputs on the host; the round scheduler (the
    clusterings above 64 x 32, or rounds above 256 x 64) returns only once every output is
    written.
    """
    t = _device.require_gpu()
    dev = t.device(device) if device is not None else t.device("cuda", t.cuda.current_device())
    if packed and all(x is None or isinstance(x, np.ndarray) for x in (reports, reputation, scaled, lo, hi)):
        reports, reputation, scaled, lo, hi = _upload_packed(
            [(reports, np.float64), (reputation, np.float64), (scaled, np.uint8), (lo, np.float64),
             (hi, np.float64)], dev)
    R = _device.as_device(reports, t.float64, dev)
    if R.dim() != 3:
        raise ValueError("reports must be (B, N, E)")
    B, N, E = R.shape
    if N < 1 or E < 1:
        raise ValueError("batched rounds need N >= 1 and E >= 1 (got %d x %d)" % (N, E))
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
    kinit = None
    k = restarts = 0
    if alg == _abi.ALG_KMEANS:
        if kmeans_init is None:
            kmeans_init = kmeans_draws(B, N)
        kinit = _device.as_device(kmeans_init, t.int32, dev)
        if kinit.dim() != 3 or kinit.shape[0] != B:
            raise ValueError("kmeans_init must be (B, restarts, k)")
        restarts, k = int(kinit.shape[1]), int(kinit.shape[2])
        if not (1 <= k <= N) or restarts < 1 or int(kinit.min()) < 0 or int(kinit.max()) >= N:
            raise ValueError("kmeans_init rows must lie in [0, N) with 1 <= k <= N")
    cthr = clusterfeck_threshold(E) if cluster_threshold is None else float(cluster_threshold)
    mc = int(max_components) if E >= int(max_components) else E  # __init__.py:134-137
    inp = _abi.Batch(B, N, E, _device.ptr(R), _device.ptr(rep), _device.ptr(sc), _device.ptr(lo_),
                     _device.ptr(hi_), shared, int(bool(int_dtype)), float(catch_tolerance),
                     float(alpha), alg, mc, float(variance_threshold), _device.ptr(aux),
                     float(hierarchy_threshold), cthr, k, restarts, _device.ptr(kinit))
    res = _abi.BatchResult()
    outs = {}
    want = [(name, kind, dt) for name, kind, dt in _abi.BATCH_OUTPUTS
            if not (name == "filled" and not filled or name == "original" and not original)
            and not (outputs is not None and name not in outputs and name not in ("filled", "original"))]
    if packed:  # one device buffer, one 16-byte-aligned view per output
        layout, off = [], 0
        for name, kind, dt in want:
            shape = _abi.out_shape(kind, B, N, E)
            nb = int(np.prod(shape)) * (8 if dt == "f8" else 4)
            layout.append((name, off, nb, dt, shape))
            off += (nb + 15) // 16 * 16
        buf = t.empty(max(off, 16), dtype=t.uint8, device=dev)
        for name, o, nb, dt, shape in layout:
            x = buf[o:o + nb].view(t.float64 if dt == "f8" else t.int32).view(shape)
            outs[name] = x
            setattr(res, name, x.data_ptr())
        outs["_packed"] = buf
        outs["_layout"] = layout
    else:
        for name, kind, dt in want:
            tdt = t.float64 if dt == "f8" else t.int32
            x = t.empty(_abi.out_shape(kind, B, N, E), dtype=tdt, device=dev)
            outs[name] = x
            setattr(res, name, x.data_ptr())
    h = _lib.bind_stream(dev.index, _device.current_stream_handle(dev))
    _lib.check(_lib.lib().pcx_consensus_batched_f64(h, C.byref(inp), C.byref(res)))
    outs["_inputs"] = (R, rep, sc, lo_, hi_, aux, kinit)  # keep inputs alive until the caller syncs
    return outs


def _upload_packed(items, dev):
    """numpy arrays (or None) -> device tensors, as views of ONE host-to-device copy."""
    t = _device.torch()
    parts, off = [], 0
    for a, dt in items:
        if a is None:
            parts.append(None)
            continue
        a = np.ascontiguousarray(a, dtype=dt)
        parts.append((a, off))
        off += (a.nbytes + 15) // 16 * 16
    host = np.empty(max(off, 16), dtype=np.uint8)
    for p in parts:
        if p is not None:
            host[p[1]:p[1] + p[0].nbytes] = p[0].reshape(-1).view(np.uint8)
    d = t.from_numpy(host).to(dev)
    tdt = {np.float64: t.float64, np.uint8: t.uint8}
    return [None if p is None else d[p[1]:p[1] + p[0].nbytes].view(tdt[dt]).view(p[0].shape)
            for p, (_, dt) in zip(parts, items)]


def unpack_round(out, b=0):
    """Round ``b`` of a ``packed=True`` result as numpy arrays, from ONE device-to-host copy."""
    host = out["_packed"].cpu().numpy()
    g = {}
    for name, o, nb, dt, shape in out["_layout"]:
        g[name] = host[o:o + nb].view(np.float64 if dt == "f8" else np.int32).reshape(shape)[b]
    return g
