"""Single-matrix consensus: tensor handoff to ``pcx_consensus_f64`` and the rank contexts.

One N x E report matrix, sharded by contiguous reporter rows over ``comm.world``
ranks (one process per GPU, or threads of one process).  The whole consensus --
stage order, scratch, and the exchange between stages -- runs inside libpcx
(``csrc/pcx_runner.cpp``); this module only builds the ``pcx_problem`` /
``pcx_result`` structs from torch tensors or numpy arrays and picks the context:

* :class:`Comm`        one rank;
* :class:`RcclComm`    one process per GPU, RCCL over xGMI inside libpcx (the unique
                       id is broadcast with torch.distributed, any backend);
* :class:`ThreadComm`  virtual ranks as threads of one process (``ThreadGroup``),
                       exchanging through host memory -- the 1-GPU rehearsal;
* :class:`CallbackComm` torch.distributed (e.g. gloo) behind libpcx's callback ops.

Reference (pyconsensus/__init__.py): interpolate :260-313, wpca :315-339,
nonconformity_rank :487-500, lie_detector tail :459-473, consensus :502-611.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from . import _abi, _device, _lib


class Comm:
    """One rank: the per-(thread, device) context of _lib."""

    world, rank = 1, 0

    def context(self, device_index):
        return _lib.context(device_index)

    @staticmethod
    def from_env(device_index=None):
        """The communicator of an initialised torch.distributed job: RCCL for the
        ``nccl`` backend (RCCL on ROCm), callbacks for any other (gloo)."""
        import torch.distributed as dist

        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return Comm()
        if device_index is None:
            device_index = _device.torch().cuda.current_device()
        if dist.get_backend() == "nccl":
            return RcclComm(dist.get_world_size(), dist.get_rank(), device_index)
        return CallbackComm(dist.get_world_size(), dist.get_rank())


class _OwnedCtx(Comm):
    _ctx = None

    def context(self, device_index):
        return self._ctx

    def close(self):
        if self._ctx:
            _lib.lib().pcx_destroy(self._ctx)
            self._ctx = None


class RcclComm(_OwnedCtx):
    """libpcx's own RCCL communicator (ncclCommInitRank); collective construction."""

    def __init__(self, world, rank, device_index):
        import torch.distributed as dist

        self.world, self.rank = int(world), int(rank)
        cid = _abi.CommId()
        if self.rank == 0:
            _lib.check(_lib.lib().pcx_comm_unique_id(C.byref(cid)))
        box = [C.string_at(C.addressof(cid), C.sizeof(cid)) if self.rank == 0 else None]  # all 128 bytes
        dist.broadcast_object_list(box, src=0)
        C.memmove(C.addressof(cid), box[0], 128)
        self.device_index = int(device_index)
        self._ctx = _lib.new_context(_lib.lib().pcx_create_rank(self.device_index, self.world, self.rank,
                                                                C.byref(cid)), "pcx_create_rank")


class ThreadGroup:
    """Shared exchange of :class:`ThreadComm` ranks (pcx_group)."""

    def __init__(self, world):
        self.world = int(world)
        self.handle = _lib.new_context(_lib.lib().pcx_group_create(self.world), "pcx_group_create")
        self.barrier = threading.Barrier(self.world)

    def __del__(self):
        try:
            _lib.lib().pcx_group_destroy(self.handle)
        except Exception:  # pragma: no cover
            pass


class ThreadComm(_OwnedCtx):
    """Virtual rank ``rank`` of a :class:`ThreadGroup` (one thread per rank, any device)."""

    def __init__(self, group, rank):
        self.g = group
        self.world, self.rank = group.world, int(rank)
        self._dev = None

    def context(self, device_index):
        if self._ctx is None or self._dev != device_index:
            self.close()
            self._ctx = _lib.new_context(_lib.lib().pcx_create_grouped(int(device_index), self.g.handle, self.rank),
                                         "pcx_create_grouped")
            self._dev = device_index
        return self._ctx

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass


class CallbackComm(_OwnedCtx):
    """torch.distributed (any backend, CPU tensors) behind libpcx's callback exchange."""

    def __init__(self, world, rank, group=None):
        import torch
        import torch.distributed as dist

        self.world, self.rank, self.group = int(world), int(rank), group
        self._dev = None

        def allreduce(user, buf, count, dtype, op):
            try:
                a = np.ctypeslib.as_array(C.cast(buf, C.POINTER(C.c_double if dtype == _abi.F64 else C.c_uint64)),
                                          shape=(count,))
                if dtype == _abi.F64:
                    t = torch.from_numpy(a)
                    o = {_abi.RED_SUM: dist.ReduceOp.SUM, _abi.RED_MIN: dist.ReduceOp.MIN,
                         _abi.RED_MAX: dist.ReduceOp.MAX}[op]
                    dist.all_reduce(t, op=o, group=self.group)
                else:  # u64: gather all ranks and reduce exactly on the host (torch has no uint64 reduce)
                    t = torch.from_numpy(a.view(np.int64).copy())
                    parts = [torch.empty_like(t) for _ in range(self.world)]
                    dist.all_gather(parts, t, group=self.group)
                    st = np.stack([p.numpy().view(np.uint64) for p in parts])
                    r = st.sum(axis=0, dtype=np.uint64) if op == _abi.RED_SUM else (
                        st.min(axis=0) if op == _abi.RED_MIN else st.max(axis=0))
                    a[:] = r
                return 0
            except Exception:  # pragma: no cover
                return 1

        def allgather(user, send, recv, nbytes):
            try:
                s = np.ctypeslib.as_array(C.cast(send, C.POINTER(C.c_uint8)), shape=(nbytes,))
                r = np.ctypeslib.as_array(C.cast(recv, C.POINTER(C.c_uint8)), shape=(nbytes * self.world,))
                t = torch.from_numpy(s.copy())
                parts = [torch.empty_like(t) for _ in range(self.world)]
                dist.all_gather(parts, t, group=self.group)
                for w, p in enumerate(parts):
                    r[w * nbytes:(w + 1) * nbytes] = p.numpy()
                return 0
            except Exception:  # pragma: no cover
                return 1

        self._cbs = (_abi.ALLREDUCE_CB(allreduce), _abi.ALLGATHER_CB(allgather))  # keep alive
        self._ops = _abi.CommOps(None, self._cbs[0], self._cbs[1])

    def context(self, device_index):
        if self._ctx is None or self._dev != device_index:
            self.close()
            self._ctx = _lib.new_context(_lib.lib().pcx_create_custom(int(device_index), self.world, self.rank,
                                                                      C.byref(self._ops)), "pcx_create_custom")
            self._dev = device_index
        return self._ctx


def progress(comm, device_index):
    """Where the single-matrix call running on ``comm``'s context is (callable from another
    thread while it runs): ``(stage name or None, host_waiting)`` (pcx_ctx_progress)."""
    st, wt = C.c_int(-1), C.c_int(0)
    _lib.check(_lib.lib().pcx_ctx_progress(comm.context(device_index), C.byref(st), C.byref(wt)))
    name = _lib.lib().pcx_stage_name(st.value).decode() if st.value >= 0 else None
    return name, bool(wt.value)


def shard_rows(N, world, rank):
    """Contiguous row block of ``rank``: (offset, count); remainder rows go to the first ranks."""
    base, rem = divmod(int(N), int(world))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def release_workspace(comm=None, device=None):
    """Free the single-matrix scratch cached in this thread's context (tens of GB at C5)."""
    t = _device.torch()
    comm = comm or Comm()
    dev = t.device(device) if device is not None else t.device("cuda", t.cuda.current_device())
    _lib.check(_lib.lib().pcx_release_workspace(comm.context(dev.index)))


clear_workspace_cache = release_workspace


def _bounds(scaled, lo, hi, conv):
    if scaled is None:
        return None, None, None
    return conv(scaled, np.uint8), conv(lo, np.float64), conv(hi, np.float64)


def _problem(n_rows, E, N, r0, P, rep, sc, lo, hi, catch_tolerance, alpha, int_dtype, algorithm, max_components,
             variance_threshold, aux, mem_kind, cluster=None):
    alg = _abi.ALGORITHMS.get(algorithm)
    if alg is None:
        raise NotImplementedError("algorithm %r is not on the GPU path" % (algorithm,))
    if alg == _abi.ALG_COKURTOSIS and aux is None:
        raise ValueError("cokurtosis needs aux_scores (this rank's rows of aux['cokurt'])")
    mc = int(max_components) if E >= int(max_components) else E  # __init__.py:134-137
    cl = cluster or {}
    kinit = cl.get("kmeans_init")  # host int32 [restarts][k], kept alive by the caller
    k, restarts = (int(kinit.shape[1]), int(kinit.shape[0])) if kinit is not None else (0, 0)
    return _abi.Problem(n_rows, E, N, r0, P, rep, sc, lo, hi, float(catch_tolerance), float(alpha),
                        int(bool(int_dtype)), alg, mc, mem_kind, float(variance_threshold), aux,
                        float(cl.get("hierarchy_threshold", 0.5)), float(cl.get("cluster_threshold", 0.0)), k,
                        restarts, None if kinit is None else kinit.ctypes.data)


def _shape_args(n_rows, comm, n_total, row_offset):
    if comm.world == 1:
        return n_rows, 0
    if n_total is None or row_offset is None:
        raise ValueError("a sharded call needs n_total and row_offset (see shard_rows)")
    return int(n_total), int(row_offset)


def consensus_matrix(reports, reputation=None, scaled=None, lo=None, hi=None, catch_tolerance=0.1,
                     alpha=0.1, int_dtype=False, algorithm="PCA", comm=None, n_total=None,
                     row_offset=None, device=None, matrices=False, profile=None, max_components=5,
                     variance_threshold=0.9, aux_scores=None, original_inplace=False):
    """Consensus of one report matrix on the GPU(s), device-resident (torch tensors).

    reports:    this rank's rows, (n_rows, E) float64 (torch tensor on the GPU, or numpy)
    reputation: RAW reputation of ALL N reporters (every rank passes the full vector), or None
    scaled/lo/hi: event bounds (E,), or None (every event binary)
    comm:       :class:`Comm` (default: single GPU); sharded calls also give n_total, row_offset
    matrices:   also return this rank's rescaled ("original") and filled reports
    original_inplace: with ``matrices``, ``original`` IS ``reports`` rescaled in place -- the
                reference's own aliasing (__init__.py:121, 266-269, 584) -- instead of a new
                tensor: only the scaled columns are written.  ``reports`` must then be a
                contiguous float64 tensor on ``device`` (it is modified)
    profile:    optional dict; receives per-stage device milliseconds (HIP events on the
                launching stream, pcx_profile_read) under the stage names of libpcx
    algorithm:  "PCA", "absolute", "big-five" (max_components, capped at E), "fixed-variance"
                (variance_threshold), "cokurtosis" (aux_scores: this rank's rows of aux["cokurt"])

    Returns (events, agents, info): event-level tensors (identical on every rank),
    this rank's per-reporter tensors, and a dict of scalars/diagnostics.
    """
    t = _device.require_gpu()
    comm = comm or Comm()
    dev = t.device(device) if device is not None else t.device("cuda", t.cuda.current_device())
    R = _device.as_device(reports, t.float64, dev)
    n_rows, E = R.shape
    N, r0 = _shape_args(n_rows, comm, n_total, row_offset)
    rep = _device.as_device(reputation, t.float64, dev)
    if rep is not None and rep.numel() != N:
        raise ValueError("reputation must hold all N=%d reporters (got %d)" % (N, rep.numel()))
    conv = lambda a, dt: _device.as_device(a, {np.uint8: t.uint8, np.float64: t.float64}[dt], dev)
    sc, lo_, hi_ = _bounds(scaled, lo, hi, conv)
    aux = None if aux_scores is None else _device.as_device(aux_scores, t.float64, dev).reshape(-1)
    if aux is not None and aux.numel() != n_rows:
        raise ValueError("aux_scores must hold this rank's %d rows" % n_rows)
    P = _device.ptr
    prob = _problem(n_rows, E, N, r0, P(R), P(rep), P(sc), P(lo_), P(hi_), catch_tolerance, alpha, int_dtype,
                    algorithm, max_components, variance_threshold, P(aux), _abi.MEM_DEVICE)
    z = lambda *shape: t.empty(shape, dtype=t.float64, device=dev)
    out = {k: z(n_rows) for k in _abi.MAT_OUTPUT_AGENTS}
    out.update({k: z(E) for k in _abi.MAT_OUTPUT_EVENTS})
    if matrices:
        if original_inplace:
            if not (isinstance(reports, t.Tensor) and reports.data_ptr() == R.data_ptr()):
                raise ValueError("original_inplace needs the reports as a contiguous float64 tensor on the device")
            out["original"], out["filled"] = R, z(n_rows, E)
        else:
            out["original"], out["filled"] = z(n_rows, E), z(n_rows, E)
    res = _abi.Result()
    for k, v in out.items():
        setattr(res, k, v.data_ptr())
    lib = _lib.lib()
    h = _lib.bind_stream(dev.index, _device.current_stream_handle(dev), comm.context(dev.index))
    if profile is not None:
        _lib.check(lib.pcx_profile_enable(h, 1))
    _lib.check(lib.pcx_consensus_f64(h, C.byref(prob), C.byref(res)))
    if profile is not None:
        ms = (C.c_double * _abi.NSTAGES)()
        _lib.check(lib.pcx_profile_read(h, ms))
        _lib.check(lib.pcx_profile_enable(h, 0))
        for k in range(_abi.NSTAGES):
            if ms[k] > 0:
                name = "M_" + lib.pcx_stage_name(k).decode()
                profile[name] = profile.get(name, 0.0) + ms[k]
    events = {k: out[k] for k in _abi.MAT_OUTPUT_EVENTS}
    agents = {k: out[k] for k in _abi.MAT_OUTPUT_AGENTS}
    for k in ("original", "filled"):
        if k in out:
            agents[k] = out[k]
    meta = _meta(res, algorithm)
    meta["inputs"] = (R, rep, sc, lo_, hi_)
    return events, agents, meta


def _meta(res, algorithm):
    return {"participation": res.participation, "avg_certainty": res.avg_certainty,
            "branch": int(res.branch), "pi_iters": int(res.pi_iters), "flags": int(res.flags),
            "components": int(res.components), "n_hard": int(res.n_hard), "sel_passes": int(res.sel_passes),
            "comm_bytes": float(res.comm_bytes), "grid_events": int(res.grid_events),
            "mixed_int8": int(res.mixed_int8), "cov_guard": int(res.cov_guard),
            "cov_guard_cols": int(res.cov_guard_cols), "cov_err_bound": float(res.cov_err_bound)}


# ---------------------------------------------------------------- host-memory entry points
def _host_call(fn_name, reports, reputation, scaled, lo, hi, device_index, outputs, catch_tolerance=0.1,
               alpha=0.1, int_dtype=False, algorithm="PCA", max_components=5, variance_threshold=0.9,
               aux_scores=None, extra=(), devices=None, hierarchy_threshold=0.5, cluster_threshold=None,
               kmeans_init=None, original_inplace=False):
    """Call a single-matrix entry point with numpy inputs / outputs (PCX_MEM_HOST: libpcx
    copies in and out).  ``outputs``: {result field: shape}.  ``devices``: a list of device
    ids -- libpcx shards the rows over them (pcx_create_devices), else one GPU."""
    _device.require_gpu()
    R = np.ascontiguousarray(reports, dtype=np.float64)
    n_rows, E = R.shape
    keep = [R]
    if original_inplace and R is not reports:
        raise ValueError("original_inplace needs the reports as a C-contiguous float64 ndarray")

    def ptr(a, dt):
        if a is None:
            return None
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a.ctypes.data

    sc, lo_, hi_ = (None, None, None) if scaled is None else (ptr(scaled, np.uint8), ptr(lo, np.float64),
                                                              ptr(hi, np.float64))
    cluster = None
    if algorithm in _abi.CLUSTER_ALGORITHMS:
        if algorithm == "k-means" and kmeans_init is None:
            from .batched import kmeans_draws

            kmeans_init = kmeans_draws(1, n_rows)[0]  # numpy's global RandomState, as scipy draws (:397)
        kinit = None if kmeans_init is None else np.ascontiguousarray(kmeans_init, dtype=np.int32)
        keep.append(kinit)
        cluster = {"hierarchy_threshold": hierarchy_threshold, "kmeans_init": kinit,
                   "cluster_threshold": 0.0 if cluster_threshold is None else cluster_threshold}
    prob = _problem(n_rows, E, n_rows, 0, R.ctypes.data, ptr(reputation, np.float64), sc, lo_, hi_,
                    catch_tolerance, alpha, int_dtype, algorithm, max_components, variance_threshold,
                    ptr(aux_scores, np.float64), _abi.MEM_HOST, cluster)
    res = _abi.Result()
    outs = {}
    for k, shape in outputs.items():
        # original_inplace: `original` is the reports array itself (pcx_result.original aliasing
        # pcx_problem.reports: the library rescales its scaled columns in place)
        outs[k] = R if (k == "original" and original_inplace) else np.empty(shape, dtype=np.float64)
        setattr(res, k, outs[k].ctypes.data)
    h = _lib.context(device_index) if devices is None else _lib.devices_context(devices)
    rc = getattr(_lib.lib(), fn_name)(h, C.byref(prob), *extra, C.byref(res))
    if rc != 0 and devices is not None and not _lib.lib().pcx_ctx_usable(h):
        # a rank failed mid-call and aborted every other rank's communicator: the context is
        # unusable, so the next call makes a fresh one.  An argument error caught before any
        # exchange leaves it usable (no costly ncclCommInitAll again).
        err = _lib.PcxError("libpcx error %d: %s" % (rc, _lib.lib().pcx_last_error().decode(errors="replace")))
        _lib.drop_devices_context(devices)
        raise err
    _lib.check(rc)
    return outs, _meta(res, algorithm)


def consensus_host(reports, reputation=None, scaled=None, lo=None, hi=None, device_index=0, matrices=True, **kw):
    """Whole consensus from host arrays (the drop-in Oracle's large-matrix path)."""
    n, E = np.shape(reports)
    shapes = {k: (n,) for k in _abi.MAT_OUTPUT_AGENTS}
    shapes.update({k: (E,) for k in _abi.MAT_OUTPUT_EVENTS})
    if matrices:
        shapes.update(original=(n, E), filled=(n, E))
    return _host_call("pcx_consensus_f64", reports, reputation, scaled, lo, hi, device_index, shapes, **kw)


def interpolate_host(reports, reputation=None, scaled=None, lo=None, hi=None, device_index=0, **kw):
    n, E = np.shape(reports)
    return _host_call("pcx_interpolate_f64", reports, reputation, scaled, lo, hi, device_index,
                      {"original": (n, E), "filled": (n, E)}, **kw)


def wpca_host(filled, reputation=None, device_index=0, **kw):
    n, E = np.shape(filled)
    return _host_call("pcx_wpca_f64", filled, reputation, None, None, None, device_index,
                      {"weighted_mean": (E,), "covariance": (E, E), "adj_first_loadings": (E,), "scores": (n,)},
                      **kw)


def lie_detector_host(filled, reputation=None, device_index=0, **kw):
    n, E = np.shape(filled)
    return _host_call("pcx_lie_detector_f64", filled, reputation, None, None, None, device_index,
                      {"adj_first_loadings": (E,), "scores": (n,), "old_rep": (n,), "this_rep": (n,),
                       "smooth_rep": (n,)}, **kw)


def nonconformity_host(scores, filled, reputation=None, rank_rule=True, device_index=0, **kw):
    n, E = np.shape(filled)
    s = np.ascontiguousarray(np.asarray(scores, dtype=np.float64).ravel())
    if s.size != n:
        raise ValueError("scores must hold one value per reporter")
    nc = np.empty(n, dtype=np.float64)
    outs, meta = _host_call("pcx_nonconformity_f64", filled, reputation, None, None, None, device_index, {},
                            extra=(s.ctypes.data, int(bool(rank_rule)), nc.ctypes.data), **kw)
    return nc, meta
