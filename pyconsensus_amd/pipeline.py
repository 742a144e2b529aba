"""Single-matrix consensus pipeline: stage sequencing, workspace and cross-rank exchange.

One N x E report matrix, sharded by reporter rows over ``comm.world`` GPUs (one
process per GPU; ``world == 1`` on a single GPU).  Each stage is one call of
``pcx_mat_stage`` (include/pcx.h, kernels in csrc/pcx_matrix.hip).  Stages that
produce per-rank partial sums write slot ``[rank]`` of a ``[world, ...]`` buffer;
:class:`Comm` sums those buffers over ranks (RCCL all-reduce via torch.distributed)
and the next stage combines the ranks in rank order, so every rank ends with the
same event-level results whatever the collective's internal order.

Reference (pyconsensus/__init__.py): interpolate :260-313, wpca :315-339,
nonconformity_rank :487-500, lie_detector tail :459-473, consensus :502-611.
"""
from __future__ import annotations

import ctypes as C
import threading

from . import _abi, _device, _lib

COL_THREADS = 256
COV_TILE = 128
COV_STAGE = 16


class Comm:
    """Cross-rank exchange used between stages.  world == 1: every call is a no-op."""

    def __init__(self, world=1, rank=0, group=None):
        self.world = int(world)
        self.rank = int(rank)
        self.group = group

    def all_reduce_sum(self, t):
        if self.world == 1:
            return
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    # [world, ...] slot buffers: other ranks' slots are zeroed before the stage writes
    # its own, so the SUM leaves every slot with exactly one contribution.
    def clear_slots(self, buf, sl=()):
        if self.world == 1:
            return
        buf[(slice(None),) + tuple(sl)] = 0

    def reduce_slots(self, buf, sl=()):
        if self.world == 1:
            return
        idx = (slice(None),) + tuple(sl)
        t = buf[idx].contiguous()
        self.all_reduce_sum(t)
        buf[idx] = t

    @staticmethod
    def from_env():
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return Comm(dist.get_world_size(), dist.get_rank())
        return Comm()


class ThreadGroup:
    """Shared state of :class:`ThreadComm` ranks (one thread per virtual shard)."""

    def __init__(self, world):
        self.world = int(world)
        self.barrier = threading.Barrier(self.world)
        self.bufs = [None] * self.world
        self.result = None


class ThreadComm(Comm):
    """Virtual shards in ONE process (one thread per rank, same or different GPUs):
    exercises the sharded stages and the slot reductions without a multi-GPU node."""

    def __init__(self, group, rank):
        super().__init__(group.world, rank)
        self.g = group

    def all_reduce_sum(self, t):
        torch = _device.torch()
        torch.cuda.synchronize()
        self.g.bufs[self.rank] = t
        self.g.barrier.wait()
        if self.rank == 0:
            acc = self.g.bufs[0].clone()
            for r in range(1, self.world):
                acc += self.g.bufs[r].to(acc.device)
            torch.cuda.synchronize()
            self.g.result = acc
        self.g.barrier.wait()
        t.copy_(self.g.result.to(t.device))
        torch.cuda.synchronize()
        self.g.barrier.wait()


def shard_rows(N, world, rank):
    """Contiguous row block of ``rank``: (offset, count); remainder rows go to the first ranks."""
    base, rem = divmod(int(N), int(world))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


class MatWorkspace:
    """Device buffers of one rank for an (n_rows x E) shard of an N x E matrix."""

    def __init__(self, n_rows, E, n_scaled, world, device):
        t = _device.torch()
        f64, u64 = t.float64, t.int64
        self.device = device
        self.n_rows, self.E, self.n_scaled, self.world = n_rows, E, n_scaled, world
        ceb = (E + COL_THREADS - 1) // COL_THREADS
        # enough row chunks to give ~2048 column-pass blocks, at least 32 rows each
        self.col_blocks = max(1, min(max(1, 2048 // ceb), (n_rows + 31) // 32, 4096))
        nb = (E + COV_TILE - 1) // COV_TILE
        self.cov_tiles = nb * (nb + 1) // 2
        # covariance operand wcd, materialised [wcd_rows][wcd_ld] (16-row stages, 128-col tiles)
        self.wcd_rows = (n_rows + COV_STAGE - 1) // COV_STAGE * COV_STAGE
        self.wcd_ld = nb * COV_TILE
        # row slices: >= ~16 workgroups per CU slot (3 per CU), each slice >= 8 stages
        stages = self.wcd_rows // COV_STAGE
        ks = -(-16 * 3 * 256 // self.cov_tiles)
        self.cov_kslices = max(1, min(32, ks, stages // 8 if stages >= 8 else 1))
        z = lambda *shape, dt=f64: t.zeros(shape, dtype=dt, device=device)
        self.rep = z(n_rows)
        self.tok = z(n_rows)
        self.T = z(max(1, n_scaled), n_rows)
        self.part = z(self.col_blocks, E, 8, 2)
        self.mpart = z(self.col_blocks, E, 4)
        self.cstat = z(world, E, 16, 2)
        self.cmax = z(world, E, 4)
        self.scal = z(world, 16, 2)
        self.spart = z(4096, 4, 2)
        self.ev = z(16, E)
        self.cslab = z(self.cov_kslices, E, E)
        self.wcd = t.empty((self.wcd_rows, self.wcd_ld), dtype=f64, device=device)
        self.tokp = t.empty((self.wcd_rows + 64,), dtype=f64, device=device)
        self.rowpart = t.empty(((self.wcd_ld + 511) // 512, self.wcd_rows, 2), dtype=t.int32, device=device)
        self.C = z(E, E)
        self.Mw = z(2 * E * E + 8 * E + 64)  # power-iteration matrices; PCX_M_EIG scratch
        self.pvec = z(4, E + 64)
        self.rowv = z(6, n_rows)
        self.rowstat = z(n_rows, 2, dt=t.int32)
        self.skey = z(world, 4, dt=u64)
        self.info = z(16, dt=u64)
        S = max(1, n_scaled)
        self.sel_sum = z(world, S, 256, 4, dt=u64)
        self.sel_min = z(world, S, 256, 2, dt=u64)
        self.sel_max = z(world, S, 256, dt=u64)
        self.sel_state = z(S, 16, dt=u64)
        self.sel_val = z(world, S, 4)

    # buffers every stage writes in full before reading: not re-zeroed on reuse
    _NO_RESET = ("wcd", "tokp", "rowpart", "T", "cslab", "C", "Mw")

    def reset(self):
        """Zero the scratch for another consensus of the same shape (reuse across calls)."""
        for name, v in vars(self).items():
            if name not in self._NO_RESET and hasattr(v, "zero_"):
                v.zero_()

    def new_outputs(self):
        """Fresh result tensors for one call (results outlive the reused scratch)."""
        t = _device.torch()
        z = lambda n: t.zeros(n, dtype=t.float64, device=self.device)
        out = {k: z(self.n_rows) for k in _abi.MAT_OUTPUT_AGENTS}
        out.update({k: z(self.E) for k in _abi.MAT_OUTPUT_EVENTS})
        return out, z(4)


_WS_CACHE = {}       # (n_rows, E, n_scaled, world, rank, device) -> MatWorkspace
_WS_CACHE_MAX = 4
_WS_LOCK = threading.Lock()


def _workspace(n_rows, E, n_scaled, world, rank, device):
    """Scratch of one rank, reused across calls of the same shape (allocating and first-touching
    tens of GB per call costs ~0.1 s at C5 sizes).  Least recently used entries are dropped."""
    key = (int(n_rows), int(E), int(n_scaled), int(world), int(rank), str(device))
    with _WS_LOCK:
        ws = _WS_CACHE.pop(key, None)
        if ws is not None and getattr(ws, "_busy", False):
            ws = None  # the same key in use on another thread: build a private one
        if ws is None:
            while len(_WS_CACHE) >= _WS_CACHE_MAX:
                _WS_CACHE.pop(next(iter(_WS_CACHE)))
            ws = MatWorkspace(n_rows, E, n_scaled, world, device)
        else:
            ws.reset()
        ws._busy = True
        _WS_CACHE[key] = ws
    return ws


def clear_workspace_cache():
    """Release every cached single-matrix workspace (device memory returns to torch's allocator)."""
    with _WS_LOCK:
        _WS_CACHE.clear()



def consensus_matrix(reports, reputation=None, scaled=None, lo=None, hi=None, catch_tolerance=0.1,
                     alpha=0.1, int_dtype=False, algorithm="PCA", comm=None, n_total=None,
                     row_offset=None, device=None, matrices=False, profile=None, max_components=5,
                     variance_threshold=0.9, aux_scores=None):
    """Consensus of one report matrix on the GPU(s).

    reports:    this rank's rows, (n_rows, E) float64 (torch tensor on the GPU, or numpy)
    reputation: RAW reputation of ALL N reporters (every rank passes the full vector), or None
    scaled/lo/hi: event bounds (E,), or None (every event binary)
    comm:       :class:`Comm` (default: single GPU)
    matrices:   also return this rank's rescaled ("original") and filled reports
    profile:    optional dict; receives per-stage device milliseconds (HIP events on the
                launching stream) under the stage names of include/pcx.h
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
    N = int(n_total) if n_total is not None else n_rows * comm.world
    r0 = int(row_offset) if row_offset is not None else comm.rank * n_rows
    rep = _device.as_device(reputation, t.float64, dev)
    if rep is not None and rep.numel() != N:
        raise ValueError("reputation must hold all N=%d reporters (got %d)" % (N, rep.numel()))
    sc = lo_ = hi_ = None
    scols = sidx = None
    n_scaled = 0
    if scaled is not None:
        sc = _device.as_device(scaled, t.uint8, dev)
        lo_ = _device.as_device(lo, t.float64, dev)
        hi_ = _device.as_device(hi, t.float64, dev)
        scl = sc.to("cpu").bool()
        cols = t.nonzero(scl).flatten().to(t.int32)
        n_scaled = int(cols.numel())
        idx = t.full((E,), -1, dtype=t.int32)
        idx[cols.long()] = t.arange(n_scaled, dtype=t.int32)
        scols = cols.to(dev)
        sidx = idx.to(dev)
    alg = _abi.ALGORITHMS.get(algorithm)
    if alg is None or algorithm in _abi.CLUSTER_ALGORITHMS:
        raise NotImplementedError("algorithm %r is not on the single-matrix path" % (algorithm,))
    aux = None
    if alg == _abi.ALG_COKURTOSIS:
        if aux_scores is None:
            raise ValueError("cokurtosis needs aux_scores (this rank's rows of aux['cokurt'])")
        aux = _device.as_device(aux_scores, t.float64, dev).reshape(-1)
        if aux.numel() != n_rows:
            raise ValueError("aux_scores must hold this rank's %d rows" % n_rows)
    algo = (alg, int(max_components) if E >= int(max_components) else E, float(variance_threshold), aux)

    ws = _workspace(n_rows, E, n_scaled, comm.world, comm.rank, dev)
    try:
        return _run(ws, R, rep, sc, lo_, hi_, scols, sidx, n_scaled, N, r0, algo, comm, dev, catch_tolerance,
                    alpha, int_dtype, matrices, profile)
    finally:
        ws._busy = False


def _run(ws, R, rep, sc, lo_, hi_, scols, sidx, n_scaled, N, r0, algo, comm, dev, catch_tolerance, alpha,
         int_dtype, matrices, profile):
    t = _device.torch()
    alg, max_components, variance_threshold, aux = algo
    n_rows, E = R.shape
    out, scalars = ws.new_outputs()
    m = _abi.Mat()
    m.n_rows, m.n_events, m.n_total, m.row_offset = n_rows, E, N, r0
    m.world, m.rank, m.int_dtype, m.algorithm = comm.world, comm.rank, int(bool(int_dtype)), alg
    m.catch_tolerance, m.alpha = float(catch_tolerance), float(alpha)
    m.n_scaled, m.sel_phase, m.col_blocks = n_scaled, 1, ws.col_blocks
    m.cov_tiles, m.cov_kslices = ws.cov_tiles, ws.cov_kslices
    m.wcd_rows, m.wcd_ld = ws.wcd_rows, ws.wcd_ld
    m.max_components, m.components, m.variance_threshold = max_components, -1, variance_threshold
    m.aux_scores = _device.ptr(aux)
    P = _device.ptr
    m.reports, m.scaled, m.lo, m.hi, m.rep_raw = P(R), P(sc), P(lo_), P(hi_), P(rep)
    m.scaled_cols, m.scaled_index = P(scols), P(sidx)
    for name in ("wcd", "tokp", "rowpart", "rep", "tok", "T", "part", "mpart", "cstat", "cmax", "scal", "spart", "ev", "cslab", "C",
                 "Mw", "pvec", "rowv", "rowstat", "skey", "info", "sel_sum", "sel_min", "sel_max", "sel_state",
                 "sel_val"):
        setattr(m, name, P(getattr(ws, name)))
    for k, v in out.items():
        setattr(m, k, P(v))
    m.scalars = P(scalars)
    mats = {}
    if matrices:
        mats = {"original": t.empty((n_rows, E), dtype=t.float64, device=dev),
                "filled": t.empty((n_rows, E), dtype=t.float64, device=dev)}
        m.original, m.filled = P(mats["original"]), P(mats["filled"])

    h = _lib.bind_stream(dev.index, _device.current_stream_handle(dev))
    lib = _lib.lib()

    names = {v: k for k, v in vars(_abi).items() if k.startswith("M_") and isinstance(v, int)}
    events = []

    def stage(s):
        if profile is not None:
            e0 = t.cuda.Event(enable_timing=True)
            e0.record()
        _lib.check(lib.pcx_mat_stage(h, C.byref(m), int(s)))
        if profile is not None:
            e1 = t.cuda.Event(enable_timing=True)
            e1.record()
            events.append((names.get(int(s), str(s)), e0, e1))

    S = slice
    # a1: reputation, tokens (__init__.py:138-146)
    comm.clear_slots(ws.scal, (S(0, 2),))
    stage(_abi.M_REPUTATION)
    comm.reduce_slots(ws.scal, (S(0, 2),))
    # a2/a3: rescale + NA + present sums (:266-299)
    comm.clear_slots(ws.cstat, (S(None), S(0, 4)))
    comm.clear_slots(ws.cmax)
    stage(_abi.M_COLSTATS)
    comm.reduce_slots(ws.cstat, (S(None), S(0, 4)))
    comm.reduce_slots(ws.cmax)
    stage(_abi.M_GUESS)
    _select(stage, m, ws, comm, phase=1)                 # scaled fills: weighted median (:300-303)
    stage(_abi.M_MEAN)
    pca = alg == _abi.ALG_PCA
    wpca = alg in (_abi.ALG_PCA, _abi.ALG_BIG_FIVE, _abi.ALG_FIXED_VARIANCE)
    if wpca:
        # a5: wcd materialised (:322); a6: covariance on fp64 MFMA (:326); a7: power iteration (:330-336)
        stage(_abi.M_WCD)
        stage(_abi.M_COV)
        stage(_abi.M_COV_REDUCE)
        comm.all_reduce_sum(ws.C)
        stage(_abi.M_COV_FINISH)
        stage(_abi.M_POWER)
        if not pca:  # big-five / fixed-variance components (:373-390, :429-451)
            stage(_abi.M_EIG)
    else:
        stage(_abi.M_ZERO_LOADING)
    comm.clear_slots(ws.skey)
    stage(_abi.M_SCORES)
    comm.reduce_slots(ws.skey)
    if alg != _abi.ALG_ABSOLUTE:
        # a8/a9: sign-choice rule (:487-500; the other algorithms: nonconformity, :475-485)
        comm.clear_slots(ws.scal, (S(2, 6),))
        stage(_abi.M_NCSUMS)
        comm.reduce_slots(ws.scal, (S(2, 6),))
        comm.clear_slots(ws.cstat, (S(None), S(4, 6)))
        stage(_abi.M_GEMV2)
        comm.reduce_slots(ws.cstat, (S(None), S(4, 6)))
        stage(_abi.M_DECIDE)
    # a10: reputation update (:460-472)
    comm.clear_slots(ws.scal, (S(6, 8),))
    stage(_abi.M_REPU)
    comm.reduce_slots(ws.scal, (S(6, 8),))
    stage(_abi.M_SMOOTH)
    # a12-a14: outcomes, participation, certainty (:510-546)
    comm.clear_slots(ws.cstat, (S(None), S(6, 14)))
    stage(_abi.M_OUTCOMES)
    comm.reduce_slots(ws.cstat, (S(None), S(6, 14)))
    stage(_abi.M_EVENTS)
    _select(stage, m, ws, comm, phase=2)                 # scaled outcomes: weighted median (:519-523)
    comm.clear_slots(ws.cstat, (S(None), S(14, 16)))
    stage(_abi.M_SCALED_CERT)
    comm.reduce_slots(ws.cstat, (S(None), S(14, 16)))
    stage(_abi.M_FINAL)
    comm.clear_slots(ws.scal, (S(8, 10),))
    stage(_abi.M_ROWSUMS)
    comm.reduce_slots(ws.scal, (S(8, 10),))
    stage(_abi.M_AGENTS)
    if matrices:
        stage(_abi.M_MATRICES)

    info = ws.info.cpu().tolist()
    if profile is not None:
        t.cuda.synchronize(dev)
        for name, e0, e1 in events:
            profile[name] = profile.get(name, 0.0) + e0.elapsed_time(e1)
    scal = scalars.cpu().tolist()
    events = {k: out[k] for k in _abi.MAT_OUTPUT_EVENTS}
    agents = {k: out[k] for k in _abi.MAT_OUTPUT_AGENTS}
    agents.update(mats)
    meta = {"participation": scal[0], "avg_certainty": scal[1],
            "branch": int(info[_abi.INFO_BRANCH]) if alg != _abi.ALG_ABSOLUTE else _abi.BRANCH_NONE,
            "pi_iters": int(info[_abi.INFO_PI_ITERS]), "flags": int(info[_abi.INFO_FLAGS]) if wpca else 0,
            "components": int(m.components),
            "filled_guess": ws.ev[0].clone(), "workspace": ws, "inputs": (R, rep, sc, lo_, hi_)}
    return events, agents, meta


def _select(stage, m, ws, comm, phase):
    """Exact weighted medians of the scaled events (weightedstats semantics)."""
    if m.n_scaled == 0:
        return
    m.sel_phase = phase
    if comm.world == 1 and m.n_rows <= _abi.SEL_EXACT_MAX:
        # small matrices: replay the reference's float walk exactly (ties included)
        stage(_abi.M_SEL_EXACT)
        stage(_abi.M_SEL_FINISH)
        return
    for b in (ws.sel_sum, ws.sel_min, ws.sel_max, ws.sel_val):
        comm.clear_slots(b)
    stage(_abi.M_SEL_INIT)
    for b in (ws.sel_sum, ws.sel_min, ws.sel_max, ws.sel_val):
        comm.reduce_slots(b)
    stage(_abi.M_SEL_START)
    if int(ws.info[_abi.INFO_SEL_ARGMAX].item()):
        comm.clear_slots(ws.sel_val)
        stage(_abi.M_SEL_ARGMAX)
        comm.reduce_slots(ws.sel_val)
        comm.clear_slots(ws.sel_val, (S_ALL, slice(2, 3)))
        stage(_abi.M_SEL_VALUE)
        comm.reduce_slots(ws.sel_val, (S_ALL, slice(2, 3)))
    for _ in range(16):  # <= 8 passes of 8 key bits each
        for b in (ws.sel_sum, ws.sel_min, ws.sel_max):
            comm.clear_slots(b)
        stage(_abi.M_SEL_HIST)
        for b in (ws.sel_sum, ws.sel_min, ws.sel_max):
            comm.reduce_slots(b)
        stage(_abi.M_SEL_STEP)
        if int(ws.info[_abi.INFO_SEL_ACTIVE].item()) == 0:
            break
    stage(_abi.M_SEL_FINISH)


S_ALL = slice(None)
