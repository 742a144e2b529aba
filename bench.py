"""Benchmark of the pyconsensus hot path on MI355X (contract: see DESIGN.md §Measurement).

Headline (BASELINE.json ``metric``): oracle rounds/sec for the batched 50 x 20
regime (config C3: 65,536 independent rounds per GPU per step, one wavefront per
round).  A "step" is one launch of ``batched_round_kernel`` over the resident
65,536-round batch: every round is a complete ``Oracle(...).consensus()``.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

``--gpus N > 1`` with no launcher (WORLD_SIZE unset) starts the second form itself as a
child job before touching the GPU; WORLD_SIZE set and different from ``--gpus`` is an
error (exit 2), so the line's ``n_gpus`` is always the number of ranks that ran.

Rounds are independent, so ranks shard them with no data-path collective
(weak scaling: every rank runs its own 65,536 rounds per step).  Rank 0 prints
ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ROUNDS, N_REP, N_EV = 65536, 50, 20
SEED = 20261015
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def round_bytes(N, E, matrices=True):
    """Algorithmic HBM bytes per round: inputs read once, outputs written once (the whole
    result dict of __init__.py:583-611, including the N x E "original" and "filled")."""
    reads = 8 * N * E + 8 * N + E * (1 + 8 + 8)          # reports, reputation, scaled/lo/hi
    writes = 8 * N * 8 + 8 * E * 9 + 8 * 2 + 4 * 3       # 8 N-vectors, 9 E-vectors, 2 f64 + 3 i32 scalars
    if matrices:
        writes += 2 * 8 * N * E                           # result["original"], result["filled"]
    return reads + writes


def host_threads():
    """The host cores this job may use: the box's share (OMP_NUM_THREADS, 16 per GPU on the
    pool) when set, else every CPU."""
    try:
        return max(1, int(os.environ["OMP_NUM_THREADS"]))
    except (KeyError, ValueError):
        return max(1, os.cpu_count() or 1)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds=12.0):
    """The C oracle (oracle/pcx_oracle_batched.c, a port of the reference algorithm)
    on this host's cores, over a bounded sample of the same workload."""
    from oracle import pcx_oracle_c as OC
    from pyconsensus_amd import synthetic

    threads = host_threads()
    R, sc, lo, hi, rep = synthetic.rounds(4096, N_REP, N_EV, seed=SEED)
    OC.batched(R[:256], sc[:256], lo[:256], hi[:256], rep[:256], threads=threads)  # warm
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        OC.batched(R, sc, lo, hi, rep, threads=threads)
        done += R.shape[0]
    el = time.perf_counter() - t0
    out = {"value": done / el, "unit": "rounds/s", "cores": threads, "kind": "port",
           "sample": "%d rounds of the C3 workload (50x20, seed %d) in %.1f s, C oracle, %d OpenMP threads"
                     % (done, SEED, el, threads),
           "host_cpus": os.cpu_count(), "cpu_model": cpu_model()}
    # SURVEY.md 8(d) asks for the box's whole host; this job may use `threads` of its cores (the
    # pool's share, OMP_NUM_THREADS), so the whole-host figure is an estimate: rounds are
    # independent, so the rate scales with cores at best linearly -- an upper bound, not measured
    out["value_all_host_cpus_linear_bound"] = out["value"] * (os.cpu_count() or threads) / threads
    # the numpy restatement (same per-round structure as the reference) for context
    from oracle.pcx_oracle import OracleCPU
    bl = synthetic.bounds_list
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 3.0:
        OracleCPU(reports=R[n], event_bounds=bl(sc[n], lo[n], hi[n]), reputation=rep[n]).consensus()
        n += 1
    out["numpy_port_rounds_per_s_1core"] = n / (time.perf_counter() - t0)
    return out


FP64_MFMA_PEAK_TFS = 78.6  # MI355X FP64 matrix peak (spec)


def bench_c5(world, rank, dev, steps, warmup, N=1_000_000, E=4096):
    """Config C5: one 1M x 4k report matrix (reputation=None), rows sharded over the
    ranks; end-to-end consensus latency (inputs resident in HBM, outputs left there)."""
    import torch

    from pyconsensus_amd import synthetic
    from pyconsensus_amd.pipeline import Comm, consensus_matrix, shard_rows

    per = 8 // world if 8 % world == 0 else None
    shards = list(range(rank * per, (rank + 1) * per)) if per else None
    off, cnt = shard_rows(N, world, rank)
    if shards is None or cnt * world != N:
        raise ValueError("C5 needs a GPU count dividing 8")
    R, sc, lo, hi, _ = synthetic.matrix_device(N, E, seed=3, n_shards=8, shards=shards, device=dev)
    comm = Comm.from_env(dev.index)  # RCCL inside libpcx for the nccl backend
    _C5_STATE["comm"], _C5_STATE["dev"] = comm, dev.index
    from pyconsensus_amd import _lib
    from pyconsensus_amd.pipeline import RcclComm

    ctx_world = int(_lib.lib().pcx_ctx_world(comm.context(dev.index)))
    if ctx_world != world:
        raise RuntimeError("libpcx context spans %d rank(s), the job %d" % (ctx_world, world))
    comm_info = {"comm": type(comm).__name__, "ctx_world": ctx_world,
                 "rccl_world": ctx_world if isinstance(comm, RcclComm) else 0}

    def run(profile=None, inplace=False):
        return consensus_matrix(R, None, sc, lo, hi, comm=comm, n_total=N, row_offset=off, device=dev,
                                profile=profile, matrices=True, original_inplace=inplace)

    _C5_STATE["phase"] = "warmup"
    for _ in range(warmup):
        run()
    _C5_STATE["phase"] = "timed steps"
    times, prof, step_prof = [], {}, []
    ev = ag = None
    for _ in range(steps):
        ev = ag = None  # drop the last step's 65 GB of outputs first (else a fresh hipMalloc is timed)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        p1 = {}
        ev, ag, meta = run(p1)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            m = torch.tensor([el], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(m, op=torch.distributed.ReduceOp.MAX)
            el = float(m.item())
        times.append(el)
        step_prof.append(p1)
        for k, v in p1.items():
            prof[k] = prof.get(k, 0.0) + v
    prof = {k: v / steps for k, v in prof.items()}
    top = [k for k, _ in sorted(prof.items(), key=lambda kv: -kv[1])[:6]]
    ev = ag = None
    inplace = c5_inplace(world, dev, steps, R, run)
    cov_ms = prof.get("M_COV", float("nan"))
    i8_ms = prof.get("M_COV_I8", float("nan"))
    # unique (j, k<=j) covariance pairs: those with a general event on fp64 MFMA (k_syrk),
    # the grid-grid pairs on int8 MFMA (k_gemm_i8); one multiply-add per pair per row
    # with mixed_int8 the general x grid pairs run on int8 too, as D digit slices of tok w
    # (D = pcx_mixed_digits(), a build parameter): int8 work = grid pairs + D x general x grid
    # per row (the digit pass k_digits is in the stage time, not in the count)
    from pyconsensus_amd import _lib

    # mixed_int8 bit 1: the general x general pairs on int8 as well, digits of tok w against digits
    # of w, the D (D + 1) / 2 digit pairs i + j < D (k_gemm_i8x): no fp64 tiles left
    ng = meta["grid_events"]
    G = E - ng
    mixed = meta.get("mixed_int8", 0)
    gg = bool(mixed & 2)
    digits = int(_lib.lib().pcx_mixed_digits())
    fp_pairs = 0 if gg else G * (G + 1) // 2 + (0 if mixed else G * ng)
    i8_pairs = (ng * (ng + 1) // 2 + (digits * G * ng if mixed else 0) +
                (digits * (digits + 1) // 2 * (G * (G + 1) // 2) if gg else 0))
    cov_flops_rank = 2.0 * cnt * fp_pairs
    i8_ops_rank = 2.0 * cnt * i8_pairs
    tfs = cov_flops_rank / (cov_ms * 1e-3) / 1e12 if cov_ms == cov_ms and fp_pairs else None
    tops = i8_ops_rank / (i8_ms * 1e-3) / 1e12 if i8_ms == i8_ms and i8_pairs else None
    del R
    return {"metric": "1M x 4k consensus latency (every output, original and filled included)", "n_gpus": world,
            **comm_info, "rows_per_gpu": cnt, "events": E,
            "latency_ms": 1e3 * sorted(times)[len(times) // 2], "latency_ms_all": [1e3 * x for x in times],
            "latency_ms_mean": 1e3 * sum(times) / len(times), "warmup_steps": warmup,
            "stage_ms_per_step": [{k: round(p.get(k, 0.0), 3) for k in top} for p in step_prof],
            "branch": meta["branch"], "pi_iters": meta["pi_iters"], "flags": meta["flags"],
            "stage_ms": {k: round(v, 3) for k, v in sorted(prof.items(), key=lambda kv: -kv[1])},
            "roofline_cov": {"bound": "mfma", "kernel": "k_syrk (none when mixed_int8 & 2)", "achieved": tfs,
                             "peak": FP64_MFMA_PEAK_TFS,
                             "unit": "TFLOP/s", "frac": (tfs / FP64_MFMA_PEAK_TFS) if tfs else None,
                             "flops_per_launch": cov_flops_rank, "traffic": load_traffic("k_syrk"),
                             "pairs": ("fp64: pairs inside the general tiles (%d positions; %d grid events on int8; mixed pairs "
                                       "on int8 slices: %s)" % (G, ng, bool(mixed)))},
            "roofline_cov_i8": {"bound": "mfma", "kernel": "k_gemm_i8 (grid + mixed launches) + k_gemm_i8x (general "
                                "pairs, when mixed_int8 & 2) + k_digits",
                                "achieved": tops, "peak": I8_MFMA_PEAK_TOPS,
                                "unit": "TOP/s", "frac": (tops / I8_MFMA_PEAK_TOPS) if tops else None,
                                "ops_per_launch": i8_ops_rank, "mixed_digits": digits,
                                "traffic": _sum_traffic(("k_gemm_i8_grid", "k_gemm_i8_mixed", "k_gemm_i8x", "k_digits"))},
            # the int8 emulation priced as the fp64 covariance it replaces: N E (E + 1) multiply-adds
            # (every unique pair, two flops each) over the M_COV_I8 stage, against the fp64 MFMA peak
            "roofline_cov_fp64_equiv": {"kernel": "M_COV_I8 (the whole covariance on int8 digit products)",
                                        "achieved": (1.0 * cnt * E * (E + 1) / (i8_ms * 1e-3) / 1e12
                                                     if i8_ms == i8_ms and gg else None),
                                        "unit": "TFLOP/s (fp64-equivalent)", "fp64_peak": FP64_MFMA_PEAK_TFS},
            "cov_guard": {"mode": meta.get("cov_guard"), "cols": meta.get("cov_guard_cols"),
                          "err_bound": meta.get("cov_err_bound"),
                          "meaning": "bound on |dC_pq| / sqrt(C_pp C_qq) of the int8 emulation (k_cov_guard); "
                                     "mode 0 = passed (<= 2^-40), 1 = every digit pair recomputed, 2 = fp64"},
            "grid_events": ng, "mixed_int8": mixed, "inplace": inplace,
            "data": "synthetic on-GPU (SURVEY.md 8(d) spec, torch Philox per 125k-row shard, seed 3), "
                    "reputation=None"}


def c5_inplace(world, dev, steps, R, run):
    """The same C5 consensus with result["original"] aliasing the reports: the reference's own
    `original` is the caller's array rescaled in place (__init__.py:121, 266-269, 584; Q2), so libpcx
    rescales the scaled columns in place and writes no copy of the matrix.  Every output is still
    produced.  The step modifies the reports, so they are restored from a device copy before each
    step, outside the timed region."""
    import torch

    R0 = R.clone()
    run(inplace=True)  # warm (the in-place outputs' allocation pattern)
    times, prof = [], {}
    for _ in range(steps):
        R.copy_(R0)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        p1 = {}
        ev, ag, meta = run(p1, inplace=True)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            m = torch.tensor([el], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(m, op=torch.distributed.ReduceOp.MAX)
            el = float(m.item())
        times.append(el)
        for k, v in p1.items():
            prof[k] = prof.get(k, 0.0) + v / steps
        ev = ag = None
    R.copy_(R0)
    del R0
    torch.cuda.empty_cache()
    return {"mode": "result['original'] aliases the reports: scaled columns rescaled in place (Q2), no matrix "
                    "copy; inputs restored from a device copy before each step, outside the timed region",
            "latency_ms": 1e3 * sorted(times)[len(times) // 2], "latency_ms_all": [1e3 * x for x in times],
            "stage_ms": {k: round(v, 3) for k, v in sorted(prof.items(), key=lambda kv: -kv[1])[:8]}}


def bench_medium(dev, B=16384, N=100, E=50, steps=3):
    """Batched rounds above one wavefront: B rounds of 100 x 50 (SURVEY.md 8(d) generator) on the
    workgroup-per-round kernel (csrc/pcx_medium.hip), every output written;
    inputs resident on the device, best of `steps` timed calls."""
    import torch

    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched

    R, sc, lo, hi, rep = synthetic.rounds(B, N, E, seed=3)
    args = [torch.as_tensor(x, device=dev) for x in (R, rep, sc.astype("uint8"), lo, hi)]
    consensus_batched(*args)
    torch.cuda.synchronize(dev)
    best = float("inf")
    for _ in range(steps):
        t0 = time.perf_counter()
        consensus_batched(*args)
        torch.cuda.synchronize(dev)
        best = min(best, time.perf_counter() - t0)
    return {"metric": "oracle rounds/sec (batched %dx%d, one workgroup per round)" % (N, E), "rounds": B,
            "rounds_per_s": B / best, "ms": best * 1e3,
            "data": "synthetic (SURVEY.md 8(d) generator, seed 3), every output written"}


def bench_c4(dev, steps=3, oracle=True):
    """Config C4: one 100k x 1k matrix (seed 2, integer reputations),
    device-resident consensus latency; the host->device copy of the reports timed apart; the
    numpy restatement (the reference's algorithm, OpenBLAS on the host cores) timed beside it on
    the same inputs, and the largest relative difference of smooth_rep against it."""
    import numpy as np
    import torch

    from pyconsensus_amd import synthetic
    from pyconsensus_amd.pipeline import consensus_matrix

    R, sc, lo, hi, rep = synthetic.matrix(100_000, 1000, seed=2)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    Rd = torch.from_numpy(R).to(dev)
    torch.cuda.synchronize(dev)
    h2d = time.perf_counter() - t0
    args = (Rd, torch.from_numpy(rep).to(dev), torch.from_numpy(sc.astype(np.uint8)).to(dev),
            torch.from_numpy(lo).to(dev), torch.from_numpy(hi).to(dev))
    consensus_matrix(*args, device=dev, matrices=True)  # warm (workspace)
    times, prof = [], {}
    for _ in range(steps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        p1 = {}
        ev, ag, meta = consensus_matrix(*args, device=dev, matrices=True, profile=p1)
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t0)
        for k, v in p1.items():
            prof[k] = prof.get(k, 0.0) + v / steps
    out = {"metric": "100k x 1k consensus latency", "latency_ms": 1e3 * sorted(times)[len(times) // 2],
           "stage_ms": {k: round(v, 3) for k, v in sorted(prof.items(), key=lambda kv: -kv[1])},
           "h2d_ms": 1e3 * h2d, "h2d_gbs": R.nbytes / h2d / 1e9, "branch": meta["branch"],
           "n_hard": meta["n_hard"], "sel_passes": meta["sel_passes"],
           "data": "synthetic (SURVEY.md 8(d), seed 2, integer reputations U[1,99])"}
    smooth = ag["smooth_rep"].cpu().numpy()
    del Rd, args, ev, ag
    torch.cuda.empty_cache()
    if oracle:
        from oracle.pcx_oracle import OracleCPU

        t0 = time.perf_counter()
        ref = OracleCPU(reports=R, event_bounds=synthetic.bounds_list(sc, lo, hi), reputation=rep).consensus()
        el = time.perf_counter() - t0
        rs = np.asarray(ref["agents"]["smooth_rep"], dtype=float)
        out["cpu_baseline"] = {"value": el * 1e3, "unit": "ms", "kind": "port", "cores": host_threads(),
                               "sample": "the whole C4 consensus, numpy restatement (oracle/pcx_oracle.py)",
                               "cpu_model": cpu_model()}
        out["smooth_rep_max_rel_diff"] = float(np.max(np.abs(smooth - rs) / np.maximum(np.abs(rs), 1e-300)))
    return out


def bench_cov_fp64(dev, N=1_000_000, E=1024, steps=2):
    """The covariance on fp64 MFMA (k_syrk), measured where it runs: a 1M x 1024 consensus whose
    every event is scaled (no grid events, so no int8 block: the general x general pairs are all of
    C, __init__.py:326).  Inputs generated in HBM (the C5 recipe's scaled columns: clip N(0.6, 0.15)
    of [lo, hi], 10% NA, reputation=None); M_COV is k_syrk alone.  2 N E (E + 1) / 2 flop."""
    import torch

    from pyconsensus_amd.pipeline import consensus_matrix

    g = torch.Generator(device=dev)
    g.manual_seed(11)
    lo = torch.rand(E, generator=g, device=dev, dtype=torch.float64) * -100.0
    hi = lo + 1.0 + 199.0 * torch.rand(E, generator=g, device=dev, dtype=torch.float64)
    z = (0.6 + 0.15 * torch.randn((N, E), generator=g, device=dev, dtype=torch.float64)).clamp_(0.001, 1.0)
    R = lo + (hi - lo) * z
    del z
    R[torch.rand((N, E), generator=g, device=dev) < 0.1] = float("nan")
    sc = torch.ones(E, dtype=torch.uint8, device=dev)
    consensus_matrix(R, None, sc, lo, hi, device=dev, matrices=False)
    ms = []
    meta = None
    for _ in range(steps):
        p1 = {}
        _, _, meta = consensus_matrix(R, None, sc, lo, hi, device=dev, matrices=False, profile=p1)
        ms.append(p1.get("M_COV", float("nan")))
    del R
    torch.cuda.empty_cache()
    cov_ms = sorted(ms)[len(ms) // 2]
    flops = 2.0 * N * E * (E + 1) / 2
    tfs = flops / (cov_ms * 1e-3) / 1e12
    return {"kernel": "k_syrk (fp64 MFMA 16x16x4, 128 x 128 tiles, split-K)", "rows": N, "events": E,
            "m_cov_ms": cov_ms, "achieved": tfs, "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
            "frac": tfs / FP64_MFMA_PEAK_TFS, "flops_per_launch": flops, "mixed_int8": meta["mixed_int8"],
            "grid_events": meta["grid_events"],
            "data": "synthetic on-GPU, every event scaled (no int8 block), 10% NA, reputation=None"}


# config C1: README.rst:28-45 (the reference's own example; scaled + binary events)
README_REPORTS = [[0.2, 0.7, 1, 1], [0.3, 0.5, 1, 1], [0.1, 0.7, 1, 1], [0.5, 0.7, 2, 1], [0.1, 0.2, 2, 2],
                  [0.1, 0.2, 2, 2]]
README_REPUTATION = [1, 2, 10, 9, 4, 2]
README_BOUNDS = [{"scaled": True, "min": 0.1, "max": 0.5}, {"scaled": True, "min": 0.2, "max": 0.7},
                 {"scaled": False, "min": 1, "max": 2}, {"scaled": False, "min": 1, "max": 2}]


def bench_dropin(dev, which, calls, oracle=True):
    """Configs C1 / C2 through the drop-in exactly as an unchanged caller of the reference runs them:
    ``Oracle(reports=<host lists / numpy>, reputation=..., event_bounds=...).consensus()`` per call,
    nothing cached across calls but libpcx's context.  Median per-call latency, the constructor and
    the host-side split (Oracle.last_info["timing_ms"]: argument preparation, the GPU call, the copy
    back, the result dict), for C2 the libpcx per-stage device times of one profiled call, and the
    numpy restatement of the same call timed beside it."""
    import numpy as np

    from pyconsensus_amd import Oracle, _abi, _lib, synthetic

    if which == "c1":
        mk = lambda: dict(reports=[list(r) for r in README_REPORTS], reputation=list(README_REPUTATION),
                          event_bounds=[dict(b) for b in README_BOUNDS])
        desc = "README.rst:28-45 example, 6 reporters x 4 events (2 scaled), host lists"
    else:
        R, sc, lo, hi, rep = synthetic.matrix(1000, 100, seed=1)
        b = synthetic.bounds_list(sc, lo, hi)
        mk = lambda: dict(reports=R.copy(), reputation=rep, event_bounds=b)
        desc = "1k x 100, 10% NA, 25% scaled, integer reputations (SURVEY.md 8(d), seed 1), numpy arrays"
    for _ in range(5):
        Oracle(**mk()).consensus()
    tot, ctor, split = [], [], []
    for _ in range(calls):
        a = mk()  # (the caller's own data; a float64 array is rescaled in place, Q2)
        t0 = time.perf_counter()
        o = Oracle(**a)
        t1 = time.perf_counter()
        o.consensus()
        t2 = time.perf_counter()
        tot.append(t2 - t0)
        ctor.append(t1 - t0)
        split.append(o.last_info["timing_ms"])
    med = lambda v: sorted(v)[len(v) // 2]
    out = {"metric": "drop-in Oracle(...).consensus() per-call latency (%s)" % which.upper(), "calls": calls,
           "latency_ms": 1e3 * med(tot), "latency_ms_min": 1e3 * min(tot), "path": o.last_info["path"],
           "split_ms": {"constructor": 1e3 * med(ctor), **{k: med([d[k] for d in split]) for k in split[0]}},
           "data": desc}
    if o.last_info["path"] == "matrix":  # libpcx's own per-stage device time of one call
        h = _lib.context(o._device_index())
        _lib.lib().pcx_profile_enable(h, 1)
        Oracle(**mk()).consensus()
        import ctypes as C

        ms = (C.c_double * _abi.NSTAGES)()
        _lib.lib().pcx_profile_read(h, ms)
        _lib.lib().pcx_profile_enable(h, 0)
        st = {_lib.lib().pcx_stage_name(k).decode(): ms[k] for k in range(_abi.NSTAGES) if ms[k] > 0}
        out["libpcx_stage_ms"] = {k: round(v, 4) for k, v in sorted(st.items(), key=lambda kv: -kv[1])[:12]}
        out["libpcx_device_ms"] = sum(v for k, v in st.items() if k not in ("H2D", "D2H", "EXCHANGE"))
    if oracle:
        from oracle.pcx_oracle import OracleCPU

        ts = []
        for _ in range(3 if which == "c2" else 20):
            a = mk()
            t0 = time.perf_counter()
            OracleCPU(**a).consensus()
            ts.append(time.perf_counter() - t0)
        out["cpu_baseline"] = {"value": 1e3 * med(ts), "unit": "ms", "kind": "port", "cores": host_threads(),
                               "sample": "the same call, numpy restatement (oracle/pcx_oracle.py)"}
    return out


def _sum_traffic(kernels, key="bytes_per_launch"):
    vals = [load_traffic(k, key) for k in kernels]
    return None if any(v is None for v in vals) else sum(vals)


def load_traffic(kernel="batched_round_kernel", key="bytes_per_launch"):
    """Per-launch PMC figure of `kernel` (HBM bytes, VALU instructions) from the committed
    rocprofv3 passes (profiles/pmc_traffic.json, `tools/gpu.sh TAG profile`), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        return d.get(kernel, {}).get(key)
    except Exception:
        return None


C5_TIMEOUT_S = 300          # multi-rank C5 watchdog (bench main)
C5_WATCHDOG_EXIT = 3        # exit status of a rank whose C5 stalled
BENCH_FAILED_EXIT = 4       # exit status after the line when a C5 / C4 / medium entry raised
C5_WARMUP = 2               # untimed C5 consensus runs (the first run allocates the workspace and outputs)
_C5_STATE = {"comm": None, "dev": None, "phase": "setup"}


def c5_stall_report(rank):
    """One line naming the rank and the libpcx stage its C5 call is in (pcx_ctx_progress)."""
    where = _C5_STATE["phase"]
    comm = _C5_STATE["comm"]
    if comm is not None:
        try:
            from pyconsensus_amd.pipeline import progress

            stage, waiting = progress(comm, _C5_STATE["dev"])
            where += ", libpcx stage %s%s" % (stage or "(none yet)", " (host waiting on the stream)" if waiting else "")
        except Exception as e:  # noqa: BLE001
            where += ", progress unavailable: %r" % (e,)
    return "rank %d stalled in C5 %s" % (rank, where)
I8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA, 2x the bf16 rate (MI355X_MICROARCH.md, Matrix cores)
VALU_ISSUE_CYCLES = 4      # a wave64 VALU instruction holds its SIMD 4 cycles
SIMDS, CLOCK_GHZ = 1024, 2.4


LAUNCHER_ENV = "PCX_BENCH_LAUNCHER"  # set by launch_ranks for its children (reported in the line)


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """``bench.py --gpus N`` without a launcher: run the driver's own N-rank command
    (torch.distributed.run, one process per GPU, rendezvous on 127.0.0.1) as a CHILD
    process and return its exit status.  Called before this process touches the GPU (no
    exec from a process that initialised HIP); rank 0 of the child job prints the line."""
    import signal
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, **{LAUNCHER_ENV: "bench.py --gpus %d (torch.distributed.run child)" % n})
    proc = subprocess.Popen(cmd, env=env)  # same process group: a group kill reaches every rank
    # a SIGTERM to this process alone is passed on (torch.distributed.run forwards it to its ranks)
    signal.signal(signal.SIGTERM, lambda s, f: proc.send_signal(s))
    try:
        return proc.wait()
    except BaseException:
        proc.terminate()
        try:
            proc.wait(timeout=30)
        except Exception:  # noqa: BLE001
            proc.kill()
        raise


def rank_devices(world, dev):
    """(rank, local device index, PCI bus id) of every rank, gathered to all ranks."""
    import torch

    p = torch.cuda.get_device_properties(dev)
    mine = {"device": dev.index, "pci_bus_id": getattr(p, "pci_bus_id", None), "name": p.name}
    if world == 1:
        return [dict(rank=0, **mine)]
    import torch.distributed as dist

    allv = [None] * world
    dist.all_gather_object(allv, mine)
    return [dict(rank=r, **v) for r, v in enumerate(allv)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=ROUNDS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c5-steps", type=int, default=3, help="timed 1M x 4k consensus runs (0 = skip)")
    ap.add_argument("--no-c4", dest="c4", action="store_false", help="skip the 100k x 1k (C4) entry")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr, flush=True)
        sys.exit(2)
    if env_world is None and args.gpus > 1:
        # no launcher: start one rank per GPU ourselves, before anything touches the GPU
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d; refusing to report a different GPU count"
              % (env_world, args.gpus), file=sys.stderr, flush=True)
        sys.exit(2)

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; PCX_DIST_BACKEND=gloo (ranks may then share a GPU) rehearses the
    # multi-rank path on a one-GPU box -- the driver's N-GPU runs use RCCL ("nccl")
    backend = os.environ.get("PCX_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local %= torch.cuda.device_count()
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    devices = rank_devices(world, dev)

    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched

    B = args.rounds
    R, sc, lo, hi, rep = synthetic.rounds(B, N_REP, N_EV, seed=SEED + rank)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt).to(dev)
    Rd, scd, lod, hid, repd = t(R), t(sc, torch.uint8), t(lo), t(hi), t(rep)
    del R

    def step(matrices=True):  # the whole result dict, "original" and "filled" included
        return consensus_batched(Rd, repd, scd, lod, hid, device=dev, filled=matrices, original=matrices)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # the vector outputs only (no N x E matrices), for reference
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(torch.cuda.current_stream(dev))
    for _ in range(5):
        step(False)
    e1.record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize(dev)
    vec_ms = e0.elapsed_time(e1) / 5

    def barrier():
        if world > 1:
            import torch.distributed as dist

            dist.barrier()
        torch.cuda.synchronize(dev)

    # kernel-only timing with HIP events on the stream the kernel runs on
    stream = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier()
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        out = step()
        e1.record(stream)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist

        m = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        elapsed = float(m.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    total_rounds = B * args.steps * world
    value = total_rounds / elapsed

    if rank == 0:
        bpl = round_bytes(N_REP, N_EV) * B
        achieved = bpl / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic()
        valu = load_traffic(key="insts_valu_per_launch")
        valu_ms = valu * VALU_ISSUE_CYCLES / (SIMDS * CLOCK_GHZ * 1e9) * 1e3 if valu else None
        line = {
            "metric": "oracle rounds/sec (batched 50x20, 1 GPU)",
            "value": value,
            "unit": "rounds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (SURVEY.md 8(d) generator: 10%% NaN, 25%% scaled events, 70/30 honest/liar, "
                     "integer reputation; seed %d + rank)") % SEED,
            "config": {"workload": "C3: %d independent 50x20 oracle rounds per GPU per step (one wavefront "
                                   "per round), inputs resident in HBM, every output of the result dict "
                                   "written (original and filled included)" % B,
                       "rounds_per_gpu": B, "reporters": N_REP, "events": N_EV,
                       "parallelism": "rounds sharded across %d GPU(s), no collective" % world},
            "roofline": {"bound": "hbm", "kernel": "batched_round_kernel", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "kernel_ms": kern_ms,
                         "algorithmic_bytes_per_launch": bpl,
                         "limiter": ("latency / instruction issue, not HBM: one wave64 per LDS-resident "
                                     "round, 14 rounds per CU (DESIGN.md 5.2)"),
                         "valu": {"insts_per_launch": valu, "issue_ms": valu_ms,
                                  "frac": (valu_ms / kern_ms) if valu_ms else None,
                                  "note": "VALU issue time of the launch's instructions (SQ_INSTS_VALU, "
                                          "profiles/pmc_traffic.json) at 4 cycles each on 1024 SIMDs at "
                                          "2.4 GHz, over the kernel time"}},
            "vectors_only_kernel_ms": vec_ms,
            "launcher": os.environ.get(LAUNCHER_ENV, "external (WORLD_SIZE=%d)" % world if world > 1 else "none"),
            "devices": devices,
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline()
    del Rd, out
    torch.cuda.empty_cache()
    c5 = c4 = None
    failed = []  # secondary entries that raised: recorded in the line, and the run exits non-zero
    if args.c5_steps > 0:
        # a failure here is recorded in the line; the C3 headline above stands.  With several
        # ranks a watchdog also guards against a stuck collective: after C5_TIMEOUT_S every rank
        # names the stage it is stuck in on stderr and exits with status C5_WATCHDOG_EXIT (the
        # run FAILS), rank 0 first printing the C3 line with the C5 entry marked as stalled.
        watchdog = None
        if world > 1:
            import threading

            def on_timeout():
                msg = c5_stall_report(rank)
                print("bench.py watchdog: %s after %d s" % (msg, C5_TIMEOUT_S), file=sys.stderr, flush=True)
                if rank == 0:
                    line["c5"] = {"metric": "1M x 4k consensus latency", "n_gpus": world,
                                  "error": "watchdog: %s after %d s" % (msg, C5_TIMEOUT_S)}
                    print(json.dumps(line), flush=True)
                os._exit(C5_WATCHDOG_EXIT)

            watchdog = threading.Timer(C5_TIMEOUT_S, on_timeout)
            watchdog.daemon = True
            watchdog.start()
        try:
            c5 = bench_c5(world, rank, dev, args.c5_steps, C5_WARMUP)
        except Exception as e:  # noqa: BLE001
            traceback.print_exc()
            failed.append("c5")
            c5 = {"metric": "1M x 4k consensus latency", "n_gpus": world, "error": repr(e)[:400]}
        if watchdog is not None:
            watchdog.cancel()
    if args.c4 and world == 1:
        try:
            c4 = bench_c4(dev, oracle=not args.no_cpu_baseline)
        except Exception as e:  # noqa: BLE001
            traceback.print_exc()
            failed.append("c4")
            c4 = {"metric": "100k x 1k consensus latency", "error": repr(e)[:400]}
    medium = None
    if args.c4 and world == 1:
        try:
            medium = bench_medium(dev)
        except Exception as e:  # noqa: BLE001
            traceback.print_exc()
            failed.append("medium")
            medium = {"metric": "oracle rounds/sec (batched 100x50)", "error": repr(e)[:400]}
    dropin = {}
    if args.c4 and world == 1:
        try:
            dropin["cov_fp64"] = bench_cov_fp64(dev)
        except Exception as e:  # noqa: BLE001
            traceback.print_exc()
            failed.append("cov_fp64")
            dropin["cov_fp64"] = {"kernel": "k_syrk", "error": repr(e)[:400]}
        for which, calls in (("c1", 200), ("c2", 30)):
            try:
                dropin[which] = bench_dropin(dev, which, calls, oracle=not args.no_cpu_baseline)
            except Exception as e:  # noqa: BLE001
                traceback.print_exc()
                failed.append(which)
                dropin[which] = {"metric": "drop-in per-call latency (%s)" % which.upper(), "error": repr(e)[:400]}
    if rank == 0:
        line.update(dropin)
        if medium is not None:
            line["medium"] = medium
        if c5 is not None:
            line["c5"] = c5
        if c4 is not None:
            line["c4"] = c4
        if c4 is not None and c5 is not None and "h2d_gbs" in c4 and "rows_per_gpu" in c5:
            # pageable host->device rate measured on C4's reports
            c5["h2d_ms_estimate"] = 8.0 * c5["rows_per_gpu"] * c5["events"] / (c4["h2d_gbs"] * 1e9) * 1e3
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    if failed:
        print("bench.py: %s raised (see the line's \"error\" entries)" % ", ".join(failed), file=sys.stderr, flush=True)
        sys.exit(BENCH_FAILED_EXIT)


if __name__ == "__main__":
    main()
