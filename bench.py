"""Benchmark of the pyconsensus hot path on MI355X (contract: see DESIGN.md §Measurement).

Headline (BASELINE.json ``metric``): oracle rounds/sec for the batched 50 x 20
regime (config C3: 65,536 independent rounds per GPU per step, one wavefront per
round).  A "step" is one launch of ``batched_round_kernel`` over the resident
65,536-round batch: every round is a complete ``Oracle(...).consensus()``.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

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

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ROUNDS, N_REP, N_EV = 65536, 50, 20
SEED = 20261015
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def round_bytes(N, E):
    """Algorithmic HBM bytes per round: inputs read once, outputs written once."""
    reads = 8 * N * E + 8 * N + E * (1 + 8 + 8)          # reports, reputation, scaled/lo/hi
    writes = 8 * N * 8 + 8 * E * 9 + 8 * 2 + 4 * 3       # 8 N-vectors, 9 E-vectors, 2 f64 + 3 i32 scalars
    return reads + writes


def cpu_baseline(seconds=12.0):
    """The C oracle (oracle/pcx_oracle_batched.c, a port of the reference algorithm)
    on this host's cores, over a bounded sample of the same workload."""
    from oracle import pcx_oracle_c as OC
    from pyconsensus_amd import synthetic

    threads = max(1, min(16, os.cpu_count() or 1))
    R, sc, lo, hi, rep = synthetic.rounds(4096, N_REP, N_EV, seed=SEED)
    OC.batched(R[:256], sc[:256], lo[:256], hi[:256], rep[:256], threads=threads)  # warm
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        OC.batched(R, sc, lo, hi, rep, threads=threads)
        done += R.shape[0]
    el = time.perf_counter() - t0
    out = {"value": done / el, "unit": "rounds/s", "cores": threads, "kind": "port",
           "sample": "%d rounds of the C3 workload (50x20, seed %d) in %.1f s, C oracle, %d OpenMP threads"
                     % (done, SEED, el, threads)}
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

    def run(profile=None):
        return consensus_matrix(R, None, sc, lo, hi, comm=comm, n_total=N, row_offset=off, device=dev,
                                profile=profile)

    for _ in range(warmup):
        run()
    times, prof = [], {}
    for _ in range(steps):
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev, ag, meta = run(prof)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            m = torch.tensor([el], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(m, op=torch.distributed.ReduceOp.MAX)
            el = float(m.item())
        times.append(el)
    prof = {k: v / steps for k, v in prof.items()}
    cov_ms = prof.get("M_COV", float("nan"))
    cov_flops_rank = float(cnt) * E * (E + 1)  # one MAC per unique (j, k<=j) pair per row
    tfs = cov_flops_rank / (cov_ms * 1e-3) / 1e12 if cov_ms == cov_ms else None
    del R
    return {"metric": "1M x 4k consensus latency", "n_gpus": world, "rows_per_gpu": cnt, "events": E,
            "latency_ms": 1e3 * sorted(times)[len(times) // 2], "latency_ms_all": [1e3 * x for x in times],
            "branch": meta["branch"], "pi_iters": meta["pi_iters"], "flags": meta["flags"],
            "stage_ms": {k: round(v, 3) for k, v in sorted(prof.items(), key=lambda kv: -kv[1])},
            "roofline_cov": {"bound": "mfma", "kernel": "k_syrk", "achieved": tfs, "peak": FP64_MFMA_PEAK_TFS,
                             "unit": "TFLOP/s", "frac": (tfs / FP64_MFMA_PEAK_TFS) if tfs else None,
                             "flops_per_launch": cov_flops_rank, "traffic": load_traffic("k_syrk")},
            "data": "synthetic on-GPU (SURVEY.md 8(d) spec, torch Philox per 125k-row shard, seed 3), "
                    "reputation=None"}


def load_traffic(kernel="batched_round_kernel"):
    """Per-launch HBM bytes of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, tools/gpu_profile.sh), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        return d.get(kernel, {}).get("bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=ROUNDS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c5-steps", type=int, default=3, help="timed 1M x 4k consensus runs (0 = skip)")
    args = ap.parse_args()

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

    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched

    B = args.rounds
    R, sc, lo, hi, rep = synthetic.rounds(B, N_REP, N_EV, seed=SEED + rank)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt).to(dev)
    Rd, scd, lod, hid, repd = t(R), t(sc, torch.uint8), t(lo), t(hi), t(rep)
    del R

    def step():
        return consensus_batched(Rd, repd, scd, lod, hid, device=dev)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

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
                                   "per round), inputs resident in HBM" % B,
                       "rounds_per_gpu": B, "reporters": N_REP, "events": N_EV,
                       "parallelism": "rounds sharded across %d GPU(s), no collective" % world},
            "roofline": {"bound": "hbm", "kernel": "batched_round_kernel", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "kernel_ms": kern_ms,
                         "algorithmic_bytes_per_launch": bpl,
                         "limiter": ("latency / VALU issue, not HBM: one wave64 per LDS-resident round, "
                                     "10 rounds per CU, SQ VALU busy ~55% "
                                     "(profiles/r1/sq_counters_batched_pass*.csv, DESIGN.md 5)")},
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline()
    del Rd, out
    torch.cuda.empty_cache()
    c5 = None
    if args.c5_steps > 0:
        c5 = bench_c5(world, rank, dev, args.c5_steps, 1)
    if rank == 0:
        if c5 is not None:
            line["c5"] = c5
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
