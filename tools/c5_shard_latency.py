"""Latency of one C5 shard (1M x 4k recipe, rows of 1/`world` of the matrix) as a one-rank
consensus on one GPU: the per-GPU compute of the N-GPU C5 run without its collectives, with
the per-stage device times, so fixed per-call costs (launches, host polls) show next to the
bandwidth / MFMA time.

usage: python tools/c5_shard_latency.py [world=8] [steps=5]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    import torch

    from pyconsensus_amd import synthetic
    from pyconsensus_amd.pipeline import consensus_matrix

    dev = torch.device("cuda", 0)
    per = 8 // world
    R, sc, lo, hi, _ = synthetic.matrix_device(1_000_000, 4096, seed=3, n_shards=8, shards=list(range(per)),
                                               device=dev)
    run = lambda prof=None: consensus_matrix(R, None, sc, lo, hi, device=dev, matrices=True, profile=prof)
    run()
    times, prof = [], {}
    for _ in range(steps):  # plain calls
        ev = ag = None
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev, ag, meta = run()
        torch.cuda.synchronize(dev)
        times.append(1e3 * (time.perf_counter() - t0))
    ev = ag = None
    run(prof)  # one call with per-stage events
    prof = {k: round(v, 3) for k, v in sorted(prof.items(), key=lambda kv: -kv[1])}
    dev_ms = sum(prof.values())
    print(json.dumps({"rows": int(R.shape[0]), "events": 4096, "latency_ms": sorted(times)[len(times) // 2],
                      "all_ms": times, "stage_sum_ms": dev_ms, "sel_passes": meta["sel_passes"],
                      "pi_iters": meta["pi_iters"], "stage_ms": prof}), flush=True)


if __name__ == "__main__":
    main()
