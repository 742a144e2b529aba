"""Throughput of batched rounds above the one-wavefront kernel: B rounds of N x E through
pcx_consensus_batched_f64 on the workgroup-per-round kernel (csrc/pcx_medium.hip), then on the
worker-stream scheduler (csrc/pcx_rounds.cpp, PCX_NO_MEDIUM=1) at several pool sizes.

usage: python tools/bench_rounds.py [B] [N] [E] [wg]   (one JSON line per path / pool size; "wg":
the workgroup kernel only)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    E = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    import torch

    from pyconsensus_amd import _lib, synthetic
    from pyconsensus_amd.batched import consensus_batched

    R, sc, lo, hi, rep = synthetic.rounds(B, N, E, seed=3)
    dev = torch.device("cuda", 0)
    Rt, rt = torch.as_tensor(R, device=dev), torch.as_tensor(rep, device=dev)
    sct, lot, hit = (torch.as_tensor(a, device=dev) for a in (sc.astype("uint8"), lo, hi))
    for _ in range(2):  # the workgroup-per-round kernel (csrc/pcx_medium.hip), N <= 256, E <= 64
        consensus_batched(Rt, rt, sct, lot, hit)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        consensus_batched(Rt, rt, sct, lot, hit)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(json.dumps({"rounds": B, "N": N, "E": E, "path": "workgroup kernel", "seconds": dt,
                      "rounds_per_s": B / dt}), flush=True)
    if len(sys.argv) > 4 and sys.argv[4] == "wg":
        return
    os.environ["PCX_NO_MEDIUM"] = "1"  # the worker-stream scheduler (csrc/pcx_rounds.cpp)
    for workers in (1, 4, 8, 16, 32):
        os.environ["PCX_ROUND_WORKERS"] = str(workers)
        _lib._ctx.clear()  # fresh context: the pool size is read when it grows
        consensus_batched(Rt[:workers], rt[:workers], sct[:workers], lot[:workers], hit[:workers])  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        consensus_batched(Rt, rt, sct, lot, hit)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"rounds": B, "N": N, "E": E, "path": "scheduler", "workers": workers, "seconds": dt,
                          "rounds_per_s": B / dt}), flush=True)


if __name__ == "__main__":
    main()
