"""The drop-in's host-memory path at C5 (1M x 4096, reputation=None): what a numpy caller of
Oracle(reports=...).consensus() pays end to end -- the reports copied to the GPU, the consensus,
every output copied back -- next to the device-resident consensus of bench.py's `c5` entry.

Two modes of result["original"]: a new host array (copy), and the reference's own aliasing (Q2,
__init__.py:121, 266-269, 584: `original` IS the caller's array, rescaled in place;
pcx_result.original == pcx_problem.reports), which the drop-in Oracle uses.  Per-stage device
times (M_H2D / M_D2H are the copies) come from libpcx's profile.

usage: python tools/c5_host_latency.py [steps=2] > out.json
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import torch

    from pyconsensus_amd import _abi, _lib, synthetic
    from pyconsensus_amd.pipeline import consensus_host

    N, E = 1_000_000, 4096
    Rd, scd, lod, hid, _ = synthetic.matrix_device(N, E, seed=3, n_shards=8, device="cuda:0")
    R0 = Rd.cpu().numpy()
    sc, lo, hi = scd.cpu().numpy(), lod.cpu().numpy(), hid.cpu().numpy()
    del Rd
    torch.cuda.empty_cache()
    out = {"rows": N, "events": E, "host_bytes_in": R0.nbytes, "modes": {}}
    h = _lib.context(0)
    for mode in ("copy", "inplace"):
        times, stages, first = [], {}, None
        for step in range(steps + 1):  # the first call allocates the workspace: reported apart
            X = R0.copy() if mode == "inplace" else R0
            _lib.check(_lib.lib().pcx_profile_enable(h, 1))
            t0 = time.perf_counter()
            outs, meta = consensus_host(X, None, sc, lo, hi, original_inplace=(mode == "inplace"))
            el = time.perf_counter() - t0
            ms = (__import__("ctypes").c_double * _abi.NSTAGES)()
            _lib.check(_lib.lib().pcx_profile_read(h, ms))
            _lib.check(_lib.lib().pcx_profile_enable(h, 0))
            del outs, X  # (before the next call: two calls' 33 GB outputs alive at once cost a reclaim)
            if step == 0:
                first = el
                continue
            times.append(el)
            for k in range(_abi.NSTAGES):
                if ms[k] > 0:
                    name = "M_" + _lib.lib().pcx_stage_name(k).decode()
                    stages[name] = stages.get(name, 0.0) + ms[k] / steps
        dev = sum(v for k, v in stages.items() if k not in ("M_H2D", "M_D2H"))
        out["modes"][mode] = {"latency_ms": 1e3 * sorted(times)[len(times) // 2],
                              "latency_ms_all": [1e3 * t for t in times],
                              "first_call_ms": 1e3 * first,  # (the device workspace and staging allocated)
                              "h2d_ms": stages.get("M_H2D"), "d2h_ms": stages.get("M_D2H"),
                              "device_stages_ms": dev,
                              "top_stages_ms": {k: round(v, 2) for k, v in
                                                sorted(stages.items(), key=lambda kv: -kv[1])[:8]}}
        print(json.dumps({"mode": mode, **out["modes"][mode]}), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
