"""Timing link between the reference and the CPU restatements ("Link to the
reference").  Runs in the BUILD container only: the reference never goes to the GPU box.

    OMP_NUM_THREADS=1 OPENBLAS_NUM_THREADS=1 python tests/golden/time_reference_vs_restatement.py

Times, on identical synthetic inputs and one core:
  * the reference `Oracle(...).consensus()` (loaded by make_golden.load_reference),
  * the numpy restatement `oracle.pcx_oracle.OracleCPU` (bench.py's C4 cpu_baseline),
  * the C restatement `oracle/pcx_oracle_batched.c` (bench.py's C3 cpu_baseline, 50x20 only),
and prints one JSON line per shape with the ratios.  Test infrastructure, not the product.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)


def _time(fn, min_s=3.0, max_n=200):
    fn()  # warm
    n, t0 = 0, time.perf_counter()
    while n < max_n:
        fn()
        n += 1
        if time.perf_counter() - t0 >= min_s:
            break
    return (time.perf_counter() - t0) / n


def main():
    import make_golden as MG

    from oracle import pcx_oracle_c as OC
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import synthetic

    ref = MG.load_reference()
    out = []
    for (N, E, seed) in ((50, 20, 20261015), (1000, 100, 1), (10000, 100, 5)):
        R, sc, lo, hi, rep = synthetic.matrix(N, E, seed=seed)
        b = synthetic.bounds_list(sc, lo, hi)
        t_ref = _time(lambda: ref.Oracle(reports=R.copy(), event_bounds=b, reputation=rep.copy()).consensus(),
                      max_n=50 if N <= 50 else 3)
        t_np = _time(lambda: OracleCPU(reports=R.copy(), event_bounds=b, reputation=rep.copy()).consensus(),
                     max_n=50 if N <= 50 else 3)
        row = {"shape": "%dx%d" % (N, E), "reference_s": t_ref, "numpy_restatement_s": t_np,
               "reference_over_numpy": t_ref / t_np}
        if N == 50 and E == 20:
            Rb, scb, lob, hib, repb = synthetic.rounds(2000, 50, 20, seed=seed)
            t0 = time.perf_counter()
            OC.batched(Rb, scb, lob, hib, repb, threads=1)
            t_c = (time.perf_counter() - t0) / 2000
            row.update(c_restatement_s=t_c, reference_over_c=t_ref / t_c)
        out.append(row)
        print(json.dumps(row), flush=True)
    return out


if __name__ == "__main__":
    main()
