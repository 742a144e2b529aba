"""The CPU oracles on the clustering algorithms of SURVEY.md 8(f) row 4 -- "k-means"
(__init__.py:392-405), "hierarchical" (:407-419), "clusterfeck" (:148-242, :421-424) --
against golden vectors produced by the reference itself (make_golden.py clusters_main ->
clusters.npz).

* oracle/pcx_oracle.py: bit for bit (k-means / hierarchical through the reference's own
  scipy.cluster calls, clusterfeck restated), with numpy's global RandomState seeded as
  the fixture was;
* oracle/pcx_oracle_batched.c (the SPEC the GPU kernel replays): the clusters exactly --
  so the per-reporter nonconformity, and from it every output, within north_star
  tolerances; the first loading (a by-product of wpca here) is the SPEC's power
  iteration, compared sign-aligned.
"""
import numpy as np

import golden_cases as G
import parity as P
from oracle import pcx_oracle_c as OC
from oracle.pcx_oracle import OracleCPU
from pyconsensus_amd.batched import kmeans_draws


def test_numpy_oracle_bitexact():
    bad = []
    for name, case in sorted(G.clusters().items()):
        kw = G.oracle_args(case)
        kw.update(G.cluster_kwargs(case))
        np.random.seed(int(case["in_np_seed"]))
        got = G.flat_result(OracleCPU(**kw).consensus())
        for k, v in got.items():
            if not np.array_equal(v, case[k], equal_nan=True):
                bad.append((name, k))
                break
    assert not bad, bad[:5]


def run_c(case):
    R = case["in_reports"][None]
    N, E = case["in_reports"].shape
    kw = {}
    if bool(case["in_has_bounds"]):
        kw.update(scaled=case["in_scaled"][None], lo=case["in_lo"][None], hi=case["in_hi"][None])
    if bool(case["in_has_rep"]):
        kw["reputation"] = case["in_reputation"][None]
    alg = str(case["in_algorithm"])
    if alg == "k-means":
        kw["kmeans_init"] = kmeans_draws(1, N, random_state=np.random.RandomState(int(case["in_np_seed"])))
    o = OC.batched(R, catch_tolerance=float(case["in_catch_tolerance"]), alpha=float(case["in_alpha"]),
                   int_dtype=bool(case["in_int_dtype"]), algorithm=alg,
                   hierarchy_threshold=float(case["in_hierarchy_threshold"]), **kw)
    return {k: v[0] for k, v in o.items()}


def test_c_oracle_vs_golden():
    fails, n = [], 0
    for name, case in sorted(G.clusters().items()):
        ours = run_c(case)
        bad, _ = P.compare(case, ours)
        n += 1
        if bad:
            fails.append((name, bad[:3]))
    print("clusters C oracle: %d cases, %d mismatches" % (n, len(fails)))
    assert not fails, fails[:8]
