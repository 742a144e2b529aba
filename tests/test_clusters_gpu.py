"""The clustering algorithms on the GPU batched kernel:
k-means (__init__.py:392-405), hierarchical (:407-419), clusterfeck (:148-242, :421-424).

* every reference golden case of clusters.npz (make_golden.py clusters_main) within the
  north_star tolerances (discrete outputs exact);
* bit-identical to the C SPEC (oracle/pcx_oracle_batched.c) on seeded synthetic batches of
  several shapes, k-means restarts drawn by the host as the reference's scipy call draws them;
* the drop-in Oracle: same results as the reference with numpy's global RandomState seeded
  alike, the clustering result containers, and the batched-only scope.
"""
import numpy as np
import pytest

import golden_cases as G
import parity as P
from oracle import pcx_oracle_c as OC

pytestmark = pytest.mark.gpu

KEYS = ("old_rep", "this_rep", "smooth_rep", "scores", "na_row", "participation_rows", "relative_part",
        "reporter_bonus", "adj_first_loadings", "outcomes_raw", "outcomes_adjusted", "outcomes_final",
        "certainty", "consensus_reward", "nas_filled", "participation_columns", "author_bonus",
        "participation", "avg_certainty", "branch", "flags", "components")


def _args(case):
    from pyconsensus_amd.batched import kmeans_draws

    N, E = case["in_reports"].shape
    kw = dict(catch_tolerance=float(case["in_catch_tolerance"]), alpha=float(case["in_alpha"]),
              int_dtype=bool(case["in_int_dtype"]), algorithm=str(case["in_algorithm"]),
              hierarchy_threshold=float(case["in_hierarchy_threshold"]))
    if bool(case["in_has_bounds"]):
        kw.update(scaled=case["in_scaled"][None], lo=case["in_lo"][None], hi=case["in_hi"][None])
    if kw["algorithm"] == "k-means":
        kw["kmeans_init"] = kmeans_draws(1, N, random_state=np.random.RandomState(int(case["in_np_seed"])))
    rep = case["in_reputation"][None] if bool(case["in_has_rep"]) else None
    return case["in_reports"][None], rep, kw


def test_golden_cases(gpu_lib):
    from pyconsensus_amd.batched import consensus_batched

    fails, n = [], 0
    for name, case in sorted(G.clusters().items()):
        R, rep, kw = _args(case)
        sc, lo, hi = kw.pop("scaled", None), kw.pop("lo", None), kw.pop("hi", None)
        out = consensus_batched(R, rep, sc, lo, hi, filled=True, original=True, **kw)
        ours = {k: v[0].cpu().numpy() for k, v in out.items() if not k.startswith("_")}
        bad, _ = P.compare(case, ours)
        n += 1
        if bad:
            fails.append((name, bad[:3]))
    print("clusters on GPU: %d cases, %d mismatches" % (n, len(fails)))
    assert not fails, fails[:8]


@pytest.mark.parametrize("alg", ["k-means", "hierarchical", "clusterfeck"])
@pytest.mark.parametrize("shape", [(512, 50, 20), (96, 64, 32), (96, 17, 5), (64, 40, 4), (64, 33, 1), (32, 1, 6)])
def test_bitexact_vs_spec(gpu_lib, alg, shape):
    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched, kmeans_draws

    B, N, E = shape
    R, sc, lo, hi, rep = synthetic.rounds(B, N, E, seed=1000 + N * E + len(alg))
    kw = dict(algorithm=alg, hierarchy_threshold=1.5 if N > 20 else 0.75)
    if alg == "k-means":
        kw["kmeans_init"] = kmeans_draws(B, N, random_state=np.random.RandomState(N + E))
    g = consensus_batched(R, rep, sc, lo, hi, **kw)
    c = OC.batched(R, sc, lo, hi, rep, threads=8, **kw)
    for k in KEYS:
        a, b = g[k].cpu().numpy(), c[k]
        same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
        assert same.all(), "%s: %d of %d entries differ from the SPEC" % (k, int((~same).sum()), same.size)


def test_oracle_dropin(gpu_lib):
    """Oracle(algorithm=...) through the GPU: reference goldens with the same global seed."""
    from pyconsensus_amd import Oracle

    cases = G.clusters()
    for name in ("readme@k-means", "readme@hierarchical", "readme@clusterfeck", "t3@k-means", "s007@k-means",
                 "s010@clusterfeck", "s011@hierarchical"):
        case = cases[name]
        kw = G.oracle_args(case)
        kw.update(G.cluster_kwargs(case))
        np.random.seed(int(case["in_np_seed"]))
        o = Oracle(**kw)
        res = o.consensus()
        ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(res).items() if k in P.ABI_NAME}
        bad, _ = P.compare(case, ours)
        assert not bad, (name, bad)
        assert res["convergence"] is True and res["components"] == -1
        assert isinstance(res["agents"]["smooth_rep"], np.ndarray)
        assert not isinstance(res["agents"]["smooth_rep"], np.ma.MaskedArray)
        assert np.all(np.asarray(res["agents"]["scores"]) == 0.0)


def test_oracle_clusters_scope(gpu_lib):
    from pyconsensus_amd import Oracle

    R = np.ones((65, 3))
    with pytest.raises(NotImplementedError):
        Oracle(reports=R, algorithm="hierarchical").consensus()
