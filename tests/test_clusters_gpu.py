"""The clustering algorithms on the GPU batched kernel:
k-means (__init__.py:392-405), hierarchical (:407-419), clusterfeck (:148-242, :421-424).

* every reference golden case of clusters.npz (make_golden.py clusters_main) within the
  north_star tolerances (discrete outputs exact);
* bit-identical to the C SPEC (oracle/pcx_oracle_batched.c) on seeded synthetic batches of
  several shapes, k-means restarts drawn by the host as the reference's scipy call draws them;
* the drop-in Oracle: same results as the reference with numpy's global RandomState seeded
  alike, and the clustering result containers;
* the single-matrix path's clustering kernels (matrices above 64 x 32): every golden case
  forced through them, and larger clustered matrices against the numpy restatement.
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


def _matrix_cluster(R, rep, sc, lo, hi, algorithm, hierarchy_threshold=0.5, kmeans_init=None, int_dtype=False,
                    catch_tolerance=0.1, alpha=0.1):
    """The single-matrix path's clustering (pcx_consensus_f64, csrc/pcx_runner.cpp cluster_nc)."""
    from pyconsensus_amd.pipeline import consensus_host

    g, meta = consensus_host(R, rep, sc, lo, hi, algorithm=algorithm, hierarchy_threshold=hierarchy_threshold,
                             kmeans_init=kmeans_init, int_dtype=int_dtype, catch_tolerance=catch_tolerance,
                             alpha=alpha)
    g["participation"] = np.array(meta["participation"])
    g["avg_certainty"] = np.array(meta["avg_certainty"])
    g["branch"] = np.array(meta["branch"])
    return g


def test_golden_cases_through_matrix_path(gpu_lib):
    """Every reference clustering golden forced through the single-matrix path (the kernels
    that serve matrices above 64 x 32): same results as the reference within the north_star
    tolerances, discrete outputs exact."""
    from pyconsensus_amd.batched import kmeans_draws

    bad_cases = {}
    for name, case in G.clusters().items():
        N, E = case["in_reports"].shape
        alg = str(case["in_algorithm"])
        sc = lo = hi = None
        if bool(case["in_has_bounds"]):
            sc, lo, hi = case["in_scaled"], case["in_lo"], case["in_hi"]
        rep = case["in_reputation"] if bool(case["in_has_rep"]) else None
        kinit = None
        if alg == "k-means":
            kinit = kmeans_draws(1, N, random_state=np.random.RandomState(int(case["in_np_seed"])))[0]
        ours = _matrix_cluster(case["in_reports"], rep, sc, lo, hi, alg,
                               hierarchy_threshold=float(case["in_hierarchy_threshold"]), kmeans_init=kinit,
                               int_dtype=bool(case["in_int_dtype"]), catch_tolerance=float(case["in_catch_tolerance"]),
                               alpha=float(case["in_alpha"]))
        bad, _ = P.compare(case, ours)
        if bad:
            bad_cases[name] = bad[:2]
    assert not bad_cases, (len(bad_cases), dict(list(bad_cases.items())[:6]))


def _clustered(N, E, seed, protos=4, flip=0.03, na=0.05, scaled_frac=0.0):
    """Binary reports around a few prototype rows (clusters of equal rows, near rows), plus
    optional scaled events: a workload where the clusterings are not all singletons."""
    rng = np.random.default_rng(seed)
    P0 = rng.integers(1, 3, (protos, E)).astype(np.float64)
    R = P0[rng.integers(0, protos, N)]
    R = np.where(rng.random((N, E)) < flip, 3.0 - R, R)
    sc = rng.random(E) < scaled_frac
    lo = np.where(sc, -10.0, 1.0)
    hi = np.where(sc, 30.0, 2.0)
    R = np.where(sc[None, :], lo + (hi - lo) * rng.uniform(0.05, 1.0, (N, E)), R)
    R[rng.random((N, E)) < na] = np.nan
    rep = rng.integers(1, 100, N).astype(np.float64)
    return R, rep, sc, lo, hi


@pytest.mark.parametrize("alg,N,E,scaled", [("hierarchical", 300, 40, 0.0), ("hierarchical", 2000, 24, 0.2),
                                            ("clusterfeck", 200, 40, 0.0), ("clusterfeck", 1500, 16, 0.2),
                                            ("k-means", 150, 20, 0.0), ("k-means", 400, 12, 0.2)])
def test_oracle_clusters_above_one_wave(gpu_lib, alg, N, E, scaled):
    """The drop-in Oracle on matrices above 64 x 32 (the single-matrix path) against the numpy
    restatement of the reference (oracle/pcx_oracle.py: scipy's own kmeans / fclusterdata and
    the restated leader clustering), numpy's global RandomState seeded alike for k-means."""
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import Oracle, synthetic

    R, rep, sc, lo, hi = _clustered(N, E, seed=N + E, scaled_frac=scaled)
    eb = synthetic.bounds_list(sc, lo, hi)
    np.random.seed(1234)
    ref = G.flat_result(OracleCPU(reports=R.copy(), event_bounds=eb, reputation=rep, algorithm=alg).consensus())
    np.random.seed(1234)
    o = Oracle(reports=R.copy(), event_bounds=eb, reputation=rep, algorithm=alg)
    res = o.consensus()
    assert o.last_info["path"] == "matrix"
    ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(res).items() if k in P.ABI_NAME}
    bad, _ = P.compare(ref, ours)
    assert not bad, bad
    assert res["convergence"] is True and np.all(np.asarray(res["agents"]["scores"]) == 0.0)
    nc_spread = np.ptp(np.asarray(res["agents"]["this_rep"], dtype=np.float64))
    assert np.isfinite(nc_spread)  # not the degenerate all-equal-sizes case


def test_oracle_clusters_refuse_sharding(gpu_lib):
    from pyconsensus_amd import _lib
    from pyconsensus_amd.pipeline import ThreadComm, ThreadGroup, consensus_matrix

    R = np.ones((100, 3))
    g = ThreadGroup(2)
    with pytest.raises(_lib.PcxError, match="one rank"):
        consensus_matrix(R, None, algorithm="hierarchical", comm=ThreadComm(g, 0), n_total=100, row_offset=0)


@pytest.mark.parametrize("name", ["readme@k-means", "readme@hierarchical", "readme@clusterfeck", "t3@k-means",
                                  "s007@k-means", "s010@clusterfeck", "s011@hierarchical"])
def test_lie_detector_stage_with_clustering(gpu_lib, name):
    """Oracle(algorithm=<clustering>).lie_detector(filled) (__init__.py:392-424): nc from the
    clusters, scores left at zeros (:357), this_rep / smooth_rep as in the reference golden
    (the golden's own filled matrix as input; numpy's global RandomState seeded alike)."""
    from pyconsensus_amd import Oracle

    case = G.clusters()[name]
    kw = G.oracle_args(case)
    kw.update(G.cluster_kwargs(case))
    o = Oracle(**kw)
    np.random.seed(int(case["in_np_seed"]))
    out = o.lie_detector(np.array(case["filled"], dtype=np.float64))
    assert np.all(np.asarray(out["scores"]) == 0.0)
    assert not isinstance(out["this_rep"], np.ma.MaskedArray)
    for k in ("this_rep", "smooth_rep"):
        np.testing.assert_allclose(np.asarray(out[k], dtype=np.float64), case["agents." + k], rtol=1e-9, atol=1e-12,
                                   err_msg="%s %s" % (name, k))
    assert o.convergence is True


def test_lie_detector_clustering_refuses_several_devices(gpu_lib):
    from pyconsensus_amd import Oracle

    with pytest.raises(NotImplementedError, match="one GPU"):
        Oracle(reports=np.ones((80, 40)), algorithm="hierarchical", devices=[0, 1]).lie_detector(np.ones((80, 40)))
