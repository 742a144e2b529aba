"""GPU parity of the batched round kernel (one wavefront per round).

* bit-for-bit against the C oracle (oracle/pcx_oracle_batched.c) on the full C3
  workload: 65,536 seeded 50 x 20 rounds, every output;
* against the reference's golden vectors (KATs, mixed shapes, 600 synthetic
  rounds) with the north_star tolerances (tests/parity.py).
"""
import numpy as np
import pytest

import golden_cases as G
import parity as P

pytestmark = pytest.mark.gpu


def _np(outs):
    return {k: v.cpu().numpy() for k, v in outs.items() if not k.startswith("_")}


def _run_gpu(case_list):
    """Rounds of one shape in one launch; case_list: list of golden dicts."""
    from pyconsensus_amd.batched import consensus_batched

    R = np.stack([c["in_reports"] for c in case_list])
    c0 = case_list[0]
    kw = {}
    if bool(c0["in_has_bounds"]):
        kw.update(scaled=np.stack([c["in_scaled"] for c in case_list]),
                  lo=np.stack([c["in_lo"] for c in case_list]), hi=np.stack([c["in_hi"] for c in case_list]))
    if bool(c0["in_has_rep"]):
        kw["reputation"] = np.stack([c["in_reputation"] for c in case_list])
    return _np(consensus_batched(R, catch_tolerance=float(c0["in_catch_tolerance"]),
                                 alpha=float(c0["in_alpha"]), int_dtype=bool(c0["in_int_dtype"]),
                                 filled=True, original=True, **kw))


def _score(cases, outs):
    """{name: mismatch kind} of the rounds of one launch, and the names run."""
    observed, ran = {}, []
    for b, (name, case) in enumerate(cases):
        ran.append(name)
        kind, _ = P.mismatch_kind(case, {k: v[b] for k, v in outs.items()})
        if kind:
            observed[name] = kind
    return observed, ran


def test_golden_synth_50x20(gpu_lib):
    st = G.synth()
    cases = [("s%03d" % b, G.unstack(st, b)) for b in range(st["branch"].shape[0])]
    P.assert_known("exact", *_score(cases, _run_gpu([c for _, c in cases])))


def test_golden_kat_and_mixed(gpu_lib):
    allc = list(G.kat().items()) + list(G.mixed().items())
    observed, ran = {}, []
    for name, case in allc:
        N, E = case["in_reports"].shape
        if name in P.EXCLUDED or N > 64 or E > 32:
            continue
        o, r = _score([(name, case)], _run_gpu([case]))
        observed.update(o)
        ran += r
    P.assert_known("exact", observed, ran)


def test_bitexact_vs_c_oracle_c3(gpu_lib):
    """Full C3 workload (65,536 x 50 x 20, seed 20261015): GPU == C oracle, bit for bit, on every
    output the bench writes -- the rescaled `original` and the `filled` matrix included."""
    from oracle import pcx_oracle_c as OC
    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched

    R, sc, lo, hi, rep = synthetic.rounds(65536, 50, 20, seed=20261015)
    g = _np(consensus_batched(R, rep, sc, lo, hi, filled=True, original=True))
    c = OC.batched(R, sc, lo, hi, rep, threads=16)
    assert set(g) <= set(c) and {"original", "filled"} <= set(g), set(g) ^ set(c)
    for k, v in g.items():
        a, b = v, c[k]
        same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
        nbad = int(np.size(same) - np.count_nonzero(same))
        assert nbad == 0, (k, nbad)


@pytest.mark.parametrize("variant", ["uniform_rep", "shared_bounds", "no_bounds", "int_dtype",
                                     "absolute", "E1", "N1", "N64_E32", "big-five", "fixed-variance",
                                     "cokurtosis", "big-five_E7", "fixed-variance_N64_E32"])
def test_variants_bitexact_vs_c_oracle(gpu_lib, variant):
    from oracle import pcx_oracle_c as OC
    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched

    N, E = {"E1": (30, 1), "N1": (1, 6), "N64_E32": (64, 32), "big-five_E7": (40, 7),
            "fixed-variance_N64_E32": (64, 32)}.get(variant, (50, 20))
    R, sc, lo, hi, rep = synthetic.rounds(512, N, E, seed=5)
    kw = dict(reputation=rep, scaled=sc, lo=lo, hi=hi)
    if variant == "uniform_rep":
        kw["reputation"] = None
    if variant == "shared_bounds":
        kw.update(scaled=sc[0], lo=lo[0], hi=hi[0])
    if variant == "no_bounds":
        kw.update(scaled=None, lo=None, hi=None)
    if variant == "int_dtype":
        R = np.where(np.isnan(R), 0.0, np.trunc(R))
        kw["int_dtype"] = True
    if variant == "absolute":
        kw["algorithm"] = "absolute"
    alg = variant.split("_")[0]
    if alg in ("big-five", "fixed-variance", "cokurtosis"):
        kw["algorithm"] = alg
        kw["max_components"] = 5
        kw["variance_threshold"] = 0.75
    if alg == "cokurtosis":
        kw["aux_scores"] = np.random.default_rng(9).normal(size=(R.shape[0], N))
    g = _np(consensus_batched(R, filled=True, original=True, **kw))
    c = OC.batched(R, **kw, threads=8)
    for k, v in g.items():
        same = (v == c[k]) | (np.isnan(v) & np.isnan(c[k])) if v.dtype.kind == "f" else (v == c[k])
        assert np.all(same), (variant, k, int(np.size(same) - np.count_nonzero(same)))


def _rounds_kw(variant, B=40, seed=77):
    from pyconsensus_amd import synthetic

    shape, *rest = variant.split("_")
    N, E = map(int, shape.split("x"))
    R, sc, lo, hi, rep = synthetic.rounds(B, N, E, seed=seed)
    kw = dict(reputation=rep, scaled=sc, lo=lo, hi=hi)
    if "uniform" in rest:
        kw["reputation"] = None
    if "shared" in rest:
        kw.update(scaled=sc[0], lo=lo[0], hi=hi[0])
    if "nobounds" in rest:
        kw.update(scaled=None, lo=None, hi=None)
    if "int" in rest:
        R = np.where(np.isnan(R), 0.0, np.trunc(R))
        kw["int_dtype"] = True
    for alg in ("big-five", "fixed-variance", "absolute", "cokurtosis"):
        if alg in rest:
            kw["algorithm"] = alg
    if kw.get("algorithm") in ("big-five", "fixed-variance"):
        kw["max_components"] = 5
        kw["variance_threshold"] = 0.75
    if kw.get("algorithm") == "cokurtosis":
        kw["aux_scores"] = np.random.default_rng(9).normal(size=(B, N))
    return R, kw


def _round_inputs(kw, b):
    sc, lo, hi = kw["scaled"], kw["lo"], kw["hi"]
    if sc is not None and sc.ndim == 2:
        sc, lo, hi = sc[b], lo[b], hi[b]
    rep = None if kw["reputation"] is None else kw["reputation"][b]
    return rep, sc, lo, hi


@pytest.mark.parametrize("variant", ["100x50", "30x40_uniform_shared", "256x64", "65x33_nobounds", "200x1",
                                     "120x20_int", "90x36_absolute", "80x40_cokurtosis", "250x60_uniform",
                                     "100x50_big-five", "70x40_fixed-variance", "150x7_big-five"])
def test_medium_rounds_bitexact_vs_spec(gpu_lib, variant):
    """Rounds above one wavefront up to 256 x 64 (every non-clustering algorithm): one workgroup per
    round (csrc/pcx_medium.hip), bit-identical to the C SPEC built for 256 reporters
    (oracle/pcx_oracle_batched.c, NMAX = 256) on every output, and within the north_star
    tolerances of the numpy restatement of the reference."""
    from oracle import pcx_oracle_c as OC
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched

    R, kw = _rounds_kw(variant)
    g = _np(consensus_batched(R, filled=True, original=True, **kw))
    c = OC.batched(R, **kw, threads=8)
    for k, v in g.items():
        same = (v == c[k]) | (np.isnan(v) & np.isnan(c[k])) if v.dtype.kind == "f" else (v == c[k])
        assert np.all(same), (variant, k, int(np.size(same) - np.count_nonzero(same)))
    alg = kw.get("algorithm", "PCA")
    if kw.get("int_dtype"):
        return  # an int matrix with a NaN fill makes the reference raise: the SPEC alone pins it
    for b in range(0, R.shape[0], 7):
        rep, sc, lo, hi = _round_inputs(kw, b)
        aux = None if alg != "cokurtosis" else {"cokurt": kw["aux_scores"][b]}
        Rb = R[b].copy()
        ref = G.flat_result(OracleCPU(reports=Rb, event_bounds=None if sc is None else synthetic.bounds_list(sc, lo, hi),
                                      reputation=rep, algorithm=alg, aux=aux, max_components=5,
                                      variance_threshold=kw.get("variance_threshold", 0.9)).consensus())
        bad, _ = P.compare(ref, {k: v[b] for k, v in g.items()})
        assert not bad, (b, bad)


@pytest.mark.parametrize("shape", [(100, 50), (250, 60), (256, 64)], ids=["100x50", "250x60", "256x64"])
def test_medium_rounds_vs_reference_goldens(gpu_lib, shape):
    """The workgroup-per-round kernel on rounds the REFERENCE computed (tests/golden/medium.npz:
    40 rounds each of 100 x 50, 250 x 60, 256 x 64, a third with reputation=None): every output
    within the north_star tolerances, fills and outcomes exact, branch codes equal."""
    import torch
    from pyconsensus_amd.batched import consensus_batched

    cases = G.medium()[shape]
    observed, ran = {}, []
    for uniform in (False, True):
        idx = [i for i, c in enumerate(cases) if ("in_reputation" not in c) == uniform]
        st = lambda k: np.stack([cases[i][k] for i in idx])
        g = _np(consensus_batched(st("in_reports"), None if uniform else st("in_reputation"), st("in_scaled"),
                                  st("in_lo"), st("in_hi"), filled=True, original=True))
        torch.cuda.synchronize()
        for t, i in enumerate(idx):
            name = "w%dx%d_%02d" % (shape[0], shape[1], i)
            ran.append(name)
            kind, _ = P.mismatch_kind(cases[i], {k: v[t] for k, v in g.items()})
            if kind:
                observed[name] = kind
    assert len(ran) == len(cases)
    P.assert_known("exact", observed, ran)


@pytest.mark.parametrize("variant", ["1x40", "2x33", "3x64_uniform", "7x50_nobounds", "9x35_absolute",
                                     "33x64_shared", "64x33_int", "65x2", "129x3", "255x63", "256x1_uniform",
                                     "5x40_big-five", "40x34_fixed-variance"])
def test_medium_rounds_edge_shapes_vs_spec(gpu_lib, variant):
    """The workgroup-per-round kernel at its edges: tiny reporter counts (one-row rounds, a
    bitonic network of two slots), E just above the one-wave limit, E = 1-3 (np.dot's ddot / dgemv
    tail orders), N just above 64 / 128 and just below 256: bit-identical to the 256-reporter SPEC
    on every output (the SPEC alone pins these; the numpy restatement is covered above)."""
    from oracle import pcx_oracle_c as OC
    from pyconsensus_amd.batched import consensus_batched

    R, kw = _rounds_kw(variant, B=24, seed=5)
    g = _np(consensus_batched(R, filled=True, original=True, **kw))
    c = OC.batched(R, **kw, threads=8)
    for k, v in g.items():
        same = (v == c[k]) | (np.isnan(v) & np.isnan(c[k])) if v.dtype.kind == "f" else (v == c[k])
        assert np.all(same), (variant, k, int(np.size(same) - np.count_nonzero(same)))


@pytest.mark.parametrize("variant", ["100x50", "30x40_uniform_shared", "200x24_big-five", "300x20"])
def test_rounds_scheduler(gpu_lib, variant, monkeypatch):
    """Rounds the workgroup kernel does not take (big-five, N > 256, or PCX_NO_MEDIUM): each runs
    as a single-matrix consensus on the worker-stream scheduler (csrc/pcx_rounds.cpp) and equals
    its own pcx_consensus_f64 call bit for bit, and the numpy restatement within tolerance."""
    import torch

    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched
    from pyconsensus_amd.pipeline import consensus_matrix

    monkeypatch.setenv("PCX_NO_MEDIUM", "1")
    R, kw = _rounds_kw(variant)
    alg = kw.get("algorithm", "PCA")
    g = _np(consensus_batched(R, filled=True, original=True, **kw))
    torch.cuda.synchronize()
    B = R.shape[0]
    for b in [0, 1, B // 2, B - 1]:
        rep, sc, lo, hi = _round_inputs(kw, b)
        ev, ag, meta = consensus_matrix(R[b], rep, sc, lo, hi, algorithm=alg, matrices=True)
        one = {k: v.cpu().numpy() for d in (ev, ag) for k, v in d.items()}
        for k, v in one.items():
            np.testing.assert_array_equal(g[k][b], v, err_msg="%s round %d" % (k, b))
        assert int(g["branch"][b]) == meta["branch"] and g["participation"][b] == meta["participation"]
    for b in range(0, B, 3):
        rep, sc, lo, hi = _round_inputs(kw, b)
        ref = G.flat_result(OracleCPU(reports=R[b].copy(), event_bounds=synthetic.bounds_list(sc, lo, hi),
                                      reputation=rep, algorithm=alg).consensus())
        bad, _ = P.compare(ref, {k: v[b] for k, v in g.items()})
        assert not bad, (b, bad)


@pytest.mark.parametrize("alg", ["hierarchical", "clusterfeck", "k-means"])
def test_rounds_above_one_wave_clustering(gpu_lib, alg):
    """The clustering algorithms in batched rounds above 64 x 32 (the scheduler's single-matrix
    consensuses): each round against the numpy restatement; k-means draws every round's
    restarts from numpy's global RandomState in round order, as B sequential reference calls."""
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched

    B, N, E = 6, 70, 12
    rng = np.random.default_rng(4)
    P0 = rng.integers(1, 3, (3, E)).astype(np.float64)
    R = P0[rng.integers(0, 3, (B, N))]
    R = np.where(rng.random((B, N, E)) < 0.03, 3.0 - R, R)
    R[rng.random((B, N, E)) < 0.05] = np.nan
    rep = rng.integers(1, 100, (B, N)).astype(np.float64)
    np.random.seed(99)
    g = _np(consensus_batched(R, rep, algorithm=alg, filled=True))
    np.random.seed(99)
    for b in range(B):
        ref = G.flat_result(OracleCPU(reports=R[b].copy(), reputation=rep[b], algorithm=alg).consensus())
        bad, _ = P.compare(ref, {k: v[b] for k, v in g.items()})
        assert not bad, (b, bad)
