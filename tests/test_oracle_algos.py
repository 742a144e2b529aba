"""The CPU oracles on the non-PCA algorithms of SURVEY.md 8(f) -- "big-five",
"fixed-variance" (__init__.py:373-390, 429-451), "cokurtosis" (:455-457) and
"absolute" (:359-362) -- against golden vectors produced by the reference itself
(tests/golden/make_golden.py algos_main -> algos.npz).

* oracle/pcx_oracle.py (numpy restatement, same LAPACK svd as the reference): bit for bit;
* oracle/pcx_oracle_batched.c (the SPEC the GPU kernel replays: Jacobi eigenpairs in place
  of gesdd, compensated dots): north_star tolerances, near ties counted separately.
"""
import numpy as np
import pytest

import golden_cases as G
import parity as P
from oracle import pcx_oracle_c as OC
from oracle.pcx_oracle import OracleCPU


def test_numpy_oracle_bitexact():
    bad = []
    for name, case in sorted(G.algos().items()):
        kw = G.oracle_args(case)
        kw.update(G.algo_kwargs(case))
        got = G.flat_result(OracleCPU(**kw).consensus())
        for k, v in got.items():
            if k == "original" and k not in case:
                continue
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
    if "in_aux_scores" in case:
        kw["aux_scores"] = case["in_aux_scores"][None]
    mc = int(case["in_max_components"])
    o = OC.batched(R, catch_tolerance=float(case["in_catch_tolerance"]), alpha=float(case["in_alpha"]),
                   int_dtype=bool(case["in_int_dtype"]), algorithm=str(case["in_algorithm"]),
                   max_components=mc if E >= mc else E, variance_threshold=float(case["in_variance_threshold"]),
                   **kw)
    return {k: v[0] for k, v in o.items()}


def test_c_oracle_vs_golden():
    observed, ran = {}, []
    for name, case in sorted(G.algos().items()):
        N, E = case["in_reports"].shape
        if N > 64 or E > 64:
            continue
        ran.append(name)
        kind, _ = P.mismatch_kind(case, run_c(case), components=True)
        if kind:
            observed[name] = kind
    P.assert_known("algos_exact", observed, ran)


@pytest.mark.parametrize("alg", ["big-five", "fixed-variance"])
def test_jacobi_eigenpairs(alg):
    """The SPEC eigen-decomposition reproduces LAPACK's spectrum: the components'
    net scores equal the numpy restatement's to 1e-9 on well-separated spectra."""
    from pyconsensus_amd import synthetic

    R, sc, lo, hi, rep = synthetic.rounds(16, 40, 12, seed=101)
    c = OC.batched(R, sc, lo, hi, rep, algorithm=alg, max_components=5)
    for b in range(R.shape[0]):
        o = OracleCPU(reports=R[b], event_bounds=synthetic.bounds_list(sc[b], lo[b], hi[b]), reputation=rep[b],
                      algorithm=alg).consensus()
        ref = np.asarray(o["agents"]["scores"], dtype=float)
        np.testing.assert_allclose(c["scores"][b], ref, rtol=1e-9, atol=1e-12 * np.max(np.abs(ref)))
        assert int(c["components"][b]) == int(o["components"])
