"""GPU parity of the non-PCA algorithms ("big-five", "fixed-variance",
"cokurtosis", plus "absolute") against the reference's golden vectors (algos.npz,
tests/golden/make_golden.py): the drop-in Oracle (batched kernel for N <= 64, E <= 32,
the staged matrix pipeline + rocSOLVER eigenpairs beyond), and the matrix pipeline forced
on the small cases.  North_star tolerances; near-tie cases (fixture flags) counted apart.
"""
import numpy as np
import pytest

import golden_cases as G
import parity as P

pytestmark = pytest.mark.gpu


def _check(cases, run, path_of):
    observed = {p: {} for p in ("algos_exact", "algos_matrix")}
    ran = {p: [] for p in observed}
    for name, case in cases:
        ours = run(case)
        path = path_of(case, ours)
        ran[path].append(name)
        kind, _ = P.mismatch_kind(case, ours, components=True)
        if kind:
            observed[path][name] = kind
    for p in observed:
        P.assert_known(p, observed[p], ran[p])


def run_oracle(case):
    from pyconsensus_amd import Oracle

    kw = G.oracle_args(case)
    kw.update(G.algo_kwargs(case))
    o = Oracle(**kw)
    res = o.consensus()
    ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(res).items() if k in P.ABI_NAME}
    ours["branch"] = np.array(o.last_info["branch"])
    ours["components"] = np.array(res["components"])
    ours["path"] = o.last_info["path"]
    assert res["convergence"] == bool(case["convergence"])
    return ours


def run_matrix(case):
    from pyconsensus_amd.pipeline import consensus_matrix

    R = case["in_reports"]
    N, E = R.shape
    bk = {}
    if bool(case["in_has_bounds"]):
        bk = dict(scaled=case["in_scaled"], lo=case["in_lo"], hi=case["in_hi"])
    rep = case["in_reputation"] if bool(case["in_has_rep"]) else None
    akw = G.algo_kwargs(case)
    ev, ag, meta = consensus_matrix(R, rep, catch_tolerance=float(case["in_catch_tolerance"]),
                                    alpha=float(case["in_alpha"]), int_dtype=bool(case["in_int_dtype"]),
                                    algorithm=str(case["in_algorithm"]), max_components=akw["max_components"],
                                    variance_threshold=akw["variance_threshold"],
                                    aux_scores=akw.get("aux", {}).get("cokurt"), matrices=True, **bk)
    out = {k: v.cpu().numpy() for k, v in list(ev.items()) + list(ag.items())}
    out["participation"] = np.array(meta["participation"])
    out["avg_certainty"] = np.array(meta["avg_certainty"])
    out["branch"] = np.array(meta["branch"])
    out["components"] = np.array(meta["components"])
    return out


@pytest.mark.parametrize("alg", ["big-five", "fixed-variance", "cokurtosis", "absolute"])
def test_oracle_algos_golden(gpu_lib, alg):
    cases = [(n, c) for n, c in sorted(G.algos().items()) if n.endswith("@" + alg)]
    _check(cases, run_oracle, lambda case, ours: "algos_exact" if ours.pop("path") == "batched" else "algos_matrix")


@pytest.mark.parametrize("alg", ["big-five", "fixed-variance", "cokurtosis"])
def test_matrix_path_algos_golden(gpu_lib, alg):
    """The staged pipeline on every case of the algorithm (small ones forced through it)."""
    cases = [(n, c) for n, c in sorted(G.algos().items()) if n.endswith("@" + alg)]
    _check(cases[::3], run_matrix, lambda case, ours: "algos_matrix")
