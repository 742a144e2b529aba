"""Readers for the golden fixtures in tests/golden/ (written by make_golden.py)."""
from __future__ import annotations

import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

AGENT_KEYS = ["old_rep", "this_rep", "smooth_rep", "na_row", "participation_rows",
              "relative_part", "reporter_bonus", "scores"]
EVENT_KEYS = ["adj_first_loadings", "outcomes_raw", "consensus_reward", "certainty",
              "NAs Filled", "participation_columns", "author_bonus",
              "outcomes_adjusted", "outcomes_final"]


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def split_cases(flat):
    """{'case/key': v} -> {case: {key: v}}"""
    out = {}
    for k, v in flat.items():
        c, kk = k.split("/", 1)
        out.setdefault(c, {})[kk] = v
    return out


def unstack(st, b):
    return {k: v[b] for k, v in st.items()}


def kat():
    return split_cases(load("kat.npz"))


def mixed():
    return split_cases(load("synth_mixed.npz"))


def synth():
    return load("synth_50x20.npz")


def c2():
    return load("c2_1000x100.npz")


def oracle_args(case):
    """Constructor kwargs equivalent to the ones the reference was run with."""
    R = case["in_reports"]
    if bool(case["in_int_dtype"]):
        R = R.astype(np.int64)
    kw = dict(reports=R)
    if bool(case["in_has_bounds"]):
        kw["event_bounds"] = [{"scaled": bool(s), "min": float(a), "max": float(b)}
                              for s, a, b in zip(case["in_scaled"], case["in_lo"], case["in_hi"])]
    if bool(case["in_has_rep"]):
        kw["reputation"] = case["in_reputation"]
    kw["catch_tolerance"] = float(case["in_catch_tolerance"])
    kw["alpha"] = float(case["in_alpha"])
    kw["algorithm"] = str(case["in_algorithm"])
    return kw


def flat_result(res):
    """Result dict -> {key: float64 array}, same keys as the fixtures."""
    f = lambda v: np.asarray(np.ma.filled(np.ma.asarray(v, dtype=np.float64), np.nan), dtype=np.float64)
    d = {"original": f(res["original"]), "filled": f(np.asarray(res["filled"]))}
    for k in AGENT_KEYS:
        d["agents." + k] = f(res["agents"][k])
    for k in EVENT_KEYS:
        d["events." + k] = f(res["events"][k])
    d["participation"] = f(res["participation"])
    d["avg_certainty"] = f(res["avg_certainty"])
    d["convergence"] = np.array(bool(res["convergence"]))
    d["components"] = np.array(int(res["components"]))
    return d


# keys whose sign follows the eigenvector sign (LAPACK-defined, quirk Q8)
SIGNED_KEYS = ("agents.scores", "events.adj_first_loadings")


def algos():
    """big-five / fixed-variance / cokurtosis / absolute cases (make_golden.py algos_main)."""
    return split_cases(load("algos.npz"))


def algo_kwargs(case):
    """Extra constructor kwargs of an algos.npz case."""
    kw = {"max_components": int(case["in_max_components"]),
          "variance_threshold": float(case["in_variance_threshold"])}
    if "in_aux_scores" in case:
        kw["aux"] = {"cokurt": case["in_aux_scores"]}
    return kw


def clusters():
    """k-means / hierarchical / clusterfeck cases (make_golden.py clusters_main)."""
    return split_cases(load("clusters.npz"))


def cluster_kwargs(case):
    """Extra constructor kwargs of a clusters.npz case (k-means also needs numpy's global
    RandomState seeded with case['in_np_seed'] before the call)."""
    return {"hierarchy_threshold": float(case["in_hierarchy_threshold"])}


# --- the workgroup-per-round golden set (make_golden.py medium_main) -------------------
MEDIUM_SHAPES = ((100, 50), (250, 60), (256, 64))
MEDIUM_ROUNDS = 40


def medium_inputs(N, E):
    """The seeded inputs of the medium golden set (synthetic.rounds: numpy's default_rng,
    identical on any host); every third round with reputation=None."""
    from pyconsensus_amd import synthetic

    R, sc, lo, hi, rep = synthetic.rounds(MEDIUM_ROUNDS, N, E, seed=5000 + N + E)
    uniform = np.arange(MEDIUM_ROUNDS) % 3 == 2
    return R, sc, lo, hi, rep, uniform


def medium():
    """{shape: [case, ...]} of medium.npz with the inputs regenerated (checked against the
    stored sha256) and the original / filled matrices rebuilt exactly: original = the
    reference's rescale (:266-269), filled = original with every missing cell of a column
    set to that column's stored fill value (:310-312)."""
    import hashlib

    flat = split_cases(load("medium.npz"))
    out = {}
    for N, E in MEDIUM_SHAPES:
        R, sc, lo, hi, rep, uniform = medium_inputs(N, E)
        cases = []
        for b in range(R.shape[0]):
            c = dict(flat["w%dx%d_%02d" % (N, E, b)])
            X = np.array(R[b], dtype=np.float64)
            assert hashlib.sha256(np.ascontiguousarray(X).tobytes()).hexdigest() == str(c["in_sha256"])
            c["in_reports"] = X.copy()
            c["in_scaled"], c["in_lo"], c["in_hi"] = sc[b].astype(bool), lo[b], hi[b]
            if not uniform[b]:
                c["in_reputation"] = rep[b]
            for j in np.nonzero(sc[b])[0]:
                X[:, j] = (X[:, j] - lo[b][j]) / float(hi[b][j] - lo[b][j])
            miss = np.isnan(X) | (X == 0.0)
            F = X.copy()
            for j in np.nonzero(miss.any(axis=0))[0]:
                F[miss[:, j], j] = c["fill_value"][j]
            c["original"], c["filled"] = X, F
            cases.append(c)
        out[(N, E)] = cases
    return out
