"""Generate the golden vectors in tests/golden/ from the reference itself.

Runs ONLY in the build container (it reads /root/reference, which never travels
to the GPU box).  The committed ``*.npz`` files are data: inputs and the
reference's outputs.  No reference source is stored anywhere in the repo; this
script reads ``/root/reference/pyconsensus/__init__.py`` as text at run time and
applies the harness of SURVEY.md Appendix A in memory:

1. ``lib2to3`` ``fix_print`` (the reference is Python 2: ``print exc`` at :332);
2. the float subscript at :312 wrapped in ``int()`` (numpy < 1.12 truncated float
   indices; numpy 2 raises);
3. ``np.matrix`` at :322 replaced by ``np.asarray`` (same BLAS arithmetic, 1-D
   vector shapes; the matrix form breaks at :492 under numpy 2.2);
4. a ``weightedstats`` module injected (the reference's unvendored, uninstalled
   dependency, ``requirements.txt:2``), restating the published pure-Python
   ``weighted_median``.

Usage:  python tests/golden/make_golden.py [algos | clusters | medium]   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import math
import os
import sys
import types
import warnings

import numpy as np

warnings.simplefilter("ignore")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
REF = "/root/reference/pyconsensus/__init__.py"


# --------------------------------------------------------------------------- harness
def _weightedstats_module():
    """Literal pure-Python restatement of weightedstats.weighted_median."""
    mod = types.ModuleType("weightedstats")

    def weighted_median(data, weights=None):
        if weights is None:
            s = sorted(data)
            n = len(s)
            return s[n // 2] if n % 2 else (s[n // 2 - 1] + s[n // 2]) / 2.0
        midpoint = 0.5 * sum(weights)
        if any([j > midpoint for j in weights]):
            wl = list(weights)
            return data[wl.index(max(wl))]
        if any([j > 0 for j in weights]):
            sorted_data, sorted_weights = zip(*sorted(zip(data, weights)))
            cumulative_weight = 0
            below = 0
            while cumulative_weight <= midpoint:
                below += 1
                cumulative_weight += sorted_weights[below - 1]
            cumulative_weight -= sorted_weights[below - 1]
            if abs(cumulative_weight - midpoint) < sys.float_info.epsilon:
                bounds = sorted_data[below - 2:below]
                return sum(bounds) / float(len(bounds))
            return sorted_data[below - 1]
        return None

    mod.weighted_median = weighted_median
    return mod


def load_reference():
    from lib2to3.refactor import RefactoringTool

    sys.modules["weightedstats"] = _weightedstats_module()
    src = open(REF).read()
    src = str(RefactoringTool(["lib2to3.fixes.fix_print"]).refactor_string(src, "pyconsensus"))
    a = "reports_copy[nan_indices[j],i] = guess"
    b = "wcd = np.matrix(reports_filled - weighted_mean)"
    assert a in src and b in src, "reference text changed; harness patches do not apply"
    src = src.replace(a, "reports_copy[int(nan_indices[j]),i] = guess")
    src = src.replace(b, "wcd = np.asarray(reports_filled - weighted_mean)")
    mod = types.ModuleType("pyconsensus_reference_harness")
    mod.__file__ = REF
    exec(compile(src, REF, "exec"), mod.__dict__)
    return mod


# --------------------------------------------------------------------------- near ties
def _normalize(v):
    v = np.abs(v)
    if np.sum(v) == 0:
        v = v + 1
    return v / np.sum(v)


def _rank_vectors(s, F, rep, dot):
    from scipy.stats import rankdata

    set1 = s + abs(s.min())
    set2 = s - s.max()
    old = dot(rep, F)
    r0 = rankdata(old)
    r1 = rankdata(dot(_normalize(set1), F) + 0.01 * old)
    r2 = rankdata(dot(_normalize(set2), F) + 0.01 * old)
    return r0, r1, r2


def _rank_decision(s, F, rep, dot):
    r0, r1, r2 = _rank_vectors(s, F, rep, dot)
    ri = np.sum(np.abs(r1 - r0)) - np.sum(np.abs(r2 - r0))
    return 0 if ri == 0 else (1 if ri < 0 else 2)


def _decision_full(s, F, rep, dot):
    """1/2: rank rule picks set1/set2; 3/4: exact rank tie, continuous rule picks set1/set2."""
    d = _rank_decision(s, F, rep, dot)
    if d:
        return d
    set1 = s + abs(s.min())
    set2 = s - s.max()
    old = dot(rep, F)
    e1 = dot(_normalize(set1), F) - old
    e2 = dot(_normalize(set2), F) - old
    if dot is _dot_exact:
        ref = math.fsum(e1 ** 2) - math.fsum(e2 ** 2)
    else:
        ref = np.sum(e1 ** 2) - np.sum(e2 ** 2)
    return 3 if ref <= 0 else 4


def _rank_neartie(s, F, rep):
    """The sign-choice rule depends on rounding: the three rank vectors from np.dot
    differ from those of correctly rounded (fsum) dots, or the decision flips when
    the dots are summed in another order."""
    a = _rank_vectors(s, F, rep, np.dot)
    b = _rank_vectors(s, F, rep, _dot_exact)
    if any(not np.array_equal(x, y) for x, y in zip(a, b)):
        return True
    dec = _decision_full(s, F, rep, np.dot)
    if any(_decision_full(s, F, rep, f) != dec for f in (_dot_exact, _dot_rev)):
        return True
    # scores are themselves BLAS/LAPACK output: the decision must survive score
    # perturbations at the 1e-13 level, and scores rounded to 12 digits (which
    # restores exact ties that rounding broke)
    rng = np.random.default_rng(0)
    trials = [np.round(s, 12)] + [s * (1.0 + 1e-13 * rng.standard_normal(s.shape)) for _ in range(6)]
    return any(_decision_full(t, F, rep, _dot_exact) != dec for t in trials)


def _dot_exact(w, F):
    return np.array([math.fsum(w * F[:, j]) for j in range(F.shape[1])])


def _dot_rev(w, F):
    return np.array([sum((w * F[:, j])[::-1].tolist()) for j in range(F.shape[1])])


def _median_margin(x, w):
    """Smallest |prefix - midpoint| over (value, weight)-sorted prefixes."""
    w = np.asarray(w, float)
    if w.size == 0:
        return np.inf
    mid = 0.5 * math.fsum(w)
    o = np.lexsort((w, np.asarray(x, float)))
    cum = np.cumsum(w[o])
    return float(np.min(np.abs(cum - mid)))


def _continuous_decision(s, F, rep, dot):
    set1 = s + abs(s.min())
    set2 = s - s.max()
    old = dot(rep, F)
    e1 = dot(_normalize(set1), F) - old
    e2 = dot(_normalize(set2), F) - old
    if dot is _dot_exact:
        ref = math.fsum(e1 ** 2) - math.fsum(e2 ** 2)
    else:
        ref = np.sum(e1 ** 2) - np.sum(e2 ** 2)
    return 3 if ref <= 0 else 4


def _continuous_neartie(s, F, rep):
    """nonconformity's decision depends on rounding: it differs under correctly
    rounded dots, or its margin is within 1e-9 of the two sums' size."""
    dec = _continuous_decision(s, F, rep, np.dot)
    if _continuous_decision(s, F, rep, _dot_exact) != dec:
        return True
    set1 = s + abs(s.min())
    set2 = s - s.max()
    old = _dot_exact(rep, F)
    a = math.fsum((_dot_exact(_normalize(set1), F) - old) ** 2)
    b = math.fsum((_dot_exact(_normalize(set2), F) - old) ** 2)
    return abs(a - b) <= 1e-9 * (a + b) or not np.all(np.isfinite(s))


def _eig_neartie(cov, algorithm, o):
    """big-five / fixed-variance results depend on LAPACK choices: a used component
    whose singular value is (nearly) repeated has no defined eigenvector; a loading
    with loading[0] ~ 0 has no defined sign (the reference flips on loading[0] < 0);
    the fixed-variance count can flip at the threshold."""
    C = np.asarray(cov, float)
    if not np.all(np.isfinite(C)):
        return True
    U, S, _ = np.linalg.svd(C)
    E = S.size
    k = min(o.max_components, E) if algorithm == "big-five" else int(o.num_components)
    scale = S[0] if S.size and S[0] > 0 else 1.0
    for i in range(min(k, E)):
        gaps = []
        if i > 0:
            gaps.append(S[i - 1] - S[i])
        if i + 1 < E:
            gaps.append(S[i] - S[i + 1])
        if S[i] > 1e-12 * scale and gaps and min(gaps) <= 1e-6 * scale:
            return True
        if S[i] > 1e-12 * scale and abs(U[0, i]) <= 1e-9:
            return True
    if algorithm == "fixed-variance":
        ve = np.cumsum(S / np.trace(C))
        if np.any(np.abs(ve - o.variance_threshold) <= 1e-9):
            return True
    return False


# --------------------------------------------------------------------------- runner
OUT_KEYS_AGENTS = ["old_rep", "this_rep", "smooth_rep", "na_row", "participation_rows",
                   "relative_part", "reporter_bonus", "scores"]
OUT_KEYS_EVENTS = ["adj_first_loadings", "outcomes_raw", "consensus_reward", "certainty",
                   "NAs Filled", "participation_columns", "author_bonus",
                   "outcomes_adjusted", "outcomes_final"]


def _f(v):
    return np.asarray(np.ma.filled(np.ma.asarray(v, dtype=np.float64), np.nan), dtype=np.float64)


def run_case(ref, reports, bounds=None, reputation=None, **kw):
    """Run the reference on one case; return a flat dict of numpy arrays."""
    cap = {}
    orig_rank = ref.Oracle.nonconformity_rank
    orig_nc = ref.Oracle.nonconformity

    def rank_hook(self, scores, F):
        cap["s"] = np.asarray(scores, float).ravel().copy()
        cap["F"] = np.asarray(F, float).copy()
        cap["rep"] = self.reputation.copy()
        cap["fallback"] = False
        return orig_rank(self, scores, F)

    def nc_hook(self, scores, F):
        cap["fallback"] = True
        if "s" not in cap:  # non-PCA algorithms call nonconformity directly (:389, :450, :456)
            cap["nc_s"] = np.asarray(scores, float).ravel().copy()
            cap["nc_F"] = np.asarray(F, float).copy()
            cap["nc_rep"] = self.reputation.copy()
        return orig_nc(self, scores, F)

    orig_wpca = ref.Oracle.wpca

    def wpca_hook(self, F):
        r = orig_wpca(self, F)
        cap["cov"] = np.asarray(r[2], float).copy()
        return r

    ref.Oracle.nonconformity_rank = rank_hook
    ref.Oracle.nonconformity = nc_hook
    ref.Oracle.wpca = wpca_hook
    try:
        if isinstance(reports, np.ndarray) and not isinstance(reports, np.ma.MaskedArray):
            arg = reports.copy()  # the reference mutates float ndarrays (Q2)
        else:
            arg = reports
        o = ref.Oracle(reports=arg, event_bounds=bounds, reputation=reputation, **kw)
        res = o.consensus()
    finally:
        ref.Oracle.nonconformity_rank = orig_rank
        ref.Oracle.nonconformity = orig_nc
        ref.Oracle.wpca = orig_wpca
    data = np.ma.getdata(reports) if isinstance(reports, np.ma.MaskedArray) else np.asarray(reports)
    d = {
        "in_reports": np.asarray(data, dtype=np.float64),
        "in_int_dtype": np.array(np.issubdtype(np.asarray(data).dtype, np.integer)),
        "in_has_bounds": np.array(bounds is not None),
        "in_has_rep": np.array(reputation is not None),
        "in_catch_tolerance": np.array(float(kw.get("catch_tolerance", 0.1))),
        "in_alpha": np.array(float(kw.get("alpha", 0.1))),
        "in_algorithm": np.array(kw.get("algorithm", "PCA")),
    }
    E = d["in_reports"].shape[1]
    if bounds is not None:
        d["in_scaled"] = np.array([bool(b["scaled"]) for b in bounds])
        d["in_lo"] = np.array([float(b["min"]) for b in bounds])
        d["in_hi"] = np.array([float(b["max"]) for b in bounds])
    if reputation is not None:
        d["in_reputation"] = np.asarray(reputation, dtype=np.float64).ravel()
    d["original"] = _f(res["original"])
    d["filled"] = _f(np.asarray(res["filled"]))
    for k in OUT_KEYS_AGENTS:
        d["agents." + k] = _f(res["agents"][k])
    for k in OUT_KEYS_EVENTS:
        d["events." + k] = _f(res["events"][k])
    for k in ("participation", "avg_certainty"):
        d[k] = np.array(float(np.ma.filled(res[k], np.nan)))
    d["convergence"] = np.array(bool(res["convergence"]))
    d["components"] = np.array(int(res["components"]))
    d["reptokens"] = np.asarray(o.reptokens, dtype=np.int64)
    # diagnostics + near-tie flags (parity reports separate these rounds)
    if "s" in cap:
        s, F, rep = cap["s"], cap["F"], cap["rep"]
        dec = _decision_full(s, F, rep, np.dot)
        assert (dec >= 3) == cap["fallback"]
        d["branch"] = np.array(dec)
        # the same decision in exact arithmetic (correctly rounded dots)
        d["branch_exact"] = np.array(_decision_full(s, F, rep, _dot_exact))
        d["neartie_rank"] = np.array(bool(_rank_neartie(s, F, rep)))
    elif "nc_s" in cap:  # continuous rule only: 3 = set1 (ref <= 0), 4 = set2
        s_, F_, rep_ = cap["nc_s"], cap["nc_F"], cap["nc_rep"]
        d["branch"] = np.array(_continuous_decision(s_, F_, rep_, np.dot))
        d["branch_exact"] = np.array(_continuous_decision(s_, F_, rep_, _dot_exact))
        d["neartie_rank"] = np.array(bool(_continuous_neartie(s_, F_, rep_)))
    else:
        d["branch"] = np.array(5)
        d["branch_exact"] = np.array(5)
        d["neartie_rank"] = np.array(False)
    d["in_max_components"] = np.array(int(kw.get("max_components", 5)))
    d["in_variance_threshold"] = np.array(float(kw.get("variance_threshold", 0.9)))
    if kw.get("aux") is not None:
        d["in_aux_scores"] = np.asarray(kw["aux"]["cokurt"], dtype=np.float64).ravel()
    d["neartie_eig"] = np.array(bool("cov" in cap and kw.get("algorithm") in ("big-five", "fixed-variance")
                                     and _eig_neartie(cap["cov"], kw.get("algorithm"), o)))
    raw = d["events.outcomes_raw"]
    tol = float(kw.get("catch_tolerance", 0.1))
    thr = np.array([1.5 - tol, 1.5 + tol])
    scaled = d.get("in_scaled", np.zeros(E, bool))
    bin_raw = raw[~scaled]
    d["neartie_catch"] = np.array(bool(bin_raw.size and np.min(np.abs(bin_raw[:, None] - thr[None, :])) < 1e-12))
    d["neartie_catch_fill"] = np.array(False)
    if "s" in cap:  # interpolation guesses of binary columns (sequential weighted means)
        X, Fm = d["original"], cap["F"]
        miss = np.isnan(X) | (X == 0.0)
        for j in np.nonzero(miss.any(axis=0) & ~scaled)[0]:
            pres = ~miss[:, j]
            if pres.any():
                g = math.fsum(cap["rep"][pres] * X[pres, j]) / math.fsum(cap["rep"][pres])
                if np.min(np.abs(g - thr)) < 1e-12:
                    d["neartie_catch_fill"] = np.array(True)
    F = d["filled"]
    sm = d["agents.smooth_rep"]
    margins = [_median_margin(F[:, j], sm) for j in np.nonzero(scaled)[0]]
    d["neartie_median"] = np.array(bool(margins and min(margins) < 1e-12))
    margins = []
    # interpolation medians (present reports, reputation weights) -- exact ties here are
    # common with integer reputations (a sorted prefix holding exactly half the weight)
    if "s" in cap:
        X = d["original"]
        miss = np.isnan(X) | (X == 0.0)
        for j in np.nonzero(miss.any(axis=0) & scaled)[0]:
            pres = ~miss[:, j]
            if pres.any():
                r = cap["rep"][pres]
                margins.append(_median_margin(X[pres, j], r / math.fsum(r)))
    d["neartie_median_fill"] = np.array(bool(margins and min(margins) < 1e-12))
    return d


def _stack(dicts):
    keys = dicts[0].keys()
    return {k: np.stack([x[k] for x in dicts]) for k in keys}


# --------------------------------------------------------------------------- cases
YES, NO, BAD, NA = 2.0, 1.0, 1.5, 0.0


def kat_cases():
    """Known-answer inputs: README, module docstring, CLI matrices, reference tests, quirks."""

    Y, N_, B, Z = YES, NO, BAD, NA
    c = {}
    # README.rst:28-45 (config C1)
    c["readme"] = dict(
        reports=[[0.2, 0.7, 1, 1], [0.3, 0.5, 1, 1], [0.1, 0.7, 1, 1],
                 [0.5, 0.7, 2, 1], [0.1, 0.2, 2, 2], [0.1, 0.2, 2, 2]],
        reputation=[1, 2, 10, 9, 4, 2],
        bounds=[{"scaled": True, "min": 0.1, "max": 0.5}, {"scaled": True, "min": 0.2, "max": 0.7},
                {"scaled": False, "min": 1, "max": 2}, {"scaled": False, "min": 1, "max": 2}])
    # module docstring, __init__.py:15-29
    c["docstring"] = dict(
        reports=[[0.2, 0.7, -1, -1], [0.3, 0.5, -1, -1], [0.1, 0.7, -1, -1],
                 [0.5, 0.7, 1, -1], [0.1, 0.2, 1, 1], [0.1, 0.2, 1, 1]],
        bounds=[{"scaled": True, "min": 0.1, "max": 0.5}, {"scaled": True, "min": 0.2, "max": 0.7},
                {"scaled": False, "min": -1, "max": 1}, {"scaled": False, "min": -1, "max": 1}])
    # CLI -t matrices (__init__.py:630-841), rebuilt from their row patterns
    r17 = [[Y, Y, N_, N_], [Y, N_, N_, N_], [Y, Y, N_, N_], [Y, Y, Y, N_], [N_, N_, Y, Y], [N_, N_, Y, Y]]
    c["t1"] = dict(reports=r17)
    c["t17"] = dict(reports=r17)
    r2 = [[Y, Y, N_, N_]] * 6 + [[Y, Y, Y, N_]] * 5
    c["t2"] = dict(reports=r2)
    c["t14"] = dict(reports=r2)
    a3 = [Y, Y, N_, N_, Y, Y, N_, N_, Y, Y, N_, N_, Y]
    b3 = [N_, N_, N_, Y, N_, N_, N_, Y, N_, N_, N_, Y, N_]
    d3 = [Y, Y, Y, N_, Y, Y, Y, N_, Y, Y, Y, N_, Y]
    c["t3"] = dict(reports=[a3] * 6 + [b3] + [d3] * 4)
    a4, b4, d4 = [Y, Y, N_, N_, Y], [N_, N_, N_, Y, N_], [Y, Y, Y, N_, Y]
    r4 = [a4] * 15 + [b4] + [d4] * 5 + [a4] * 4
    c["t4"] = dict(reports=r4)
    c["t15"] = dict(reports=r4)
    c["t5"] = dict(reports=[
        [B, N_, N_, Y, N_, N_, Y, Y, B, B], [B, B, N_, B, B, Y, Y, B, Y, B],
        [N_, Y, B, B, N_, Y, N_, N_, B, B], [B, B, B, B, B, N_, N_, N_, B, Y],
        [N_, Y, Y, B, B, Y, B, Y, B, Y], [N_, Y, Y, Y, N_, B, N_, B, B, B],
        [N_, N_, N_, Y, N_, N_, N_, Y, B, Y], [B, B, B, Y, B, Y, B, B, Y, N_],
        [B, B, B, N_, B, Y, Y, N_, N_, B], [B, Y, B, Y, N_, N_, Y, Y, N_, B],
        [Y, Y, B, B, B, Y, B, B, Y, Y], [Y, B, Y, N_, Y, B, Y, N_, Y, B]]
        + [[N_, N_, N_, Y, Y, Y, B, Y, B, N_]] * 7 + [[B, B, B, Y, B, Y, B, B, Y, N_]])
    r6 = ([[N_, N_, Y, Y, N_, Y, N_, N_, N_, N_], [Y, Y, N_, N_, N_, Y, Y, Y, N_, Y],
           [Y, Y, N_, Y, N_, Y, Y, N_, Y, Y], [N_, Y, N_, N_, Y, N_, Y, N_, N_, Y],
           [N_, N_, Y, N_, Y, N_, N_, N_, N_, N_], [N_, Y, N_, N_, N_, Y, Y, N_, Y, Y],
           [Y, N_, N_, Y, Y, N_, Y, N_, N_, N_], [Y, Y, N_, N_, Y, N_, Y, Y, Y, N_]]
          + [[Y, N_, N_, Y, N_, Y, N_, N_, N_, Y]] * 11 + [[N_, Y, N_, N_, Y, N_, Y, N_, N_, Y]])
    c["t6"] = dict(reports=r6)
    c["t16"] = dict(reports=r6)
    c["t7"] = dict(reports=[[Y] * 6, [Y, Y, Y, N_, N_, N_], [Z] * 6])
    c["t8"] = dict(reports=[[Y] * 6, [Y, Y, Y, N_, Z, Z], [Y, Y, Y, Z, Z, N_]])
    c["t9"] = dict(reports=[[Y] * 6, [Y, Y, Y, N_, Z, Z], [Y, Y, Y, N_, Z, Z]])
    c["t10"] = dict(reports=[[Y, Y, Y, N_, Y, Y], [Y, Y, Y, N_, Z, Z], [Y, Y, Y, N_, Z, Z]])
    c["t11"] = dict(reports=[[Y] * 6, [Z] * 6, [Y, Y, Y, N_, N_, N_]])
    c["t12"] = dict(reports=[[Y, Y, Y, N_, N_, N_]] * 3)
    c["t13"] = dict(reports=[[Y, Y, Y, N_, N_, N_]])
    c["t18"] = dict(reports=[[Y, Y, N_, N_], [Y, N_, N_, N_]] + [[Z] * 4] * 14)
    # CLI -m (:863-876) and -s (:877-895)
    c["missing"] = dict(
        reports=[[Y, Y, N_, Z], [Y, N_, N_, N_], [Y, Y, N_, N_], [Y, Y, Y, N_], [Z, N_, Y, Y], [N_, N_, Y, Y]],
        reputation=[2, 10, 4, 2, 7, 1])
    c["scaled_cli"] = dict(
        reports=[[Y, Y, N_, N_, 233, 16027.59], [Y, N_, N_, N_, 199, Z], [Y, Y, N_, N_, 233, 16027.59],
                 [Y, Y, Y, N_, 250, Z], [N_, N_, Y, Y, 435, 8001.00], [N_, N_, Y, Y, 435, 19999.00]],
        bounds=[{"scaled": False, "min": N_, "max": 1}] * 4 + [
            {"scaled": True, "min": 0, "max": 435}, {"scaled": True, "min": 8000, "max": 20000}])
    # reference tests (test_consensus.py:28-158): 0/1 convention (0 == NA here)
    base = [[1, 1, 0, 0], [1, 0, 0, 0], [1, 1, 0, 0], [1, 1, 1, 0], [0, 0, 1, 1], [0, 0, 1, 1]]
    nanr = [[1, 1, 0, 0], [1, 0, 0, 0], [1, 1, np.nan, 0], [1, 1, 1, 0], [0, 0, 1, 1], [0, 0, 1, 1]]
    sc = [[0.3, 0.2, 0, 0], [0.5, 0.3, 0, 0], [0.4, 0.1, 0, 0], [0.2, 0.7, 1, 0], [0.1, 0.3, 1, 1], [0.15, 0.2, 1, 1]]
    scn = [[0.3, 0.2, 0, 0], [0.5, 0.3, np.nan, 0], [0.4, 0.1, 0, 0], [0.2, 0.7, 1, 0], [0.1, 0.3, 1, 1], [0.15, 0.2, 1, 1]]
    sb = [{"scaled": True, "min": 0.1, "max": 0.5}, {"scaled": True, "min": 0.2, "max": 0.7},
          {"scaled": False, "min": 0, "max": 1}, {"scaled": False, "min": 0, "max": 1}]
    c["test_base_int"] = dict(reports=base)
    c["test_base_weighted"] = dict(reports=base, reputation=np.array([1, 1, 1, 1, 1, 1]))
    c["test_nans"] = dict(reports=np.array(nanr))
    c["test_nans_weighted"] = dict(reports=np.array(nanr), reputation=np.array([1] * 6))
    c["test_scaled"] = dict(reports=sc, bounds=sb)
    c["test_scaled_nans"] = dict(reports=np.array(scn), bounds=sb)
    c["test_weighted_scaled_nans"] = dict(reports=np.array(scn), bounds=sb, reputation=np.array([1] * 6))
    c["test_array"] = dict(reports=np.array(base))
    c["test_masked"] = dict(reports=np.ma.masked_array(base, np.isnan(base)))
    # the same tests shifted to the current 1/2 convention (binary columns + 1)
    c["test_base_shift"] = dict(reports=(np.array(base, float) + 1.0))
    c["test_nans_shift"] = dict(reports=(np.array(nanr, float) + 1.0))
    # quirks
    c["q_catch_tol"] = dict(reports=r17, catch_tolerance=0.3)
    c["q_alpha"] = dict(reports=r17, reputation=[2, 10, 4, 2, 7, 1], alpha=0.25)
    c["q_int_fill"] = dict(reports=[[2, 2, 1, 0], [2, 1, 1, 1], [1, 2, 0, 2], [2, 2, 2, 1], [1, 1, 2, 2], [1, 1, 2, 2]])
    # int dtype + scaled: rescaled values truncate to 0 (-> missing) unless == max
    c["q_int_scaled"] = dict(reports=[[3, 2, 1, 10], [8, 1, 1, 1], [4, 2, 0, 2], [8, 2, 2, 7], [1, 1, 2, 10], [7, 1, 2, 0]],
                             bounds=[{"scaled": True, "min": 1, "max": 8}, {"scaled": False, "min": 1, "max": 2},
                                     {"scaled": False, "min": 1, "max": 2}, {"scaled": True, "min": 0, "max": 10}])
    c["q_scaled_eq_min"] = dict(reports=[[0.1, 1, 2], [0.3, 2, 2], [0.5, 1, 1], [0.1, 2, 1], [0.4, 2, 2]],
                                bounds=[{"scaled": True, "min": 0.1, "max": 0.5},
                                        {"scaled": False, "min": 1, "max": 2}, {"scaled": False, "min": 1, "max": 2}])
    c["q_all_missing_col"] = dict(reports=[[2, np.nan, 1], [1, np.nan, 1], [2, np.nan, 2], [2, np.nan, 1]],
                                  reputation=[3, 1, 2, 5])
    c["q_all_missing_scaled_col"] = dict(
        reports=[[2, np.nan, 1, 0.4], [1, np.nan, 1, 0.2], [2, np.nan, 2, 0.9], [2, np.nan, 1, 0.7]],
        bounds=[{"scaled": False, "min": 1, "max": 2}, {"scaled": True, "min": 0, "max": 1},
                {"scaled": False, "min": 1, "max": 2}, {"scaled": True, "min": 0, "max": 1}],
        reputation=[3, 1, 2, 5])
    c["q_single_reporter"] = dict(reports=[[2.0, 1.0, 2.0, 1.0]])
    c["q_identical_rows_scaled"] = dict(reports=[[0.3, 2.0, 0.7]] * 5,
                                        bounds=[{"scaled": True, "min": 0, "max": 1},
                                                {"scaled": False, "min": 1, "max": 2},
                                                {"scaled": True, "min": 0, "max": 1}])
    c["q_half_median"] = dict(reports=[[0.2, 1], [0.4, 1], [0.6, 2], [0.8, 2]],
                              bounds=[{"scaled": True, "min": 0, "max": 1}, {"scaled": False, "min": 1, "max": 2}])
    c["q_float_rep"] = dict(reports=r17, reputation=[0.3, 1.7, 2.25, 0.05, 1.0, 3.3])
    return c


def main():
    ref = load_reference()
    from pyconsensus_amd import synthetic

    out = {}
    for name, spec in kat_cases().items():
        kw = {k: v for k, v in spec.items() if k not in ("reports", "bounds", "reputation")}
        d = run_case(ref, spec["reports"], spec.get("bounds"), spec.get("reputation"), **kw)
        for k, v in d.items():
            out[name + "/" + k] = v
    np.savez_compressed(os.path.join(HERE, "kat.npz"), **out)
    print("kat cases:", len(kat_cases()))

    # seeded synthetic 50x20 rounds (the C3 round shape), 600 rounds, seed 7
    R, scaled, lo, hi, rep = synthetic.rounds(600, 50, 20, seed=7)
    rows = []
    for b in range(R.shape[0]):
        d = run_case(ref, R[b], synthetic.bounds_list(scaled[b], lo[b], hi[b]), rep[b])
        del d["original"]  # = rescaled inputs; kept for the small suites only (size)
        rows.append(d)
    st = _stack(rows)
    np.savez_compressed(os.path.join(HERE, "synth_50x20.npz"), **st)
    print("synth_50x20: branch counts", np.bincount(st["branch"].astype(int)),
          "exact-arith branch differs", int(np.sum(st["branch"] != st["branch_exact"])),
          "fill near-ties catch/median", st["neartie_catch_fill"].sum(), st["neartie_median_fill"].sum(),
          "near-ties rank/catch/median", st["neartie_rank"].sum(), st["neartie_catch"].sum(),
          st["neartie_median"].sum())

    # mixed small shapes (batched-kernel generality), uniform and weighted reputation
    rng = np.random.default_rng(11)
    mixed = {}
    for k in range(120):
        n = int(rng.integers(2, 65))
        e = int(rng.integers(2, 33))
        Rm, sm, lom, him, repm = synthetic.rounds(1, n, e, seed=1000 + k, reputation=bool(k % 3))
        d = run_case(ref, Rm[0], synthetic.bounds_list(sm[0], lom[0], him[0]) if k % 4 else None,
                     None if repm is None else repm[0])
        for kk, v in d.items():
            mixed["m%03d/%s" % (k, kk)] = v
    np.savez_compressed(os.path.join(HERE, "synth_mixed.npz"), **mixed)
    print("synth_mixed: 120 cases")

    algos_main(ref)

    # config C2: 1000 x 100, seed 1
    Rc, sc_, loc, hic, repc = synthetic.matrix(1000, 100, seed=1)
    d = run_case(ref, Rc, synthetic.bounds_list(sc_, loc, hic), repc)
    np.savez_compressed(os.path.join(HERE, "c2_1000x100.npz"), **d)
    print("c2 done; branch", d["branch"])


def algos_main(ref):
    """algorithm = big-five / fixed-variance / cokurtosis:
    KAT matrices, seeded 50 x 20 rounds, mixed small shapes, and matrix-path sizes."""
    from pyconsensus_amd import synthetic

    out = {}
    algos = ("big-five", "fixed-variance", "cokurtosis")

    def add(name, reports, bounds, rep, alg, seed, **extra):
        N = np.asarray(reports).shape[0]
        kw = dict(algorithm=alg, **extra)
        if alg == "cokurtosis":
            kw["aux"] = {"cokurt": np.random.default_rng(seed).normal(0.0, 1.0, N)}
        d = run_case(ref, reports, bounds, rep, **kw)
        for k, v in d.items():
            out[name + "/" + k] = v

    kats = kat_cases()
    for nm in ("readme", "docstring", "t1", "t3", "t5", "t6", "t8", "missing", "scaled_cli", "test_base_shift",
               "q_float_rep", "q_alpha"):
        spec = kats[nm]
        kw = {k: v for k, v in spec.items() if k not in ("reports", "bounds", "reputation")}
        for a_i, alg in enumerate(algos):
            add("%s@%s" % (nm, alg), spec["reports"], spec.get("bounds"), spec.get("reputation"), alg,
                1000 + a_i, **kw)
    # CLI -x (__init__.py:849-862): the "absolute" branch (no nonconformity, Q13)
    add("x_example@absolute", kats["t1"]["reports"], None, [2, 10, 4, 2, 7, 1], "absolute", 0)
    add("missing@absolute", kats["missing"]["reports"], None, kats["missing"]["reputation"], "absolute", 0)
    for a_i, alg in enumerate(algos):
        R, sc, lo, hi, rep = synthetic.rounds(120, 50, 20, seed=8 + a_i)
        for b in range(R.shape[0]):
            add("s%03d@%s" % (b, alg), R[b], synthetic.bounds_list(sc[b], lo[b], hi[b]), rep[b], alg, 77 * b + a_i)
        rng = np.random.default_rng(31 + a_i)
        for k in range(30):
            n, e = int(rng.integers(3, 65)), int(rng.integers(2, 33))
            Rm, sm, lom, him, repm = synthetic.rounds(1, n, e, seed=5000 + 100 * a_i + k, reputation=bool(k % 3))
            extra = {"max_components": int(rng.integers(1, 7))} if alg == "big-five" else {}
            if alg == "fixed-variance":
                extra = {"variance_threshold": float(rng.choice([0.5, 0.75, 0.9, 0.99]))}
            add("m%03d@%s" % (k, alg), Rm[0], synthetic.bounds_list(sm[0], lom[0], him[0]) if k % 4 else None,
                None if repm is None else repm[0], alg, 9000 + k, **extra)
        for (n, e) in ((300, 40), (1200, 64)):  # matrix-path sizes
            Rb, sb, lb, hb, rb = synthetic.matrix(n, e, seed=n + e + a_i)
            add("big%dx%d@%s" % (n, e, alg), Rb, synthetic.bounds_list(sb, lb, hb), rb, alg, n)
    np.savez_compressed(os.path.join(HERE, "algos.npz"), **out)
    cases = split_keys(out)
    nt = sum(bool(v.get("neartie_rank", False)) or bool(v.get("neartie_eig", False)) for v in cases.values())
    print("algos: %d cases, %d flagged near-tie" % (len(cases), nt))


def clusters_main(ref):
    """algorithm = k-means / hierarchical / clusterfeck (__init__.py:392-428):
    KAT matrices, seeded 50 x 20 rounds and mixed small shapes (the batched regime).  k-means
    draws its initial code books from numpy's global RandomState (scipy.cluster.vq.kmeans,
    seed=None): every case seeds it first and records the seed (in_np_seed)."""
    from pyconsensus_amd import synthetic

    out = {}
    algos = ("k-means", "hierarchical", "clusterfeck")

    def add(name, reports, bounds, rep, alg, seed, **extra):
        kw = dict(algorithm=alg, **extra)
        np.random.seed(seed)
        d = run_case(ref, reports, bounds, rep, **kw)
        d["in_np_seed"] = np.array(seed)
        d["in_hierarchy_threshold"] = np.array(float(extra.get("hierarchy_threshold", 0.5)))
        for k, v in d.items():
            out[name + "/" + k] = v

    kats = kat_cases()
    for nm in ("readme", "docstring", "t1", "t2", "t3", "t4", "t5", "t6", "t8", "t10", "missing", "scaled_cli",
               "test_base_shift", "q_float_rep", "q_alpha"):
        if nm not in kats:
            continue
        spec = kats[nm]
        kw = {k: v for k, v in spec.items() if k not in ("reports", "bounds", "reputation")}
        for a_i, alg in enumerate(algos):
            extra = dict(kw)
            if alg == "hierarchical":
                extra["hierarchy_threshold"] = 1.5
            add("%s@%s" % (nm, alg), spec["reports"], spec.get("bounds"), spec.get("reputation"), alg,
                2000 + a_i, **extra)
    thr = (0.5, 1.5, 2.5, 3.5)
    for a_i, alg in enumerate(algos):
        R, sc, lo, hi, rep = synthetic.rounds(120, 50, 20, seed=40 + a_i)
        for b in range(R.shape[0]):
            extra = {"hierarchy_threshold": thr[b % 4]} if alg == "hierarchical" else {}
            add("s%03d@%s" % (b, alg), R[b], synthetic.bounds_list(sc[b], lo[b], hi[b]), rep[b], alg,
                100 * b + a_i, **extra)
        rng = np.random.default_rng(61 + a_i)
        for k in range(40):
            n, e = int(rng.integers(2, 65)), int(rng.integers(1, 33))
            Rm, sm, lom, him, repm = synthetic.rounds(1, n, e, seed=7000 + 100 * a_i + k, reputation=bool(k % 3))
            extra = {"hierarchy_threshold": float(rng.choice(thr))} if alg == "hierarchical" else {}
            add("m%03d@%s" % (k, alg), Rm[0], synthetic.bounds_list(sm[0], lom[0], him[0]) if k % 4 else None,
                None if repm is None else repm[0], alg, 9100 + k, **extra)
    np.savez_compressed(os.path.join(HERE, "clusters.npz"), **out)
    cases = split_keys(out)
    print("clusters: %d cases" % len(cases))


def medium_main(ref):
    """Rounds of 100 x 50, 250 x 60 and 256 x 64 (the workgroup-per-round kernel's shapes,
    csrc/pcx_medium.hip), 40 each, PCA, from the reference itself.  Only OUTPUTS are stored
    (plus a checksum of the regenerated inputs): the reports come from medium_inputs(), and
    the filled matrix is stored as its per-column fill value (every missing cell of a column
    takes the same guess, :310-312), which with the inputs gives it back exactly."""
    import hashlib

    sys.path.insert(0, os.path.join(REPO, "tests"))
    from golden_cases import MEDIUM_SHAPES, medium_inputs

    out = {}
    for N, E in MEDIUM_SHAPES:
        R, sc, lo, hi, rep, uniform = medium_inputs(N, E)
        from pyconsensus_amd import synthetic

        for b in range(R.shape[0]):
            d = run_case(ref, R[b], synthetic.bounds_list(sc[b], lo[b], hi[b]), None if uniform[b] else rep[b])
            X, F = d.pop("original"), d.pop("filled")
            miss = np.isnan(X) | (X == 0.0)
            fill = np.full(E, np.nan)
            for j in np.nonzero(miss.any(axis=0))[0]:
                vals = F[miss[:, j], j]
                assert np.all((vals == vals[0]) | (np.isnan(vals) & np.isnan(vals[0])))
                fill[j] = vals[0]
            d["fill_value"] = fill
            d["in_sha256"] = np.array(hashlib.sha256(np.ascontiguousarray(d.pop("in_reports")).tobytes()).hexdigest())
            for k in [k for k in d if k.startswith("in_") and k not in ("in_sha256", "in_has_rep", "in_has_bounds",
                                                                        "in_catch_tolerance", "in_alpha",
                                                                        "in_int_dtype", "in_algorithm")]:
                del d[k]  # regenerated with the reports
            for k, v in d.items():
                out["w%dx%d_%02d/%s" % (N, E, b, k)] = v
        print("medium %dx%d: %d rounds" % (N, E, R.shape[0]))
    np.savez_compressed(os.path.join(HERE, "medium.npz"), **out)


def split_keys(flat):
    res = {}
    for k, v in flat.items():
        c, kk = k.split("/", 1)
        res.setdefault(c, {})[kk] = v
    return res


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "algos":
        algos_main(load_reference())
    elif len(sys.argv) > 1 and sys.argv[1] == "clusters":
        clusters_main(load_reference())
    elif len(sys.argv) > 1 and sys.argv[1] == "medium":
        medium_main(load_reference())
    else:
        main()
