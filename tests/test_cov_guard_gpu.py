"""The int8-emulated covariance against the entries it approximates (k_cov_guard).

The general x grid and general x general blocks of the covariance (pyconsensus/__init__.py:326)
run on int8 MFMA over six balanced base-254 digit slices of tok * w at one fixed-point scale per
column, set by the column's largest |F - mu|.  A column where all but a few rows share one value
(the "concentrated" columns below) has that scale set by its outliers, so the majority's tiny
|w| keeps only its top digits and the dropped digit pairs (i + j >= 6) leave the same error on
every row: linear in the rows, ~5e-9 of C_pp at 1M rows.  The guard (k_cov_guard) bounds the
emulation's error against every entry and recomputes when the bound exceeds 2^-40:
  * cov_guard 1: the remaining digit pairs (every digit product exact);
  * cov_guard 2: the general pairs on fp64 (k_syrk), when the digit strings' own residues are
    what the bound cannot hold (majority values spread below the digits' resolution).
Each case checks the covariance ELEMENT-WISE against a reference summed in numpy's pairwise order
(error <= ~30 u sum tok |w_p||w_q| <= ~3e-15 sqrt(C_pp C_qq) by Cauchy-Schwarz):
|dC_pq| <= 1e-12 sqrt(C_pp C_qq) wherever the int8 emulation produced the entry, and the fp64
class bound of the reference's own dgemm (2e-10 sqrt(C_pp C_qq) here) where the fallback did.
The whole consensus of concentrated scaled events is checked against the numpy oracle at the
north-star tolerance (1e-9), at one and two ranks (the guard's sums travel with the covariance).
"""
import numpy as np
import pytest

import golden_cases as G
import parity as P

pytestmark = pytest.mark.gpu

EPS_INT8 = 1e-12
EPS_FP64 = 2e-10


def _tokens(N, rep):
    r = np.full(N, 1.0 / N) if rep is None else rep / rep.sum()
    return np.array([int(x * 1e6) for x in r], dtype=np.float64)  # self.reptokens (:146)


def _ref_entries(F, tok, mu, rows, denom):
    """C[p, :] for p in rows: sum_i fl(tok_i w_ip) w_iq / denom with w = fl(F - mu) (wcd, :322;
    np.ma.multiply(wcd.T, tokens), :326), each row of products summed by np.sum along its
    contiguous axis (numpy's pairwise sum)."""
    N, E = F.shape
    out = np.empty((len(rows), E))
    for a, p in enumerate(rows):
        tw = tok * (F[:, p] - mu[p])
        for q0 in range(0, E, 16):
            q1 = min(E, q0 + 16)
            W = np.ascontiguousarray((F[:, q0:q1] - mu[q0:q1]).T)
            out[a, q0:q1] = (W * tw[None, :]).sum(axis=1)
    return out / denom


def _ref_diag(F, tok, mu, denom):
    E = F.shape[1]
    d = np.empty(E)
    for q0 in range(0, E, 16):
        q1 = min(E, q0 + 16)
        W = np.ascontiguousarray((F[:, q0:q1] - mu[q0:q1]).T)
        d[q0:q1] = ((W * tok[None, :]) * W).sum(axis=1)
    return d / denom


def _concentrated(N, E, n_general, n_conc, seed, noise=0.0, rep_kind=None):
    """Filled matrix (no NA, no bounds): grid columns on {1, 1.5, 2}, general columns uniform on
    [1, 2], and n_conc general columns equal to one value on every row but 1-5 outliers
    (noise > 0: that value plus uniform noise of that size on every row)."""
    rng = np.random.default_rng(seed)
    F = rng.choice([1.0, 1.5, 2.0], size=(N, E), p=[0.45, 0.1, 0.45])
    gen = np.sort(rng.choice(E, n_general, replace=False))
    F[:, gen] = 1.0 + rng.random((N, n_general))
    conc = gen[:n_conc]
    for c in conc:
        F[:, c] = 1.0 + rng.random()
        if noise:
            F[:, c] += noise * (rng.random(N) - 0.5)
        k = int(rng.integers(1, 6))
        F[rng.choice(N, k, replace=False), c] = 1.0 + rng.random(k)
    rep = None if rep_kind is None else rng.integers(1, 100, N).astype(np.float64)
    return F, gen, conc, rep


def _check(F, rep, gen, conc, outs, meta, eps):
    N, E = F.shape
    tok = _tokens(N, rep)
    mu = outs["weighted_mean"]
    C = outs["covariance"]
    rng = np.random.default_rng(1)
    rows = sorted(set(conc.tolist()) | set(rng.choice(gen, min(8, len(gen)), replace=False).tolist()))
    ref = _ref_entries(F, tok, mu, rows, tok.sum() - 1.0)
    diag = _ref_diag(F, tok, mu, tok.sum() - 1.0)
    worst = 0.0
    for a, p in enumerate(rows):
        scale = np.sqrt(np.abs(diag[p] * diag))
        err = np.abs(C[p] - ref[a])
        nz = scale > 0
        assert np.all(err[~nz] == 0.0), (p, err[~nz].max())
        rel = err[nz] / scale[nz]
        worst = max(worst, float(rel.max()))
    np.testing.assert_array_equal(C, C.T)
    print("max |dC_pq| / sqrt(C_pp C_qq) over the checked rows:", worst, "guard:", meta["cov_guard"],
          meta["cov_guard_cols"], meta["cov_err_bound"])
    assert worst <= eps, worst
    return worst


@pytest.mark.timeout(600)
def test_concentrated_columns_take_every_digit_pair(gpu_lib):
    """1M rows, reputation=None (every token 1), 8 of 60 general columns concentrated: the dropped
    pairs' bound trips (the bound of the 21 pairs is reported), the remaining pairs run, and every
    checked entry is within 1e-12 of sqrt(C_pp C_qq)."""
    from pyconsensus_amd.pipeline import wpca_host

    F, gen, conc, rep = _concentrated(1_000_000, 200, 60, 8, seed=11)
    outs, meta = wpca_host(F, rep)
    assert meta["mixed_int8"] == 3, meta
    assert meta["cov_guard"] == 1, meta
    assert meta["cov_err_bound"] > 2.0 ** -40 and meta["cov_guard_cols"] >= len(conc), meta
    _check(F, rep, gen, conc, outs, meta, EPS_INT8)


@pytest.mark.timeout(600)
def test_concentrated_noisy_columns_fall_back_to_fp64(gpu_lib):
    """The same with the majority value spread by 1e-9 on every row: the digit strings' own
    residues are no longer constant, the bound cannot hold 2^-40 and the general pairs run on
    fp64 MFMA (mixed_int8 0)."""
    from pyconsensus_amd.pipeline import wpca_host

    F, gen, conc, rep = _concentrated(1_000_000, 200, 60, 8, seed=12, noise=1e-9)
    outs, meta = wpca_host(F, rep)
    assert meta["cov_guard"] == 2 and meta["mixed_int8"] == 0, meta
    _check(F, rep, gen, conc, outs, meta, EPS_FP64)


@pytest.mark.timeout(600)
def test_uniform_columns_pass_the_guard(gpu_lib):
    """No concentrated column (the C5 recipe's kind of data, 1M rows, tokens 1): the guard passes
    on the 21 pairs and the entries are within 1e-12 of sqrt(C_pp C_qq)."""
    from pyconsensus_amd.pipeline import wpca_host

    F, gen, conc, rep = _concentrated(1_000_000, 200, 60, 0, seed=13)
    outs, meta = wpca_host(F, rep)
    assert meta["mixed_int8"] == 3 and meta["cov_guard"] == 0, meta
    assert 0.0 < meta["cov_err_bound"] <= 2.0 ** -40, meta
    _check(F, rep, gen, conc, outs, meta, EPS_INT8)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n_conc", [0, 6])
def test_tokens_near_63(gpu_lib, n_conc):
    """C4-style integer reputations with the largest token near the int8 path's limit of 63
    (32,000 rows, reputations 1..99: tokens up to ~61), 2 digit strings (tok w and w)."""
    from pyconsensus_amd.pipeline import wpca_host

    F, gen, conc, rep = _concentrated(32_000, 300, 150, n_conc, seed=14 + n_conc, rep_kind="int")
    tok = _tokens(F.shape[0], rep)
    assert 55 <= tok.max() <= 63, tok.max()
    outs, meta = wpca_host(F, rep)
    assert meta["mixed_int8"] in (0, 3), meta
    if meta["cov_guard"] != 2:
        assert meta["mixed_int8"] == 3
    _check(F, rep, gen, conc, outs, meta, EPS_FP64 if meta["cov_guard"] == 2 else EPS_INT8)


def _conc_reports(N, E, seed):
    """Reports with scaled events in [0, 100], a quarter of them concentrated (every report the
    same but 1-5), 10% NA elsewhere; binary events 1 / 2; reputation None."""
    rng = np.random.default_rng(seed)
    R = rng.choice([1.0, 2.0], size=(N, E))
    sc = np.zeros(E, dtype=bool)
    sc[rng.choice(E, E // 3, replace=False)] = True
    lo = np.zeros(E)
    hi = np.where(sc, 100.0, 1.0)
    hi[~sc] = 1.0
    scols = np.flatnonzero(sc)
    R[:, scols] = np.round(rng.normal(60.0, 15.0, (N, len(scols))).clip(0.0, 100.0), 3)
    for c in scols[: len(scols) // 4]:
        R[:, c] = 37.5
        k = int(rng.integers(1, 6))
        R[rng.choice(N, k, replace=False), c] = np.round(rng.random(k) * 100.0, 3)
    na = rng.random((N, E)) < 0.1
    na[:, scols[: len(scols) // 4]] = False
    R[na] = np.nan
    return R, sc, lo, hi


_REF = {}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [1, 2])
def test_consensus_concentrated_vs_oracle(gpu_lib, world):
    """The whole consensus of 400k x 192 reports with concentrated scaled events (reputation None)
    against the numpy oracle, north-star tolerances, at one and two ranks."""
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import Oracle, synthetic
    from test_matrix_gpu import _sharded

    N, E = 400_000, 192
    if "c" not in _REF:
        R, sc, lo, hi = _conc_reports(N, E, seed=21)
        ref = G.flat_result(OracleCPU(reports=R, event_bounds=synthetic.bounds_list(sc, lo, hi)).consensus())
        _REF["c"] = (R, sc, lo, hi, ref)
    R, sc, lo, hi, ref = _REF["c"]
    if world == 1:
        o = Oracle(reports=R.copy(), event_bounds=synthetic.bounds_list(sc, lo, hi))
        res = o.consensus()
        ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(res).items() if k in P.ABI_NAME}
        info = o.last_info
        assert info["mixed_int8"] in (0, 3) and info["cov_guard"] in (1, 2), info
    else:
        ours, info = _sharded(R, None, sc, lo, hi, world)
    print(world, {k: info.get(k) for k in ("mixed_int8", "cov_guard", "cov_guard_cols", "cov_err_bound")})
    bad, sign = P.compare(ref, ours)
    assert not bad, bad
