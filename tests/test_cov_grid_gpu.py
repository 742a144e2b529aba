"""Covariance tiles on int8 MFMA (M_COV_PLAN / M_COV_I8).

Binary events whose filled values all lie on {1, 1.5, 2} ("grid" events) take the wcd
positions after the general events; the covariance tiles made only of grid positions are
P = sum tok z z^T on int8 MFMA with z = 2 (F - 1), combined with the exact T and Z sums;
the general x grid pairs multiply PCX_NDIG (6) base-254 int8 digit slices of tok w (w = F - mu) with z,
and when the general events fill whole 256-event tiles the general x general pairs multiply those
digits with PCX_NDIG digit slices of w (k_gemm_i8x; pcx_result.mixed_int8 == 3), over 256-position
tiles that reach into the next digit's positions when the general events fill an odd number of
128-event tiles.
The wpca entry's covariance is checked against the reference formula
(pyconsensus/__init__.py:317-326) evaluated in numpy: all-general, mixed, all-grid,
varying tokens (tok * z operand), off-grid values and tokens above 63 (no int8 path).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ref(F, rep):
    """weighted_mean, covariance_matrix of Oracle.wpca (:317-326) in numpy.  The mean is
    summed in extended precision: np.ma.average's row-sequential sum is off by up to
    ~N ulps, libpcx's compensated one is within an ulp of exact."""
    N = F.shape[0]
    r = np.full(N, 1.0 / N) if rep is None else rep / rep.sum()
    tok = np.array([int(x * 1e6) for x in r], dtype=np.float64)  # self.reptokens (:146)
    rl = r.astype(np.longdouble)
    mu = ((F.astype(np.longdouble) * rl[:, None]).sum(axis=0) / rl.sum()).astype(np.float64)
    wcd = F - mu
    return mu, (wcd.T * tok) @ wcd / (tok.sum() - 1)


def _filled(N, E, seed, frac_scaled=0.25, offgrid=()):
    rng = np.random.default_rng(seed)
    F = rng.choice([1.0, 1.5, 2.0], size=(N, E), p=[0.45, 0.1, 0.45])
    sc = rng.random(E) < frac_scaled
    F[:, sc] = 1.0 + rng.random((N, int(sc.sum())))
    for c in offgrid:
        F[rng.integers(0, N), c] = 1.25
    return F, sc


CASES = {
    # name: N, E, scaled fraction, reputation kind, off-grid events, expect int8 path
    "mixed_uniform": (40000, 300, 0.25, None, (), True),
    "all_grid": (40000, 200, 0.0, None, (), True),
    "mixed_int_rep": (40000, 300, 0.25, "int", (), True),
    "offgrid_events": (40000, 300, 0.25, None, (3, 150, 299), True),
    "tokens_above_63": (3000, 300, 0.25, "int", (), False),
    "single_tile": (20000, 100, 0.3, None, (), True),  # general and grid share the one tile: fp64
    "two_tiles": (20000, 200, 0.3, None, (), True),
    # 256 and 512 general positions (1 and 2 whole 256-position tiles)
    "gg_int8_one_tile": (40000, 700, 0.33, None, (), True),
    "gg_int8_int_rep": (40000, 900, 0.5, "int", (), True),
    # every token int(1/N 1e6) = 1: the general pairs take the tok w digits for both operands
    "gg_int8_tokens_one": (600000, 300, 0.5, None, (), True),
    # every token int(1/N 1e6) = 16, a power of two: tok w 2^-e = w 2^-f, the same shortcut
    "gg_int8_tokens_pow2": (62500, 700, 0.33, None, (), True),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_wpca_covariance_grid(name):
    from pyconsensus_amd.pipeline import wpca_host

    N, E, fs, rk, og, expect = CASES[name]
    F, sc = _filled(N, E, seed=N + E, frac_scaled=fs, offgrid=og)
    rep = None if rk is None else np.random.default_rng(7).integers(1, 100, N).astype(np.float64)
    outs, meta = wpca_host(F, rep)
    mu, cov = _ref(F, rep)
    n_grid = int(E - sc.sum() - len([c for c in og if not sc[c]]))
    gb = -(-(E - n_grid) // 128) * 128  # general events take the first 128-event tiles
    assert meta["grid_events"] == (max(0, E - gb) if expect else 0), (meta["grid_events"], n_grid)
    # general x grid and general x general pairs on int8 digit slices whenever both kinds of tile
    # are present
    assert meta["mixed_int8"] == (3 if expect and 0 < gb < E else 0), (meta["mixed_int8"], gb)
    np.testing.assert_allclose(outs["weighted_mean"], mu, rtol=1e-14, atol=0)
    scale = np.abs(cov).max()
    err = np.abs(outs["covariance"] - cov).max() / scale
    print(name, "grid events", meta["grid_events"], "max err / max|C|", err)
    assert err < 1e-12
    np.testing.assert_array_equal(outs["covariance"], outs["covariance"].T)
