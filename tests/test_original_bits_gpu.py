"""`original` keeps the caller's bits of every missing report, and the compact passes agree with
the oracle, on a matrix large enough for every int8 block.

`original` is the rescaled reports (__init__.py:266-269), so an unscaled column's cells -- a NaN,
a negative NaN, a NaN with a payload, a zero (missing by the reference's own rule, :278), a -0.0
-- come back bit for bit.  1024 events, 283 of them scaled: the general tiles end at 384, so 101
grid events sit in them (positions [n_general, gb)), whose outcome / GEMV2 sums take the 2-bit codes
k_wcd keeps for them (zbg) on int8 MFMA.  E <= 1024 also runs the power iteration's presquaring,
whose scratch once overwrote the plan's general count that those passes read (a C4 failure at
world 1).  Checked at one rank (the drop-in, host arrays) and two (device arrays).
"""
import numpy as np
import pytest

import golden_cases as G
import parity as P

pytestmark = pytest.mark.gpu


def _matrix(N, E, seed):
    rng = np.random.default_rng(seed)
    R = rng.choice([1.0, 1.5, 2.0], size=(N, E), p=[0.45, 0.1, 0.45])
    sc = rng.random(E) < 0.25
    lo = np.where(sc, rng.uniform(-10.0, 0.0, E), 1.0)
    hi = np.where(sc, lo + rng.uniform(1.0, 20.0, E), 2.0)
    R[:, sc] = lo[sc] + (hi[sc] - lo[sc]) * np.clip(rng.normal(0.6, 0.15, (N, int(sc.sum()))), 0.001, 1.0)
    R[rng.random((N, E)) < 0.1] = np.nan
    grid = np.flatnonzero(~sc)
    odd = {}
    # a grid column with zeros among its missing reports, one with negative NaNs, one with a payload
    c_zero, c_neg, c_pay = grid[3], grid[7], grid[11]
    rows = rng.choice(N, 40, replace=False)
    R[rows, c_zero] = 0.0
    R[rows[:20], c_zero] = -0.0
    odd["zero"] = c_zero
    u = R[:, c_neg].view(np.uint64)
    m = np.isnan(R[:, c_neg])
    u[m] = np.uint64(0xFFF8000000000000)  # -NaN
    odd["neg"] = c_neg
    u = R[:, c_pay].view(np.uint64)
    m = np.isnan(R[:, c_pay])
    u[m] = np.uint64(0x7FF8000000000123)  # quiet NaN with a payload
    odd["payload"] = c_pay
    return R, sc, lo, hi, odd


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [1, 2])
def test_grid_codes_original_bits_and_oracle(gpu_lib, world):
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import Oracle, synthetic

    from test_matrix_gpu import _sharded

    N, E = 16400, 1024  # 16.8M cells >= 2^24: the codes path
    R, sc, lo, hi, odd = _matrix(N, E, seed=11)
    b = synthetic.bounds_list(sc, lo, hi)
    ref = G.flat_result(OracleCPU(reports=R.copy(), event_bounds=b, reputation=None).consensus())
    if world == 1:
        o = Oracle(reports=R.copy(), event_bounds=b, reputation=None)
        ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(o.consensus()).items() if k in P.ABI_NAME}
        info = o.last_info
    else:
        ours, info = _sharded(R, None, sc, lo, hi, world)
    assert info.get("mixed_int8", 0) & 1 and info.get("grid_events", 0) > 0, info
    bad, _ = P.compare(ref, ours)
    assert not bad, bad
    # `original`: the input's own bits on every unscaled column (the odd columns included)
    orig = np.asarray(ours["original"])
    for name, c in odd.items():
        np.testing.assert_array_equal(orig[:, c].view(np.uint64), R[:, c].view(np.uint64), err_msg=name)
    un = np.flatnonzero(~sc)
    np.testing.assert_array_equal(orig[:, un].view(np.uint64), R[:, un].view(np.uint64))
