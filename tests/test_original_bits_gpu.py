"""`original` keeps the caller's bits of every missing report, and the compact passes agree with
the oracle, on a matrix large enough for every int8 block and the int8-MFMA weighted counts
(DESIGN.md 5.1, round 6).

`original` is the rescaled reports (__init__.py:266-269), so an unscaled column's cells -- a NaN,
a negative NaN, a NaN with a payload, a zero (missing by the reference's own rule, :278), a -0.0
-- come back bit for bit.  1024 events, 265 of them scaled: the general tiles end at 384, so 119
grid events sit in them (positions [n_general, gb)), whose outcome / GEMV2 sums take the 2-bit codes
k_zbg keeps for them on int8 MFMA.  E <= 1024 also runs the power iteration's presquaring,
whose scratch once overwrote the plan's general count that those passes read (a C4 failure at
world 1).  Checked at one rank (the drop-in, host arrays) and two (device arrays).
"""
import numpy as np
import pytest

import golden_cases as G
import parity as P

pytestmark = pytest.mark.gpu


def _matrix(N, E, seed):
    """The synthetic recipe (truth per event, 10 % NaN, 25 % scaled) with three
    grid columns' missing reports re-encoded: zeros (+0.0 and -0.0), negative NaNs, NaNs with a
    payload."""
    from pyconsensus_amd import synthetic

    R, sc, lo, hi, _ = synthetic.matrix(N, E, seed=seed)
    sc = np.asarray(sc, dtype=bool)
    rng = np.random.default_rng(seed + 1)
    grid = np.flatnonzero(~sc)
    odd = {}
    c_zero, c_neg, c_pay = grid[3], grid[7], grid[11]
    m = np.isnan(R[:, c_zero])
    z = np.where(m)[0]
    R[z, c_zero] = np.where(rng.random(z.size) < 0.5, 0.0, -0.0)
    odd["zero"] = c_zero
    u = R[:, c_neg].view(np.uint64)
    u[np.isnan(R[:, c_neg])] = np.uint64(0xFFF8000000000000)  # -NaN
    odd["neg"] = c_neg
    u = R[:, c_pay].view(np.uint64)
    u[np.isnan(R[:, c_pay])] = np.uint64(0x7FF8000000000123)  # quiet NaN with a payload
    odd["payload"] = c_pay
    return R, sc, lo, hi, odd


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [1, 2])
def test_grid_codes_original_bits_and_oracle(gpu_lib, world):
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import Oracle, synthetic

    from test_matrix_gpu import _sharded

    N, E = 220_000, 1024  # N x 640 grid positions >= 2^27: the int8-MFMA weighted counts (wdig_fits)
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
