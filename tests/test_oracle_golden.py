"""The CPU oracle (oracle/pcx_oracle.py) against the reference's golden vectors.

The fixtures were produced by running the reference itself (tests/golden/make_golden.py);
on the same numpy/OpenBLAS the restatement must agree bit for bit.
"""
import numpy as np
import pytest

import golden_cases as G
from oracle.pcx_oracle import OracleCPU, weighted_median


def _check(case, res, exact=True):
    got = G.flat_result(res)
    for k, v in got.items():
        if k == "original" and k not in case:
            continue
        ref = case[k]
        if exact:
            np.testing.assert_array_equal(v, ref, err_msg=k)
        else:
            np.testing.assert_allclose(v, ref, rtol=1e-12, atol=1e-14, err_msg=k)


@pytest.mark.parametrize("name", sorted(G.kat().keys()))
def test_kat(name):
    case = G.kat()[name]
    o = OracleCPU(**G.oracle_args(case))
    _check(case, o.consensus())
    np.testing.assert_array_equal(o.reptokens, case["reptokens"])


def test_mixed_shapes():
    for name, case in G.mixed().items():
        _check(case, OracleCPU(**G.oracle_args(case)).consensus())


def test_synth_50x20():
    st = G.synth()
    for b in range(st["branch"].shape[0]):
        case = G.unstack(st, b)
        o = OracleCPU(**G.oracle_args(case))
        _check(case, o.consensus())
        assert o.diag["branch"] in (1, 2, 3, 4)


def test_c2():
    case = G.c2()
    _check(case, OracleCPU(**G.oracle_args(case)).consensus())


@pytest.mark.parametrize("shape", G.MEDIUM_SHAPES, ids=["%dx%d" % s for s in G.MEDIUM_SHAPES])
def test_medium_shapes(shape):
    """Rounds of the workgroup-per-round shapes, 40 each (medium.npz, reference-generated):
    at 250 x 60 and 256 x 64 (N*E >= 9216) the reference's np.dot is multi-threaded OpenBLAS."""
    for case in G.medium()[shape]:
        _check(case, OracleCPU(**G.oracle_args(case)).consensus())


def test_weighted_median_branches():
    # dominant weight
    assert weighted_median([5.0, 1.0, 3.0], [0.1, 0.7, 0.2]) == 1.0
    # crossing
    assert weighted_median([1.0, 2.0, 3.0, 4.0], [0.3, 0.1, 0.35, 0.25]) == 3.0
    # exact half -> mean of the straddling pair
    assert weighted_median([1.0, 2.0, 3.0, 4.0], [0.25, 0.25, 0.25, 0.25]) == 2.5
    # no positive weight
    assert weighted_median([1.0, 2.0], [0.0, 0.0]) is None


def test_appendix_c_anchor():
    """SURVEY.md Appendix C values (README example, C1)."""
    case = G.kat()["readme"]
    res = OracleCPU(**G.oracle_args(case)).consensus()
    np.testing.assert_allclose(np.asarray(res["agents"]["smooth_rep"]),
                               [0.038501766886541035, 0.07693012197380761, 0.3809800680761801,
                                0.31073090020632843, 0.12857142857142856, 0.06428571428571428], rtol=0, atol=0)
    assert res["events"]["outcomes_final"] == [0.5, 0.7, 1.5, 1.0]
