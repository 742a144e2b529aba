"""The closed-form sequential sums behind the equal-weight weighted median
(csrc/pcx_seqsum.h, exported as pcx_seqsum_const / pcx_seqsum_first_above).

weightedstats' walk (__init__.py:303, :520-523) and the interpolation total (:294) add
weights one at a time in float arithmetic; with equal weights (reputation=None) the
library replays those sums by binade stepping instead of N additions.  Checked here
against the plain left-to-right loop (np.cumsum adds sequentially) for the weights the
reference actually produces: 1/N, (1/N)/S(n) (a phase-1 interpolation weight), and
arbitrary doubles, over counts up to 3 million."""
import numpy as np
import pytest

from pyconsensus_amd import _lib


def _weights():
    cs = []
    for N in (3, 7, 10, 999, 1000, 123457, 250000, 1000000, 1048576):
        c = 1.0 / float(N)
        cs.append(c)
        present = N - N // 10
        tot = np.cumsum(np.full(present, c))[-1]
        cs.append(c / tot)
    rng = np.random.default_rng(7)
    cs += list(np.ldexp(rng.uniform(0.5, 1.0, 24), -rng.integers(0, 40, 24)))
    cs += [0.1, 1.0 / 3.0, 3.0, 2.0 ** -30, 5e-324 * 2 ** 40]
    return cs


@pytest.mark.parametrize("c", _weights())
def test_seqsum_matches_sequential_loop(c):
    lib = _lib.lib()
    K = 3_000_000
    pre = np.concatenate([[0.0], np.cumsum(np.full(K, c))])
    rng = np.random.default_rng(int(abs(np.log2(c)) * 1000) % 2 ** 31)
    ks = list(range(12)) + list(rng.integers(0, K + 1, 40)) + [K]
    for k in ks:
        assert lib.pcx_seqsum_const(c, int(k)) == pre[k], (c, k)
        for t in (pre[k], np.nextafter(pre[k], 0.0), np.nextafter(pre[k], np.inf), 0.5 * pre[K]):
            want = int(np.searchsorted(pre[1:], t, side="right")) + 1  # least k >= 1 with pre[k] > t
            got = lib.pcx_seqsum_first_above(c, float(t), K)
            assert got == (want if want <= K else K + 1), (c, k, t)


def test_seqsum_degenerate():
    lib = _lib.lib()
    assert lib.pcx_seqsum_const(0.0, 10) == 0.0
    assert lib.pcx_seqsum_const(1.5, 0) == 0.0
    assert np.isnan(lib.pcx_seqsum_const(float("nan"), 10))
    assert lib.pcx_seqsum_first_above(0.0, 0.5, 100) == 101
    assert lib.pcx_seqsum_first_above(0.25, -1.0, 100) == 1
