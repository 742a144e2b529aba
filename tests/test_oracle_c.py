"""The C oracle (oracle/pcx_oracle_batched.c, the batched-round spec the GPU kernel
replays bit for bit) against the reference's golden vectors."""
import numpy as np
import pytest

import golden_cases as G
import parity as P
from oracle import pcx_oracle_c as OC


def run_c(case):
    R = case["in_reports"][None]
    kw = {}
    if bool(case["in_has_bounds"]):
        kw.update(scaled=case["in_scaled"][None], lo=case["in_lo"][None], hi=case["in_hi"][None])
    if bool(case["in_has_rep"]):
        kw["reputation"] = case["in_reputation"][None]
    o = OC.batched(R, catch_tolerance=float(case["in_catch_tolerance"]), alpha=float(case["in_alpha"]),
                   int_dtype=bool(case["in_int_dtype"]), **kw)
    return {k: v[0] for k, v in o.items()}


def _suite(cases):
    """Run the SPEC on the cases; {name: mismatch kind} and the names run."""
    observed, ran = {}, []
    for name, case in cases:
        N, E = case["in_reports"].shape
        if name in P.EXCLUDED or N > 64 or E > 64:
            continue
        ran.append(name)
        kind, _ = P.mismatch_kind(case, run_c(case))
        if kind:
            observed[name] = kind
    return observed, ran


def test_kat():
    P.assert_known("exact", *_suite(G.kat().items()))


def test_mixed_shapes():
    P.assert_known("exact", *_suite(G.mixed().items()))


def test_synth_50x20():
    st = G.synth()
    P.assert_known("exact", *_suite(("s%03d" % b, G.unstack(st, b)) for b in range(st["branch"].shape[0])))


@pytest.mark.parametrize("name", P.DEGENERATE_MASKED)
def test_masked_data_case(name):
    """The SPEC on the reference's degenerate all-missing scaled column (parity.DEGENERATE_MASKED):
    every output, numpy.ma's masked-data ones included, and the branch, as the reference."""
    P.assert_full(name, G.kat()[name], run_c(G.kat()[name]))


def test_threads_deterministic():
    from pyconsensus_amd import synthetic
    R, sc, lo, hi, rep = synthetic.rounds(64, 50, 20, seed=3)
    a = OC.batched(R, sc, lo, hi, rep, threads=1)
    b = OC.batched(R, sc, lo, hi, rep, threads=4)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_openblas_gemv_order_model():
    """The np.dot operation-order model the SPEC and the batched kernel replay (ob_vecmat)
    matches numpy bit for bit on this host, when its OpenBLAS core is the goldens' one."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import probe_openblas_order as PO

    arch, ver = PO.blas_core()
    if arch != "SkylakeX" or ver != "0.3.29":
        pytest.skip("host OpenBLAS core %s %s differs from the goldens' (SkylakeX 0.3.29)" % (arch, ver))
    bad, tot = PO.check(max_n=40, max_e=12, trials=1)
    assert bad == 0, (bad, tot)


@pytest.mark.parametrize("N,E,uniform", [(100, 50, False), (256, 64, False), (30, 40, True), (200, 1, False)])
def test_spec256_matches_numpy_restatement(N, E, uniform):
    """The C SPEC built for 256 reporters (oracle/lib/libpcx_oracle256.so: the bitwise target of
    the workgroup-per-round kernel) against the numpy restatement of the reference, north_star
    tolerances."""
    import golden_cases as G
    import parity as P
    from oracle import pcx_oracle_c as OC
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import synthetic

    R, sc, lo, hi, rep = synthetic.rounds(4, N, E, seed=N + E)
    if uniform:
        rep = None
    o = OC.batched(R, sc, lo, hi, rep, threads=2)
    for b in range(R.shape[0]):
        ref = G.flat_result(OracleCPU(reports=R[b].copy(), event_bounds=synthetic.bounds_list(sc[b], lo[b], hi[b]),
                                      reputation=None if rep is None else rep[b]).consensus())
        bad, _ = P.compare(ref, {k: v[b] for k, v in o.items()})
        assert not bad, (b, bad)


def _medium_batch(cases, uniform):
    idx = [i for i, c in enumerate(cases) if ("in_reputation" not in c) == uniform]
    st = lambda k: np.stack([cases[i][k] for i in idx])
    rep = None if uniform else st("in_reputation")
    return idx, st("in_reports"), st("in_scaled"), st("in_lo"), st("in_hi"), rep


@pytest.mark.parametrize("shape", [(100, 50), (250, 60), (256, 64)], ids=["100x50", "250x60", "256x64"])
def test_spec256_vs_reference_medium_goldens(shape):
    """The 256-reporter SPEC (the workgroup-per-round kernel's bitwise target) against rounds the
    REFERENCE computed at 100 x 50, 250 x 60 and 256 x 64 (tests/golden/medium.npz; at the two
    larger shapes N*E >= 9216, where the reference's dgemv is multi-threaded): no mismatch,
    branch codes included."""
    import golden_cases as G

    cases = G.medium()[shape]
    observed, ran = {}, []
    for uniform in (False, True):
        idx, R, sc, lo, hi, rep = _medium_batch(cases, uniform)
        o = OC.batched(R, sc, lo, hi, rep, threads=8)
        for t, i in enumerate(idx):
            name = "w%dx%d_%02d" % (shape[0], shape[1], i)
            ran.append(name)
            kind, _ = P.mismatch_kind(cases[i], {k: v[t] for k, v in o.items()})
            if kind:
                observed[name] = kind
    assert len(ran) == len(cases)
    P.assert_known("exact", observed, ran)
