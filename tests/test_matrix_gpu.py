"""GPU parity of the single-matrix pipeline (csrc/pcx_matrix.hip via pipeline.py).

* golden vectors (KATs, mixed shapes, synthetic 50x20, C2 1000x100) forced through
  the matrix path, north_star tolerances, near-tie rounds counted separately;
* larger matrices against the numpy CPU oracle run on the box;
* virtual row shards (2 and 3 ranks in one process) against the 1-rank result.
"""
import numpy as np
import pytest

import golden_cases as G
import parity as P

pytestmark = pytest.mark.gpu


def run_matrix(case, **kw):
    from pyconsensus_amd.pipeline import consensus_matrix

    R = case["in_reports"]
    bk = {}
    if bool(case["in_has_bounds"]):
        bk = dict(scaled=case["in_scaled"], lo=case["in_lo"], hi=case["in_hi"])
    rep = case["in_reputation"] if bool(case["in_has_rep"]) else None
    ev, ag, meta = consensus_matrix(R, rep, catch_tolerance=float(case["in_catch_tolerance"]),
                                    alpha=float(case["in_alpha"]), int_dtype=bool(case["in_int_dtype"]),
                                    matrices=True, **bk, **kw)
    out = {k: v.cpu().numpy() for k, v in list(ev.items()) + list(ag.items())}
    out["participation"] = np.array(meta["participation"])
    out["avg_certainty"] = np.array(meta["avg_certainty"])
    out["branch"] = np.array(meta["branch"])
    return out


def _suite(cases):
    stats = dict(n=0, neartie=0, neartie_match=0, sign=0)
    fails = []
    for name, case in cases:
        if name in P.EXCLUDED:
            continue
        ours = run_matrix(case)
        bad, sign = P.compare(case, ours)
        stats["n"] += 1
        stats["sign"] += sign
        ok = not bad and P.branch_matches(case, ours, sign)
        if P.is_neartie(case, "matrix_small"):
            stats["neartie"] += 1
            stats["neartie_match"] += ok
        elif not ok:
            fails.append((name, int(ours["branch"]), int(case["branch"]), bad[:3]))
    return stats, fails


def test_matrix_golden_kat(gpu_lib):
    stats, fails = _suite(G.kat().items())
    print("matrix kat", stats)
    assert not fails, fails[:4]


def test_matrix_golden_mixed(gpu_lib):
    stats, fails = _suite(G.mixed().items())
    print("matrix mixed", stats)
    assert not fails, fails[:4]


def test_matrix_golden_synth(gpu_lib):
    st = G.synth()
    stats, fails = _suite((b, G.unstack(st, b)) for b in range(0, st["branch"].shape[0], 5))
    print("matrix synth", stats)
    assert not fails, fails[:4]


def test_matrix_golden_c2(gpu_lib):
    """Config C2 (1000 x 100, 10% NA, mixed bounds) through the drop-in Oracle."""
    from pyconsensus_amd import Oracle

    case = G.c2()
    res = Oracle(**G.oracle_args(case)).consensus()
    ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(res).items() if k in P.ABI_NAME}
    bad, sign = P.compare(case, ours)
    assert not bad, bad


@pytest.mark.parametrize("shape", [(3000, 150), (20000, 400),
                                   pytest.param((100_000, 1000), id="C4_100k_x_1k")])
def test_matrix_vs_numpy_oracle(gpu_lib, shape):
    """Against the numpy restatement run on the box; (100_000, 1000) is BASELINE config C4
    at full size (the oracle takes ~35 s there)."""
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import Oracle, synthetic

    N, E = shape
    R, sc, lo, hi, rep = synthetic.matrix(N, E, seed=N + E)
    if N > 8192:
        # the selection path computes medians in exact arithmetic; with integer
        # reputations exact half-weight prefixes (rounding-decided in the reference)
        # are common, so the large case uses continuous reputations
        rep = np.random.default_rng(N).uniform(0.5, 99.5, N)
    b = synthetic.bounds_list(sc, lo, hi)
    ref = G.flat_result(OracleCPU(reports=R, event_bounds=b, reputation=rep).consensus())
    res = Oracle(reports=R.copy(), event_bounds=b, reputation=rep).consensus()
    ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(res).items() if k in P.ABI_NAME}
    bad, sign = P.compare(ref, ours)
    assert not bad, bad


def test_virtual_shards_match_single(gpu_lib):
    """2 and 3 row shards (ThreadComm, one GPU) reproduce the 1-rank result."""
    import threading

    import torch
    from pyconsensus_amd import synthetic
    from pyconsensus_amd.pipeline import ThreadComm, ThreadGroup, consensus_matrix, shard_rows

    N, E = 5000, 120
    R, sc, lo, hi, rep = synthetic.matrix(N, E, seed=17)
    ev1, ag1, m1 = consensus_matrix(R, rep, sc, lo, hi)
    ref_ev = {k: v.cpu().numpy() for k, v in ev1.items()}
    ref_ag = {k: v.cpu().numpy() for k, v in ag1.items()}
    for world in (2, 3):
        grp = ThreadGroup(world)
        res = [None] * world
        errs = []

        def worker(r):
            try:
                torch.cuda.set_device(0)
                off, cnt = shard_rows(N, world, r)
                ev, ag, meta = consensus_matrix(R[off:off + cnt], rep, sc, lo, hi, comm=ThreadComm(grp, r),
                                                n_total=N, row_offset=off)
                res[r] = ({k: v.cpu().numpy() for k, v in ev.items()},
                          {k: v.cpu().numpy() for k, v in ag.items()}, meta["branch"])
            except Exception as e:  # pragma: no cover
                errs.append(e)
                grp.barrier.abort()

        th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
        [x.start() for x in th]
        [x.join() for x in th]
        assert not errs, errs
        for r in range(world):
            ev, ag, br = res[r]
            assert br == m1["branch"]
            for k in ref_ev:
                np.testing.assert_allclose(ev[k], ref_ev[k], rtol=1e-12, atol=1e-14, err_msg=k)
            for k in ("outcomes_adjusted", "outcomes_final"):
                np.testing.assert_array_equal(ev[k], ref_ev[k], err_msg=k)
        for k in ref_ag:
            got = np.concatenate([res[r][1][k] for r in range(world)])
            np.testing.assert_allclose(got, ref_ag[k], rtol=1e-12, atol=1e-14, err_msg=k)
