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
    stats = dict(n=0, neartie=0, neartie_match=0, sign=0)
    fails = []
    for name, case in cases:
        N, E = case["in_reports"].shape
        if name in P.EXCLUDED or N > 64 or E > 64:
            continue
        ours = run_c(case)
        bad, sign = P.compare(case, ours)
        stats["n"] += 1
        stats["sign"] += sign
        branch_ok = P.branch_matches(case, ours, sign)
        if P.is_neartie(case):
            stats["neartie"] += 1
            stats["neartie_match"] += (not bad) and branch_ok
        elif bad or not branch_ok:
            fails.append((name, int(ours["branch"]), int(case["branch"]), bad[:3]))
    return stats, fails


def test_kat():
    stats, fails = _suite(G.kat().items())
    assert not fails, fails


def test_mixed_shapes():
    stats, fails = _suite(G.mixed().items())
    assert not fails, fails
    assert stats["neartie"] < 0.25 * stats["n"]


def test_synth_50x20():
    st = G.synth()
    stats, fails = _suite((b, G.unstack(st, b)) for b in range(st["branch"].shape[0]))
    assert not fails, fails
    assert stats["neartie"] <= 0.08 * stats["n"], stats
    assert stats["sign"] >= 0.98 * stats["n"], stats


def test_threads_deterministic():
    from pyconsensus_amd import synthetic
    R, sc, lo, hi, rep = synthetic.rounds(64, 50, 20, seed=3)
    a = OC.batched(R, sc, lo, hi, rep, threads=1)
    b = OC.batched(R, sc, lo, hi, rep, threads=4)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
