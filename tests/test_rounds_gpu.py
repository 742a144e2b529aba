"""The round scheduler (csrc/pcx_rounds.cpp: rounds above 256 x 64 and the clusterings above
64 x 32, each a single-matrix consensus on a pool of worker contexts) when a worker's workspace
does not fit: the worker reports PCX_ENOMEM, frees its workspace, leaves the pool and hands its
round back; the batch completes on the other workers and the handed-back round runs afterwards.
The fault is injected by the test-only entry point pcx_test_inject_enomem(ctx, k) (worker k's first
round of the next call reports PCX_ENOMEM without running), and the results must equal a run
without it bit for bit.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ("old_rep", "this_rep", "smooth_rep", "scores", "na_row", "participation_rows", "relative_part",
        "reporter_bonus", "adj_first_loadings", "outcomes_raw", "outcomes_adjusted", "outcomes_final",
        "certainty", "consensus_reward", "nas_filled", "participation_columns", "author_bonus",
        "participation", "avg_certainty", "branch", "flags")


def _run(R, rep, sc, lo, hi, env, fault_worker=None):
    import torch

    from pyconsensus_amd import _lib
    from pyconsensus_amd.batched import consensus_batched

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        if fault_worker is not None:
            _lib.check(_lib.lib().pcx_test_inject_enomem(_lib.context(torch.cuda.current_device()), fault_worker))
        out = consensus_batched(R, rep, sc, lo, hi)
        torch.cuda.synchronize()
        return {k: out[k].cpu().numpy() for k in KEYS if k in out}
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("worker", [0, 2])
def test_enomem_handback_completes_identically(gpu_lib, worker):
    from pyconsensus_amd import synthetic

    B, N, E = 7, 300, 20  # N > 256: the round scheduler
    R, sc, lo, hi, rep = synthetic.rounds(B, N, E, seed=20261017)
    base = _run(R, rep, sc, lo, hi, {"PCX_ROUND_WORKERS": "3"})
    faulted = _run(R, rep, sc, lo, hi, {"PCX_ROUND_WORKERS": "3"}, fault_worker=worker)
    assert set(base) == set(faulted) and len(base) >= 15
    for k in base:
        np.testing.assert_array_equal(faulted[k], base[k], err_msg=k)
    # and the pool still serves a normal call afterwards
    again = _run(R, rep, sc, lo, hi, {"PCX_ROUND_WORKERS": "3"})
    for k in base:
        np.testing.assert_array_equal(again[k], base[k], err_msg=k)
