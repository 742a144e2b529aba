"""Context lifecycle (pcx_api.cpp / pcx_runner.cpp / pcx_rounds.cpp): the host resources a context
gathers over mixed calls are each freed once, whatever the order they were made in.

Round 5 shipped a stray hipHostFree of the pinned staging slots inside the medium-scratch growth
branch (found by inspection, not by a test): a host-memory call with large outputs (pinned slots),
then a workgroup-per-round batch larger than the context's scratch, then another host call, then
pcx_destroy freed the slots twice.  This runs exactly that sequence -- plus a batched round above
the one-block selection limit, which takes the pipelined selection's pinned info words on a worker
context of the round scheduler (freed by rounds_free) -- in a fresh process, twice over with
pcx_release_workspace between, and requires a clean exit with every result still correct.  Each
cycle also runs the host path in place (the chunked H2D with its host rewrite threads, round 6).
"""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

SCRIPT = textwrap.dedent(r"""
    import numpy as np
    from pyconsensus_amd import _lib, synthetic
    from pyconsensus_amd.batched import consensus_batched
    from pyconsensus_amd.pipeline import consensus_host

    # 140k x 240: original / filled of 269 MB each, above the 256 MB staging threshold (pinned slots)
    R, sc, lo, hi, rep = synthetic.matrix(140_000, 240, seed=5)
    ref, _ = consensus_host(R.copy(), rep, sc, lo, hi)
    h = _lib.context(0)
    for cycle in range(2):
        for B, N, E in ((32, 100, 50), (300, 250, 64)):  # workgroup-per-round scratch grows
            Rb, scb, lob, hib, repb = synthetic.rounds(B, N, E, seed=B)
            out = consensus_batched(Rb, repb, scb, lob, hib)
            assert np.isfinite(out["smooth_rep"].cpu().numpy()).all()
        # rounds of 9000 rows (above SEL_EXACT_MAX): the round scheduler's worker contexts run the
        # pipelined selection (pinned info words + events per worker context)
        Rb, scb, lob, hib, repb = synthetic.rounds(2, 9000, 40, seed=9)
        out = consensus_batched(Rb, repb, scb, lob, hib)
        assert np.isfinite(out["smooth_rep"].cpu().numpy()).all()
        got, _ = consensus_host(R.copy(), rep, sc, lo, hi)
        for k in ref:
            assert np.array_equal(got[k].view(np.int64), ref[k].view(np.int64)), k
        # in place (the reports' H2D in row chunks, each rewritten by host threads as it lands;
        # `filled` copied back on the context's side stream): the same bits
        X = R.copy()
        got, _ = consensus_host(X, rep, sc, lo, hi, original_inplace=True)
        assert got["original"] is X
        for k in ref:
            assert np.array_equal(got[k].view(np.int64), ref[k].view(np.int64)), k
        if cycle == 0:
            _lib.check(_lib.lib().pcx_release_workspace(h))
    _lib.lib().pcx_destroy(h)
    _lib._ctx.clear()
    print("lifecycle ok")
""")


@pytest.mark.timeout(300)
def test_context_lifecycle_clean_exit(gpu_lib):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    p = subprocess.run([sys.executable, "-c", SCRIPT], cwd=root, env=env, capture_output=True, text=True,
                       timeout=280)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    assert "lifecycle ok" in p.stdout
