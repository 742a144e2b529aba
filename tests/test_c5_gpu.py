"""Config C5 at its full size (1M reporters x 4096 events, reputation=None) on one MI355X.

The numpy oracle cannot run at this size (>= 6 fp64 copies of 32 GB), so
parity here rests on size-independent properties (the same matrix as `bench.py`'s C5 line,
generated on the GPU shard by shard):

* reputation vectors are distributions (non-negative, sum to 1);
* binary outcomes are catch values {1, 1.5, 2}; scaled outcomes lie inside their bounds;
* row-shard invariance: 2, 4 and 8 virtual ranks (ThreadComm, each generating its own
  8/N of the 8 row shards, exactly what rank r of `bench.py --gpus N` builds) reproduce
  the 1-rank result -- the multi-GPU C5 configurations rehearsed at full size on one device.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, E = 1_000_000, 4096


def _np(d):
    return {k: v.cpu().numpy() for k, v in d.items()}


def test_c5_full_size_properties_and_shard_invariance(gpu_lib):
    import torch

    from pyconsensus_amd import synthetic
    from pyconsensus_amd.pipeline import consensus_matrix, release_workspace

    dev = torch.device("cuda:0")
    R, sc, lo, hi, _ = synthetic.matrix_device(N, E, seed=3, n_shards=8, device=dev)
    ev, ag, meta = consensus_matrix(R, None, sc, lo, hi, device=dev)
    ref_ev, ref_ag, branch = _np(ev), _np(ag), meta["branch"]
    scaled = sc.cpu().numpy().astype(bool)
    lo_, hi_ = lo.cpu().numpy(), hi.cpu().numpy()
    del R, ev, ag, meta
    release_workspace()
    torch.cuda.empty_cache()

    # reputation vectors are distributions
    for k in ("this_rep", "smooth_rep"):
        v = ref_ag[k]
        assert v.shape == (N,) and np.all(v >= 0), k
        assert abs(v.sum() - 1.0) < 1e-9, (k, v.sum())
    # outcomes: catch values for binary events, inside the bounds for scaled ones
    fin = ref_ev["outcomes_final"]
    assert fin.shape == (E,) and np.all(np.isfinite(fin))
    assert np.all(np.isin(fin[~scaled], (1.0, 1.5, 2.0)))
    assert np.all((fin[scaled] >= lo_[scaled]) & (fin[scaled] <= hi_[scaled]))
    assert branch in (1, 2, 3, 4)

    for world in (2, 4, 8):  # the N of the driver's scaling runs
        _check_world(world, dev, ref_ev, ref_ag, branch)


def _check_world(world, dev, ref_ev, ref_ag, branch):
    import torch

    from pyconsensus_amd import synthetic
    from pyconsensus_amd.pipeline import ThreadComm, ThreadGroup, consensus_matrix, shard_rows

    grp = ThreadGroup(world)
    res = [None] * world
    errs = []

    def worker(r):
        try:
            torch.cuda.set_device(0)
            per = 8 // world
            Rr, scr, lor, hir, _ = synthetic.matrix_device(N, E, seed=3, n_shards=8,
                                                           shards=list(range(r * per, (r + 1) * per)), device=dev)
            off, cnt = shard_rows(N, world, r)
            assert Rr.shape[0] == cnt
            comm = ThreadComm(grp, r)
            e, a, m = consensus_matrix(Rr, None, scr, lor, hir, comm=comm, n_total=N, row_offset=off, device=dev)
            res[r] = (_np(e), _np(a), m["branch"], m["comm_bytes"])
            del Rr, e, a
            comm.close()  # frees this virtual rank's scratch
        except Exception as ex:  # pragma: no cover
            errs.append(ex)
            grp.barrier.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    [x.start() for x in th]
    [x.join() for x in th]
    torch.cuda.empty_cache()
    assert not errs, errs
    cb = max(res[r][3] for r in range(world))
    print("C5 world %d: collective bytes per rank %.1f MB" % (world, cb / 1e6))
    if world == 8:  # the sharded consensus exchanges < 300 MB per rank at C5
        assert cb < 300e6, cb
    for r in range(world):
        e, a, br, _ = res[r]
        assert br == branch
        for k in ref_ev:
            np.testing.assert_allclose(e[k], ref_ev[k], rtol=1e-12, atol=1e-14, err_msg=k)
        for k in ("outcomes_adjusted", "outcomes_final"):
            np.testing.assert_array_equal(e[k], ref_ev[k], err_msg=k)
    for k in ref_ag:
        got = np.concatenate([res[r][1][k] for r in range(world)])
        np.testing.assert_allclose(got, ref_ag[k], rtol=1e-12, atol=1e-14, err_msg=k)
