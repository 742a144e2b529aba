"""The row-sharded consensus across real processes (torch.distributed), on one GPU.

Two ranks, one process each, both on cuda:0, exchanging through pipeline.Comm with
the gloo backend (RCCL refuses two ranks on one device; the driver's multi-GPU runs
use RCCL with the same Comm calls).  Every rank must end with the 1-rank result:
event outputs on every rank, agent outputs for its own rows.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, E = 6000, 96


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist

        from pyconsensus_amd import synthetic
        from pyconsensus_amd.pipeline import Comm, consensus_matrix, shard_rows

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        R, sc, lo, hi, rep = synthetic.matrix(N, E, seed=23)
        off, cnt = shard_rows(N, world, rank)
        ev, ag, meta = consensus_matrix(R[off:off + cnt], rep, sc, lo, hi, comm=Comm.from_env(),
                                        n_total=N, row_offset=off)
        out = {"ev": {k: v.cpu().numpy() for k, v in ev.items()},
               "ag": {k: v.cpu().numpy() for k, v in ag.items()},
               "branch": meta["branch"], "off": off, "cnt": cnt}
        dist.barrier()
        dist.destroy_process_group()
        if rank == 0:
            ev1, ag1, m1 = consensus_matrix(R, rep, sc, lo, hi)
            out["single"] = {"ev": {k: v.cpu().numpy() for k, v in ev1.items()},
                             "ag": {k: v.cpu().numpy() for k, v in ag1.items()}, "branch": m1["branch"]}
        q.put((rank, out))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc() + repr(e)))


def test_two_process_shards_match_single(gpu_lib):
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=110) for _ in range(world))
    [p.join(timeout=30) for p in ps]
    for r in range(world):
        assert isinstance(res[r], dict), res[r]
    ref = res[0]["single"]
    for r in range(world):
        o = res[r]
        assert o["branch"] == ref["branch"]
        for k, v in ref["ev"].items():
            np.testing.assert_allclose(o["ev"][k], v, rtol=1e-12, atol=1e-14, err_msg=k)
        for k in ("outcomes_adjusted", "outcomes_final"):
            np.testing.assert_array_equal(o["ev"][k], ref["ev"][k], err_msg=k)
        sl = slice(o["off"], o["off"] + o["cnt"])
        for k, v in ref["ag"].items():
            if v.shape[0] != N:
                continue
            np.testing.assert_allclose(o["ag"][k], v[sl], rtol=1e-12, atol=1e-14, err_msg=k)
