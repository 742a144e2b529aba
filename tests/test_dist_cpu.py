"""The N>1 path's host protocol on CPU with torch.distributed gloo, world_size 2.

pipeline.Comm is what the sharded consensus uses between stages: each rank writes
its partial into slot [rank] of a [world, ...] buffer; clear_slots + reduce_slots
(all-reduce SUM) must leave every slot holding exactly its owner's values on every
rank, for whole buffers and for sub-slices (the stages reuse one buffer for several
slot ranges), and a full-buffer SUM (the covariance) must add the ranks.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pyconsensus_amd.pipeline import Comm, shard_rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        comm = Comm.from_env()
        assert comm.world == world and comm.rank == rank
        # a [world, E, 16, 2] column-stat buffer reused for two slot ranges
        E = 5
        buf = torch.zeros(world, E, 16, 2, dtype=torch.float64)
        comm.clear_slots(buf, (slice(None), slice(0, 4)))
        buf[rank, :, 0:4] = rank + 1.0
        comm.reduce_slots(buf, (slice(None), slice(0, 4)))
        for w in range(world):
            assert torch.all(buf[w, :, 0:4] == w + 1.0)
        # second stage writes another slot range; the first range must stay intact
        comm.clear_slots(buf, (slice(None), slice(4, 6)))
        buf[rank, :, 4:6] = 10.0 * (rank + 1)
        comm.reduce_slots(buf, (slice(None), slice(4, 6)))
        for w in range(world):
            assert torch.all(buf[w, :, 0:4] == w + 1.0)
            assert torch.all(buf[w, :, 4:6] == 10.0 * (w + 1))
        # uint64 key slots (score min/max) survive the SUM exactly
        sk = torch.zeros(world, 4, dtype=torch.int64)
        comm.clear_slots(sk)
        sk[rank, 0] = -1 - rank  # ~0ull-style patterns
        sk[rank, 1] = (1 << 62) + rank
        comm.reduce_slots(sk)
        for w in range(world):
            assert sk[w, 0].item() == -1 - w and sk[w, 1].item() == (1 << 62) + w
        # plain all-reduce (covariance partials)
        C = torch.full((3, 3), float(rank + 1), dtype=torch.float64)
        comm.all_reduce_sum(C)
        assert torch.all(C == sum(range(1, world + 1)))
        # row shards tile [0, N)
        N = 1001
        spans = [shard_rows(N, world, r) for r in range(world)]
        assert spans[0][0] == 0 and sum(c for _, c in spans) == N
        assert all(spans[r][0] + spans[r][1] == spans[r + 1][0] for r in range(world - 1))
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2])
def test_slot_protocol_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = [q.get(timeout=120) for _ in range(world)]
    [p.join(timeout=60) for p in ps]
    assert all(r[1] == "ok" for r in res), res


def test_shard_rows_uneven():
    for N in (1, 7, 1000, 1000000):
        for world in (1, 2, 3, 8):
            if N < world:
                continue
            spans = [shard_rows(N, world, r) for r in range(world)]
            assert sum(c for _, c in spans) == N
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
