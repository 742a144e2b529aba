"""The N>1 host path on CPU with torch.distributed gloo, world_size 2.

libpcx's sharded consensus exchanges per-rank partials through a communicator; the
callback backend (pipeline.CallbackComm) carries those exchanges over torch.distributed.
Its two callbacks are exercised here exactly as libpcx calls them -- host buffers, in
place -- with the data kinds the consensus exchanges: u64 selection limbs / counts (SUM,
exact even near 2^64), u64 key ranges (MIN / MAX), f64 covariance partials (SUM) and
rank-ordered all-gathers of dd slot blocks.  Row sharding math is checked too."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from pyconsensus_amd import _abi
from pyconsensus_amd.pipeline import CallbackComm, shard_rows


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
        comm = CallbackComm(world, rank)
        ar, ag = comm._cbs
        p = lambda a: a.ctypes.data_as(C.c_void_p)
        # u64 limbs and counts: exact SUM (no float rounding, no int64 overflow issues)
        big = np.array([2 ** 62 + rank, 12345 + rank, (1 << 43) - 1], dtype=np.uint64)
        assert ar(None, p(big), big.size, _abi.U64, _abi.RED_SUM) == 0
        assert big.tolist() == [sum(2 ** 62 + r for r in range(world)), sum(12345 + r for r in range(world)),
                                world * ((1 << 43) - 1)]
        keys = np.array([0xFFFF000000000000 - rank, 5 + rank], dtype=np.uint64)
        mn = keys.copy()
        assert ar(None, p(mn), 2, _abi.U64, _abi.RED_MIN) == 0
        assert mn.tolist() == [0xFFFF000000000000 - (world - 1), 5]
        mx = keys.copy()
        assert ar(None, p(mx), 2, _abi.U64, _abi.RED_MAX) == 0
        assert mx.tolist() == [0xFFFF000000000000, 5 + world - 1]
        # f64 covariance partials
        cov = np.full((3, 3), rank + 1.0)
        assert ar(None, p(cov), cov.size, _abi.F64, _abi.RED_SUM) == 0
        assert np.all(cov == sum(range(1, world + 1)))
        # all-gather of dd slot blocks: rank order
        blk = np.arange(6, dtype=np.float64) + 100 * rank
        out = np.zeros(6 * world)
        assert ag(None, p(blk), p(out), blk.nbytes) == 0
        assert np.array_equal(out, np.concatenate([np.arange(6.0) + 100 * r for r in range(world)]))
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc() + repr(e)))


@pytest.mark.parametrize("world", [2])
def test_callback_exchange_gloo(world):
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
            assert spans[0][0] == 0 and sum(c for _, c in spans) == N
            assert all(spans[r][0] + spans[r][1] == spans[r + 1][0] for r in range(world - 1))
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
