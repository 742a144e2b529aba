"""Device-memory handoff through torch (allocation, host<->device copies, streams)."""
from __future__ import annotations

import numpy as np


def torch():
    import torch as _t

    return _t


def require_gpu():
    t = torch()
    if not t.cuda.is_available():
        from ._lib import PcxError

        raise PcxError("no GPU visible: pyconsensus_amd runs on MI355X only (no CPU fallback)")
    return t


def as_device(x, dtype, device):
    """numpy / list / torch -> contiguous torch tensor on ``device`` (no copy if already there)."""
    t = torch()
    if x is None:
        return None
    if isinstance(x, t.Tensor):
        return x.to(device=device, dtype=dtype).contiguous()
    a = np.ascontiguousarray(np.asarray(x), dtype={t.float64: np.float64, t.uint8: np.uint8,
                                                    t.int32: np.int32}[dtype])
    return t.from_numpy(a).to(device, non_blocking=False)


def ptr(x):
    return None if x is None else x.data_ptr()


def current_stream_handle(device):
    return torch().cuda.current_stream(device).cuda_stream


def synchronize(device):
    torch().cuda.synchronize(device)
