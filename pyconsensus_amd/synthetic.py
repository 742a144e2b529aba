"""Synthetic report matrices.

The reference has no data generator: its callers are user code and the external
Simulator.jl Monte Carlo driver (README.rst:52-56), which loops
``Oracle(...).consensus()`` over random rounds.  This module draws report
matrices with the shape of that workload so that the bench and the parity tests
run on the same inputs:

* per event: ``scaled ~ Bernoulli(0.25)``; scaled bounds ``lo ~ U(-100, 0)``,
  ``hi = lo + U(1, 200)``; binary truth in {1.0, 2.0} (NO/YES,
  ``pyconsensus/__init__.py:65-67``);
* per reporter: 70 % honest (flip probability 0.1), 30 % liars (0.6);
* scaled values ``lo + (hi - lo) * clip(N(0.6, 0.15), 0.001, 1)`` (never exactly
  ``lo``, so the NA==0.0 quirk of ``__init__.py:278`` is not hit by accident);
* 10 % of cells NaN (missing);
* reputation: integers U[1, 99] (``None`` = uniform, ``__init__.py:138-141``).

Two generators:

* :func:`rounds` / :func:`matrix` -- numpy ``default_rng`` (host), used for every
  size the CPU oracle can check (C1-C4 and the batched C3 block).
* :func:`matrix_device` -- torch on the GPU (Philox), used for the 1M x 4k C5
  matrix that is generated straight into HBM, one independent stream per
  125k-row shard so the matrix does not depend on the GPU count.
"""
from __future__ import annotations

import numpy as np

HONEST_FRAC = 0.7
FLIP_HONEST = 0.1
FLIP_LIAR = 0.6
SCALED_FRAC = 0.25
NA_FRAC = 0.1


def _events(rng, shape):
    """Per-event parameters for a leading ``shape`` (rounds) and E events."""
    scaled = rng.random(shape) < SCALED_FRAC
    lo = np.where(scaled, rng.uniform(-100.0, 0.0, shape), 1.0)
    hi = np.where(scaled, lo + rng.uniform(1.0, 200.0, shape), 2.0)
    truth = rng.integers(1, 3, shape).astype(np.float64)
    return scaled, lo, hi, truth


def _reports(rng, scaled, lo, hi, truth, n_rows, na_frac):
    """Reporter rows for event parameters of shape (..., E) -> (..., N, E)."""
    lead = scaled.shape[:-1]
    E = scaled.shape[-1]
    honest = rng.random(lead + (n_rows,)) < HONEST_FRAC
    p_flip = np.where(honest, FLIP_HONEST, FLIP_LIAR)[..., None]
    flip = rng.random(lead + (n_rows, E)) < p_flip
    t = truth[..., None, :]
    binary = np.where(flip, 3.0 - t, t)
    z = np.clip(rng.normal(0.6, 0.15, lead + (n_rows, E)), 0.001, 1.0)
    sc = lo[..., None, :] + (hi - lo)[..., None, :] * z
    R = np.where(scaled[..., None, :], sc, binary)
    R[rng.random(lead + (n_rows, E)) < na_frac] = np.nan
    return R


def rounds(B, N=50, E=20, seed=20261015, na_frac=NA_FRAC, reputation=True):
    """B independent N x E oracle rounds (config C3 is B=65536, N=50, E=20).

    Returns ``reports (B,N,E) f64``, ``scaled (B,E) bool``, ``lo (B,E)``,
    ``hi (B,E)``, ``reputation (B,N) f64 or None``.
    """
    rng = np.random.default_rng(seed)
    scaled, lo, hi, truth = _events(rng, (B, E))
    R = _reports(rng, scaled, lo, hi, truth, N, na_frac)
    rep = rng.integers(1, 100, (B, N)).astype(np.float64) if reputation else None
    return R, scaled, lo, hi, rep


def matrix(N, E, seed=1, na_frac=NA_FRAC, reputation=True):
    """One N x E report matrix (C2: 1000x100 seed 1; C4: 100000x1000 seed 2)."""
    R, scaled, lo, hi, rep = rounds(1, N, E, seed=seed, na_frac=na_frac, reputation=reputation)
    return R[0], scaled[0], lo[0], hi[0], (rep[0] if rep is not None else None)


def bounds_list(scaled, lo, hi):
    """Reference-style ``event_bounds`` list of dicts (``__init__.py:108-114``)."""
    return [{"scaled": bool(s), "min": float(a), "max": float(b)} for s, a, b in zip(scaled, lo, hi)]


def matrix_device(N, E, seed=3, n_shards=8, shards=None, device="cuda", reputation=False):
    """C5-style matrix generated on the GPU, ``n_shards`` independent row blocks.

    Event parameters come from the numpy stream of ``SeedSequence(seed)``; each
    shard's rows come from a torch Philox generator seeded from that shard's
    spawned child, so shard ``k`` is identical whichever GPU generates it.
    ``shards`` selects which shard indices to build (default: all), returning the
    concatenated rows.  Returns torch tensors ``R (rows,E)``, ``scaled (E,) u8``,
    ``lo``, ``hi`` and ``rep`` (``None`` unless ``reputation``).
    """
    import torch

    ss = np.random.SeedSequence(seed)
    children = ss.spawn(1 + n_shards)
    ev_rng = np.random.default_rng(children[0])
    scaled, lo, hi, truth = _events(ev_rng, (E,))
    rows_per = N // n_shards
    assert rows_per * n_shards == N, "N must split evenly into shards"
    shards = list(range(n_shards)) if shards is None else list(shards)
    dev = torch.device(device)
    sc_t = torch.as_tensor(scaled, device=dev)
    lo_t = torch.as_tensor(lo, device=dev)
    hi_t = torch.as_tensor(hi, device=dev)
    tr_t = torch.as_tensor(truth, device=dev)
    R = torch.empty((rows_per * len(shards), E), dtype=torch.float64, device=dev)
    reps = []
    for k, s in enumerate(shards):
        g = torch.Generator(device=dev)
        g.manual_seed(int(children[1 + s].generate_state(1, dtype=np.uint64)[0] & 0x7FFFFFFFFFFFFFFF))
        blk = R[k * rows_per:(k + 1) * rows_per]
        honest = torch.rand((rows_per, 1), generator=g, device=dev, dtype=torch.float64) < HONEST_FRAC
        p_flip = torch.where(honest, FLIP_HONEST, FLIP_LIAR)
        # build column-chunked to bound temporaries (a 125k x 4k f64 block is 4 GB)
        step = max(1, (1 << 27) // rows_per)
        for c0 in range(0, E, step):
            c1 = min(E, c0 + step)
            u = torch.rand((rows_per, c1 - c0), generator=g, device=dev, dtype=torch.float64)
            t = tr_t[c0:c1]
            binary = torch.where(u < p_flip, 3.0 - t, t)
            z = torch.randn((rows_per, c1 - c0), generator=g, device=dev, dtype=torch.float64)
            z.mul_(0.15).add_(0.6).clamp_(0.001, 1.0)
            sc = lo_t[c0:c1] + (hi_t[c0:c1] - lo_t[c0:c1]) * z
            out = torch.where(sc_t[c0:c1].bool(), sc, binary)
            na = torch.rand((rows_per, c1 - c0), generator=g, device=dev, dtype=torch.float64) < NA_FRAC
            out.masked_fill_(na, float("nan"))
            blk[:, c0:c1] = out
            del u, binary, z, sc, out, na
        if reputation:
            reps.append(torch.randint(1, 100, (rows_per,), generator=g, device=dev).to(torch.float64))
    rep = torch.cat(reps) if reputation else None
    return R, sc_t.to(torch.uint8), lo_t, hi_t, rep
