"""Fit of the operation order of ``np.dot(v, F)`` (v: (N,), F: (N, E) C-contiguous) in the
build container -- numpy 2.2.6 on OpenBLAS 0.3.29, DYNAMIC_ARCH with SkylakeX kernels --
the machine the golden vectors were generated on (make_golden.py).

The reference's discontinuous decisions (the rank rule, __init__.py:490-498; catch of the
raw outcomes, :510, :531) read ``np.dot(rep, F)``, ``np.dot(normalize(set), F)`` and
``np.dot(smooth_rep, F)``.  OpenBLAS does not document its summation order, so it was
measured: random inputs with a wide exponent range make every association visible, and
the model below (restated in C in oracle/pcx_oracle_batched.c ob_vecmat and in HIP in
csrc/pcx_batched.hip) reproduces numpy bit for bit.  Run as a script it prints the
mismatch count; tests/test_oracle_c.py runs it when the host's OpenBLAS core is SkylakeX.
"""
from __future__ import annotations

import math

import numpy as np


def fma(a, b, c):
    """Correctly rounded a*b + c (Python 3.10 has no math.fma): exact integer arithmetic."""
    a, b, c = float(a), float(b), float(c)
    if a == 0 or b == 0 or not (math.isfinite(a) and math.isfinite(b) and math.isfinite(c)):
        return a * b + c
    ma, ea = math.frexp(a)
    mb, eb = math.frexp(b)
    ma, ea, mb, eb = int(ma * (1 << 53)), ea - 53, int(mb * (1 << 53)), eb - 53
    if c == 0:
        p, e = ma * mb, ea + eb
    else:
        mc, ec = math.frexp(c)
        mc, ec = int(mc * (1 << 53)), ec - 53
        e = min(ea + eb, ec)
        p = (ma * mb << (ea + eb - e)) + (mc << (ec - e))
    if p == 0:
        return 0.0
    return float(p << e) if e >= 0 else p / (1 << -e)


def ob_ddot(a, x):
    """E == 1: numpy's ddot -- 4 x 8 fma lanes per 32 elements, folded to 4 x 4 lanes,
    16 per step, lanes summed (0+2)+(1+3), then a sequential fma tail."""
    n = len(x)
    acc8 = [[0.0] * 8 for _ in range(4)]
    n32, n16 = n & -32, n & -16
    for i in range(0, n32, 32):
        for k in range(32):
            acc8[k // 8][k % 8] = fma(a[i + k], x[i + k], acc8[k // 8][k % 8])
    acc4 = [[acc8[r][q] + acc8[r][q + 4] for q in range(4)] for r in range(4)]
    for i in range(n32, n16, 16):
        for k in range(16):
            acc4[k // 4][k % 4] = fma(a[i + k], x[i + k], acc4[k // 4][k % 4])
    A = [((acc4[0][q] + acc4[1][q]) + acc4[2][q]) + acc4[3][q] for q in range(4)]
    d = (A[0] + A[2]) + (A[1] + A[3])
    for i in range(n16, n):
        d = fma(a[i], x[i], d)
    return d


def ob_vecmat(v, F):
    """The model: cblas_dgemv(RowMajor, Trans) = column-major dgemv_n on the E x N matrix."""
    N, E = F.shape
    v = [float(t) for t in v]
    out = np.empty(E)
    for j in range(E):
        a = [float(t) for t in F[:, j]]
        if E == 1:
            out[j] = ob_ddot(a, v)
        elif j < (E & ~3):  # 4-row vector kernel
            y, n = 0.0, 0
            while n + 4 <= N:
                t = a[n + 1] * v[n + 1]
                for k in (0, 2, 3):
                    t = fma(a[n + k], v[n + k], t)
                y, n = y + t, n + 4
            if n + 2 <= N:
                y, n = y + fma(a[n], v[n], a[n + 1] * v[n + 1]), n + 2
            if n < N:
                y = y + a[n] * v[n]
            out[j] = y
        else:  # scalar tail rows
            t, i = 0.0, 0
            if E in (2, 3):
                while i + 4 <= N:
                    t = t + fma(a[i], v[i], a[i + 1] * v[i + 1])
                    t = t + fma(a[i + 2], v[i + 2], a[i + 3] * v[i + 3])
                    i += 4
            while i < N:
                t, i = fma(a[i], v[i], t), i + 1
            out[j] = t
    return out


def check(max_n=64, max_e=32, trials=2, seed=0):
    """Number of mismatching outputs of the model against np.dot on random inputs."""
    rng = np.random.default_rng(seed)
    bad = tot = 0
    for E in range(1, max_e + 1):
        for N in range(1, max_n + 1):
            for _ in range(trials):
                v = rng.uniform(0.5, 1, N) * np.exp2(rng.integers(-20, 20, N)) * rng.choice([-1, 1], N)
                F = rng.uniform(0.5, 1, (N, E)) * np.exp2(rng.integers(-20, 20, (N, E))) * rng.choice([-1, 1], (N, E))
                bad += int(np.sum(ob_vecmat(v, F) != np.dot(v, F)))
                tot += E
    return bad, tot


def blas_core():
    try:
        from threadpoolctl import threadpool_info

        for d in threadpool_info():
            if d.get("internal_api") == "openblas":
                return d.get("architecture"), d.get("version")
    except Exception:  # pragma: no cover
        pass
    return None, None


if __name__ == "__main__":
    print(blas_core(), check())
