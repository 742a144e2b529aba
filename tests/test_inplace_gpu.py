"""`original` aliasing the reports (pcx_result.original == pcx_problem.reports): the reference's
own `original` is the caller's array rescaled in place (__init__.py:121, 266-269, 584; Q2), so
libpcx rescales the scaled columns in place instead of writing a copy of every column.  Every
output must equal the copy mode's bit for bit, and the reports buffer must afterwards hold the
copy mode's `original` bit for bit -- through the fused k_wcd pass (PCA), the k_matrices pass
(algorithms without wpca, the interpolate entry), device and host memory, one and two ranks.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.int64) if a.dtype == np.float64 else a


def _same(a, b, what):
    np.testing.assert_array_equal(_bits(a), _bits(b), err_msg=what)


def _device_run(R, rep, sc, lo, hi, inplace, **kw):
    import torch

    from pyconsensus_amd.pipeline import consensus_matrix

    Rd = torch.as_tensor(R).to("cuda:0").contiguous()
    t = lambda x, dt=torch.float64: None if x is None else torch.as_tensor(x, dtype=dt).to("cuda:0")
    ev, ag, meta = consensus_matrix(Rd, t(rep), t(sc, torch.uint8), t(lo), t(hi), matrices=True,
                                    original_inplace=inplace, **kw)
    torch.cuda.synchronize()
    out = {k: v.cpu().numpy() for k, v in list(ev.items()) + list(ag.items())}
    out["branch"] = np.array(meta["branch"])
    out["reports_after"] = Rd.cpu().numpy()
    if inplace:
        assert ag["original"].data_ptr() == Rd.data_ptr()
    return out


@pytest.mark.parametrize("shape,algorithm,int_dtype,repnone", [
    ((20000, 400), "PCA", False, False),
    ((16648, 2048), "PCA", False, True),    # int8 grid + mixed blocks, compact passes
    ((3000, 150), "PCA", True, False),      # int dtype: truncated rescale (Q3)
    ((5000, 120), "absolute", False, False),  # no wpca: k_matrices writes at the end
])
def test_inplace_equals_copy_device(gpu_lib, shape, algorithm, int_dtype, repnone):
    from pyconsensus_amd import synthetic

    N, E = shape
    R, sc, lo, hi, rep = synthetic.matrix(N, E, seed=N + 7)
    if int_dtype:
        R = np.where(np.isnan(R), np.nan, np.round(R))
    rep = None if repnone else rep
    kw = dict(algorithm=algorithm, int_dtype=int_dtype)
    a = _device_run(R, rep, sc, lo, hi, False, **kw)
    b = _device_run(R, rep, sc, lo, hi, True, **kw)
    for k in a:
        if k == "reports_after":
            continue
        _same(b[k], a[k], k)
    _same(b["reports_after"], a["original"], "reports rescaled in place == original")
    _same(a["reports_after"], R, "copy mode leaves the reports alone")
    # binary columns are untouched bits (NaN payloads included)
    _same(b["reports_after"][:, ~sc.astype(bool)], R[:, ~sc.astype(bool)], "binary columns")


def test_inplace_host_and_two_ranks(gpu_lib):
    """Host memory (the drop-in's path, also the multi-device context sharding the rows over two
    ranks on device 0): `original` comes back as the caller's own array."""
    from pyconsensus_amd import synthetic
    from pyconsensus_amd.pipeline import consensus_host, interpolate_host

    R, sc, lo, hi, rep = synthetic.matrix(6000, 90, seed=31)
    for devices in (None, [0, 0]):  # (two ranks sum the covariance in another order: own reference)
        ref, _ = consensus_host(R.copy(), rep, sc, lo, hi, devices=devices)
        X = R.copy()
        got, _ = consensus_host(X, rep, sc, lo, hi, original_inplace=True, devices=devices)
        assert got["original"] is X
        for k in ref:
            _same(got[k], ref[k], "%s devices=%s" % (k, devices))
    X = R.copy()
    iref, _ = interpolate_host(R.copy(), rep, sc, lo, hi)
    ig, _ = interpolate_host(X, rep, sc, lo, hi, original_inplace=True)
    assert ig["original"] is X
    _same(X, iref["original"], "interpolate in place")
    _same(ig["filled"], iref["filled"], "interpolate filled")


def test_dropin_rescales_caller_array(gpu_lib):
    """Oracle on a float64 ndarray above the batched limits: the caller's array IS result['original']
    and carries the rescaled scaled columns (Q2), with no second host copy."""
    from pyconsensus_amd import Oracle, synthetic

    R, sc, lo, hi, rep = synthetic.matrix(2000, 60, seed=44)
    raw = R.copy()
    res = Oracle(reports=R, event_bounds=synthetic.bounds_list(sc, lo, hi), reputation=rep).consensus()
    assert np.shares_memory(res["original"], R)
    cols = np.nonzero(sc)[0]
    assert not np.array_equal(R[:, cols][~np.isnan(raw[:, cols])], raw[:, cols][~np.isnan(raw[:, cols])])
    _same(R[:, ~sc.astype(bool)], raw[:, ~sc.astype(bool)], "binary columns untouched")


def test_inplace_without_filled(gpu_lib):
    """`original` aliased and `filled` NULL: the interpolate entry and a consensus without wpca
    (no k_wcd pass: M_ZERO_LOADING) must still rescale the scaled columns in place (k_matrices
    runs for the in-place rescale alone)."""
    from pyconsensus_amd import _abi, synthetic
    from pyconsensus_amd.pipeline import _host_call, consensus_host, interpolate_host

    R, sc, lo, hi, rep = synthetic.matrix(5000, 120, seed=52)
    iref, _ = interpolate_host(R.copy(), rep, sc, lo, hi)
    X = R.copy()
    got, _ = _host_call("pcx_interpolate_f64", X, rep, sc, lo, hi, 0, {"original": X.shape}, original_inplace=True)
    assert got["original"] is X
    _same(X, iref["original"], "interpolate in place, no filled")
    n, E = R.shape
    shapes = {k: (n,) for k in _abi.MAT_OUTPUT_AGENTS}
    shapes.update({k: (E,) for k in _abi.MAT_OUTPUT_EVENTS})
    cref, _ = consensus_host(R.copy(), rep, sc, lo, hi, algorithm="absolute")
    X = R.copy()
    shapes["original"] = X.shape
    got, _ = _host_call("pcx_consensus_f64", X, rep, sc, lo, hi, 0, shapes, algorithm="absolute", original_inplace=True)
    _same(X, cref["original"], "absolute consensus in place, no filled")
    for k in cref:
        if k not in ("original", "filled"):
            _same(got[k], cref[k], k)
