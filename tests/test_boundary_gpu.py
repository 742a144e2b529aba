"""The single-matrix C-ABI driven from plain C (tests/c/consensus_abi.c): one call of
pcx_consensus_f64 per rank, host buffers, no Python or torch in the caller -- at world 1
(pcx_create) and as 2 / 3 in-process virtual ranks (pcx_group, each passing only its rows),
against the numpy oracle.  Also: the reference's stage methods on the drop-in Oracle
(interpolate / wpca / lie_detector / nonconformity(_rank), __init__.py:260-500) against the
numpy restatement, and the RCCL communicator itself (a one-rank RCCL context runs every
exchange of the sharded path) against the plain context."""
import os
import subprocess

import numpy as np
import pytest

import golden_cases as G
import parity as P

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def c_exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("cabi")
    exe = str(d / "consensus_abi")
    lib = os.path.join(ROOT, "pyconsensus_amd")
    subprocess.check_call(["gcc", "-O1", "-std=c99", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "consensus_abi.c"), "-o", exe, "-L", lib, "-lpcx",
                           "-lpthread", "-Wl,-rpath," + lib])
    return exe, d


def _write_case(path, R, rep, sc, lo, hi):
    N, E = R.shape
    with open(path, "wb") as f:
        np.array([N, E, rep is not None, sc is not None], dtype=np.int64).tofile(f)
        np.ascontiguousarray(R, dtype=np.float64).tofile(f)
        if rep is not None:
            np.asarray(rep, dtype=np.float64).tofile(f)
        if sc is not None:
            np.asarray(sc, dtype=np.uint8).tofile(f)
            np.asarray(lo, dtype=np.float64).tofile(f)
            np.asarray(hi, dtype=np.float64).tofile(f)


def _read_out(path, N, E):
    a = np.fromfile(path, dtype=np.float64)
    out, o = {}, 0
    for k in G.AGENT_KEYS[:0] or ["old_rep", "this_rep", "smooth_rep", "scores", "na_row", "participation_rows",
                                  "relative_part", "reporter_bonus"]:
        out[k] = a[o:o + N]
        o += N
    for k in ["adj_first_loadings", "outcomes_raw", "outcomes_adjusted", "outcomes_final", "certainty",
              "consensus_reward", "nas_filled", "participation_columns", "author_bonus"]:
        out[k] = a[o:o + E]
        o += E
    out["filled"] = a[o:o + N * E].reshape(N, E)
    o += N * E
    out["participation"], out["avg_certainty"] = a[o], a[o + 1]
    return out, {"branch": int(a[o + 2]), "n_hard": int(a[o + 4]), "sel_passes": int(a[o + 5])}


@pytest.mark.parametrize("world", [1, 2, 3])
def test_c_program_calls_single_matrix_abi(gpu_lib, c_exe, world):
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import synthetic

    exe, d = c_exe
    N, E = 9000, 130
    R, sc, lo, hi, rep = synthetic.matrix(N, E, seed=31)
    ref = G.flat_result(OracleCPU(reports=R, event_bounds=synthetic.bounds_list(sc, lo, hi),
                                  reputation=rep).consensus())
    inp, outp = str(d / ("in%d.bin" % world)), str(d / ("out%d.bin" % world))
    _write_case(inp, R, rep, sc, lo, hi)
    r = subprocess.run([exe, inp, outp, str(world)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    ours, info = _read_out(outp, N, E)
    print(r.stdout.strip(), info)
    bad, _ = P.compare(ref, ours)
    assert not bad, bad


@pytest.mark.parametrize("devices", ["0", "0,0", "0,0,0"])
def test_c_program_multi_device_context(gpu_lib, c_exe, devices):
    """ONE pcx_consensus_f64 call on a pcx_create_devices context with the whole host matrix:
    the library shards the rows over the listed devices (worker threads; RCCL ncclCommInitAll
    for distinct ids -- "0" is a one-rank RCCL communicator -- host exchange when an id
    repeats).  Equals the one-device call: discrete outputs exactly, continuous ones within the
    north_star tolerance (the covariance partials are summed across ranks)."""
    from pyconsensus_amd import synthetic

    exe, d = c_exe
    N, E = 9000, 130
    R, sc, lo, hi, rep = synthetic.matrix(N, E, seed=31)
    inp = str(d / "in_dev.bin")
    _write_case(inp, R, rep, sc, lo, hi)
    o1, on = str(d / "out_dev1.bin"), str(d / ("out_dev_%s.bin" % devices.replace(",", "_")))
    r = subprocess.run([exe, inp, o1, "1"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    world = devices.count(",") + 1
    r = subprocess.run([exe, inp, on, str(world), devices], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    print(r.stdout.strip())
    # the sharded covariance is one f64 SUM all-reduce of per-rank partials: continuous
    # outputs agree with the one-device call to rounding, discrete ones exactly
    one, _ = _read_out(o1, N, E)
    many, info = _read_out(on, N, E)
    ref = {g: one[a] for g, a in P.ABI_NAME.items() if a in one}
    bad, _ = P.compare(ref, many)
    assert not bad, bad
    for k in ("na_row", "nas_filled", "outcomes_adjusted", "outcomes_final", "filled"):
        np.testing.assert_array_equal(many[k], one[k], err_msg=k)
    assert info["branch"] == _read_out(o1, N, E)[1]["branch"]


def test_oracle_devices_matches_one_gpu(gpu_lib):
    """Oracle(devices=[0, 0]): the drop-in's row-sharded multi-GPU path (rehearsed on one
    GPU: two ranks on device 0) equals Oracle() -- fills and discrete outputs exactly, the
    rest within the north_star tolerance -- for consensus and the stage methods."""
    from pyconsensus_amd import Oracle, _lib, synthetic

    R, sc, lo, hi, rep = synthetic.matrix(3001, 70, seed=12)
    eb = synthetic.bounds_list(sc, lo, hi)
    one = Oracle(reports=R.copy(), event_bounds=eb, reputation=rep).consensus()
    o2 = Oracle(reports=R.copy(), event_bounds=eb, reputation=rep, devices=[0, 0])
    two = o2.consensus()
    assert o2.last_info["devices"] == [0, 0] and o2.last_info["comm_bytes"] > 0
    f1, f2 = G.flat_result(one), G.flat_result(two)
    bad, _ = P.compare(f1, {a: f2[g] for g, a in P.ABI_NAME.items()})
    assert not bad, bad
    g1 = Oracle(reports=R.copy(), event_bounds=eb, reputation=rep)
    g2 = Oracle(reports=R.copy(), event_bounds=eb, reputation=rep, devices=[0, 0, 0])
    F1, F2 = g1.interpolate(g1.reports), g2.interpolate(g2.reports)
    np.testing.assert_array_equal(F2, F1)  # fills are exact on any rank count
    s1, s2 = g1.lie_detector(F1), g2.lie_detector(F2)
    for k in ("this_rep", "smooth_rep"):
        np.testing.assert_allclose(np.asarray(s2[k]), np.asarray(s1[k]), rtol=1e-9, atol=1e-12, err_msg=k)
    with pytest.raises(_lib.PcxError, match="fewer rows than devices"):
        Oracle(reports=np.ones((66, 2)), devices=[0] * 70).lie_detector(np.ones((66, 2)))


def test_devices_context_survives_a_failed_call(gpu_lib):
    """A bad argument on a multi-device context (non-finite catch_tolerance, a clustering
    algorithm on several ranks) fails before any worker starts -- no abort of the context's
    exchange -- and the next call on the same cached context succeeds with the one-device
    result."""
    from pyconsensus_amd import _lib, synthetic
    from pyconsensus_amd.pipeline import consensus_host

    R, sc, lo, hi, rep = synthetic.matrix(500, 40, seed=21)
    h0 = _lib.devices_context([0, 0])
    with pytest.raises(_lib.PcxError, match="catch_tolerance"):
        consensus_host(R, rep, sc, lo, hi, devices=[0, 0], catch_tolerance=float("nan"))
    with pytest.raises(_lib.PcxError, match="one rank"):
        consensus_host(R, rep, sc, lo, hi, devices=[0, 0], algorithm="hierarchical")
    # the argument errors came before any exchange: the cached context is kept, not recreated
    assert _lib.devices_context([0, 0]) == h0 and _lib.lib().pcx_ctx_usable(h0) == 1
    two, m2 = consensus_host(R, rep, sc, lo, hi, devices=[0, 0])
    one, m1 = consensus_host(R, rep, sc, lo, hi)
    assert m2["branch"] == m1["branch"]
    np.testing.assert_array_equal(two["outcomes_final"], one["outcomes_final"])
    np.testing.assert_allclose(two["smooth_rep"], one["smooth_rep"], rtol=1e-9, atol=1e-12)


def _small_oracles(name):
    from oracle.pcx_oracle import OracleCPU
    from pyconsensus_amd import Oracle, synthetic

    if name == "readme":
        case = G.kat()["readme"]
        kw = G.oracle_args(case)
    else:
        R, sc, lo, hi, rep = synthetic.matrix(2000, 90, seed=77)
        kw = dict(reports=R, event_bounds=synthetic.bounds_list(sc, lo, hi), reputation=rep)
    cpu = OracleCPU(**{k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in kw.items()})
    gpu = Oracle(**{k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in kw.items()})
    return cpu, gpu


@pytest.mark.parametrize("name", ["readme", "2000x90"])
def test_stage_methods_match_restatement(gpu_lib, name):
    cpu, gpu = _small_oracles(name)
    # interpolate (:260-313): filled matrix exact, scaled events rescaled in place
    Fc = cpu.interpolate(cpu.reports)
    Fg = gpu.interpolate(gpu.reports)
    np.testing.assert_array_equal(np.asarray(Fg, float), np.asarray(Fc, float))
    np.testing.assert_array_equal(np.ma.getdata(gpu.reports), np.ma.getdata(cpu.reports))
    F = np.asarray(Fc, dtype=np.float64)
    # wpca (:315-339): mean, covariance, loading (up to the LAPACK sign, Q8), scores
    mc, wc, cc, lc, sc_ = cpu.wpca(F)
    mg, wg, cg, lg, sg = gpu.wpca(F)
    np.testing.assert_allclose(np.asarray(mg), np.asarray(mc), rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(np.asarray(wg), np.asarray(wc), rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(np.asarray(cg), np.asarray(cc), rtol=1e-11, atol=1e-14)
    lcv, lgv = np.asarray(lc, float), np.asarray(lg, float)
    sign = -1.0 if np.dot(lcv, lgv) < 0 else 1.0
    np.testing.assert_allclose(sign * lgv, lcv, rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(sign * np.asarray(sg, float).ravel(), np.asarray(sc_, float).ravel(), rtol=1e-9,
                               atol=1e-11)
    # nonconformity (:475-485) and nonconformity_rank (:487-500) on the reference's scores
    s = np.asarray(sc_, float).ravel()
    np.testing.assert_allclose(gpu.nonconformity(s, F), cpu.nonconformity(s, F), rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(gpu.nonconformity_rank(s, F), cpu.nonconformity_rank(s, F), rtol=1e-12, atol=1e-14)
    # lie_detector (:341-473): reputations
    ld_c = cpu.lie_detector(F)
    ld_g = gpu.lie_detector(F)
    for k in ("this_rep", "smooth_rep", "old_rep"):
        np.testing.assert_allclose(np.asarray(ld_g[k], float), np.asarray(ld_c[k], float), rtol=1e-9, atol=1e-12,
                                   err_msg=k)
    assert isinstance(ld_g["smooth_rep"], np.ma.MaskedArray)


def test_rccl_communicator_one_rank(gpu_lib):
    """A one-rank RCCL context (ncclCommInitRank through libpcx) runs every collective of the
    sharded path -- u64 SUM / MIN / MAX, f64 SUM, in-place and packed all-gathers, the
    selection passes -- and must give the plain context's result bit for bit."""
    import socket

    import torch
    import torch.distributed as dist
    from pyconsensus_amd import synthetic
    from pyconsensus_amd.pipeline import RcclComm, consensus_matrix

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        R, sc, lo, hi, rep = synthetic.matrix(12000, 100, seed=5)
        ev1, ag1, m1 = consensus_matrix(R, rep, sc, lo, hi)
        comm = RcclComm(1, 0, torch.cuda.current_device())
        ev2, ag2, m2 = consensus_matrix(R, rep, sc, lo, hi, comm=comm, n_total=R.shape[0], row_offset=0)
        comm.close()
        assert m2["sel_passes"] > 0  # the exchanged selection ran (not the one-rank shortcut)
        for d1, d2 in ((ev1, ev2), (ag1, ag2)):
            for k in d1:
                np.testing.assert_array_equal(d2[k].cpu().numpy(), d1[k].cpu().numpy(), err_msg=k)
    finally:
        dist.destroy_process_group()
