"""The drop-in Oracle (pyconsensus_amd.Oracle) on the GPU: reference API, result
containers and golden values."""
import numpy as np
import pytest

import golden_cases as G
import parity as P

pytestmark = pytest.mark.gpu


def test_readme_example(gpu_lib):
    """README.rst:28-45 (config C1): SURVEY.md Appendix C anchor values."""
    from pyconsensus_amd import Oracle

    reports = [[0.2, 0.7, 1, 1], [0.3, 0.5, 1, 1], [0.1, 0.7, 1, 1],
               [0.5, 0.7, 2, 1], [0.1, 0.2, 2, 2], [0.1, 0.2, 2, 2]]
    bounds = [{"scaled": True, "min": 0.1, "max": 0.5}, {"scaled": True, "min": 0.2, "max": 0.7},
              {"scaled": False, "min": 1, "max": 2}, {"scaled": False, "min": 1, "max": 2}]
    o = Oracle(reports=reports, reputation=[1, 2, 10, 9, 4, 2], event_bounds=bounds)
    r = o.consensus()
    np.testing.assert_allclose(np.asarray(r["agents"]["smooth_rep"]),
                               [0.038501766886541035, 0.07693012197380761, 0.3809800680761801,
                                0.31073090020632843, 0.12857142857142856, 0.06428571428571428], rtol=1e-12)
    assert r["events"]["outcomes_final"] == [0.5, 0.7, 1.5, 1.0]
    assert r["events"]["outcomes_adjusted"] == [1.0, 1.0, 1.5, 1.0]
    np.testing.assert_allclose(r["participation"], 0.8083264115523836, rtol=1e-12)
    assert np.isnan(r["events"]["certainty"][2])
    assert o.reptokens == [35714, 71428, 357142, 321428, 142857, 71428]
    assert isinstance(r["agents"]["smooth_rep"], np.ma.MaskedArray)
    assert set(r) == {"original", "filled", "agents", "events", "participation", "avg_certainty",
                      "convergence", "components"}


@pytest.mark.parametrize("name", sorted(k for k in G.kat().keys() if k not in P.EXCLUDED))
def test_kat_through_oracle(gpu_lib, name):
    from pyconsensus_amd import Oracle

    case = G.kat()[name]
    o = Oracle(**G.oracle_args(case))
    res = o.consensus()
    ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(res).items() if k in P.ABI_NAME}
    ours["branch"] = np.array(o.last_info["branch"])
    kind, bad = P.mismatch_kind(case, ours)
    path = "exact" if o.last_info["path"] == "batched" else "matrix"
    assert kind == P.KNOWN_MISMATCH[path].get(name, (None,))[0], (path, kind, bad)


@pytest.mark.parametrize("name", P.DEGENERATE_MASKED)
def test_masked_data_case(gpu_lib, name):
    """The degenerate all-missing scaled column (parity.DEGENERATE_MASKED) through the drop-in
    Oracle (batched kernel) and forced through the single-matrix pipeline: every output,
    numpy.ma's masked-data ones included, and the branch, as the reference."""
    from pyconsensus_amd import Oracle
    from test_matrix_gpu import run_matrix

    case = G.kat()[name]
    o = Oracle(**G.oracle_args(case))
    res = o.consensus()
    ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(res).items() if k in P.ABI_NAME}
    ours["branch"] = np.array(o.last_info["branch"])
    P.assert_full(name, case, ours)
    P.assert_full(name, case, run_matrix(case))


def test_caller_array_rescaled_in_place(gpu_lib):
    """Quirk Q2: a float ndarray passed as reports is rescaled in place."""
    from pyconsensus_amd import Oracle

    R = np.array([[0.2, 1.0], [0.4, 2.0], [0.3, 2.0]])
    Oracle(reports=R, event_bounds=[{"scaled": True, "min": 0.0, "max": 0.8},
                                    {"scaled": False, "min": 1, "max": 2}]).consensus()
    np.testing.assert_allclose(R[:, 0], [0.25, 0.5, 0.375])
