"""CLI parity: the reference's -t/-x/-m/-s runner
(pyconsensus/__init__.py:613-898).  CPU: the test matrices equal the KAT inputs taken
from the reference; GPU: each CLI run reproduces the reference's golden results."""
import numpy as np
import pytest

import golden_cases as G
import parity as P


@pytest.mark.parametrize("k", list(range(1, 19)))
def test_test_matrices_match_reference(k):
    from pyconsensus_amd.cli import test_matrix

    np.testing.assert_array_equal(test_matrix(k), G.kat()["t%d" % k]["in_reports"])


def test_help_and_bad_option(capsys):
    from pyconsensus_amd.cli import main

    assert main(["prog", "-h"]) == 0
    assert "test matrix" in capsys.readouterr().out
    assert main(["prog", "--nope"]) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("k", list(range(1, 19)))
def test_cli_t_runs_golden(gpu_lib, k, capsys):
    from pyconsensus_amd import Oracle
    from pyconsensus_amd.cli import main, test_matrix

    assert main(["prog", "-t", str(k)]) == 0
    out = capsys.readouterr().out
    assert "outcomes_final" in out and "smooth_rep" in out
    case = G.kat()["t%d" % k]
    o = Oracle(reports=test_matrix(k))
    res = o.consensus()
    ours = {P.ABI_NAME[kk]: v for kk, v in G.flat_result(res).items() if kk in P.ABI_NAME}
    ours["branch"] = np.array(o.last_info["branch"])
    kind, bad = P.mismatch_kind(case, ours)
    path = "exact" if o.last_info["path"] == "batched" else "matrix"
    assert kind == P.KNOWN_MISMATCH[path].get("t%d" % k, (None,))[0], (path, kind, bad)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["-x", "-m", "-s"])
def test_cli_examples_run(gpu_lib, opt, capsys):
    from pyconsensus_amd.cli import main

    assert main(["prog", opt]) == 0
    assert "smooth_rep" in capsys.readouterr().out
