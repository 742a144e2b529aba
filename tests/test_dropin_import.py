"""The reference's import path: ``from pyconsensus import Oracle, main``
(/root/reference/test/test_consensus.py:23) resolves to the MI355X implementation.

CPU: the names resolve to pyconsensus_amd's, ``main`` handles -h / a bad option as the
reference's (__init__.py:613-627), ``fold`` (:75-86).  GPU: the README example and
``main(["pyconsensus", "-t", "1"])`` through that import path, against the reference goldens."""
import os
import subprocess
import sys

import numpy as np
import pytest

import golden_cases as G
import parity as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_names_resolve_to_the_gpu_implementation():
    import pyconsensus
    import pyconsensus_amd
    from pyconsensus import Oracle, main
    from pyconsensus_amd.cli import main as amd_main

    assert Oracle is pyconsensus_amd.Oracle
    assert main is amd_main
    assert (pyconsensus.NO, pyconsensus.YES, pyconsensus.BAD, pyconsensus.NA) == (1.0, 2.0, 1.5, 0.0)


def test_main_help_and_bad_option(capsys):
    from pyconsensus import main

    assert main(argv=("", "-h")) == 0
    assert "test matrix" in capsys.readouterr().out
    assert main(argv=("", "-q")) == 2


def test_fold():
    from pyconsensus import fold

    assert fold([1, 2, 3, 4, 5, 6], 3) == [[1, 2, 3], [4, 5, 6]]
    with pytest.raises(Exception, match="not divisible"):
        fold([1, 2, 3], 2)


def test_module_entry_point_help():
    out = subprocess.run([sys.executable, "-m", "pyconsensus", "-h"], capture_output=True, text=True,
                         cwd=ROOT, timeout=120)
    assert out.returncode == 0 and "test matrix" in out.stdout


@pytest.mark.gpu
def test_readme_example_via_reference_import(gpu_lib):
    """README.rst:28-45 through ``from pyconsensus import Oracle``."""
    from pyconsensus import Oracle

    reports = [[0.2, 0.7, 1, 1], [0.3, 0.5, 1, 1], [0.1, 0.7, 1, 1],
               [0.5, 0.7, 2, 1], [0.1, 0.2, 2, 2], [0.1, 0.2, 2, 2]]
    bounds = [{"scaled": True, "min": 0.1, "max": 0.5}, {"scaled": True, "min": 0.2, "max": 0.7},
              {"scaled": False, "min": 1, "max": 2}, {"scaled": False, "min": 1, "max": 2}]
    r = Oracle(reports=reports, reputation=[1, 2, 10, 9, 4, 2], event_bounds=bounds).consensus()
    np.testing.assert_allclose(np.asarray(r["agents"]["smooth_rep"]),
                               [0.038501766886541035, 0.07693012197380761, 0.3809800680761801,
                                0.31073090020632843, 0.12857142857142856, 0.06428571428571428], rtol=1e-12)
    assert r["events"]["outcomes_final"] == [0.5, 0.7, 1.5, 1.0]


@pytest.mark.gpu
def test_main_t1_via_reference_import(gpu_lib, capsys):
    """``main(["pyconsensus", "-t", "1"])`` prints the tables; the same matrix through
    ``pyconsensus.Oracle`` matches the reference golden t1."""
    from pyconsensus import Oracle, main
    from pyconsensus_amd.cli import test_matrix

    assert main(["pyconsensus", "-t", "1"]) == 0
    out = capsys.readouterr().out
    assert "outcomes_final" in out and "smooth_rep" in out
    o = Oracle(reports=test_matrix(1))
    res = o.consensus()
    ours = {P.ABI_NAME[k]: v for k, v in G.flat_result(res).items() if k in P.ABI_NAME}
    ours["branch"] = np.array(o.last_info["branch"])
    kind, bad = P.mismatch_kind(G.kat()["t1"], ours)
    assert kind is None, bad
