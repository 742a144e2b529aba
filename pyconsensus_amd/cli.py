"""Command-line runner with the reference CLI's options (pyconsensus/__init__.py:613-898).

    python -m pyconsensus_amd -t N      # test matrix N = 1..18, algorithm "PCA" (:628-847)
    python -m pyconsensus_amd -x        # example, algorithm "absolute" (:849-862)
    python -m pyconsensus_amd -m        # missing reports, weighted (:863-876)
    python -m pyconsensus_amd -s        # scaled events (:877-895)
    python -m pyconsensus_amd -h        # help

Every consensus runs on the GPU through :class:`pyconsensus_amd.Oracle`; the output is the
reference's: the report matrix (``-t``), then the ``events`` and ``agents`` tables as pandas
DataFrames.  ``--algorithm`` (an addition) selects any GPU-path algorithm for ``-t``.
"""
from __future__ import annotations

import getopt
import sys

import numpy as np

YES, NO, BAD, NA = 2.0, 1.0, 1.5, 0.0  # __init__.py:65-68
_CODE = {"Y": YES, "N": NO, "B": BAD, "Z": NA}


def _rows(*patterns):
    """Report rows from compact patterns: 'Y' = YES, 'N' = NO, 'B' = BAD, 'Z' = NA;
    ``("YYNN", 6)`` repeats a row."""
    out = []
    for p in patterns:
        pat, times = (p, 1) if isinstance(p, str) else p
        out.extend([[_CODE[c] for c in pat]] * times)
    return np.array(out, dtype=np.float64)


def test_matrix(k):
    """The reference's -t test matrices (:630-841), by number."""
    m1 = ("YYNN", "YNNN", "YYNN", "YYYN", "NNYY", "NNYY")
    m2 = (("YYNN", 6), ("YYYN", 5))
    m4 = (("YYNNY", 15), "NNNYN", ("YYYNY", 5), ("YYNNY", 4))
    m6 = ("NNYYNYNNNN", "YYNNNYYYNY", "YYNYNYYNYY", "NYNNYNYNNY", "NNYNYNNNNN", "NYNNNYYNYY",
          "YNNYYNYNNN", "YYNNYNYYYN", ("YNNYNYNNNY", 11), "NYNNYNYNNY")
    table = {
        1: m1, 17: m1, 2: m2, 14: m2, 4: m4, 15: m4, 6: m6, 16: m6,
        3: (("YYNNYYNNYYNNY", 6), "NNNYNNNYNNNYN", ("YYYNYYYNYYYNY", 4)),
        5: ("BNNYNNYYBB", "BBNBBYYBYB", "NYBBNYNNBB", "BBBBBNNNBY", "NYYBBYBYBY", "NYYYNBNBBB",
            "NNNYNNNYBY", "BBBYBYBBYN", "BBBNBYYNNB", "BYBYNNYYNB", "YYBBBYBBYY", "YBYNYBYNYB",
            ("NNNYYYBYBN", 7), "BBBYBYBBYN"),
        7: ("YYYYYY", "YYYNNN", "ZZZZZZ"),
        8: ("YYYYYY", "YYYNZZ", "YYYZZN"),
        9: ("YYYYYY", "YYYNZZ", "YYYNZZ"),
        10: ("YYYNYY", "YYYNZZ", "YYYNZZ"),
        11: ("YYYYYY", "ZZZZZZ", "YYYNNN"),
        12: (("YYYNNN", 3),),
        13: ("YYYNNN",),
        18: ("YYNN", "YNNN", ("ZZZZ", 14)),
    }
    if k not in table:
        raise ValueError("no test matrix %r (1..18)" % (k,))
    return _rows(*table[k])


def _tables(result):
    import pandas as pd

    return pd.DataFrame(result["events"]), pd.DataFrame(result["agents"])


def main(argv=None):
    from . import Oracle

    argv = sys.argv if argv is None else argv
    try:
        opts, _ = getopt.getopt(argv[1:], "hxmst:a:", ["help", "example", "missing", "scaled", "test=",
                                                        "algorithm="])
    except getopt.GetoptError as e:
        sys.stderr.write(e.msg)
        sys.stderr.write("for help use --help")
        return 2
    algorithm = "PCA"
    for opt, arg in opts:
        if opt in ("-a", "--algorithm"):
            algorithm = arg
    for opt, arg in opts:
        if opt in ("-h", "--help"):
            print(__doc__)
            return 0
        if opt in ("-t", "--test"):
            reports = test_matrix(int(arg))
            res = Oracle(reports=reports.copy(), algorithm=algorithm).consensus()
            ev, ag = _tables(res)
            print(reports)
            print(ev)
            print()
            print(ag)
        elif opt in ("-x", "--example"):
            reports = test_matrix(1)
            res = Oracle(reports=reports, reputation=[2, 10, 4, 2, 7, 1], algorithm="absolute").consensus()
            ev, ag = _tables(res)
            print(ev)
            print(ag)
        elif opt in ("-m", "--missing"):
            reports = _rows("YYNZ", "YNNN", "YYNN", "YYYN", "ZNYY", "NNYY")
            res = Oracle(reports=reports, reputation=[2, 10, 4, 2, 7, 1], algorithm="PCA").consensus()
            ev, ag = _tables(res)
            print(ev)
            print(ag)
        elif opt in ("-s", "--scaled"):
            reports = np.array([[YES, YES, NO, NO, 233, 16027.59], [YES, NO, NO, NO, 199, NA],
                                [YES, YES, NO, NO, 233, 16027.59], [YES, YES, YES, NO, 250, NA],
                                [NO, NO, YES, YES, 435, 8001.00], [NO, NO, YES, YES, 435, 19999.00]])
            bounds = [{"scaled": False, "min": NO, "max": 1}] * 4 + [
                {"scaled": True, "min": 0, "max": 435}, {"scaled": True, "min": 8000, "max": 20000}]
            res = Oracle(reports=reports, event_bounds=bounds).consensus()
            ev, ag = _tables(res)
            print(ev)
            print(ag)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
