"""``pyconsensus`` -- the reference's import path, served by the MI355X implementation.

The reference's callers and tests do ``from pyconsensus import Oracle, main``
(/root/reference/test/test_consensus.py:23; ``Oracle`` at pyconsensus/__init__.py:100,
``main`` at :613).  This package keeps that line working unchanged: ``Oracle`` and ``main``
are :class:`pyconsensus_amd.Oracle` and :func:`pyconsensus_amd.cli.main`, so every consensus
runs on libpcx's HIP kernels.  The module constants (:65-68) and ``fold`` (:73-84) are the
reference's plain helpers.
"""
from pyconsensus_amd import Oracle, consensus_batched  # noqa: F401
from pyconsensus_amd.cli import main  # noqa: F401

__title__ = "pyconsensus"
__version__ = "0.5.7"  # the reference release this drop-in follows (__init__.py:54)

NO = 1.0
YES = 2.0
BAD = 1.5
NA = 0.0


def fold(arr, num_cols):
    """Row-major list -> list of rows of ``num_cols`` (__init__.py:75-86), same error."""
    n = len(arr) / float(num_cols)
    if n != int(n):
        raise Exception("array length (%i) not divisible by %i" % (len(arr), num_cols))
    return [list(arr[i * num_cols:(i + 1) * num_cols]) for i in range(int(n))]


__all__ = ["Oracle", "main", "fold", "NO", "YES", "BAD", "NA", "consensus_batched"]
