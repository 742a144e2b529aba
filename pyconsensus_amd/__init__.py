"""pyconsensus_amd -- MI355X-native Oracle.consensus() (PCA path) behind the pyconsensus API.

    from pyconsensus_amd import Oracle
    Oracle(reports, event_bounds=..., reputation=...).consensus()

Batched Monte Carlo rounds: :func:`consensus_batched`.  Single huge matrices,
row-sharded over GPUs: :func:`pyconsensus_amd.pipeline.consensus_matrix`.
"""
__version__ = "0.1.0"

from .batched import consensus_batched  # noqa: E402,F401
from .oracle import Oracle  # noqa: E402,F401
