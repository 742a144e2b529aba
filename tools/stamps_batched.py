"""Diagnostic: per-phase shader-clock breakdown of batched_round_kernel on the C3 workload
(PCX_STAMPS=1 makes the library stamp s_memtime at phase boundaries; printed to stderr)."""
import os
import sys

os.environ["PCX_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pyconsensus_amd import synthetic  # noqa: E402
from pyconsensus_amd.batched import consensus_batched  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
R, sc, lo, hi, rep = synthetic.rounds(B, 50, 20, seed=20261015)
t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt).cuda()
args = (t(R), t(rep), t(sc, torch.uint8), t(lo), t(hi))
for _ in range(2):
    consensus_batched(*args)
    torch.cuda.synchronize()
