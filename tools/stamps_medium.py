"""Diagnostic: per-phase shader-clock breakdown of medium_round_kernel (csrc/pcx_medium.hip)
(PCX_STAMPS=1 makes the library stamp s_memtime at phase boundaries; printed to stderr).

usage: python tools/stamps_medium.py [B] [N] [E]
"""
import os
import sys
import time

os.environ["PCX_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pyconsensus_amd import synthetic  # noqa: E402
from pyconsensus_amd.batched import consensus_batched  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 100
E = int(sys.argv[3]) if len(sys.argv) > 3 else 50
R, sc, lo, hi, rep = synthetic.rounds(B, N, E, seed=3)
t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt).cuda()
args = (t(R), t(rep), t(sc, torch.uint8), t(lo), t(hi))
print(f"B={B} N={N} E={E} scaled columns={int(sc.sum())}/{sc.size}", flush=True)
for _ in range(2):
    t0 = time.perf_counter()
    consensus_batched(*args)
    torch.cuda.synchronize()
    print(f"  {B / (time.perf_counter() - t0):.0f} rounds/s (stamped)", flush=True)
