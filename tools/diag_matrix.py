"""Diagnostic: matrix-path intermediates vs the numpy oracle for one golden case (GPU box)."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
import golden_cases as G
from oracle.pcx_oracle import OracleCPU
from pyconsensus_amd.pipeline import consensus_matrix

which = sys.argv[1] if len(sys.argv) > 1 else "m051"
if which.startswith("m"):
    case = G.mixed()[which]
else:
    case = G.unstack(G.synth(), int(which))
kw = G.oracle_args(case)
o = OracleCPU(**kw)
F = o.interpolate(o.reports)
wm, wcd, cov, ld, sc = o.wpca(F)
bk = {}
if bool(case["in_has_bounds"]):
    bk = dict(scaled=case["in_scaled"], lo=case["in_lo"], hi=case["in_hi"])
rep = case["in_reputation"] if bool(case["in_has_rep"]) else None
ev, ag, meta = consensus_matrix(case["in_reports"], rep, matrices=True, **bk)
ws = meta["workspace"]
E = F.shape[1]
mu = ws.ev[1].cpu().numpy()
C = ws.C.cpu().numpy()
L = ws.ev[3].cpu().numpy()
print("flags", meta["flags"], "iters", meta["pi_iters"], "branch", meta["branch"])
print("filled max diff", np.nanmax(np.abs(ag["filled"].cpu().numpy() - F)))
print("mu rel diff", np.max(np.abs(mu - np.asarray(wm)) / np.abs(np.asarray(wm))))
covn = np.asarray(cov)
print("C max abs diff", np.max(np.abs(C - covn)), "max |C|", np.max(np.abs(covn)))
i, j = np.unravel_index(np.argmax(np.abs(C - covn)), C.shape)
print("worst entry", i, j, C[i, j], covn[i, j])
ldn = np.asarray(ld)
s = np.sign(np.dot(L, ldn))
print("loading max diff", np.max(np.abs(L * s - ldn)))
print("tokens", ws.tok.cpu().numpy()[:5], o.reptokens[:5], "denom", ws.scal[0, 0].cpu().numpy())
