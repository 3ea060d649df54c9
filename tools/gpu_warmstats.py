"""Warm-start statistics of a c2 batch: cold QPs per problem by SCP count; the
indices of the problems with the most IPM iterations (for CPU studies)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
import numpy as np, torch
from oracle import scp_reference as R
from scpqp import batch as BT
from scpqp.solver import ScpQpSolver
sc = R.circle_scenario(4, Hp=20)
bt = BT.make_batch(sc, 1024, base_seed=0)
S = ScpQpSolver(sc, max_batch=1024)
out = S.solve(bt.x0, bt.u0, bt.ec_noise); torch.cuda.synchronize()
ns, ni, nw = out.n_scp.cpu().numpy(), out.n_ipm.cpu().numpy(), out.n_warm.cpu().numpy()
for k in range(1, 21):
    sel = ns == k
    if sel.any():
        cold = k - nw[sel]
        print(f"nscp {k:2d}: {sel.sum():4d}  cold QPs mean {cold.mean():5.2f}  ipm {ni[sel].mean():6.1f}  ipm/cold {ni[sel].sum() / max(cold.sum(), 1):5.1f}")
top = np.argsort(-ni)[:10]
print("most IPM iterations: idx nscp nwarm nipm", [(int(i), int(ns[i]), int(nw[i]), int(ni[i])) for i in top])
