"""A/B timing of library variants on the c2 bench config (interleaved rounds, one process)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")
sys.path.insert(0, PKG)
import numpy as np, torch
from scpqp import _lib as LB
from oracle import scp_reference as R
from scpqp import batch as BT
from scpqp.solver import ScpQpSolver
libs = sys.argv[1:] or ["libscpqp.so"]
sc = R.circle_scenario(4, Hp=20)
bt = BT.make_batch(sc, 1024, base_seed=0)
solvers = {}
for name in libs:
    LB._lib = None
    LB._lib = LB.load(os.path.join(PKG, "scpqp", name))
    S = ScpQpSolver(sc, max_batch=1024)
    out = S.solve(bt.x0, bt.u0, bt.ec_noise); torch.cuda.synchronize()
    solvers[name] = (S, out)
times = {n: [] for n in libs}
for rnd in range(5):
    for name, (S, out) in solvers.items():
        torch.cuda.synchronize(); t = time.time()
        S.solve(bt.x0, bt.u0, bt.ec_noise, out=out); torch.cuda.synchronize()
        times[name].append(time.time() - t)
ref = None
for name, (S, out) in solvers.items():
    u = out.u.cpu().numpy()
    if ref is None: ref = u
    print(f"{name:24s} median {np.median(times[name])*1e3:7.2f} ms  min {min(times[name])*1e3:7.2f} ms  "
          f"solves/s {1024/np.median(times[name]):9.0f}  max|du| vs first {np.abs(u-ref).max():.1e}  res {S.resources()}")
