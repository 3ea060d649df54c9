"""Diagnostic: run one edge case of tests/test_gpu_parity.py::test_edge_cases per process."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd"))
import numpy as np, torch
from oracle import scp_reference as R
from scpqp import batch as BT
from scpqp.solver import ScpQpSolver
case = sys.argv[1]
t = time.time()
HPS = {"badhp": [20, 21, 0, 20], "hp1": [1, 1, 1, 1], "hp20": [20, 20, 20, 20], "zero1": [0],
       "zero2": [20, 0], "big2": [20, 21]}
if case in HPS:
    sc = R.circle_scenario(4, Hp=20)
    hp = np.array(HPS[case], np.int32)
    B = len(hp)
    S = ScpQpSolver(sc, max_batch=B)
    bt = BT.make_batch(sc, B, base_seed=1)
    out = S.solve(bt.x0, bt.u0, bt.ec_noise, hp=hp)
else:
    sc = R.circle_scenario(1, Hp=64)
    S = ScpQpSolver(sc, max_batch=2)
    bt = BT.make_batch(sc, 2, base_seed=3)
    out = S.solve(bt.x0, bt.u0, bt.ec_noise)
torch.cuda.synchronize()
print(case, "ok %.2fs" % (time.time() - t), out.status.tolist(), out.n_scp.tolist(), out.n_ipm.tolist(), flush=True)
