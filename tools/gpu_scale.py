"""Throughput vs batch size (diagnostic): does a second workgroup per CU add throughput?"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd"))
import numpy as np, torch
from oracle import scp_reference as R
from scpqp import batch as BT
from scpqp.solver import ScpQpSolver
nv, hp = int(sys.argv[1]) if len(sys.argv) > 1 else 4, int(sys.argv[2]) if len(sys.argv) > 2 else 20
sc = R.circle_scenario(nv, Hp=hp)
base = BT.make_batch(sc, 1024, base_seed=0)
S = ScpQpSolver(sc, max_batch=4096)
print("resources", S.resources())
for B in (1, 64, 128, 256, 512, 768, 1024, 2048, 4096):
    idx = np.arange(B) % 1024
    x0 = torch.as_tensor(base.x0[idx], device="cuda"); u0 = torch.as_tensor(base.u0[idx], device="cuda")
    ec = torch.as_tensor(base.ec_noise[idx], device="cuda")
    out = S.alloc_out(B)
    S.solve(x0, u0, ec, out=out); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        S.solve(x0, u0, ec, out=out)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print(f"B={B:5d}: {ms:8.2f} ms  {B / ms * 1e3:9.0f} solves/s  mean ipm/problem {out.n_ipm.float().mean().item():.1f}", flush=True)
