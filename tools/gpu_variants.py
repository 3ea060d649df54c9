"""Time library builds x memory plans on c2 batches (one process, interleaved rounds).

    python tools/gpu_variants.py B1,B2,.. lib[:plan] [lib[:plan] ...]

lib is a file under scpqp/ (e.g. libscpqp.so, libscpqp_nt128.so); plan sets
SCPQP_PLAN (0 all LDS, 1 vectors in the workspace, ...) for that handle.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")
sys.path[:0] = [ROOT, PKG]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import scp_reference as R  # noqa: E402
from scpqp import _lib as LB  # noqa: E402
from scpqp import batch as BT  # noqa: E402
from scpqp.solver import ScpQpSolver  # noqa: E402

batches = [int(b) for b in sys.argv[1].split(",")]
specs = sys.argv[2:] or ["libscpqp.so"]
nveh = int(os.environ.get("NVEH", 4))
hp = int(os.environ.get("HP", 20))
sc = R.circle_scenario(nveh, Hp=hp)
bt = BT.make_batch(sc, max(batches), base_seed=0)
for B in batches:
    sub = bt.slice(0, B)
    runs = {}
    for spec in specs:
        name, _, plan = spec.partition(":")
        if plan:
            os.environ["SCPQP_PLAN"] = plan
        else:
            os.environ.pop("SCPQP_PLAN", None)
        LB._lib = None
        LB._lib = LB.load(os.path.join(PKG, "scpqp", name))
        S = ScpQpSolver(sc, max_batch=B)
        out = S.solve(sub.x0, sub.u0, sub.ec_noise)
        torch.cuda.synchronize()
        runs[spec] = (S, out, [])
    for rnd in range(4):
        for spec, (S, out, ts) in runs.items():
            torch.cuda.synchronize()
            t = time.perf_counter()
            S.solve(sub.x0, sub.u0, sub.ec_noise, out=out)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
    ref = None
    for spec, (S, out, ts) in runs.items():
        u = out.u.cpu().numpy()
        ref = u if ref is None else ref
        med = float(np.median(ts))
        nipm = out.n_ipm.cpu().numpy().sum() / out.n_scp.cpu().numpy().sum()
        nw = out.n_warm.cpu().numpy().sum() / out.n_scp.cpu().numpy().sum() if hasattr(out, "n_warm") else -1
        print(f"B={B:5d} {spec:26s} {med * 1e3:8.2f} ms {B / med:9.0f} solves/s  "
              f"max|du| {np.abs(u - ref).max():.1e} ipm/qp {nipm:.2f} warm {nw:.2f} {S.resources()}", flush=True)
        S.close()
