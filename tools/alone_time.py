"""Diagnostic: latency of single c2 problems solved alone (B = 1) against the whole batch.

The c2 makespan is its slowest problem's chain; this times that problem on an
otherwise idle GPU, i.e. without co-resident problems on its CU.
    python tools/alone_time.py [problem ...]      (default: 271 0)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]


def main():
    import torch
    from oracle import scp_reference as R
    from scpqp import shard
    from scpqp.solver import ScpQpSolver
    probs = [int(a) for a in sys.argv[1:]] or [271, 0]
    sc = R.circle_scenario(4, Hp=20)
    bt = shard.shard_batch(sc, 1024, 0, base_seed=0)
    S = ScpQpSolver(sc, max_batch=1024)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        S.solve(bt.x0, bt.u0, bt.ec_noise)
    torch.cuda.synchronize()
    e0.record()
    out = S.solve(bt.x0, bt.u0, bt.ec_noise)
    e1.record()
    torch.cuda.synchronize()
    print(f"batch of 1024: {e0.elapsed_time(e1):.3f} ms")
    ns, ni = out.n_scp.cpu().numpy(), out.n_ipm.cpu().numpy()
    S1 = ScpQpSolver(sc, max_batch=1)
    for p in probs:
        x0, u0, ec = (a[p:p + 1].copy() for a in (bt.x0, bt.u0, bt.ec_noise))
        for _ in range(2):
            S1.solve(x0, u0, ec)
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            e0.record()
            o1 = S1.solve(x0, u0, ec)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f"problem {p}: n_scp {int(ns[p])} n_ipm {int(ni[p])} (alone: {int(o1.n_scp[0])} / {int(o1.n_ipm[0])}); "
              f"alone {min(ts):.3f}-{max(ts):.3f} ms")


if __name__ == "__main__":
    main()
