"""Diagnostic: one solve and one evaluate of the c2-shaped batch of size B on a given build.
    python tools/eval_time.py <lib.so> <B>"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]


def main():
    import torch
    from oracle import scp_reference as R
    from scpqp import _lib, shard
    from scpqp.solver import ScpQpSolver
    _lib.use_build(sys.argv[1])
    B = int(sys.argv[2])
    sc = R.circle_scenario(4, Hp=20)
    bt = shard.shard_batch(sc, B, 0, base_seed=0)
    S = ScpQpSolver(sc, max_batch=B)
    out = S.solve(bt.x0, bt.u0, bt.ec_noise)
    torch.cuda.synchronize()
    print("solved", B, flush=True)
    t = time.perf_counter()
    ev = S.evaluate(out.u, bt.x0, bt.u0, bt.ec_noise)
    print(f"evaluate B {B}: {1e3 * (time.perf_counter() - t):.2f} ms, obj equal "
          f"{bool(torch.allclose(ev['obj'], out.obj, rtol=1e-12, atol=0))}", flush=True)
    S.close()


if __name__ == "__main__":
    main()
