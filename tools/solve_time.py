"""Diagnostic: one solve of a configuration's batch on a given build, timed (wall).
    python tools/solve_time.py <lib.so> <c2|c4|c3|c5> [reps]"""
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
    cfg = sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    nv, hp, B, rank, mixed = {"c2": (4, 20, 1024, 0, None), "c4": (4, 20, 8192, 7, None),
                              "c3": (8, 30, 4096, 0, None), "c5": (4, 30, 3072, 0, (10, 20, 30))}[cfg]
    sc = R.circle_scenario(nv, Hp=hp)
    bt = shard.shard_batch(sc, B, rank, base_seed=0, mixed_hp=mixed)
    S = ScpQpSolver(sc, max_batch=B)
    for r in range(reps):
        t = time.perf_counter()
        out = S.solve(bt.x0, bt.u0, bt.ec_noise, hp=bt.hp if mixed else None, trace=(r == 0))
        torch.cuda.synchronize()
        print(f"{cfg} B {B} rep {r}: {1e3 * (time.perf_counter() - t):.1f} ms, mean SCP "
              f"{float(out.n_scp.float().mean()):.3f}", flush=True)
    if hasattr(_lib.load(), "scpqp_diag_reduce_check"):
        import ctypes
        c = (ctypes.c_ulonglong * 2)()
        _lib.load().scpqp_diag_reduce_check(c, 0)
        print("reduction check counters", c[0], c[1])
    S.close()


if __name__ == "__main__":
    main()
