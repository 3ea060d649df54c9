"""c5 (4 vehicles, Hp {10, 20, 30} mixed, B = 3072) by horizon class: kernel time of the
mixed launch (one hp_max = 30 plan for every problem) against one launch per class, each
with the plan of its own horizon (hp_max = 10 / 20 / 30 solvers on that class's problems).
    python tools/c5_classes.py [reps]
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd"))
import numpy as np
import torch

import Scenarios
from scpqp import shard
from scpqp.solver import ScpQpSolver


def scen(hp, nv=4):
    sc = Scenarios.Scenario(False)
    sc.Hp = sc.Hu = hp
    sc.get_circle_scenario([2 * math.pi / nv * (i + 1) for i in range(nv)])
    sc.complete_scenario()
    return sc


def timed(S, args, hp=None, reps=3):
    out = S.alloc_out(args[0].shape[0])
    S.solve(*args, hp=hp, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        S.solve(*args, hp=hp, out=out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, out


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    sc30 = scen(30)
    B = 3072
    bt = shard.shard_batch(sc30, B, 0, base_seed=0, mixed_hp=(10, 20, 30))
    x0 = torch.as_tensor(bt.x0, device=dev)
    u0 = torch.as_tensor(bt.u0, device=dev)
    ec = torch.as_tensor(bt.ec_noise, device=dev)
    hp = np.asarray(bt.hp)
    S = ScpQpSolver(sc30, max_batch=B, device=dev)
    ms_mixed, out = timed(S, (x0, u0, ec), hp=torch.as_tensor(hp, device=dev), reps=reps)
    ipm_mixed = out.n_ipm.cpu().numpy()
    print(f"mixed launch: {ms_mixed:.2f} ms  {B / ms_mixed * 1e3:.0f} solves/s", flush=True)
    tot = 0.0
    for h in (30, 20, 10):
        idx = np.nonzero(hp == h)[0]
        it = torch.as_tensor(idx, device=dev)
        Sh = ScpQpSolver(scen(h), max_batch=len(idx), device=dev)
        ms, o = timed(Sh, (x0[it], u0[it], ec[it]), reps=reps)
        tot += ms
        print(f"class hp={h}: {len(idx)} problems, {ms:.2f} ms, ipm {o.n_ipm.sum().item()} "
              f"(mixed launch: {ipm_mixed[idx].sum()})", flush=True)
    print(f"per-class launches back to back: {tot:.2f} ms  {B / tot * 1e3:.0f} solves/s")


if __name__ == "__main__":
    main()
