"""A/B of run-time solver parameters on the shipped library (one process, interleaved).

    python tools/gpu_param_ab.py c2:10 "polish_delta=3e-7" "polish_delta=1e-8" ...

For each parameter set: solves/s over the timed steps, SCP / IPM / polish-solve counts,
and the largest |u - u_first| against the first set on the problems whose SCP count
agrees (the certified polish point is the QP's unique minimiser, so a parameter of the
polish may change the path, not the answer).
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
from scpqp import batch as BT  # noqa: E402
from scpqp import shard  # noqa: E402
from scpqp.solver import ScpQpSolver  # noqa: E402
from oracle import scp_reference as R  # noqa: E402

CFG = {"c2": (4, 20, 1024), "c3": (8, 30, 4096), "c4": (4, 20, 8192), "c5": (4, 30, 3072)}


def parse(spec):
    kw = {}
    for item in spec.split(","):
        if item:
            k, v = item.split("=")
            kw[k] = int(v) if k in ("polish_refine", "max_ipm_iter") else float(v)
    return kw


def main():
    cfg, steps = sys.argv[1].split(":")
    steps = int(steps)
    V, H, B = CFG[cfg]
    sc = R.circle_scenario(V, Hp=H)
    mixed = (10, 20, 30) if cfg == "c5" else None   # bench.py's c5: mixed horizons
    bt = shard.shard_batch(sc, B, 0, base_seed=0, mixed_hp=mixed) if mixed else BT.make_batch(sc, B, base_seed=0)
    hpt = torch.as_tensor(bt.hp, device=torch.device("cuda", 0)) if mixed else None
    dev = torch.device("cuda", 0)
    x0 = torch.as_tensor(bt.x0, device=dev)
    u0 = torch.as_tensor(bt.u0, device=dev)
    ec = torch.as_tensor(bt.ec_noise, device=dev)
    ref = None
    for rep in range(2):
        for spec in sys.argv[2:]:
            S = ScpQpSolver(sc, max_batch=B, device=dev, **parse(spec))
            out = S.alloc_out(B)
            S.solve(x0, u0, ec, hp=hpt, out=out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                S.solve(x0, u0, ec, hp=hpt, out=out)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            u = out.u.cpu().numpy().reshape(B, -1)
            nscp = out.n_scp.cpu().numpy()
            nqp = max(int(nscp.sum()), 1)
            st = out.status.cpu().numpy()
            line = (f"{cfg} [{spec}] {B / dt:9.0f} solves/s  ms {dt * 1e3:8.2f}  scp {nscp.mean():.3f}  "
                    f"ipm/qp {out.n_ipm.cpu().numpy().sum() / nqp:.2f}  "
                    f"polish solves/qp {out.n_refine.cpu().numpy().sum() / nqp:.2f}  "
                    f"warm ok/qp {out.n_warm.cpu().numpy().sum() / nqp:.3f}  conv {np.mean((st & 0xff) == 0):.4f}  rej {np.mean((st & 0x100) != 0):.4f}")
            if ref is None and os.environ.get("CMP"):   # first set of another library's run
                z = np.load(os.environ["CMP"])
                ref = (z["u"], z["nscp"], z["st"])
            if ref is None:
                ref = (u, nscp, st)
                if os.environ.get("SAVE"):
                    np.savez(os.environ["SAVE"], u=u, nscp=nscp, st=st)
            else:
                same = nscp == ref[1]
                du = np.abs(u[same] - ref[0][same]).max() if same.any() else float("nan")
                line += f"  |du| {du:.1e} on {int(same.sum())}/{B} (nscp differs on {int((~same).sum())})"
                cv = same & ((st & 0xff) == 0) & ((ref[2] & 0xff) == 0)
                if cv.any():
                    line += f"  |du| converged {np.abs(u[cv] - ref[0][cv]).max():.1e} on {int(cv.sum())}"
            print(line, flush=True)
            if os.environ.get("DETAIL"):
                nref = out.n_refine.cpu().numpy(); npol = out.n_polish.cpu().numpy()
                nipm = out.n_ipm.cpu().numpy(); nwarm = out.n_warm.cpu().numpy()
                for b in np.argsort(-nref)[:12]:
                    print(f"    b {b:5d} nscp {nscp[b]:3d} ipm {nipm[b]:4d} rounds {npol[b]:4d} "
                          f"solves {nref[b]:5d} warm_ok {nwarm[b]:3d} status {st[b]:#x}")
                print(f"    solves per problem: p50 {np.median(nref):.0f} p90 {np.percentile(nref, 90):.0f} "
                      f"p99 {np.percentile(nref, 99):.0f} max {nref.max()}")
            S.close()


if __name__ == "__main__":
    main()
