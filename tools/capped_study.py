"""Capped problems (20 QPs without meeting the stopping rule): per SCP iteration, the
device's distance to the restatement's exact-polish run (ed) next to the distance between
the restatement's own two polish modes (em, exact vs the device's regularised one), for
every capped problem of the c2 batch and of the first 32 c3 problems.
    python tools/capped_study.py
"""
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import scp_parity as SP  # noqa: E402
from oracle import scp_reference as R  # noqa: E402
from scpqp import _lib as LB  # noqa: E402
from scpqp import shard  # noqa: E402
from scpqp.solver import ScpQpSolver  # noqa: E402
from test_gpu_configs import _oracle_modes_job  # noqa: E402


def main():
    for nV, Hp, B in ((4, 20, 1024), (8, 30, 32)):
        sc = R.circle_scenario(nV, Hp=Hp)
        bt = shard.shard_batch(sc, B, 0, base_seed=0)
        S = ScpQpSolver(sc, max_batch=B)
        out = S.solve(bt.x0, bt.u0, bt.ec_noise, trace=True)
        torch.cuda.synchronize()
        st = out.status.cpu().numpy()
        capped = np.flatnonzero((st & 0xff) == LB.ST_MAX_SCP).tolist()
        jobs = [(nV, Hp, bt.x0[b], bt.u0[b], bt.ec_noise[b]) for b in capped]
        with mp.get_context("spawn").Pool(min(16, max(1, len(jobs)))) as pool:
            res = pool.map(_oracle_modes_job, jobs)
        N = nV * Hp
        for b, (rx, rr) in zip(capped, res):
            tr = SP.device_trace(out, b, nV, 0, Hp, Hp)
            ed = [float(np.max(np.abs(tr[it]["z"][:N] - rx.history[it]["z"][:N]))) for it in range(20)]
            em = [float(np.max(np.abs(rr.history[it]["z"][:N] - rx.history[it]["z"][:N])))
                  if it < rr.n_scp else float("nan") for it in range(20)]
            dm = [float(np.max(np.abs(tr[it]["z"][:N] - rr.history[it]["z"][:N])))
                  if it < rr.n_scp else float("nan") for it in range(20)]
            print(f"{nV} veh problem {b}: exact n_scp {rx.n_scp} reg n_scp {rr.n_scp} device "
                  f"{int(out.n_scp[b].item())}; max ed {max(ed):.2e} max em {np.nanmax(em):.2e} "
                  f"max |dev - reg| {np.nanmax(dm):.2e}")
            print("   ed " + " ".join(f"{v:.0e}" for v in ed))
            print("   em " + " ".join(f"{v:.0e}" for v in em))
            print("   dr " + " ".join(f"{v:.0e}" for v in dm))
        S.close()


if __name__ == "__main__":
    main()
