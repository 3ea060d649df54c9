"""Generate the golden parity fixtures (tests/golden/*.npz) from the CPU restatement.

    python tests/golden/make_golden.py

The reference itself could not be executed here (denied), so the
fixtures are produced by ``oracle/scp_reference.py`` in faithful mode (dense
tensors exactly as QCQP_formulate) where that fits in memory, else structured
mode (c3).  The oracle is pinned by the known-answer tests and KKT
certificates in tests/test_oracle_*.py.  Each fixture holds the problem inputs
(in the C-ABI batch layout), the final outputs, the stage intermediates of
problem 0 and, for small configs, the per-SCP-iteration rows of problem 0.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd"))

from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT          # noqa: E402

CONFIGS = {
    # name: (scenario builder, B, mode, mixed horizons, keep SCP history of problem 0)
    "c1_circle1_hp10": (lambda: R.circle_scenario(1, Hp=10), 4, "faithful", None, True),
    "c2_circle4_hp20": (lambda: R.circle_scenario(4, Hp=20), 8, "faithful", None, True),
    "c3_circle8_hp30": (lambda: R.circle_scenario(8, Hp=30), 1, "structured", None, False),
    "c5_circle4_mixed": (lambda: R.circle_scenario(4, Hp=30), 3, "faithful", (10, 20, 30), False),
    "frog_hp10": (lambda: R.frog_scenario(Hp=10), 2, "faithful", None, True),
    "parallel5_hp10": (lambda: R.parallel_scenario(5, Hp=10), 2, "faithful", None, True),
    # per-iteration histories of the MFMA-factor configurations (round 3): c3 problem 0,
    # and every problem of the c5 batch (one per horizon class 10 / 20 / 30, all in
    # hp_max = 30 slots); the inputs are those of the fixtures above (same seed)
    "c3_circle8_hp30_hist": (lambda: R.circle_scenario(8, Hp=30), 1, "structured", None, "all"),
    "c5_circle4_mixed_hist": (lambda: R.circle_scenario(4, Hp=30), 3, "faithful", (10, 20, 30), "all"),
}
BASE_SEED = 20240


def make(name):
    build, B, mode, mixed, hist = CONFIGS[name]
    sc = build()
    bt = BT.make_batch(sc, B, base_seed=BASE_SEED, mixed_hp=mixed)
    nV, Hm = sc.nVeh, bt.hp_max
    u = np.zeros((B, nV * Hm))
    traj = np.zeros((B, Hm * 2 * nV))
    ref = np.zeros((B, Hm * 2 * nV))
    n_scp = np.zeros(B, np.int32)
    n_ipm = np.zeros(B, np.int32)
    obj = np.zeros(B)
    maxv = np.zeros(B)
    sumv = np.zeros(B)
    feas = np.zeros(B, np.int32)
    extra = {}
    for b in range(B):
        H = int(bt.hp[b])
        nO = sc.nObst
        ob = bt.obst[b].reshape(-1)[:nO * 2 * H].reshape(nO, 2, H)
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=H, obst=ob)
        keep = hist == "all" or (hist and b == 0)
        r = R.scp_solve(p, mode=mode, keep_history=keep)
        u[b, :nV * H] = r.u
        traj[b, :H * 2 * nV] = r.traj.reshape(-1)
        ref[b, :H * 2 * nV] = p.ref_points.reshape(-1)
        n_scp[b], n_ipm[b] = r.n_scp, r.n_ipm
        obj[b], maxv[b], sumv[b], feas[b] = r.obj, r.max_violation, r.sum_violations, r.feasible
        if b == 0:
            L = r.lin
            extra.update(lin_Ad=L.Ad, lin_Bd=L.Bd, lin_Ed=L.Ed, lin_g=L.g, lin_const=L.const,
                         lin_Phi0=L.Phi0, lin_Psi0=L.Psi0, lin_gamma0=L.gamma0)
        if keep:
            # problem 0 under "hist_*", problem b > 0 under "hist{b}_*"
            pre = "hist" if b == 0 else f"hist{b}"
            extra[pre + "_u_lin"] = np.array([h["u_lin"] for h in r.history])
            extra[pre + "_A"] = np.array([h["A"] for h in r.history])
            extra[pre + "_b"] = np.array([h["b"] for h in r.history])
            extra[pre + "_z"] = np.array([h["z"] for h in r.history])
            extra[pre + "_obj"] = np.array([h["obj"] for h in r.history])
            extra[pre + "_maxviol"] = np.array([h["maxviol"] for h in r.history])
            kkt = np.array([[h["certificate"][k] for k in
                             ("stationarity", "primal", "dual", "complementarity")]
                            for h in r.history])
            extra[pre + "_kkt"] = kkt
    out = os.path.join(HERE, name + ".npz")
    np.savez_compressed(out, scenario=name, mode=mode, n_veh=nV, n_obst=sc.nObst, hp_max=Hm,
                        x0=bt.x0, u0=bt.u0, ec_noise=bt.ec_noise, hp=bt.hp, obst=bt.obst,
                        seeds=bt.seeds, ref_points=ref, u=u, traj=traj, n_scp=n_scp, n_ipm=n_ipm,
                        obj=obj, max_violation=maxv, sum_violations=sumv, feasible=feas, **extra)
    print(f"{name}: B={B} n_scp={n_scp.tolist()} -> {os.path.getsize(out)} bytes", flush=True)


if __name__ == "__main__":
    names = sys.argv[1:] or list(CONFIGS)
    for nm in names:
        make(nm)
