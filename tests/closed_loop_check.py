"""Closed-loop parity of ``ClosedLoopBatch`` (main.py:98-206 on the device)
against the CPU restatement, for long runs (the reference's Nsim = 50).

Two comparisons per realisation and MPC step:

1. **Step parity on the device's own inputs** (never skipped): the restated
   SCP solve (oracle structured mode, keep_history) on the device's delay-
   compensated x0, held command u0, warm start and obstacle prediction, against
   the device solve, per SCP iteration where the counts differ
   (tests/scp_parity.py); the restated plant (the reference's dopri5 call,
   main.py:184-191) from the device's start state with the device's control
   ticks, against the device plant path.
2. **Independent closed loop**: the restated ``ClosedLoop`` run on its own from
   the same initial state.  Its per-step state / control differences to the
   device run are reported; they stay at integration-tolerance level as long as
   both loops take the same SCP iteration counts, and a stop flip (a threshold
   straddle, explained in 1.) legitimately moves the two loops apart afterwards.
3. **Independent closed loop on the device's integrator** (``rk4_loop``): the
   same restated loop with the reference's scipy integrator calls replaced by
   the restated fixed-step RK4 of csrc/plant.hip (oracle/plant_reference.py
   ``plant="rk4"``).  Where loop 2 parts from the device loop only because the
   two integrators differ by ~1e-12 m (the noise-free circle's mirror-symmetric
   bifurcation), loop 3 keeps following the device loop.

Used by tests/test_gpu_closed_loop.py and tools/closed_loop_parity.py (which
writes the profiles/ record).  The oracle runs in a spawned process pool, one
realisation per task.
"""
from __future__ import annotations

import math
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")

X0_SIGMA = np.array([0.05, 0.05, 0.005, 0.02, 0.0, 0.002])
PLANT_TOL = 1e-6       # device RK4 vs the reference's dopri5 at 1e-8


def _paths():
    for p in (HERE, ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)


def scenario(case):
    """main8: the reference's __main__ configuration (main.py:234-255: 8 vehicles
    on the circle, Hp = 10, is_noise False).  c2: 4-vehicle circle, Hp = 20."""
    _paths()
    from oracle import scp_reference as R
    if case == "main8":
        return R.circle_scenario(8, Hp=10)
    if case == "c2":
        return R.circle_scenario(4, Hp=20)
    if case == "circle4_hp10":
        return R.circle_scenario(4, Hp=10)
    if case == "frog":
        return R.frog_scenario(Hp=10)
    if case == "parallel5":
        return R.parallel_scenario(5, Hp=10)
    raise ValueError(case)


def initial_states(case, B, seed=2024):
    sc = scenario(case)
    base = np.array(sc.x0, float)
    x = np.repeat(base[None], B, 0)
    if case != "main8":            # Monte-Carlo realisations: perturbed initial states
        rng = np.random.default_rng(seed)
        x = x + rng.standard_normal(x.shape) * X0_SIGMA
    return x


def run_device(case, B, steps, device):
    """The device closed loop; returns per-realisation numpy step records."""
    _paths()
    from scpqp.rollout import ClosedLoopBatch
    sc = scenario(case)
    x_init = initial_states(case, B)
    cl = ClosedLoopBatch(sc, B, device=device, keep_path=True, trace=True)
    cl.reset(x_init)
    hist = cl.run(steps)
    nV, Hp = sc.nVeh, sc.Hp
    recs = []
    for b in range(B):
        rb = []
        for h in hist:
            rb.append(dict(
                x0=h["x0"][b].cpu().numpy(), u0=h["u0"][b].cpu().numpy(),
                u_warm=None if h["u_warm"] is None else h["u_warm"][b].cpu().numpy(),
                obst=None if h["obst"] is None else h["obst"][b].cpu().numpy(),
                u=h["u"][b].cpu().numpy(), n_scp=int(h["n_scp"][b]),
                trace=h["trace"][b].cpu().numpy(), traj=h["traj"][b].cpu().numpy(),
                U=h["U"][b].cpu().numpy().reshape(nV, Hp).T,
                x_start=h["x_start"][b].cpu().numpy(), u_tick=h["u_tick"][b].cpu().numpy(),
                path=h["path"][b].cpu().numpy()))
        recs.append(rb)
    cl.close()
    return x_init, recs


def check_realisation(args):
    """Oracle work for one realisation (runs in a worker).  Returns per-step metrics."""
    case, x_init, recs, mirror_steps = args[:4]
    rk4_loop = len(args) > 4 and args[4]
    _paths()
    from oracle import plant_reference as PR
    from oracle import scp_reference as R
    from scpqp import trace as TR
    import scp_parity as SP
    sc = scenario(case)
    nV, nO, Hp, tps = sc.nVeh, sc.nObst, sc.Hp, sc.ticks_per_sim
    ref = PR.ClosedLoop(sc, x_init=x_init)
    ref4 = PR.ClosedLoop(sc, x_init=x_init, plant="rk4") if rk4_loop else None
    steps = []
    same_counts = True
    same_counts4 = True
    for i, d in enumerate(recs):
        m = dict(step=i, n_scp_dev=d["n_scp"])
        # 1a. solve parity on the device's inputs
        p = R.make_problem(sc, d["x0"], d["u0"], np.zeros((nV, 2)), Hp=Hp,
                           obst=d["obst"] if nO else None)
        r = R.scp_solve(p, u_warm=d["u_warm"], mode="structured", keep_history=True)
        u = d["u"][:nV * Hp]
        tr = TR.decode(d["trace"], d["n_scp"], nV, nO, Hp, Hp)
        m["n_scp_oracle_same_inputs"] = r.n_scp
        try:
            res = SP.compare(u, d["traj"], d["n_scp"], tr, r, nV, Hp, what=f"step {i}")
            m["solve"] = "flip" if res["mismatch"] else "equal"
            m["solve_u_err"] = res["u_err"]
            if res["mismatch"]:
                m["flip_margin"] = res["margin"]
        except AssertionError as e:
            mirror = float(np.max(np.abs(u + r.u)))
            if i in mirror_steps and mirror <= SP.U_TOL:
                m["solve"] = "mirror"
                m["solve_u_err"] = mirror
            else:
                m["solve"] = "FAIL"
                m["error"] = str(e)
        # 1b. plant parity on the device's inputs (the reference's dopri5 call)
        perr = 0.0
        for v in range(nV):
            ms = PR.plant_step(sc, v, d["x_start"][v], i * sc.dt, d["u_tick"][v])
            perr = max(perr, float(np.max(np.abs(ms - d["path"][v]))))
        m["plant_err"] = perr
        # 2. the independent restated loop
        rr = ref.step(i)
        # the symmetric (noise-free) circle can settle in the mirror branch on either
        # side; the loops then run mirrored and are no longer compared entry-wise
        mirrored = (np.max(np.abs(rr["U"] + d["U"])) < np.max(np.abs(rr["U"] - d["U"]))
                    and np.max(np.abs(rr["U"] - d["U"])) > 1e-4)
        m["loop_mirrored"] = bool(mirrored)
        same_counts = same_counts and rr["n_scp"] == d["n_scp"] and not mirrored
        m["n_scp_oracle_loop"] = rr["n_scp"]
        m["same_counts_so_far"] = same_counts
        m["loop_x0_diff"] = float(np.max(np.abs(rr["x0"] - d["x0"])))
        m["loop_U_diff"] = float(np.max(np.abs(rr["U"] - d["U"])))
        want = ref.path[:, :, i * tps:(i + 1) * tps + 1].transpose(1, 2, 0)
        m["loop_path_diff"] = float(np.max(np.abs(want - d["path"])))
        # 3. the independent restated loop on the device's integrator
        if ref4 is not None:
            r4 = ref4.step(i)
            mir4 = (np.max(np.abs(r4["U"] + d["U"])) < np.max(np.abs(r4["U"] - d["U"]))
                    and np.max(np.abs(r4["U"] - d["U"])) > 1e-4)
            same_counts4 = same_counts4 and r4["n_scp"] == d["n_scp"] and not mir4
            m["rk4_loop_mirrored"] = bool(mir4)
            m["rk4_n_scp_oracle_loop"] = r4["n_scp"]
            m["rk4_same_counts_so_far"] = same_counts4
            m["rk4_loop_x0_diff"] = float(np.max(np.abs(r4["x0"] - d["x0"])))
            m["rk4_loop_U_diff"] = float(np.max(np.abs(r4["U"] - d["U"])))
            w4 = ref4.path[:, :, i * tps:(i + 1) * tps + 1].transpose(1, 2, 0)
            m["rk4_loop_path_diff"] = float(np.max(np.abs(w4 - d["path"])))
        steps.append(m)
    return steps


def run(case, B, steps, device, workers=16, mirror_steps=(), rk4_loop=False):
    x_init, recs = run_device(case, B, steps, device)
    ctx = mp.get_context("spawn")
    tasks = [(case, x_init[b], recs[b], tuple(mirror_steps), rk4_loop) for b in range(B)]
    with ctx.Pool(min(workers, B)) as pool:
        per = pool.map(check_realisation, tasks)
    return per


def summary(per):
    allm = [m for rb in per for m in rb]
    kinds = {}
    for m in allm:
        kinds[m["solve"]] = kinds.get(m["solve"], 0) + 1
    agree = [m for m in allm if m["same_counts_so_far"]]
    return dict(
        realisations=len(per), steps=len(per[0]) if per else 0, solve_kinds=kinds,
        max_solve_u_err=max((m["solve_u_err"] for m in allm if "solve_u_err" in m), default=0.0),
        max_plant_err=max(m["plant_err"] for m in allm),
        min_flip_margin=min((m["flip_margin"] for m in allm if "flip_margin" in m),
                            default=math.inf),
        loop_steps_with_same_counts=len(agree),
        loop_max_path_diff_same_counts=max((m["loop_path_diff"] for m in agree), default=0.0),
        loop_max_U_diff_same_counts=max((m["loop_U_diff"] for m in agree), default=0.0),
        loop_max_path_diff_all=max(m["loop_path_diff"] for m in allm),
        loop_max_U_diff_all=max(m["loop_U_diff"] for m in allm),
        **(dict(rk4_loop_steps_with_same_counts=sum(m["rk4_same_counts_so_far"] for m in allm),
                rk4_loop_mirrored_steps=sum(m["rk4_loop_mirrored"] for m in allm),
                rk4_loop_max_path_diff_all=max(m["rk4_loop_path_diff"] for m in allm),
                rk4_loop_max_U_diff_all=max(m["rk4_loop_U_diff"] for m in allm),
                rk4_loop_max_x0_diff_all=max(m["rk4_loop_x0_diff"] for m in allm))
           if allm and "rk4_loop_path_diff" in allm[0] else {}))
