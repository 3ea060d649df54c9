"""Per-SCP-iteration parity between the device and the CPU restatement.

The SCP stopping rule (SCP_controller.py:191-195) is a threshold test,
``|delta| < 1e-3 and max_violation <= 4.2e-3``.  Two correct solvers whose
iterates agree to 1e-9 can still stop one iteration apart when delta (or the
violation) of some iteration lies within that distance of its threshold.  Such
a problem is not skipped: both runs are compared iteration by iteration up to
the shorter count, and the first iteration where exactly one side stops must
be explained by a stopping-rule term that straddles its threshold, i.e. one
whose distance to the threshold is no larger than the two sides' difference
in it (plus a rounding floor).  Reference loop: SCP_controller.py:92-197.
"""
from __future__ import annotations

import numpy as np

from oracle import scp_reference as R
from scpqp import trace as TR

U_TOL = 1e-7          # rad, end to end / per iteration
TRAJ_TOL = 1e-6       # m
OBJ_RTOL = 1e-8
FLIP_FLOOR = 1e-9     # rounding floor of a threshold straddle


def stops(delta, maxviol, nV):
    if nV == 1 and abs(delta) < R.DELTA_TOL and maxviol > R.CONSTRAINT_TOL:
        return True
    return abs(delta) < R.DELTA_TOL and maxviol <= R.CONSTRAINT_TOL


def flip_explained(d_dev, d_orc, mv_dev, mv_orc):
    """The stopping decision differs: some term sits on its threshold within the
    two sides' disagreement in that term.  Returns (explained, margin)."""
    dd = abs(abs(d_dev) - abs(d_orc)) + FLIP_FLOOR
    dm = abs(mv_dev - mv_orc) + FLIP_FLOOR
    m_delta = min(abs(abs(d_dev) - R.DELTA_TOL), abs(abs(d_orc) - R.DELTA_TOL))
    m_viol = min(abs(mv_dev - R.CONSTRAINT_TOL), abs(mv_orc - R.CONSTRAINT_TOL))
    straddle_d = (abs(d_dev) < R.DELTA_TOL) != (abs(d_orc) < R.DELTA_TOL)
    straddle_v = (mv_dev <= R.CONSTRAINT_TOL) != (mv_orc <= R.CONSTRAINT_TOL)
    ok = (straddle_d and m_delta <= dd) or (straddle_v and m_viol <= dm)
    return ok, min(m_delta if straddle_d else np.inf, m_viol if straddle_v else np.inf)


def compare(dev_u, dev_traj, dev_nscp, dev_trace, r, nV, H, what=""):
    """Device result of one problem against the oracle's SCPResult ``r`` (run with
    keep_history=True).  dev_trace: decoded trace (scpqp.trace.decode) or None.
    Equal SCP counts: final u / traj.  Different counts: per iteration up to the
    shorter count, then the flip explanation.  Returns a dict of what was checked."""
    if dev_nscp == r.n_scp:
        eu = float(np.max(np.abs(dev_u - r.u)))
        et = float(np.max(np.abs(dev_traj - r.traj)))
        assert eu <= U_TOL, f"{what}: |u| err {eu:.2e}"
        assert et <= TRAJ_TOL, f"{what}: |traj| err {et:.2e}"
        return dict(mismatch=False, u_err=eu, traj_err=et)
    assert dev_trace is not None, f"{what}: n_scp {dev_nscp} vs {r.n_scp} and no device trace"
    assert r.history, f"{what}: oracle run without keep_history"
    n = min(dev_nscp, r.n_scp)
    worst = 0.0
    for it in range(n):
        t, h = dev_trace[it], r.history[it]
        e = float(np.max(np.abs(t["z"][:nV * H] - h["z"][:nV * H])))
        worst = max(worst, e)
        assert e <= U_TOL, f"{what}: iteration {it} |u| err {e:.2e}"
        assert abs(t["obj"] - h["obj"]) <= OBJ_RTOL * max(1.0, abs(h["obj"])), \
            f"{what}: iteration {it} obj {t['obj']} vs {h['obj']}"
    last = n - 1
    t, h = dev_trace[last], r.history[last]
    assert stops(t["delta"], t["maxviol"], nV) != stops(h["delta"], h["maxviol"], nV), \
        f"{what}: counts differ but iteration {last} decides the same on both sides"
    ok, margin = flip_explained(t["delta"], h["delta"], t["maxviol"], h["maxviol"])
    assert ok, (f"{what}: unexplained stop flip at iteration {last}: delta {t['delta']:.12g} vs "
                f"{h['delta']:.12g}, maxviol {t['maxviol']:.6g} vs {h['maxviol']:.6g}")
    return dict(mismatch=True, iters_compared=n, u_err=worst, flip_iter=last, margin=margin)


def device_trace(out, b, nV, nO, H, hp_max):
    if out.trace is None:
        return None
    return TR.decode(out.trace[b].cpu().numpy(), int(out.n_scp[b].item()), nV, nO, H, hp_max)


def oracle_job(args):
    """One oracle SCP solve with its per-iteration history, for a spawn pool:
    ``args`` = (n_veh, Hp, x0, u0, ec_noise[, scenario Hp])."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (here, root, os.path.join(root, "senquential-convex-programming-for-trajectory-planning_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import scp_reference as R_
    single_thread_blas()
    n_veh, hp, x0, u0, ec = args[:5]
    sc = R_.circle_scenario(n_veh, Hp=args[5] if len(args) > 5 else hp)
    p = R_.make_problem(sc, x0, u0, ec, Hp=hp)
    return R_.scp_solve(p, mode="structured", keep_history=True)


def single_thread_blas():
    """One BLAS thread in a pool worker (the pools run one worker per core of the box's
    CPU share; a multithreaded BLAS per worker on small matrices oversubscribes it)."""
    try:
        import threadpoolctl
        threadpoolctl.threadpool_limits(1)
    except ImportError:
        pass
