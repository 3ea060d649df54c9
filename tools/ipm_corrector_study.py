"""CPU study: fewer cold-IPM iterations through extra centrality correctors.

Every QP of a c2 problem's SCP loop (oracle arithmetic, the kernel's scaled form)
is solved by the kernel's Mehrotra predictor-corrector (R.qp_ipm) and by variants:

  gondzio K   up to K Gondzio multiple-centrality correctors per iteration
              (Gondzio 1996; Colombo & Gondzio 2008 for QP): after the Mehrotra
              direction with step a, aim at the enlarged step a~ = min(1, a + da),
              project the trial complementarity products onto [bmin sigma mu,
              bmax sigma mu] and solve once more with the projection's defect added
              to the complementarity right-hand side; keep the corrected direction
              only if its step grows by at least gamma da.

A corrector costs one more triangular-solve pair and one vector phase on the
factor the iteration already has; an iteration costs the assembly, the
factorisation, two solve pairs and two vector phases.  The cost model below
uses the B = 1 phase stamps of the shipped kernel (profiles/r03_phases.txt).

    python tools/ipm_corrector_study.py [n_problems] [c2|c3|hp10|hp30|frog|par5] [seed]

The kernel's round-3 rules are "round-3 start + adaptive step + split primal / dual steps"
(DESIGN §3).
"""
import os
import sys

import numpy as np
import scipy.linalg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT  # noqa: E402

# cycles (B = 1, c2): assembly 29k + factorisation 65k + init/top ~2k per iteration,
# a solve pair ~10.5k, a vector phase (back + rhs or back + update) ~14.5k
C_ITER = 29e3 + 65e3 + 2e3 + 2 * (10.5e3 + 14.5e3)
C_CORR = 10.5e3 + 14.5e3


def ipm(P, q, G, h, K=0, da=0.1, bmin=0.1, bmax=10.0, gamma=0.1, tol=R.IPM_TOL, maxit=60,
        sig_pow=3, init="cvxopt", floor=1e-2, lam0=1.0, woff=1.0, shift=0.0, ulin=None, clip=0.9,
        eta="fixed", lam_box=None, start=None, split=False):
    mc = len(h)
    x = np.linalg.solve(P + G.T @ G, -q + G.T @ h)
    s = h - G @ x
    lam = -s.copy()
    if init == "cvxopt":
        ts = -s.min()
        if ts >= -1e-8 * max(np.linalg.norm(s), 1.0):
            s = s + (1 + ts)
        tz = -lam.min()
        if tz >= -1e-8 * max(np.linalg.norm(lam), 1.0):
            lam = lam + (1 + tz)
    elif init.startswith("mehrotra"):
        # Mehrotra (1992) starting point: shift to positivity, then balance the products
        s = s + max(-1.5 * s.min(), 0.0) + 1e-8
        lam = lam + max(-1.5 * lam.min(), 0.0) + 1e-8
        sl = s @ lam
        s, lam = s + 0.5 * sl / lam.sum(), lam + 0.5 * sl / s.sum()
    elif init.startswith("omega") or init in ("lin", "zero"):
        # controls from the omega-free normal system, the slack at its smallest feasible
        # value (+1), the omega bound's multiplier carrying the slack weight
        N = len(q) - 1
        Gu = G[:, :N]
        if init == "lin":   # the SCP linearisation point (no initial solve)
            xu = np.clip(ulin, -clip, clip)
            init = "omega-floor"
        elif init == "zero":
            xu = np.zeros(N)
            init = "omega-floor"
        else:
            xu = np.linalg.solve(P[:N, :N] + Gu.T @ Gu, -q[:N] + Gu.T @ h)
        r = Gu @ xu - h                       # omega rows: a_r u - b_r - omega <= 0 scaled
        col = G[:, N]
        viol = np.where(col < 0, r / np.where(col < 0, -col, 1.0), -np.inf)[:-1]
        om = max(0.0, viol.max()) + woff
        x = np.append(xu, om)
        s = h - G @ x
        s = s + max(-1.5 * s.min(), 0.0) + (1.0 if init == "omega" else shift)
        s = np.maximum(s, floor * max(1.0, s.max()) if init == "omega-floor" else s)
        lam = np.full(len(h), lam0 if lam0 > 0 else -lam0 * abs(q[N]) / len(h))
        if lam_box is not None:   # box rows: the rows without an omega coefficient
            lam[:-1][col[:-1] == 0] = lam_box
        lam[-1] = abs(q[N]) / -col[-1]
        if init == "omega-bal":
            mu0 = (s @ lam) / len(h)
            lam = np.maximum(lam, mu0 / s)
    elif init.startswith("dual"):
        # dual-feasible multipliers from the least-squares stationarity of rd = 0
        lam = np.linalg.lstsq(G.T, -(P @ x + q), rcond=None)[0]
        s = s + max(-1.5 * s.min(), 0.0) + 1e-8
        lam = lam + max(-1.5 * lam.min(), 0.0) + 1e-8
        sl = s @ lam
        s, lam = s + 0.5 * sl / lam.sum(), lam + 0.5 * sl / s.sum()
    if start is not None:            # explicit (x, s, lam), e.g. a warm start
        x, s, lam = (np.array(v, float) for v in start)
    qn = max(1.0, np.abs(q).max()); hn = max(1.0, np.abs(h).max())
    ncorr = 0
    for it in range(maxit):
        rd = P @ x + q + G.T @ lam
        rp = G @ x + s - h
        gap = s @ lam
        pobj = 0.5 * x @ P @ x + q @ x
        if (np.abs(rp).max() <= tol * hn and np.abs(rd).max() <= tol * qn
                and gap <= tol * max(1.0, abs(pobj))):
            return x, s, lam, it, 1, ncorr
        mu = gap / mc
        d = lam / s
        try:
            L = np.linalg.cholesky(P + G.T @ (d[:, None] * G))
        except np.linalg.LinAlgError:
            return x, s, lam, it, 2, ncorr

        def solve(rc):
            dx = scipy.linalg.cho_solve((L, True), -rd - G.T @ (d * rp - rc / s))
            ds = -rp - G @ dx
            return dx, ds, -(rc + lam * ds) / s

        dx, ds, dl = solve(s * lam)
        a = R._max_step(s, ds, lam, dl)
        if split == "both":   # split affine steps in the centring estimate as well
            apa = R._max_step(s, ds, np.ones_like(lam), np.zeros_like(dl))
            ada = R._max_step(np.ones_like(s), np.zeros_like(ds), lam, dl)
            sigma = ((s + apa * ds) @ (lam + ada * dl) / mc / mu) ** sig_pow
        else:
            sigma = ((s + a * ds) @ (lam + a * dl) / mc / mu) ** sig_pow
        rc = s * lam + ds * dl - sigma * mu
        dx, ds, dl = solve(rc)
        a = R._max_step(s, ds, lam, dl)
        for _ in range(K):
            if a >= 1.0:
                break
            at = min(1.0, a + da)
            v = (s + at * ds) * (lam + at * dl)
            lo, hi = bmin * sigma * mu, bmax * sigma * mu
            t = np.clip(v, lo, hi) - v
            t = np.maximum(t, -hi)            # do not pull large products down too far
            ncorr += 1
            dx2, ds2, dl2 = solve(rc - t)
            a2 = R._max_step(s, ds2, lam, dl2)
            if a2 >= a + gamma * da:
                dx, ds, dl, a = dx2, ds2, dl2, a2
            else:
                break
        if eta == "fixed":
            a = min(1.0, 0.99 * a)
        elif eta == "adaptive":      # step factor max(0.99, 1 - mu)
            a = min(1.0, max(0.99, 1.0 - mu) * a)
        elif isinstance(eta, tuple):  # (floor, scale): max(floor, 1 - scale * mu)
            a = min(1.0, max(eta[0], 1.0 - eta[1] * mu) * a)
        else:                        # max(0.95, 1 - 10 mu): damped further from the path
            a = min(1.0, max(0.95, 1.0 - 10 * mu) * a)
        if split:   # separate primal (x, s) and dual (lam) step lengths
            ap = R._max_step(s, ds, np.ones_like(lam), np.zeros_like(dl))
            ad = R._max_step(np.ones_like(s), np.zeros_like(ds), lam, dl)
            f = max(eta[0], 1.0 - eta[1] * mu) if isinstance(eta, tuple) else max(0.99, 1.0 - mu)
            ap, ad = min(1.0, f * ap), min(1.0, f * ad)
            x = x + ap * dx; s = s + ap * ds; lam = lam + ad * dl
            continue
        x = x + a * dx; s = s + a * ds; lam = lam + a * dl
    return x, s, lam, maxit, 0, ncorr


SCEN = {   # name: (scenario, Hp)
    "c2": (lambda: R.circle_scenario(4, Hp=20), 20),
    "c3": (lambda: R.circle_scenario(8, Hp=30), 30),
    "hp10": (lambda: R.circle_scenario(4, Hp=10), 10),
    "hp30": (lambda: R.circle_scenario(4, Hp=30), 30),
    "frog": (lambda: R.frog_scenario(Hp=10), 10),
    "par5": (lambda: R.parallel_scenario(5, Hp=10), 10),
}


def collect(nprob, scen="c2", seed=0):
    mk, Hp = SCEN[scen]
    sc = mk()
    nv = sc.nVeh
    N = nv * Hp
    bt = BT.make_batch(sc, nprob, base_seed=seed)
    qps = []
    for b in range(nprob):
        obst = bt.obst[b] if sc.nObst else None
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=Hp, obst=obst)
        r = R.scp_solve(p, mode="structured", keep_history=True)
        lin = r.lin
        Phi0 = np.zeros((N, N)); Psi0 = np.zeros(N)
        for v in range(nv):
            Phi0[Hp * v:Hp * v + Hp, Hp * v:Hp * v + Hp] = lin.Phi0[v]
            Psi0[Hp * v:Hp * v + Hp] = lin.Psi0[v]
        for h in r.history:
            Pm, qv, G, hv = R.qp_matrices(Phi0, Psi0, h["A"], h["b"], sc.uLim)
            qps.append(R.qp_scale(Pm, qv, G, hv, sc.uLim, N) + (np.asarray(h["u_lin"], float) / sc.uLim,))
    return qps


def main():
    nprob = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    scen = sys.argv[2] if len(sys.argv) > 2 else "c2"
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    qps = collect(nprob, scen, seed)
    new = dict(init="omega-floor", floor=0.1, lam0=-0.3)     # the kernel's starting point
    new = dict(init="omega-floor", floor=0.1, lam0=-0.3)     # the kernel's starting point
    new = dict(init="omega-floor", floor=0.1, lam0=-0.3)     # the kernel's starting point
    new = dict(init="omega-floor", floor=0.1, lam0=-0.3)     # the kernel's starting point
    new = dict(init="omega-floor", floor=0.1, lam0=-0.3, eta="adaptive")   # the kernel (round 3)
    new = dict(init="omega-floor", floor=0.1, lam0=-0.3, eta="adaptive")   # the kernel (round 3)
    new = dict(init="omega-floor", floor=0.1, lam0=-0.3, eta="adaptive")   # the kernel (round 3)
    start = dict(init="omega-floor", floor=0.1, lam0=-0.3)               # ph_init_b
    kernel = dict(start, eta="adaptive")                                   # + step_factor
    start = dict(init="omega-floor", floor=0.1, lam0=-0.3)               # ph_init_b
    kernel = dict(start, eta="adaptive")                                   # + step_factor
    start = dict(init="omega-floor", floor=0.1, lam0=-0.3)               # ph_init_b
    adaptive = dict(start, eta="adaptive")                                 # + step_factor
    kernel = dict(adaptive, split=True)                                    # + split steps
    variants = [("cvxopt start, 0.99 step (round 2)", {}), ("round-3 start, 0.99 step", start),
                ("round-3 start + adaptive step", adaptive),
                ("  + split primal / dual steps (kernel)", kernel),
                ("  + 1 Gondzio corrector", dict(kernel, K=1)), ("  + sigma^2", dict(kernel, sig_pow=2)),
                ("  slack floor .05", dict(kernel, floor=0.05)), ("  lam0 .2", dict(kernel, lam0=-0.2)),
                ("  box-row lam0 10", dict(kernel, lam_box=10.0)),
                ("  start at the linearisation point", dict(kernel, init="lin")),
                ("  step max(.99, 1 - .1 mu)", dict(start, eta=(0.99, 0.1))),
                ("  step max(.995, 1 - mu)", dict(start, eta=(0.995, 1.0))),
                ("  step max(.95, 1 - 10 mu)", dict(start, eta="damped"))]
    base = None
    print(f"{len(qps)} QPs ({nprob} {scen} problems, every SCP iteration)")
    for name, kw in variants:
        its = corr = cert = worst = 0
        dz = 0.0
        for (Ps, qs, Gs, hs, sv, rn, ulin) in qps:
            if kw.get("init") == "lin":
                kw = dict(kw, ulin=ulin)
            x, s, lam, it, st, nc = ipm(Ps, qs, Gs, hs, **kw)
            its += it; corr += nc; worst = max(worst, it)
            pol = R.qp_polish_regularised(Ps, qs, Gs, hs, x, s, lam, nref=40)
            if pol is not None:
                cert += 1
                x0, s0, l0, _, _ = R.qp_ipm(Ps, qs, Gs, hs)
                ref = R.qp_polish_regularised(Ps, qs, Gs, hs, x0, s0, l0, nref=40)
                if ref is not None:
                    dz = max(dz, float(np.abs(pol[0] - ref[0]).max()))
        cost = its * C_ITER + corr * C_CORR
        base = base or cost
        print(f"{name:20s} iters/QP {its / len(qps):5.2f} (max {worst:2d})  correctors/QP "
              f"{corr / len(qps):5.2f}  certified {cert}/{len(qps)}  max|dz| {dz:.1e}  "
              f"model cycles {cost / base:5.3f}")


if __name__ == "__main__":
    main()
