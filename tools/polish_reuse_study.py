"""CPU study (round 4): the first polish round on the IPM's own last normal matrix.

After a cold IPM converges, the polish (proximal method of multipliers on the active set
A = {lam > s}) assembles and factors K_p = P + rho I + G_A' G_A / delta.  The IPM's last
factor K = P + G' diag(d) G, d = lam / s of its last iterate, already weights the active
rows heavily.  A multiplier iteration with per-row penalties d on A,
    x+ = K^-1 (-q - G_A' y + G_A' d_A h_A + G_I' d_I G_I x),   y+ = y + d_A (G_A x+ - h_A),
has the same fixed point (the KKT point of the QP restricted to A: the inactive rows'
terms cancel at x+ = x), so it can run on the IPM's factor with no new assembly or
factorisation.  Question: how often does it certify in the first round, in how many
solves, and does it land on the same minimiser as the exact polish?

    python tools/polish_reuse_study.py [nprob]

Result (c2, 8 problems, 57 cold QPs): the first round certifies 3 of 57 and runs into the
40-solve cap on almost all of them (the weights lam / s of the IPM's last iterate are far
from a contraction for the multiplier update).  Not built.
"""
import os
import sys

import numpy as np
import scipy.linalg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT  # noqa: E402


def ipm_last_factor(P, q, G, h, tol=R.IPM_TOL, maxit=60):
    """qp_ipm(init='omega') that also returns the weights d and Cholesky factor of its
    last factorisation."""
    mc = len(h)
    x, s, lam = R.ipm_start_omega(P, q, G, h)
    qn = max(1.0, np.abs(q).max()); hn = max(1.0, np.abs(h).max())
    last = None
    for it in range(maxit):
        rd = P @ x + q + G.T @ lam
        rp = G @ x + s - h
        gap = s @ lam
        pobj = 0.5 * x @ P @ x + q @ x
        if (np.abs(rp).max() <= tol * hn and np.abs(rd).max() <= tol * qn
                and gap <= tol * max(1.0, abs(pobj))):
            return x, s, lam, it, 1, last
        mu = gap / mc
        d = lam / s
        try:
            Lc = np.linalg.cholesky(P + G.T @ (d[:, None] * G))
        except np.linalg.LinAlgError:
            return x, s, lam, it, 2, last
        last = (d.copy(), Lc)

        def solve(rc):
            dx = scipy.linalg.cho_solve((Lc, True), -rd - G.T @ (d * rp - rc / s))
            ds = -rp - G @ dx
            return dx, ds, -(rc + lam * ds) / s
        dx, ds, dl = solve(s * lam)
        a = R._max_step(s, ds, lam, dl)
        sigma = ((s + a * ds) @ (lam + a * dl) / mc / mu) ** 3
        dx, ds, dl = solve(s * lam + ds * dl - sigma * mu)
        eta = max(0.99, 1.0 - mu)
        ap = min(1.0, eta * R._max_step(s, ds, np.ones_like(lam), np.zeros_like(dl)))
        ad = min(1.0, eta * R._max_step(np.ones_like(s), np.zeros_like(ds), lam, dl))
        x = x + ap * dx; s = s + ap * ds; lam = lam + ad * dl
    return x, s, lam, maxit, 0, last


def polish_reuse(P, q, G, h, x, s, lam, last, nref=40):
    """One round of the weighted multiplier iteration on the IPM's factor; returns
    (x, lam_full, solves) if it certifies, else (None, solves)."""
    d, Lc = last
    act = lam > s
    ina = ~act
    Ga, ha, Gi = G[act], h[act], G[ina]
    da, di = d[act], d[ina]
    y = lam[act].copy()
    xk = x.copy()
    conv = False
    nsol = 0
    for k in range(nref):
        rhs = -q - Ga.T @ y + Ga.T @ (da * ha) + Gi.T @ (di * (Gi @ xk))
        xn = scipy.linalg.cho_solve((Lc, True), rhs)
        nsol += 1
        y = y + da * (Ga @ xn - ha)
        step = np.abs(xn - xk).max()
        xk = xn
        if k >= 1 and step <= R.POLISH_TOL * max(1.0, np.abs(xk).max()):
            conv = True
            break
    if not np.all(np.isfinite(xk)):
        return None, nsol
    ok, _ = R._pdas_update(G, h, act, xk, y)
    if ok and conv:
        lam_full = np.zeros_like(lam); lam_full[act] = y
        return (xk, lam_full), nsol
    return None, nsol


def main():
    nprob = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    nveh = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    hp = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    sc = R.circle_scenario(nveh, Hp=hp)
    bt = BT.make_batch(sc, nprob, base_seed=77)
    N = nveh * hp
    n_qp = n_cert = 0
    sol_reuse, sol_std, errs = [], [], []
    for b in range(nprob):
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=hp)
        r = R.scp_solve(p, mode="structured", keep_history=True)
        lin = R.linearise(p, "structured")
        Phi0 = np.zeros((N, N)); Psi0 = np.zeros(N)
        for v in range(nveh):
            Phi0[hp * v:hp * (v + 1), hp * v:hp * (v + 1)] = lin.Phi0[v]
            Psi0[hp * v:hp * (v + 1)] = lin.Psi0[v]
        for hh in r.history:
            P, q, G, h = R.qp_matrices(Phi0, Psi0, hh["A"], hh["b"], p.u_lim)
            Ps, qs, Gs, hs, sv, rn = R.qp_scale(P, q, G, h, p.u_lim, N)
            x, s, lam, it, st, last = ipm_last_factor(Ps, qs, Gs, hs)
            if last is None:
                continue
            n_qp += 1
            ref = R.qp_polish_exact(Ps, qs, Gs, hs, x, s, lam)
            pr, ns = polish_reuse(Ps, qs, Gs, hs, x, s, lam, last)
            sol_reuse.append(ns)
            if pr is not None:
                n_cert += 1
                if ref is not None:
                    errs.append(float(np.abs(pr[0] - ref[0]).max()))
    e = np.array(errs) if errs else np.array([np.nan])
    print(f"{nprob} problems ({nveh} veh, Hp {hp}), {n_qp} cold QPs: first polish round on the IPM's "
          f"factor certifies {n_cert}/{n_qp}, solves mean {np.mean(sol_reuse):.2f} max {max(sol_reuse)}, "
          f"|x - exact polish| max {np.nanmax(e):.2e}")


if __name__ == "__main__":
    main()
