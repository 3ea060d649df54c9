"""CPU study: IPM iterations from the CVXOPT cold start vs a shifted warm start
from the previous SCP iteration's QP solution (x, s, lam), on c2 problems."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT  # noqa: E402


def ipm_from(P, q, G, h, x, s, lam, tol=1e-9, maxit=60):
    mc = len(h)
    qn = max(1.0, np.abs(q).max()); hn = max(1.0, np.abs(h).max())
    import scipy.linalg
    for it in range(maxit):
        rd = P @ x + q + G.T @ lam
        rp = G @ x + s - h
        gap = s @ lam
        pobj = 0.5 * x @ P @ x + q @ x
        if (np.abs(rp).max() <= tol * hn and np.abs(rd).max() <= tol * qn
                and gap <= tol * max(1.0, abs(pobj))):
            return x, s, lam, it, 1
        mu = gap / mc
        d = lam / s
        try:
            L = np.linalg.cholesky(P + G.T @ (d[:, None] * G))
        except np.linalg.LinAlgError:
            return x, s, lam, it, 2

        def solve(rc):
            dx = scipy.linalg.cho_solve((L, True), -rd - G.T @ (d * rp - rc / s))
            ds = -rp - G @ dx
            return dx, ds, -(rc + lam * ds) / s
        dx, ds, dl = solve(s * lam)
        a = R._max_step(s, ds, lam, dl)
        sigma = ((s + a * ds) @ (lam + a * dl) / mc / mu) ** 3
        dx, ds, dl = solve(s * lam + ds * dl - sigma * mu)
        a = min(1.0, 0.99 * R._max_step(s, ds, lam, dl))
        x = x + a * dx; s = s + a * ds; lam = lam + a * dl
    return x, s, lam, maxit, 0


def main():
    nprob = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    thetas = [float(t) for t in sys.argv[2:]] or [1e-1, 1e-2, 1e-3]
    sc = R.circle_scenario(4, Hp=20)
    bt = BT.make_batch(sc, nprob, base_seed=1234)
    res = {t: [] for t in thetas}
    cold = []
    for b in range(nprob):
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=20)
        r = R.scp_solve(p, mode="structured", keep_history=True)
        lin = R.linearise(p, "structured")
        N = 80
        Phi0 = np.zeros((N, N)); Psi0 = np.zeros(N)
        for v in range(4):
            Phi0[20 * v:20 * v + 20, 20 * v:20 * v + 20] = lin.Phi0[v]
            Psi0[20 * v:20 * v + 20] = lin.Psi0[v]
        prev = None
        for ih, hh in enumerate(r.history):
            P, q, G, h = R.qp_matrices(Phi0, Psi0, hh["A"], hh["b"], p.u_lim)
            Ps, qs, Gs, hs, sv, rn = R.qp_scale(P, q, G, h, p.u_lim, N)
            x, s, lam, it, st = R.qp_ipm(Ps, qs, Gs, hs)
            pol = R.qp_polish_exact(Ps, qs, Gs, hs, x, s, lam)
            cold.append(it)
            if prev is not None:
                xp, lp = prev
                for t in thetas:
                    s0 = np.maximum(hs - Gs @ xp, t)
                    l0 = np.maximum(lp, t)
                    xw, sw, lw, itw, stw = ipm_from(Ps, qs, Gs, hs, xp.copy(), s0, l0)
                    polw = R.qp_polish_exact(Ps, qs, Gs, hs, xw, sw, lw)
                    ok = polw is not None and pol is not None and np.abs(polw[0] - pol[0]).max() < 1e-8
                    res[t].append((ih, it, itw, ok))
            prev = (pol[0], pol[1]) if pol is not None else (x, lam)
    print(f"cold IPM iterations: mean {np.mean(cold):.2f}")
    for t in thetas:
        a = np.array(res[t], float)
        print(f"theta {t:.0e}: warm IPM its mean {a[:, 2].mean():.2f} (cold on same QPs {a[:, 1].mean():.2f}) "
              f"polish same answer {int(a[:, 3].sum())}/{len(a)}")
        for k in (1, 2, 3):
            sel = a[:, 0] == k if k < 3 else a[:, 0] >= 3
            print(f"    qp index {k}{'+' if k == 3 else ''}: warm {a[sel, 2].mean():.2f} cold {a[sel, 1].mean():.2f}")


if __name__ == "__main__":
    main()
