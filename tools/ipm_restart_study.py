"""CPU study: the cold IPM after a failed active-set warm start (QP k >= 2 whose
previous active set does not certify), against IPM starts built from the previous
QP's solution.  The IPM is the kernel's (oracle qp_ipm init="omega": Mehrotra,
step factor max(0.99, 1 - mu), separate primal and dual steps), run from
  cold: ipm_start_omega (what the kernel does now);
  W1:   x = x_prev (omega re-derived as in the cold start), s / lam as the cold start;
  W2:   x = x_prev, s as the cold start, lam = max(lam_prev, th * lam0);
  W3:   x = x_prev, s = max(h - G x, th), lam = max(lam_prev, th).
    python tools/ipm_restart_study.py [n_problems] [th]
"""
import os
import sys

import numpy as np
import scipy.linalg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pdas_study import pdas_exact  # noqa: E402


def ipm(P, q, G, h, x, s, lam, tol=R.IPM_TOL, maxit=60):
    mc = len(h)
    qn = max(1.0, np.abs(q).max()); hn = max(1.0, np.abs(h).max())
    for it in range(maxit):
        rd = P @ x + q + G.T @ lam
        rp = G @ x + s - h
        gap = s @ lam
        pobj = 0.5 * x @ P @ x + q @ x
        if (np.abs(rp).max() <= tol * hn and np.abs(rd).max() <= tol * qn
                and gap <= tol * max(1.0, abs(pobj))):
            return it, 1, x
        mu = gap / mc
        d = lam / s
        try:
            L = np.linalg.cholesky(P + G.T @ (d[:, None] * G))
        except np.linalg.LinAlgError:
            return it, 2, x

        def solve(rc):
            dx = scipy.linalg.cho_solve((L, True), -rd - G.T @ (d * rp - rc / s))
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
    return maxit, 0, x


def start_from(P, q, G, h, xprev, lam_prev, kind, th):
    x0, s0, l0 = R.ipm_start_omega(P, q, G, h)
    N = len(q) - 1
    x = xprev.copy()
    r = G[:, :N] @ x[:N] - h
    col = G[:, N]
    coll = col[:-1] < 0
    x[N] = max(0.0, float(np.max(r[:-1][coll] / -col[:-1][coll]))) + 1.0
    sr = h - G @ x
    if kind == "W1" or kind == "W2":
        s = sr + max(-1.5 * sr.min(), 0.0)
        s = np.maximum(s, 0.1 * max(1.0, s.max()))
        lam = l0 if kind == "W1" else np.maximum(lam_prev, th * l0)
    else:
        s = np.maximum(sr, th)
        lam = np.maximum(lam_prev, th)
    return x, s, lam


def main():
    nprob = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    th = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
    sc = R.circle_scenario(4, Hp=20)
    bt = BT.make_batch(sc, nprob, base_seed=0)
    N = 80
    res = {k: [] for k in ("cold", "W1", "W2", "W3")}
    for b in range(nprob):
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=20)
        r = R.scp_solve(p, mode="structured", keep_history=True)
        lin = r.lin
        Phi0 = np.zeros((N, N)); Psi0 = np.zeros(N)
        for v in range(4):
            Phi0[20 * v:20 * v + 20, 20 * v:20 * v + 20] = lin.Phi0[v]
            Psi0[20 * v:20 * v + 20] = lin.Psi0[v]
        prev = None
        for k, hk in enumerate(r.history):
            P, q, G, h = R.qp_matrices(Phi0, Psi0, hk["A"], hk["b"], p.u_lim)
            Ps, qs, Gs, hs, sv, rn = R.qp_scale(P, q, G, h, p.u_lim, N)
            xs = hk["z"] / sv
            # the QP's own multipliers (exact polish on its active set)
            act = Gs @ xs - hs >= -1e-7
            _, xchk = pdas_exact(Ps, qs, Gs, hs, act.copy())
            if prev is not None and k >= 2:
                xprev, aprev, lprev = prev
                rp, _ = pdas_exact(Ps, qs, Gs, hs, aprev.copy(), cap=8)
                if rp < 0:    # the warm start fails: the kernel runs the cold IPM
                    for kind in res:
                        if kind == "cold":
                            x, s, lam = R.ipm_start_omega(Ps, qs, Gs, hs)
                        else:
                            x, s, lam = start_from(Ps, qs, Gs, hs, xprev, lprev, kind, th)
                        it, st, xf = ipm(Ps, qs, Gs, hs, x, s, lam)
                        res[kind].append((it, st, float(np.abs(xf - xs).max())))
            # multipliers of this QP on the scaled rows (least squares on the active rows)
            Ga = Gs[act]
            lam_a = np.linalg.lstsq(Ga.T, -(Ps @ xs + qs), rcond=None)[0] if act.any() else np.zeros(0)
            lam_full = np.zeros(len(hs)); lam_full[act] = np.maximum(lam_a, 0.0)
            prev = (xs, act, lam_full)
    for kind, v in res.items():
        a = np.array(v)
        if len(a):
            print(f"{kind:5s}: {len(a)} failed-warm QPs, IPM iterations mean {a[:, 0].mean():.2f} "
                  f"max {a[:, 0].max():.0f}, converged {np.mean(a[:, 1] == 1):.2f}, "
                  f"max |x - x*| {a[:, 2].max():.1e}")


if __name__ == "__main__":
    main()
