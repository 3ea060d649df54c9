"""CPU study: how early can the cold IPM hand over to the active-set polish?

For the cold QPs of c2 problems (oracle arithmetic, the kernel's algorithm):
IPM iterations needed to reach scaled tolerance `tol`, and whether the
regularised polish from that point certifies the same minimiser as from the
1e-9 point.  Also an active-set-stability stop: hand over once {lam > s} is
unchanged for `k` consecutive iterations and the gap is below `gtol`.

    python tools/ipm_tol_study.py [n_problems]
"""
import os
import sys

import numpy as np
import scipy.linalg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT  # noqa: E402


def ipm_trace(P, q, G, h, maxit=60):
    """qp_ipm with the per-iteration (x, s, lam, scaled residuals) recorded."""
    mc = len(h)
    x = np.linalg.solve(P + G.T @ G, -q + G.T @ h)
    s = h - G @ x
    lam = -s.copy()
    ts = -s.min()
    if ts >= -1e-8 * max(np.linalg.norm(s), 1.0):
        s = s + (1 + ts)
    tz = -lam.min()
    if tz >= -1e-8 * max(np.linalg.norm(lam), 1.0):
        lam = lam + (1 + tz)
    qn = max(1.0, np.abs(q).max()); hn = max(1.0, np.abs(h).max())
    out = []
    for it in range(maxit):
        rd = P @ x + q + G.T @ lam
        rp = G @ x + s - h
        gap = s @ lam
        pobj = 0.5 * x @ P @ x + q @ x
        res = max(np.abs(rp).max() / hn, np.abs(rd).max() / qn, gap / max(1.0, abs(pobj)))
        out.append((x.copy(), s.copy(), lam.copy(), res, gap / mc))
        if res <= 1e-9:
            break
        mu = gap / mc
        d = lam / s
        try:
            L = np.linalg.cholesky(P + G.T @ (d[:, None] * G))
        except np.linalg.LinAlgError:
            break

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
    return out


def main():
    nprob = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    sc = R.circle_scenario(4, Hp=20)
    bt = BT.make_batch(sc, nprob, base_seed=0)
    tols = [1e-9, 1e-7, 1e-6, 1e-5, 1e-4, 1e-3]
    stats = {t: [0, 0, 0, 0.0] for t in tols}          # iters, certified, total, max dz
    stab = {k: [0, 0, 0, 0.0] for k in (2, 3)}
    nqp = 0
    for b in range(nprob):
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=20)
        r = R.scp_solve(p, mode="structured", keep_history=True)
        lin = r.lin
        Phi0 = np.zeros((80, 80)); Psi0 = np.zeros(80)
        for v in range(4):
            Phi0[20 * v:20 * v + 20, 20 * v:20 * v + 20] = lin.Phi0[v]
            Psi0[20 * v:20 * v + 20] = lin.Psi0[v]
        for h in r.history:
            Pm, qv, G, hv = R.qp_matrices(Phi0, Psi0, h["A"], h["b"], sc.uLim)
            Ps, qs, Gs, hs, sv, rn = R.qp_scale(Pm, qv, G, hv, sc.uLim, 80)
            tr = ipm_trace(Ps, qs, Gs, hs)
            ref = R.qp_polish_regularised(Ps, qs, Gs, hs, *tr[-1][:3])
            if ref is None:
                continue
            nqp += 1
            zref = ref[0]
            for t in tols:
                k = next((i for i, e in enumerate(tr) if e[3] <= t), len(tr) - 1)
                pol = R.qp_polish_regularised(Ps, qs, Gs, hs, *tr[k][:3])
                st = stats[t]
                st[0] += k; st[2] += 1
                if pol is not None:
                    st[1] += 1
                    st[3] = max(st[3], float(np.abs(pol[0] - zref).max()))
            for kk in stab:
                acts = [e[2] > e[1] for e in tr]
                j = next((i for i in range(kk, len(tr)) if all(np.array_equal(acts[i], acts[i - d])
                                                                for d in range(1, kk + 1))
                          and tr[i][4] < 1e-3), len(tr) - 1)
                pol = R.qp_polish_regularised(Ps, qs, Gs, hs, *tr[j][:3])
                st = stab[kk]
                st[0] += j; st[2] += 1
                if pol is not None:
                    st[1] += 1
                    st[3] = max(st[3], float(np.abs(pol[0] - zref).max()))
    print(f"{nqp} QPs (cold IPM from every SCP iteration of {nprob} c2 problems)")
    for t, (it, ok, n, dz) in stats.items():
        print(f"tol {t:7.0e}: mean IPM iters {it / n:5.2f}  polish certified {ok}/{n}  max|dz| {dz:.1e}")
    for k, (it, ok, n, dz) in stab.items():
        print(f"active set stable {k} its (mu<1e-3): mean IPM iters {it / n:5.2f}  certified {ok}/{n}  max|dz| {dz:.1e}")


if __name__ == "__main__":
    main()
