"""CPU study (verdict r05 item 5): can more IPM iterations replace the active-set polish?

For the cold QPs of c2 problems (oracle arithmetic, the kernel's IPM): run the IPM past the
kernel's 1e-9 scaled tolerance, without a polish, and record per tolerance how many QPs reach
it before the normal matrix breaks down, the extra iterations beyond 1e-9, and how far the
IPM iterate is from the polished (certified) minimiser, in rad (scaled u x u_lim).  The single-
QP parity bar is 1e-8 rad.

    python tools/ipm_nopolish_study.py [n_problems]
"""
import os
import sys

import numpy as np
import scipy.linalg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT  # noqa: E402

TOLS = [1e-9, 1e-10, 1e-11, 1e-12, 1e-13]


def ipm_trace(P, q, G, h, stop=1e-14, maxit=80):
    """The kernel's Mehrotra IPM (tools/ipm_tol_study.py's restatement) run to `stop`,
    every iterate recorded with its scaled KKT residual."""
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
        out.append((x.copy(), s.copy(), lam.copy(), res))
        if res <= stop:
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
    st = {t: [0, 0, 0.0, 0.0] for t in TOLS}   # reached, extra its, max err, sum err
    nqp, its9 = 0, 0
    for b in range(nprob):
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=20)
        r = R.scp_solve(p, mode="structured", keep_history=True)
        lin = r.lin
        Phi0 = np.zeros((80, 80)); Psi0 = np.zeros(80)
        for v in range(4):
            Phi0[20 * v:20 * v + 20, 20 * v:20 * v + 20] = lin.Phi0[v]
            Psi0[20 * v:20 * v + 20] = lin.Psi0[v]
        for hh in r.history:
            Pm, qv, G, hv = R.qp_matrices(Phi0, Psi0, hh["A"], hh["b"], sc.uLim)
            Ps, qs, Gs, hs, sv, rn = R.qp_scale(Pm, qv, G, hv, sc.uLim, 80)
            tr = ipm_trace(Ps, qs, Gs, hs)
            k9 = next((i for i, e in enumerate(tr) if e[3] <= 1e-9), None)
            if k9 is None:
                continue
            ref = R.qp_polish_regularised(Ps, qs, Gs, hs, *tr[k9][:3])
            if ref is None:
                continue
            nqp += 1
            its9 += k9
            zref = ref[0]
            for t in TOLS:
                k = next((i for i, e in enumerate(tr) if e[3] <= t), None)
                if k is None:
                    continue
                err = float(np.abs(tr[k][0][:80] - zref[:80]).max()) * sc.uLim
                a = st[t]
                a[0] += 1; a[1] += k - k9; a[2] = max(a[2], err); a[3] += err
    print(f"{nqp} cold QPs of {nprob} c2 problems; IPM iterations to 1e-9: {its9 / nqp:.2f} per QP")
    for t, (n, ex, mx, sm) in st.items():
        if n == 0:
            print(f"tol {t:7.0e}: reached by 0/{nqp}")
            continue
        print(f"tol {t:7.0e}: reached by {n}/{nqp} QPs, {ex / n:4.2f} iterations beyond 1e-9, "
              f"|u_ipm - u_polished| mean {sm / n:.1e} max {mx:.1e} rad")


if __name__ == "__main__":
    main()
