"""CPU study: how far is each SCP iteration's QP from the previous one's active set?

For c2 problems, the exact oracle SCP loop is replayed QP by QP.  For every QP k >= 1
(scaled form, qp_scale), the exact primal-dual active-set method (direct KKT solve per
round, oracle _pdas_update) is started from
  prev: the previous QP's certified active set (what the kernel's warm start uses),
  pred: the rows active or violated at the previous solution under the new rows
        (G_k x_{k-1} - h_k >= -tau),
and the rounds to certification are counted (cap 20), next to the cold IPM's count
(the kernel's start, oracle qp_ipm init="omega").
    python tools/pdas_study.py [n_problems] [tau]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT  # noqa: E402


def pdas_exact(P, q, G, h, act, cap=20):
    n = len(q)
    for rnd in range(cap):
        Ga, ha = G[act], h[act]
        na = int(act.sum())
        K = np.zeros((n + na, n + na))
        K[:n, :n] = P
        K[:n, n:] = Ga.T
        K[n:, :n] = Ga
        sol = np.linalg.lstsq(K, np.concatenate([-q, ha]), rcond=None)[0]
        xp, la = sol[:n], sol[n:]
        ok, nxt = R._pdas_update(G, h, act, xp, la)
        if ok:
            return rnd + 1, xp
        if np.array_equal(nxt, act):
            return -(rnd + 1), xp
        act = nxt
    return -cap, None


def main():
    nprob = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    tau = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-6
    sc = R.circle_scenario(4, Hp=20)
    bt = BT.make_batch(sc, nprob, base_seed=0)
    N = 80
    rows = []
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
            x, s, lam, it, st = R.qp_ipm(Ps, qs, Gs, hs, init="omega")
            xs = hk["z"] / sv
            act = Gs @ xs - hs >= -1e-7
            if prev is not None:
                xprev, aprev = prev
                r_prev, _ = pdas_exact(Ps, qs, Gs, hs, aprev.copy())
                pred = Gs @ xprev - hs >= -tau
                r_pred, _ = pdas_exact(Ps, qs, Gs, hs, pred)
                diff = int((act != aprev).sum())
                rows.append((b, k, it, int(act.sum()), diff, r_prev, r_pred))
            prev = (xs, act)
    print(" prob qp cold_ipm |A| |A^A_prev| pdas(prev) pdas(pred)   (negative: stuck / cap)")
    for rw in rows:
        print(" %4d %2d %8d %3d %10d %10d %10d" % rw)
    a = np.array([rw[2:] for rw in rows], float)
    for k in (1, 2, 3):
        m = np.array([rw[1] == k for rw in rows])
        if m.any():
            sub = a[m]
            print(f"QP{k}: cold IPM {sub[:, 0].mean():.2f}; pdas(prev) certified {np.mean(sub[:, 3] > 0):.2f} "
                  f"mean rounds {sub[sub[:, 3] > 0, 3].mean() if (sub[:, 3] > 0).any() else 0:.2f}; "
                  f"pdas(pred) certified {np.mean(sub[:, 4] > 0):.2f} mean rounds "
                  f"{sub[sub[:, 4] > 0, 4].mean() if (sub[:, 4] > 0).any() else 0:.2f}")


if __name__ == "__main__":
    main()
