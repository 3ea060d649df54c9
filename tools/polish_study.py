"""CPU study of the active-set polish cost on c2 problems (oracle arithmetic).

For every convexified QP of a few c2 problems: cold IPM + regularised polish
(what the kernel runs after a failed warm start) and the warm polish from the
previous QP's certified active set.  Prints solves per round / QP for a set of
(delta, tol) choices so the kernel's polish parameters can be picked on the CPU.

    python tools/polish_study.py [n_problems] [delta ...]
"""
import os
import sys

import numpy as np
import scipy.linalg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT  # noqa: E402


def polish(P, q, G, h, act, y_all, x, delta, rho=1e-12, nref=40, rounds=6, tol=1e-10, early=0.0, why=None,
           stall=False):
    """Mirror of qp_polish_regularised from an explicit active set; returns
    (x, lam, n_solves, n_rounds) or (None, ..)."""
    xk = x.copy()
    L = None
    solves = 0
    extended = False
    prev_chg = 1 << 30
    for rnd in range(rounds):
        Ga, ha = G[act], h[act]
        y = y_all[act].copy()
        if L is None:
            L = np.linalg.cholesky(P + rho * np.eye(len(q)) + Ga.T @ Ga / delta)
        conv = False
        for k in range(nref):
            xn = scipy.linalg.cho_solve((L, True), -q - Ga.T @ y + Ga.T @ ha / delta + rho * xk)
            solves += 1
            y = y + (Ga @ xn - ha) / delta
            step = np.abs(xn - xk).max()
            xk = xn
            if k >= 1 and step <= tol * max(1.0, np.abs(xk).max()):
                conv = True
                break
            if early > 0 and k >= 1:
                r = Ga @ xk - ha
                rall = G @ xk - h
                if (rall[~act] > early).any() or (y < -early).any():
                    break
        ok, nxt = R._pdas_update(G, h, act, xk, y)
        if ok and conv:
            lam = np.zeros(len(h)); lam[act] = y
            return xk, lam, solves, rnd + 1
        y_all = np.zeros(len(h)); y_all[act] = y
        if np.array_equal(nxt, act):
            if conv or extended:
                if why is not None: why.append('stuck')
                return None, None, solves, rnd + 1
            extended = True
            continue
        y_all[~nxt] = 0.0
        nchg = int((nxt != act).sum())
        if stall and rnd >= 1 and nchg >= prev_chg:
            if why is not None: why.append('stall')
            return None, None, solves, rnd + 1
        prev_chg = nchg
        act = nxt
        L = None
    if why is not None: why.append('rounds')
    return None, None, solves, rounds


def main():
    nprob = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    deltas = [3e-7]
    global NREF, ROUNDS, EARLY, WHY
    NREF, ROUNDS, EARLY = int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
    global STALL; STALL = os.environ.get("STALL") == "1"
    WHY = []
    global TRACE; TRACE = []
    global WROUNDS; WROUNDS = []
    global COARSE, CTOLS; COARSE = {}; CTOLS = [1e-3, 1e-4, 1e-5, 1e-6, 1e-7]
    sc = R.circle_scenario(4, Hp=20)
    bt = BT.make_batch(sc, nprob, base_seed=1234)
    pick = os.environ.get("PROBLEMS")      # e.g. "1008,958": problems of the c2 bench batch
    if pick:
        idx = np.array([int(i) for i in pick.split(",")])
        bt = BT.make_batch(sc, int(idx.max()) + 1, base_seed=0).slice(0, int(idx.max()) + 1)
        bt = type(bt)(bt.x0[idx], bt.u0[idx], bt.ec_noise[idx], bt.hp[idx], bt.obst[idx], bt.hp_max,
                      bt.seeds[idx])
        nprob = len(idx)
    for delta in deltas:
        cold_s, warm_s, warm_ok, nqp, cold_r, warm_r, err = [], [], 0, 0, [], [], 0.0
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
                act = lam > s
                xc, lc, ns, nr = polish(Ps, qs, Gs, hs, act, np.where(act, lam, 0.0), x, delta)
                for ctol in CTOLS:
                    x2, s2, l2, it2, st2 = R.qp_ipm(Ps, qs, Gs, hs, tol=ctol)
                    a2 = l2 > s2
                    xq, lq, nsq, nrq = polish(Ps, qs, Gs, hs, a2, np.where(a2, l2, 0.0), x2, delta, rounds=8)
                    COARSE.setdefault(ctol, []).append((it, it2, xq is not None, nsq, nrq))
                cold_s.append(ns); cold_r.append(nr)
                nqp += 1
                if xc is not None:
                    err = max(err, np.abs(xc * sv - hh["z"]).max())
                if prev is not None:
                    pact, plam, px = prev
                    xw, lw, nsw, nrw = polish(Ps, qs, Gs, hs, pact, plam, px, delta, nref=NREF, rounds=ROUNDS, early=EARLY, why=WHY, stall=STALL)
                    warm_s.append(nsw); warm_r.append(nrw)
                    WROUNDS.append((nrw, xw is not None))
                    warm_ok += xw is not None
                    TRACE.append((b, ih, len(r.history), xw is not None, nsw, int(pact.sum()), int((lc > 0).sum()) if xc is not None else -1, int((pact != (lc > 0)).sum()) if xc is not None else -1))
                prev = (lc > 0, lc, xc) if xc is not None else None
        print(f"delta {delta:.1e}: {nqp} QPs  cold polish solves mean {np.mean(cold_s):.2f} "
              f"(max {max(cold_s)}) rounds {np.mean(cold_r):.2f} | warm solves mean "
              f"{np.mean(warm_s):.2f} rounds {np.mean(warm_r):.2f} ok {warm_ok}/{len(warm_s)} "
              f"| max |z - z_exact| {err:.1e}")
        import collections; print('   warm failures', collections.Counter(WHY)); print('   warm solves hist', collections.Counter(warm_s))
        for ct, v in COARSE.items():
            v = np.array(v, float)
            print(f'   ipm tol {ct:.0e}: ipm its {v[:,1].mean():.2f} (full {v[:,0].mean():.2f}) polish ok {int(v[:,2].sum())}/{len(v)} solves {v[:,3].mean():.2f} rounds {v[:,4].mean():.2f} max rounds {v[:,4].max():.0f}')
        wr = np.array(WROUNDS, float)
        print(f"   warm rounds total {wr[:, 0].sum():.0f}  (successful attempts {wr[wr[:, 1] == 1, 0].sum():.0f}, failed {wr[wr[:, 1] == 0, 0].sum():.0f})")
        import collections
        agg = collections.defaultdict(lambda: [0, 0, 0])
        for t in TRACE:
            a = agg[min(t[1], 5)]; a[0] += 1; a[1] += int(t[3]); a[2] += t[4]
        for k in sorted(agg):
            a = agg[k]; print(f'   qp index {k}{"+" if k == 5 else ""}: warm ok {a[1]}/{a[0]}  solves/attempt {a[2] / a[0]:.1f}')
        hist = np.bincount(cold_s)
        print("   cold solves histogram", {i: int(c) for i, c in enumerate(hist) if c})


if __name__ == "__main__":
    main()
