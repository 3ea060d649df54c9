"""CPU study: does scaling the slack variable omega (omega = kappa omega') change the
number of cold IPM iterations of the scaled QP?  (It does not help: DESIGN.md §3.)

    python tools/slack_scale_study.py [n_problems]
"""
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, 'senquential-convex-programming-for-trajectory-planning_amd'), HERE]
from oracle import scp_reference as R
from scpqp import batch as BT
import ipm_tol_study as S

nprob = int(sys.argv[1]) if len(sys.argv)>1 else 6
sc = R.circle_scenario(4, Hp=20)
bt = BT.make_batch(sc, nprob, base_seed=0)
kappas = [1e-5, 1e-3, 1e-2, 1e-1, 1.0, 3.0, 1e1, 1e2, 1e3]
its = {k: [] for k in kappas}; bad = {k: 0 for k in kappas}
for b in range(nprob):
    p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=20)
    r = R.scp_solve(p, mode="structured", keep_history=True)
    lin = r.lin
    Phi0 = np.zeros((80, 80)); Psi0 = np.zeros(80)
    for v in range(4):
        Phi0[20*v:20*v+20, 20*v:20*v+20] = lin.Phi0[v]; Psi0[20*v:20*v+20] = lin.Psi0[v]
    for h in r.history:
        Pm, qv, G, hv = R.qp_matrices(Phi0, Psi0, h["A"], h["b"], sc.uLim)
        for k in kappas:
            sv = np.ones(81); sv[:80] = sc.uLim; sv[80] = k
            Ps = Pm * sv[:, None] * sv[None, :]; qs = qv * sv; Gs = G * sv[None, :]
            rn = np.sqrt((Gs**2).sum(1)); rn[rn == 0] = 1
            Gs = Gs / rn[:, None]; hs = hv / rn
            tr = S.ipm_trace(Ps, qs, Gs, hs)
            its[k].append(len(tr) - 1)
            pol = R.qp_polish_regularised(Ps, qs, Gs, hs, *tr[-1][:3])
            if pol is None or np.abs(pol[0][:80]*sc.uLim - h["z"][:80]).max() > 1e-8: bad[k] += 1
for k in kappas:
    a = np.array(its[k])
    print(f"kappa {k:7.0e}: IPM its mean {a.mean():5.2f}  first-QP {a[0]}  max {a.max()}  polish mismatches {bad[k]}/{len(a)}")
