"""Stage-by-stage GPU-vs-oracle probe (diagnostic; prints max errors)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd"))
import torch
from oracle import scp_reference as R
from scpqp import batch as BT
from scpqp.solver import ScpQpSolver, unpack_problem

def run(nv, hp, B, nchk, mixed=None):
    sc = R.circle_scenario(nv, Hp=hp)
    bt = BT.make_batch(sc, B, base_seed=1000, mixed_hp=mixed)
    S = ScpQpSolver(sc, max_batch=B, hp_max=bt.hp_max)
    print(f"== nv={nv} hp={hp} B={B} resources={S.resources()}", flush=True)
    hpa = bt.hp if mixed else None
    lin = S.linearize(bt.x0, bt.u0, bt.ec_noise, hp=hpa)
    errs = {}
    for b in range(nchk):
        H = int(bt.hp[b])
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=H)
        L = R.linearise(p, "faithful")
        def e(name, a, ref):
            errs[name] = max(errs.get(name, 0.0), float(np.max(np.abs(a - ref)) / max(1.0, np.max(np.abs(ref)))))
        e("Ad", lin["Ad"][b].cpu().numpy(), L.Ad)
        e("Bd", lin["Bd"][b].cpu().numpy(), L.Bd)
        e("Ed", lin["Ed"][b].cpu().numpy(), L.Ed)
        g = lin["g"][b].reshape(-1)[:nv*H*2].reshape(nv, H, 2).cpu().numpy()
        e("g", g, L.g)
        ct = lin["const_term"][b].reshape(-1)[:nv*H*2].reshape(nv, H*2).cpu().numpy()
        e("const", ct, L.const)
        ps = lin["psi0"][b].reshape(-1)[:nv*H].reshape(nv, H).cpu().numpy()
        e("psi0", ps, L.Psi0)
        rp = lin["ref_points"][b].reshape(-1)[:H*2*nv].reshape(H, 2, nv).cpu().numpy()
        e("ref", rp, p.ref_points)
    print("  linearize rel errs:", {k: f"{v:.1e}" for k, v in errs.items()}, flush=True)
    # evaluate at random u
    rng = np.random.default_rng(0)
    U = rng.uniform(-0.05, 0.05, size=(B, nv * bt.hp_max))
    ev = S.evaluate(U, bt.x0, bt.u0, bt.ec_noise, hp=hpa)
    eo = 0.0; ec = 0.0
    for b in range(nchk):
        H = int(bt.hp[b])
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=H)
        L = R.linearise(p, "faithful")
        q = R.qcqp_formulate(p, L)
        r = R.qcqp_evaluate_dense(q, U[b, :nv*H], nv, H, 0)
        eo = max(eo, abs(ev["obj"][b].item() - r.obj) / max(1, abs(r.obj)))
        cv = ev["c_veh"][b].reshape(-1)[:nv*nv*H].reshape(nv, nv, H).cpu().numpy()
        fin = np.isfinite(r.c_veh)
        ec = max(ec, float(np.max(np.abs(cv[fin] - r.c_veh[fin]))) if fin.any() else 0.0)
        assert np.all(np.isinf(cv[~fin]))
    print(f"  evaluate: obj rel {eo:.1e}  c_veh abs {ec:.1e}", flush=True)
    # one QP (max_scp=1) from cold start
    torch.cuda.synchronize()
    out1 = S.solve(bt.x0, bt.u0, bt.ec_noise, hp=hpa, max_scp_iter=1)
    torch.cuda.synchronize()
    eu = 0.0
    for b in range(nchk):
        H = int(bt.hp[b])
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=H)
        r = R.scp_solve(p, mode="structured", max_scp=1)
        u, tr = unpack_problem(out1, b, nv, H)
        eu = max(eu, float(np.max(np.abs(u.cpu().numpy() - r.u))))
    print(f"  one QP: u abs err {eu:.1e}  status {out1.status[:nchk].tolist()} nipm {out1.n_ipm[:nchk].tolist()}", flush=True)
    # full SCP
    torch.cuda.synchronize(); t = time.time()
    out = S.solve(bt.x0, bt.u0, bt.ec_noise, hp=hpa)
    torch.cuda.synchronize(); dt = time.time() - t
    eu = et = 0.0; mism = 0
    for b in range(nchk):
        H = int(bt.hp[b])
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=H)
        r = R.scp_solve(p, mode="structured")
        u, tr = unpack_problem(out, b, nv, H)
        if out.n_scp[b].item() != r.n_scp:
            mism += 1
            continue
        eu = max(eu, float(np.max(np.abs(u.cpu().numpy() - r.u))))
        et = max(et, float(np.max(np.abs(tr.cpu().numpy() - r.traj))))
    ts = []
    for _ in range(3):
        torch.cuda.synchronize(); t = time.time()
        S.solve(bt.x0, bt.u0, bt.ec_noise, hp=hpa, out=out)
        torch.cuda.synchronize(); ts.append(time.time() - t)
    dt = min(ts)
    st = out.status.cpu().numpy()
    print(f"  full SCP: u err {eu:.1e} traj err {et:.1e} nscp-mismatch {mism}/{nchk}; "
          f"status hist {np.unique(st, return_counts=True)}; nscp mean {out.n_scp.float().mean().item():.2f} "
          f"nipm mean {out.n_ipm.float().mean().item():.1f}; wall {dt*1e3:.1f} ms for B={B}", flush=True)

if __name__ == "__main__":
    run(1, 10, 4, 4)
    run(4, 20, 64, 8)
    run(4, 20, 1024, 4)
    run(4, 30, 48, 3, mixed=[10, 20, 30])
    run(8, 30, 16, 2)
