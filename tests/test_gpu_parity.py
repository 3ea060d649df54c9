"""GPU parity: the HIP kernels (through the C-ABI) against the CPU restatement
and the committed golden fixtures.

Tolerances (SURVEY.md §8d, fp64 throughout):
  * stage intermediates (Ad, Bd, Ed, g_m, const_term, Psi_0): 1e-12 relative;
  * one QP from the same linearisation point: |u| <= 1e-8 rad;
  * end-to-end on problems with equal SCP iteration count: |Traj| <= 1e-6 m,
    |U| <= 1e-7 rad; a problem whose SCP count differs is compared iteration by
    iteration (device trace vs oracle history) up to the shorter count, and its
    stop flip must straddle the threshold (tests/scp_parity.py) — none is skipped;
  * integer outputs (n_scp, status, feasibility) exact where the iterates agree.
"""
import multiprocessing as mp
import os

import numpy as np
import pytest
import torch

from oracle import scp_reference as R
from scpqp import _lib as LB
from scpqp import batch as BT
from scpqp.solver import ScpQpSolver, unpack_problem

import scp_parity as SP

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BUILDERS = {
    "c1_circle1_hp10": lambda: R.circle_scenario(1, Hp=10),
    "c2_circle4_hp20": lambda: R.circle_scenario(4, Hp=20),
    "c3_circle8_hp30": lambda: R.circle_scenario(8, Hp=30),
    "c5_circle4_mixed": lambda: R.circle_scenario(4, Hp=30),
    "frog_hp10": lambda: R.frog_scenario(Hp=10),
    "parallel5_hp10": lambda: R.parallel_scenario(5, Hp=10),
}
TRAJ_TOL = 1e-6
U_TOL = 1e-7
QP_TOL = 1e-8


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b))))


def oracle_problem(sc, bt, b):
    H = int(bt.hp[b])
    ob = bt.obst[b].reshape(-1)[:sc.nObst * 2 * H].reshape(sc.nObst, 2, H)
    return R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=H, obst=ob), H


def cases():
    return {
        "c2": (R.circle_scenario(4, Hp=20), dict()),
        "c5_mixed": (R.circle_scenario(4, Hp=30), dict(mixed_hp=(10, 20, 30))),
        "frog": (R.frog_scenario(Hp=10), dict()),
        "parallel5": (R.parallel_scenario(5, Hp=10), dict()),
        # mixed horizons WITH obstacles: the obstacle slot [nObst][2][hp_b] is read packed
        # inside the hp_max slot (SCP_controller.py:106-114, MPC_Iter.py:45-51)
        "frog_mixed": (R.frog_scenario(Hp=20), dict(mixed_hp=(10, 15, 20))),
        "parallel5_mixed": (R.parallel_scenario(5, Hp=14), dict(mixed_hp=(6, 10, 14))),
    }


ALL_CASES = ["c2", "c5_mixed", "frog", "parallel5", "frog_mixed", "parallel5_mixed"]


@pytest.mark.parametrize("case", ALL_CASES)
def test_linearize_parity(gpu, case):
    sc, kw = cases()[case]
    bt = BT.make_batch(sc, 12, base_seed=101, **kw)
    S = ScpQpSolver(sc, max_batch=12, hp_max=bt.hp_max)
    lin = S.linearize(bt.x0, bt.u0, bt.ec_noise, hp=bt.hp, obst=bt.obst)
    nV = sc.nVeh
    for b in range(12):
        p, H = oracle_problem(sc, bt, b)
        L = R.linearise(p, "faithful")
        assert rel(lin["Ad"][b].cpu().numpy(), L.Ad) <= 1e-12
        assert rel(lin["Bd"][b].cpu().numpy(), L.Bd) <= 1e-12
        assert np.max(np.abs(lin["Ed"][b].cpu().numpy() - L.Ed)) <= 1e-12
        g = lin["g"][b].reshape(-1)[:nV * H * 2].reshape(nV, H, 2).cpu().numpy()
        assert rel(g, L.g) <= 1e-12
        ct = lin["const_term"][b].reshape(-1)[:nV * H * 2].reshape(nV, 2 * H).cpu().numpy()
        assert rel(ct, L.const) <= 1e-12
        ps = lin["psi0"][b].reshape(-1)[:nV * H].reshape(nV, H).cpu().numpy()
        assert rel(ps, L.Psi0) <= 1e-10
        rp = lin["ref_points"][b].reshape(-1)[:H * 2 * nV].reshape(H, 2, nV).cpu().numpy()
        assert np.max(np.abs(rp - p.ref_points)) <= 1e-12
    S.close()


@pytest.mark.parametrize("case", ALL_CASES)
@pytest.mark.parametrize("quirk", [True, False])
def test_evaluate_parity(gpu, case, quirk):
    sc, kw = cases()[case]
    B = 8
    bt = BT.make_batch(sc, B, base_seed=202, **kw)
    S = ScpQpSolver(sc, max_batch=B, hp_max=bt.hp_max, obstacle_quirk=quirk)
    nV, nO = sc.nVeh, sc.nObst
    g = np.random.default_rng(0)
    U = g.uniform(-sc.uLim, sc.uLim, (B, nV * bt.hp_max))
    ev = S.evaluate(U, bt.x0, bt.u0, bt.ec_noise, hp=bt.hp, obst=bt.obst)
    for b in range(B):
        p, H = oracle_problem(sc, bt, b)
        L = R.linearise(p, "structured")
        r = R.evaluate_structured(p, L, U[b, :nV * H], obst_quirk=quirk)
        assert ev["obj"][b].item() == pytest.approx(r.obj, rel=1e-12)
        assert ev["max_violation"][b].item() == pytest.approx(r.max_violation, rel=1e-10, abs=1e-12)
        assert ev["sum_violations"][b].item() == pytest.approx(r.sum_violations, rel=1e-10, abs=1e-12)
        assert bool(ev["feasible"][b].item()) == r.feasible
        cv = ev["c_veh"][b].reshape(-1)[:nV * nV * H].reshape(nV, nV, H).cpu().numpy()
        fin = np.isfinite(r.c_veh)
        assert np.array_equal(np.isfinite(cv), fin)
        if fin.any():
            assert np.max(np.abs(cv[fin] - r.c_veh[fin])) <= 1e-10
        if nO:
            co = ev["c_obs"][b].reshape(-1)[:nV * nO * H].reshape(nV, nO, H).cpu().numpy()
            fin = np.isfinite(r.c_obs)
            assert np.array_equal(np.isfinite(co), fin)
            if fin.any():
                assert np.max(np.abs(co[fin] - r.c_obs[fin])) <= 1e-10
        tr = ev["traj"][b].reshape(-1)[:H * 2 * nV].reshape(H, 2, nV).cpu().numpy()
        tro, _ = R.forward_u(L, U[b, :nV * H], nV, H)
        assert np.max(np.abs(tr - tro)) <= 1e-12 * 30
    S.close()


@pytest.mark.parametrize("case", ALL_CASES)
def test_single_qp_parity(gpu, case):
    sc, kw = cases()[case]
    B = 32
    bt = BT.make_batch(sc, B, base_seed=303, **kw)
    S = ScpQpSolver(sc, max_batch=B, hp_max=bt.hp_max)
    out = S.solve(bt.x0, bt.u0, bt.ec_noise, hp=bt.hp, obst=bt.obst, max_scp_iter=1)
    torch.cuda.synchronize()
    for b in range(0, B, 4):
        p, H = oracle_problem(sc, bt, b)
        r = R.scp_solve(p, mode="structured", max_scp=1)
        u, _ = unpack_problem(out, b, sc.nVeh, H)
        assert np.max(np.abs(u.cpu().numpy() - r.u)) <= QP_TOL
    S.close()


@pytest.mark.parametrize("name", sorted(BUILDERS))
def test_solve_matches_golden(gpu, name):
    f = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    sc = BUILDERS[name]()
    nV = sc.nVeh
    B = f["x0"].shape[0]
    S = ScpQpSolver(sc, max_batch=B, hp_max=int(f["hp_max"]))
    obst = f["obst"] if sc.nObst else None
    out = S.solve(f["x0"], f["u0"], f["ec_noise"], hp=f["hp"], obst=obst, trace=True)
    ref = S.sample_reference(f["x0"], hp=f["hp"])
    torch.cuda.synchronize()
    for b in range(B):
        H = int(f["hp"][b])
        rp = ref[b].reshape(-1)[:H * 2 * nV].cpu().numpy()
        assert np.max(np.abs(rp - f["ref_points"][b, :H * 2 * nV])) <= 1e-12
        if out.n_scp[b].item() != f["n_scp"][b]:
            # stop flip: per-iteration comparison against the oracle's history
            ob = f["obst"][b].reshape(-1)[:sc.nObst * 2 * H].reshape(sc.nObst, 2, H)
            p = R.make_problem(sc, f["x0"][b], f["u0"][b], f["ec_noise"][b], Hp=H, obst=ob)
            r = R.scp_solve(p, mode="structured", keep_history=True)
            u, tr = unpack_problem(out, b, nV, H)
            SP.compare(u.cpu().numpy(), tr.cpu().numpy(), int(out.n_scp[b].item()),
                       SP.device_trace(out, b, nV, sc.nObst, H, S.hp_max), r, nV, H,
                       what=f"{name}[{b}]")
            continue
        u, tr = unpack_problem(out, b, nV, H)
        assert np.max(np.abs(u.cpu().numpy() - f["u"][b, :nV * H])) <= U_TOL
        assert np.max(np.abs(tr.cpu().numpy().reshape(-1) - f["traj"][b, :H * 2 * nV])) <= TRAJ_TOL
        assert bool(out.feasible[b].item()) == bool(f["feasible"][b])
        assert out.obj[b].item() == pytest.approx(float(f["obj"][b]), rel=1e-8, abs=1e-6)
    S.close()


def test_c2_full_batch_properties_and_sample_parity(gpu):
    """BASELINE c2 at full size: 1024 problems in one launch.  Size-independent
    properties on all problems; oracle parity on a sample."""
    sc = R.circle_scenario(4, Hp=20)
    B = 1024
    bt = BT.make_batch(sc, B, base_seed=0)
    S = ScpQpSolver(sc, max_batch=B)
    out = S.solve(bt.x0, bt.u0, bt.ec_noise, trace=True)
    torch.cuda.synchronize()
    u = out.u.cpu().numpy()
    st = out.status.cpu().numpy()
    n_scp = out.n_scp.cpu().numpy()
    assert np.all(np.isfinite(u))
    assert np.all(np.abs(u) <= sc.uLim * (1 + 1e-9))
    assert np.all((n_scp >= 1) & (n_scp <= 20))
    assert np.mean((st & 0xff) == LB.ST_CONVERGED) >= 0.99
    # forward_U consistency: the evaluator on the returned u reproduces traj / obj / maxviol
    ev = S.evaluate(out.u, bt.x0, bt.u0, bt.ec_noise)
    assert torch.max(torch.abs(ev["traj"] - out.traj)).item() <= 1e-12 * 30
    assert torch.allclose(ev["obj"], out.obj, rtol=1e-12, atol=0)
    assert torch.equal(ev["feasible"], out.feasible)
    # oracle parity on a deterministic sample of 128 (every 8th problem): every sampled
    # problem compared, per iteration where the SCP counts differ
    idx = list(range(0, B, 8))
    jobs = [(4, 20, bt.x0[b], bt.u0[b], bt.ec_noise[b]) for b in idx]
    with mp.get_context("spawn").Pool(16) as pool:
        res = pool.map(SP.oracle_job, jobs)
    for b, r in zip(idx, res):
        H = 20
        ub, tb = unpack_problem(out, b, 4, H)
        SP.compare(ub.cpu().numpy(), tb.cpu().numpy(), int(n_scp[b]),
                   SP.device_trace(out, b, 4, 0, H, 20), r, 4, H, what=f"c2[{b}]")
    S.close()


def test_batch_invariance_and_determinism(gpu):
    sc = R.circle_scenario(4, Hp=20)
    B = 96
    bt = BT.make_batch(sc, B, base_seed=9)
    S = ScpQpSolver(sc, max_batch=B)
    a = S.solve(bt.x0, bt.u0, bt.ec_noise)
    ua = a.u.clone()
    b_ = S.solve(bt.x0, bt.u0, bt.ec_noise)
    torch.cuda.synchronize()
    assert torch.equal(ua, b_.u) and torch.equal(a.n_ipm, b_.n_ipm)
    sub = bt.slice(37, 41)
    c = S.solve(sub.x0, sub.u0, sub.ec_noise)
    torch.cuda.synchronize()
    assert torch.equal(c.u, ua[37:41])
    S.close()


def test_warm_start_and_eps_nudge(gpu):
    sc = R.circle_scenario(4, Hp=20)
    B = 8
    bt = BT.make_batch(sc, B, base_seed=21)
    S = ScpQpSolver(sc, max_batch=B)
    cold = S.solve(bt.x0, bt.u0, bt.ec_noise)
    uw = cold.u.clone()
    warm = S.solve(bt.x0, bt.u0, bt.ec_noise, u_warm=uw, trace=True)
    torch.cuda.synchronize()
    for b in range(B):
        p, H = oracle_problem(sc, bt, b)
        r = R.scp_solve(p, u_warm=uw[b].cpu().numpy(), mode="structured", keep_history=True)
        ub, tb = unpack_problem(warm, b, 4, H)
        SP.compare(ub.cpu().numpy(), tb.cpu().numpy(), int(warm.n_scp[b].item()),
                   SP.device_trace(warm, b, 4, 0, H, 20), r, 4, H, what=f"warm[{b}]")
    assert warm.n_scp.float().mean().item() <= cold.n_scp.float().mean().item()
    S.close()


def test_edge_cases(gpu):
    sc = R.circle_scenario(4, Hp=20)
    S = ScpQpSolver(sc, max_batch=4)
    bt = BT.make_batch(sc, 4, base_seed=1)
    # empty batch: no launch, no error
    S.solve(bt.x0[:0], bt.u0[:0], bt.ec_noise[:0])
    # too large a batch: API error, nothing launched
    big = BT.make_batch(sc, 5, base_seed=1)
    with pytest.raises(ValueError):
        S.solve(big.x0, big.u0, big.ec_noise)
    # a horizon outside [1, hp_max] is reported per problem, never used for indexing
    bad = S.solve(bt.x0, bt.u0, bt.ec_noise, hp=np.array([20, 21, 0, 20], np.int32))
    torch.cuda.synchronize()
    assert bad.status.cpu().tolist()[1:3] == [LB.ST_INVALID, LB.ST_INVALID]
    assert (bad.status[0].item() & 0xff) == LB.ST_CONVERGED
    # minimal horizon hp = 1 inside a hp_max = 20 slot
    out = S.solve(bt.x0, bt.u0, bt.ec_noise, hp=np.ones(4, np.int32))
    torch.cuda.synchronize()
    for b in range(4):
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=1)
        r = R.scp_solve(p, mode="structured")
        u, _ = unpack_problem(out, b, 4, 1)
        assert np.max(np.abs(u.cpu().numpy() - r.u)) <= U_TOL
    S.close()
    # maximum horizon: 1 vehicle, Hp = 64 (SCPQP_MAX_HP)
    sc1 = R.circle_scenario(1, Hp=64)
    S1 = ScpQpSolver(sc1, max_batch=2)
    b1 = BT.make_batch(sc1, 2, base_seed=3)
    o1 = S1.solve(b1.x0, b1.u0, b1.ec_noise)
    torch.cuda.synchronize()
    for b in range(2):
        p = R.make_problem(sc1, b1.x0[b], b1.u0[b], b1.ec_noise[b], Hp=64)
        r = R.scp_solve(p, mode="structured")
        assert o1.n_scp[b].item() == r.n_scp
        assert np.max(np.abs(o1.u[b].cpu().numpy() - r.u)) <= U_TOL
    S1.close()


def test_sampler_quirks(gpu):
    # B.1 alternation past the end of the line, and the 3-point '^' flag (B.2)
    sc = R.circle_scenario(2, Hp=8)
    S = ScpQpSolver(sc, max_batch=2)
    x0 = np.array(sc.x0, float)[None].repeat(2, 0)
    x0[0, 0, 0:2] = [25.0, 0.3]                  # vehicle 0 drives (30,0) -> (-30,0): on the line
    x0[1, 0, 0:2] = [-29.5, 0.0]                 # 0.5 m before its end: B.1 overshoot alternation
    ref = S.sample_reference(x0).cpu().numpy()
    for b in range(2):
        for v in range(2):
            want = R.sample_reference(8, sc.referenceTrajectories[v], x0[b, v, 0], x0[b, v, 1],
                                      x0[b, v, 3] * sc.dt)
            assert np.max(np.abs(ref[b, :, :, v] - want)) <= 1e-12
    S.close()
