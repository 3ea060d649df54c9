"""GPU parity of the plant kernels (csrc/plant.hip) and the
closed-loop rollout against the CPU restatement (oracle/plant_reference.py).

Tolerances: the device integrates with fixed-step RK4 (h <= 2.5 ms); against
the integration-error-free DOP853 solution at rtol = atol = 1e-13 the states
agree to 1e-9; against the reference's own scipy calls (odeint at 1.49e-8,
dopri5 at 1e-8) to 1e-6.  Clipping is min/max arithmetic: bit-exact.
"""
import math

import numpy as np
import pytest
import torch

from oracle import plant_reference as PR
from oracle import scp_reference as R
from scpqp import plant as PL

pytestmark = pytest.mark.gpu


def _states(rng, B, V):
    x = np.zeros((B, V, 6))
    x[..., 0] = rng.uniform(-30, 30, (B, V))
    x[..., 1] = rng.uniform(-30, 30, (B, V))
    x[..., 2] = rng.uniform(-math.pi, math.pi, (B, V))
    x[..., 3] = rng.uniform(2.0, 6.0, (B, V))
    x[..., 4] = rng.uniform(-0.5, 0.5, (B, V))
    x[..., 5] = rng.uniform(-0.05, 0.05, (B, V))
    return x


def test_delay_compensate_parity(gpu):
    sc = R.circle_scenario(4, Hp=20)
    rng = np.random.default_rng(11)
    B, V = 24, 4
    xm = _states(rng, B, V)
    uh = rng.uniform(-0.05, 0.05, (B, V))
    p = PL.plant_params(sc.Lf, sc.Lr)
    x0, traj = PL.delay_compensate(p, xm, uh, PR.delay_horizon(sc), device=gpu)
    x0, traj = x0.cpu().numpy(), traj.cpu().numpy()
    worst_exact = worst_ref = 0.0
    for b in range(B):
        xe, te = PR.delay_compensate_exact(sc, xm[b], uh[b])
        xr, _, tr = PR.delay_compensate(sc, xm[b], uh[b])
        worst_exact = max(worst_exact, np.abs(traj[b] - te).max(), np.abs(x0[b] - xe).max())
        worst_ref = max(worst_ref, np.abs(traj[b] - tr).max())
        assert np.array_equal(traj[b, -1].T, x0[b])
    assert worst_exact < 1e-9, worst_exact
    assert worst_ref < 1e-6, worst_ref


def test_delay_compensate_noise_terms(gpu):
    """Constant noise on dx[0], dx[1] shifts x, y by noise * T exactly (Model.py:84-86)."""
    sc = R.circle_scenario(2, Hp=10)
    p = PL.plant_params(sc.Lf, sc.Lr)
    xm = np.array([[[0.0, 0.0, 0.3, 4.0, 0.0, 0.0], [1.0, 2.0, -0.3, 3.0, 0.0, 0.0]]])
    nz = np.array([[[3e-6, -2e-6], [1e-6, 1e-6]]])
    a, _ = PL.delay_compensate(p, xm, np.zeros((1, 2)), 0.43, device=gpu)
    b, _ = PL.delay_compensate(p, xm, np.zeros((1, 2)), 0.43, noise=nz, device=gpu)
    d = (b - a).cpu().numpy()[0]
    assert np.allclose(d[:, :2], nz[0] * 0.43, atol=1e-15)
    assert np.all(d[:, 2:] == 0)


def test_plant_step_parity(gpu):
    sc = R.circle_scenario(4, Hp=20)
    rng = np.random.default_rng(5)
    B, V, K = 6, 4, sc.ticks_per_sim + 1
    xs = _states(rng, B, V)
    ut = rng.uniform(-0.05, 0.05, (B, V, K))
    p = PL.plant_params(sc.Lf, sc.Lr)
    path = PL.plant_step(p, xs, ut, sc.tick_length, device=gpu).cpu().numpy()
    assert path.shape == (B, V, K, 6)
    worst_exact = worst_ref = 0.0
    for b in range(2):
        for v in range(V):
            ex = PR.plant_step_exact(sc, v, xs[b, v], 1.2, ut[b, v])
            rf = PR.plant_step(sc, v, xs[b, v], 1.2, ut[b, v])
            worst_exact = max(worst_exact, np.abs(path[b, v] - ex).max())
            worst_ref = max(worst_ref, np.abs(path[b, v] - rf).max())
    assert np.array_equal(path[:, :, 0], xs)
    assert worst_exact < 1e-9, worst_exact
    assert worst_ref < 1e-6, worst_ref


def test_clip_controls_bit_exact(gpu):
    rng = np.random.default_rng(2)
    B, V, Hp = 16, 4, 20
    u = rng.uniform(-0.2, 0.2, (B, V * Hp))
    u0 = rng.uniform(-0.05, 0.05, (B, V))
    um = rng.uniform(0.02, 0.06, (B, V))
    du = math.pi / 180 * 6
    ut = torch.as_tensor(u, device=gpu).contiguous()
    PL.clip_controls(ut, u0, um, V, Hp, du)
    got = ut.cpu().numpy()
    for b in range(B):
        want = PR.clip_controls(u[b].reshape(V, Hp).T, u0[b], um[b], du).T.reshape(-1)
        assert np.array_equal(got[b], want)


def test_empty_batches(gpu):
    p = PL.plant_params([0.34], [0.34])
    x0, traj = PL.delay_compensate(p, np.zeros((0, 1, 6)), np.zeros((0, 1)), 0.43, device=gpu)
    assert x0.shape == (0, 1, 6) and traj.shape == (0, 10, 6, 1)
    out = PL.plant_step(p, np.zeros((0, 1, 6)), np.zeros((0, 1, 41)), 0.01, device=gpu)
    assert out.shape == (0, 1, 41, 6)
    with pytest.raises(ValueError):
        PL.delay_compensate(p, np.zeros((2, 2, 6)), np.zeros((2, 2)), 0.43, device=gpu)


def test_closed_loop_rollout_matches_restatement(gpu):
    """Five MPC steps of main.py:98-191 for four realisations (perturbed initial
    states): every step's solve and plant step on the device's own inputs, and the
    independent restated loop (tests/closed_loop_check.py; none skipped)."""
    import closed_loop_check as CC
    per = CC.run("circle4_hp10", 4, 5, gpu, workers=4)
    s = CC.summary(per)
    assert s["solve_kinds"].get("FAIL", 0) == 0 and s["solve_kinds"].get("mirror", 0) == 0
    assert s["max_plant_err"] <= CC.PLANT_TOL
    assert s["loop_max_path_diff_same_counts"] <= 1e-5
    assert s["loop_max_U_diff_same_counts"] <= 1e-6


def test_dropin_delay_compensation_matches_straight_line_and_odeint(gpu):
    """MPC_Iter.delay_compensate (the drop-in IterClass path) runs on the device."""
    import MPC_Iter
    import Scenarios
    from scpqp import batch as BT
    sc = Scenarios.Scenario(False)
    sc.Hp = sc.Hu = 20
    sc.get_circle_scenario([2 * math.pi / 4 * (i + 1) for i in range(4)])
    sc.complete_scenario()
    nT = sc.ticks_delay_x + sc.ticks_per_sim + sc.ticks_delay_u
    x_meas = np.array(sc.x0).reshape(4, 6)
    u_path = np.zeros((4, nT))
    x0, u0, traj = MPC_Iter.delay_compensate(sc, x_meas, u_path)
    assert np.allclose(x0, BT.delay_compensated_nominal(sc), atol=1e-10)
    assert traj.shape == (10, 6, 4) and np.array_equal(traj[-1].T, x0)
    assert np.all(u0 == 0)
    u_path[:, -1] = [0.01, -0.02, 0.03, 0.0]
    x0, u0, traj = MPC_Iter.delay_compensate(sc, x_meas, u_path)
    osc = R.circle_scenario(4, Hp=20)
    xr, _, tr = PR.delay_compensate(osc, x_meas, u_path[:, -1])
    assert np.abs(traj - tr).max() < 1e-6 and np.allclose(u0[:, 0], u_path[:, -1])
    with pytest.raises(AssertionError):
        MPC_Iter.delay_compensate(sc, x_meas, np.zeros((4, nT + 1)))


@pytest.mark.parametrize("kind", ["frog", "parallel5"])
def test_closed_loop_rollout_with_obstacles(gpu, kind):
    """Closed loop on the obstacle scenarios (Scenarios.py:127-201): obstacle
    predictions from the constant-velocity obstacle paths (main.py:61-71,
    MPC_Iter.py:45-51) feed the solve and the evaluation; every step checked on
    the device's own inputs (tests/closed_loop_check.py)."""
    import closed_loop_check as CC
    per = CC.run(kind, 2, 4, gpu, workers=2)
    s = CC.summary(per)
    assert s["solve_kinds"].get("FAIL", 0) == 0 and s["solve_kinds"].get("mirror", 0) == 0
    assert s["max_plant_err"] <= CC.PLANT_TOL
    assert s["loop_max_path_diff_same_counts"] <= 1e-5
    from scpqp.rollout import ClosedLoopBatch
    sc = CC.scenario(kind)
    x_init = CC.initial_states(kind, 2)
    cl = ClosedLoopBatch(sc, 2, device=gpu)
    cl.reset(x_init)
    hist = cl.run(2)
    for b in range(2):
        ref = PR.ClosedLoop(sc, x_init=x_init[b])
        for i in range(2):
            r = ref.step(i)
            if int(hist[i]["n_scp"][b]) != r["n_scp"]:
                break
            ev, rev = hist[i]["evaluation"], r["evaluation"]     # SCP_controller.py:343-400
            assert bool(ev["predictionFeasible"][b]) == rev["predictionFeasible"]
            assert np.abs(ev["constraintValuesObstacle"][b].cpu().numpy()
                          - rev["constraintValuesObstacle"]).max() < 1e-6
            for k in ("predictionObjectiveValueX", "predictionObjectiveValueU"):
                assert abs(float(ev[k][b]) - rev[k]) <= 1e-6 * max(1.0, abs(rev[k]))
    cl.close()


def test_result_for_plot_matches_restatement(gpu, tmp_path):
    """f3 at batch scale: ClosedLoopBatch.result_for_plot(b) (main.py:213-225's
    result_for_plot1) against the restatement's, field by field, and dump_result
    readable by json with draw_video.py:44-56's reshapes."""
    import json
    from scpqp.rollout import ClosedLoopBatch
    sc = R.frog_scenario(Hp=10)
    rng = np.random.default_rng(11)
    B, steps, nV = 2, 2, sc.nVeh
    x_init = np.array(sc.x0)[None] + rng.normal(0, 1, (B, nV, 6)) * np.array(
        [0.05, 0.05, 0.005, 0.02, 0, 0.002])
    cl = ClosedLoopBatch(sc, B, device=gpu, keep_path=True, timing=True)
    cl.reset(x_init)
    cl.run(steps)
    compared = 0
    for b in range(B):
        ref = PR.ClosedLoop(sc, x_init=x_init[b])
        for i in range(steps):
            ref.step(i)
        if [int(h["n_scp"][b]) for h in cl.history] != [r["n_scp"] for r in ref.records]:
            continue
        compared += 1
        got, want = cl.result_for_plot(b), ref.result_for_plot()
        assert set(got) == set(want)
        tol = dict(vehiclePathFullRes=1e-5, obstaclePathFullRes=1e-12, controlPathFullRes=1e-6,
                   controlPredictions=1e-6, trajectoryPredictions=1e-5, initial_pos=1e-6,
                   ReferenceTrajectory=1e-6, MPC_delay_compensation_trajectory=1e-6)
        for k, t in tol.items():
            g, w = np.asarray(got[k]), np.asarray(want[k])
            assert g.shape == w.shape, k
            assert np.array_equal(np.isnan(g), np.isnan(w)), k
            assert np.nanmax(np.abs(g - w)) < t, k
        assert np.allclose(got["evaluations_obj_value"], want["evaluations_obj_value"], rtol=1e-6)
        assert np.all(got["stepTime"][:steps] > 0) and np.all(got["stepTime"][steps:] == 0)
        p = tmp_path / f"frog_{b}.json"
        with open(p, "w") as fp:
            cl.dump_result(fp, b)
        back = json.load(open(p))
        veh = np.reshape(back["vehiclePathFullRes"], (6, nV, sc.ticks_total + 1), order="F")
        assert np.array_equal(veh, got["vehiclePathFullRes"], equal_nan=True)
    assert compared >= 1
    cl.close()
