"""The plant restatement (oracle/plant_reference.py) pinned
by closed-form solutions of the bicycle model, and its scipy calls checked
against each other.  CPU only.

Known answers (Model.py:61-87, noise off):
* delta = u_ref = 0, a = 0: straight line at the rear-axle speed;
* steering: d(delta)/dt = (u_ref - delta) / 0.1 -> first-order lag, exact
  exponential;
* delta = u_ref != 0 held, a = 0: a circle of radius v_c / psi_dot around a
  fixed centre, heading rate psi_dot = v_c tan(delta) cos(beta) / L.
"""
import math

import numpy as np
import pytest

from oracle import plant_reference as PR
from oracle import scp_reference as R


def _sc(n=2, hp=10):
    return R.circle_scenario(n, Hp=hp)


def straight(x, t):
    out = np.array(x, float)
    out[0] += x[3] * t * math.cos(x[2])
    out[1] += x[3] * t * math.sin(x[2])
    return out


def circle(x, t, L):
    x = np.asarray(x, float)
    rho = 0.5
    tu = math.tan(x[5])
    beta = math.atan(rho * tu)
    vc = x[3] * math.sqrt(1 + (rho * tu) ** 2)
    w = vc * tu * math.cos(beta) / L
    out = x.copy()
    out[2] = x[2] + w * t
    out[0] = x[0] + vc / w * (math.sin(x[2] + beta + w * t) - math.sin(x[2] + beta))
    out[1] = x[1] - vc / w * (math.cos(x[2] + beta + w * t) - math.cos(x[2] + beta))
    return out


def test_delay_compensation_straight_line():
    sc = _sc()
    xm = np.array([[1.0, -2.0, 0.3, 4.0, 0.0, 0.0], [0.0, 5.0, -1.2, 3.5, 0.0, 0.0]])
    x0, u0, traj = PR.delay_compensate(sc, xm, np.zeros(2))
    T = PR.delay_horizon(sc)
    assert abs(T - 0.43) < 1e-15
    for v in range(2):
        assert np.allclose(x0[v], straight(xm[v], T), atol=1e-7)   # odeint rtol/atol 1.5e-8
        for j, t in enumerate(np.linspace(0, T, PR.DELAY_STEPS)):
            assert np.allclose(traj[j, :, v], straight(xm[v], t), atol=1e-7)
    xe, te = PR.delay_compensate_exact(sc, xm, np.zeros(2))
    assert np.allclose(xe, [straight(xm[v], T) for v in range(2)], atol=1e-12)
    assert traj.shape == te.shape == (10, 6, 2) and np.array_equal(u0, np.zeros(2))


def test_steering_lag_is_exponential():
    sc = _sc()
    xm = np.array([[0.0, 0.0, 0.0, 0.0, 0.0, 0.02], [0.0, 0.0, 0.0, 0.0, 0.0, -0.01]])
    u = np.array([-0.03, 0.04])
    x0, _, _ = PR.delay_compensate(sc, xm, u)
    xe, _ = PR.delay_compensate_exact(sc, xm, u)
    T = PR.delay_horizon(sc)
    want = u + (xm[:, 5] - u) * math.exp(-T / 0.1)
    assert np.allclose(xe[:, 5], want, atol=1e-13)
    assert np.allclose(x0[:, 5], want, atol=1e-8)
    assert np.all(xe[:, :2] == 0.0)      # speed 0: no motion


@pytest.mark.parametrize("delta", [0.02, -0.05])
def test_held_steering_drives_a_circle(delta):
    sc = _sc()
    xm = np.array([[3.0, 1.0, 0.7, 4.0, 0.0, delta]] * 2)
    xe, te = PR.delay_compensate_exact(sc, xm, np.full(2, delta))
    for j, t in enumerate(np.linspace(0, PR.delay_horizon(sc), PR.DELAY_STEPS)):
        assert np.allclose(te[j, :, 0], circle(xm[0], t, 0.68), atol=1e-11)
    x0, _, _ = PR.delay_compensate(sc, xm, np.full(2, delta))
    assert np.allclose(x0, xe, atol=1e-6)


def test_plant_step_matches_exact_flow():
    sc = _sc()
    rng = np.random.default_rng(3)
    x = np.array([2.0, -1.0, 0.4, 4.0, 0.1, 0.01])
    u = rng.uniform(-0.05, 0.05, sc.ticks_per_sim + 1)
    got = PR.plant_step(sc, 0, x, 0.8, u)
    ref = PR.plant_step_exact(sc, 0, x, 0.8, u)
    assert got.shape == (sc.ticks_per_sim + 1, 6)
    assert np.array_equal(got[0], x)
    assert np.max(np.abs(got - ref)) < 1e-6         # dopri5 at rtol = atol = 1e-8


def test_clip_controls_known_answers():
    U = np.array([[0.2, -0.2], [0.2, -0.01], [-0.2, 0.0]])
    got = PR.clip_controls(U, u0=np.array([0.0, 0.0]), umax=np.array([0.05, 0.05]), du_lim=0.1)
    want = np.array([[0.05, -0.05], [0.05, -0.01], [-0.05, 0.0]])
    assert np.allclose(got, want)
    got = PR.clip_controls(U, u0=np.array([0.0, 0.0]), umax=np.array([1.0, 1.0]), du_lim=0.1)
    assert np.allclose(got[:, 0], [0.1, 0.2, 0.1]) and np.allclose(got[:, 1], [-0.1, -0.01, 0.0])


def test_steering_limit_and_control_index():
    sc = _sc()
    assert PR.steering_limit(sc, 4.0, 0) == sc.mechanicalSteeringLimit   # atan(4.905*.68/16) > 3 deg
    assert PR.steering_limit(sc, 20.0, 0) == pytest.approx(math.atan(4.905 * 0.68 / 400))
    assert PR.control_tick_index(sc, 0.0) == 1
    assert PR.control_tick_index(sc, 0.4) == 41
    assert PR.control_tick_index(sc, 1e9) == sc.ticks_total


@pytest.mark.slow
def test_closed_loop_restatement_two_steps():
    sc = _sc(2, hp=10)
    cl = PR.ClosedLoop(sc)
    r0 = cl.step(0)
    r1 = cl.step(1)
    tps = sc.ticks_per_sim
    assert np.all(np.isfinite(cl.path[:, :, :2 * tps + 1]))
    assert np.all(np.isnan(cl.path[:, :, 2 * tps + 1:]))
    # step 0 holds u0 = 0 over the delay: x0 is the straight-line nominal state
    x_init = np.array(sc.x0)
    for v in range(2):
        assert np.allclose(r0["x0"][v], straight(x_init[v], 0.43), atol=1e-7)
    # the command applied after the actuator delay is the first clipped control
    assert np.allclose(cl.control[:, 1 + sc.ticks_delay_u + tps], r0["U"][0])
    assert np.all(np.abs(r1["U"]) <= sc.mechanicalSteeringLimit + 1e-12)


@pytest.mark.parametrize("tdx", [0, 2])
def test_held_command_tick_matches_main_py_slicing(tdx):
    """The rollout's held-command index (scpqp/rollout.py) against main.py:101-117's
    u_path construction, over a whole simulation including the truncated end."""
    from scpqp.rollout import held_command_tick
    sc = _sc()
    tps, tdu, tt = sc.ticks_per_sim, sc.ticks_delay_u, sc.ticks_total
    control = np.arange(tt + 1, dtype=float) + 1.0          # tick k holds k + 1
    truncated = 0
    for i in range(sc.Nsim):
        now = i * tps
        meas = max(0, now - tdx)
        act = min(tt + 1, now + 1 + tdu + tps)
        u_path = np.zeros(tdx + tps + tdu)
        lo = max(tdx - now, 0)
        u_path[lo:lo + act - 1 - meas] = control[meas + 1:act]
        k = held_command_tick(now, tdx, tdu, tps, tt)
        if k is None:
            truncated += 1
            assert u_path[-1] == 0.0
        else:
            assert u_path[-1] == control[k]
    assert truncated >= 1            # the last MPC step of main.py holds u = 0


@pytest.mark.slow
def test_result_for_plot_has_main_py_schema():
    """oracle ClosedLoop.result_for_plot: the keys, shapes and NaN/zero fill of
    main.py:213-225, round-tripped through json and read back with
    draw_video.py:44-56's reshapes."""
    import json
    sc = R.frog_scenario(Hp=10)
    cl = PR.ClosedLoop(sc)
    cl.step(0)
    res = cl.result_for_plot()
    nV, Hp, Nsim, T = sc.nVeh, sc.Hp, sc.Nsim, sc.ticks_total
    txt = json.dumps({k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in res.items()})
    back = json.loads(txt)
    shapes = dict(vehiclePathFullRes=(6, nV, T + 1), obstaclePathFullRes=(sc.nObst, 2, T + 1),
                  controlPathFullRes=(nV, T + 1), controlPredictions=(Hp, nV, Nsim),
                  trajectoryPredictions=(Hp, 2, nV, Nsim), initial_pos=(1, 2, nV, Nsim),
                  MPC_delay_compensation_trajectory=(10, 6, nV, Nsim),
                  evaluations_obj_value=(1, 1), controllerRuntime=(Nsim, 1),
                  stepTime=(Nsim, 1), ReferenceTrajectory=(Hp, 2, nV, Nsim))
    assert set(back) == set(shapes)
    for k, shp in shapes.items():
        a = np.reshape(back[k], shp, order="F")
        if k not in ("initial_pos", "evaluations_obj_value"):
            assert np.array_equal(a, res[k], equal_nan=True), k
    tps = sc.ticks_per_sim
    veh = res["vehiclePathFullRes"]
    assert np.all(np.isfinite(veh[:, :, :tps + 1])) and np.all(np.isnan(veh[:, :, tps + 1:]))
    assert np.all(res["controlPredictions"][:, :, 1:] == 0)
    assert np.allclose(res["obstaclePathFullRes"][:, :, 0], np.array(sc.obstacles)[:, 0:2])
