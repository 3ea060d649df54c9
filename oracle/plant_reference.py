"""CPU restatement of the plant around the SCP solve.

TEST INFRASTRUCTURE ONLY — the product never imports this file; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` may.

The reference integrates the bicycle model (Model.py:61-87) with scipy:

* delay compensation, ``IterClass`` (MPC_Iter.py:24-33): ``scipy.integrate.
  odeint(model.ode, x_measured[v], linspace(0, delay_x + dt + delay_u, 10),
  args=(u_path[v, -1], Lf[v], Lr[v]))`` — LSODA at its default rtol = atol =
  1.49012e-8;
* the plant, ``Simulation.runsimulation`` (main.py:184-191): ``scipy.integrate.
  ode(model.odes_).set_integrator('dopri5', atol=1e-8, rtol=1e-8)``, restarted
  at t0 = i*dt for every output time of the step with the control value of that
  tick;
* steering-limit enforcement (main.py:164-174) and the control-path bookkeeping
  with the actuator delay (main.py:101-117, 176-182).

The scipy calls below are the reference's own third-party calls with the same
arguments (scipy 1.15 here; the reference pins no version).  ``*_exact`` runs
the same initial value problems at rtol = atol = 1e-13 (DOP853) as the
integration-error-free truth the GPU's fixed-step RK4 is checked against.
``is_noise`` is False in main.py:235, so the plant is deterministic.
"""
from __future__ import annotations

import math
import warnings

import numpy as np
import scipy.integrate

from . import scp_reference as R

DELAY_STEPS = 10                          # MPC_Iter.py:21
LATERAL_ACC_LIMIT = 9.81 / 2              # Scenarios.py:48
NX = 6


def _ode(x, t, u_ref, Lf, Lr):
    """Model.ode with odeint's f(x, t, *args) signature (Model.py:61-87)."""
    return R.bicycle_rhs(x, u_ref, Lf, Lr)


def _odes(t, x, u_ref, Lf, Lr):
    """Model.odes_ with scipy.integrate.ode's f(t, x, *args) signature (Model.py:89-114)."""
    return R.bicycle_rhs(x, u_ref, Lf, Lr)


def delay_horizon(sc):
    """delay_x + dt + delay_u (MPC_Iter.py:28)."""
    return sc.delay_x + sc.dt + sc.delay_u


def delay_compensate(sc, x_measured, u_hold, steps=DELAY_STEPS):
    """MPC_Iter.py:24-33.  x_measured [nVeh, 6], u_hold [nVeh] (= u_path[:, -1])
    -> x0 [nVeh, 6], u0 [nVeh], trajectory [steps, 6, nVeh]."""
    nV = len(u_hold)
    times = np.linspace(0, delay_horizon(sc), steps)
    x0 = np.zeros((nV, NX))
    traj = np.zeros((steps, NX, nV))
    for v in range(nV):
        Y = scipy.integrate.odeint(_ode, np.asarray(x_measured[v], float), times,
                                   args=(float(u_hold[v]), sc.Lf[v], sc.Lr[v]))
        x0[v] = Y[-1]
        traj[:, :, v] = Y
    return x0, np.asarray(u_hold, float).copy(), traj


def delay_compensate_exact(sc, x_measured, u_hold, steps=DELAY_STEPS):
    """The same initial value problem at rtol = atol = 1e-13 (DOP853)."""
    nV = len(u_hold)
    times = np.linspace(0, delay_horizon(sc), steps)
    traj = np.zeros((steps, NX, nV))
    for v in range(nV):
        sol = scipy.integrate.solve_ivp(_odes, (0.0, times[-1]), np.asarray(x_measured[v], float),
                                        method="DOP853", t_eval=times, rtol=1e-13, atol=1e-13,
                                        args=(float(u_hold[v]), sc.Lf[v], sc.Lr[v]))
        traj[:, :, v] = sol.y.T
    return traj[-1].T.copy(), traj


def plant_step(sc, v, x_start, t0, u_of_k):
    """main.py:184-191 for vehicle v: ``model_step [ticks_per_sim + 1, 6]``;
    output k restarts dopri5 at t0 and integrates to timelist[k] with the
    constant control u_of_k[k]."""
    K = sc.ticks_per_sim + 1
    timelist = np.linspace(t0, t0 + sc.dt, K)
    out = np.zeros((K, NX))
    for k in range(K):
        ode = scipy.integrate.ode(_odes).set_integrator("dopri5", atol=1e-8, rtol=1e-8)
        ode.set_initial_value(np.asarray(x_start, float), t=t0).set_f_params(
            float(u_of_k[k]), sc.Lf[v], sc.Lr[v])
        with warnings.catch_warnings():   # k = 0 integrates over a zero span, as the reference does
            warnings.simplefilter("ignore", UserWarning)
            out[k] = ode.integrate(timelist[k])
    return out


def plant_step_exact(sc, v, x_start, t0, u_of_k):
    """plant_step at rtol = atol = 1e-13 (DOP853)."""
    K = sc.ticks_per_sim + 1
    timelist = np.linspace(t0, t0 + sc.dt, K)
    out = np.zeros((K, NX))
    out[0] = x_start
    for k in range(1, K):
        sol = scipy.integrate.solve_ivp(_odes, (t0, timelist[k]), np.asarray(x_start, float),
                                        method="DOP853", rtol=1e-13, atol=1e-13,
                                        args=(float(u_of_k[k]), sc.Lf[v], sc.Lr[v]))
        out[k] = sol.y[:, -1]
    return out


# ---------------------------------------------------------------------------
# The device's integrator restated (csrc/plant.hip): classical RK4 with equal steps of
# at most H_MAX over each span.  Used by ClosedLoop(plant="rk4") to run the restated
# closed loop on the device's plant arithmetic instead of the reference's scipy calls,
# so that a divergence between the device loop and the restated loop can be pinned on
# the integrator (dopri5 / LSODA vs RK4, ~1e-12 m) rather than on the solver.
# ---------------------------------------------------------------------------
H_MAX = 2.5e-3            # scpqp/plant.py H_MAX (a quarter tick)


def _rk4_steps(T, hmax=H_MAX):
    """plant.hip steps_for: ceil(|T| / hmax - 1e-9), at least 1."""
    return max(1, int(math.ceil(abs(T) / hmax - 1e-9)))


def _rk4_flow(x, T, u_ref, Lf, Lr, n):
    """plant.hip flow(): n RK4 steps of h = T / n from x (Model.py:61-87 right-hand side)."""
    x = np.array(x, float)
    h = T / n
    for _ in range(n):
        k1 = R.bicycle_rhs(x, u_ref, Lf, Lr)
        k2 = R.bicycle_rhs(x + 0.5 * h * k1, u_ref, Lf, Lr)
        k3 = R.bicycle_rhs(x + 0.5 * h * k2, u_ref, Lf, Lr)
        k4 = R.bicycle_rhs(x + h * k3, u_ref, Lf, Lr)
        x = x + h / 6.0 * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
    return x


def delay_compensate_rk4(sc, x_measured, u_hold, steps=DELAY_STEPS):
    """delay_compensate on the device's integrator (plant.hip delay_kernel): the
    outputs linspace(0, horizon, steps), each span integrated from the previous output."""
    nV = len(u_hold)
    span = delay_horizon(sc) / (steps - 1)
    n = _rk4_steps(span)
    traj = np.zeros((steps, NX, nV))
    for v in range(nV):
        x = np.asarray(x_measured[v], float)
        traj[0, :, v] = x
        for j in range(1, steps):
            x = _rk4_flow(x, span, float(u_hold[v]), sc.Lf[v], sc.Lr[v], n)
            traj[j, :, v] = x
    return traj[-1].T.copy(), np.asarray(u_hold, float).copy(), traj


def plant_step_rk4(sc, v, x_start, t0, u_of_k):
    """plant_step on the device's integrator (plant.hip plant_kernel): output k
    integrates k ticks from x_start with the control of tick k."""
    K = sc.ticks_per_sim + 1
    out = np.zeros((K, NX))
    out[0] = x_start
    for k in range(1, K):
        T = k * sc.tick_length
        out[k] = _rk4_flow(x_start, T, float(u_of_k[k]), sc.Lf[v], sc.Lr[v], _rk4_steps(T))
    return out


def clip_controls(U, u0, umax, du_lim):
    """main.py:164-174 on U [Hp, nVeh] (a copy is returned)."""
    U = np.array(U, float, copy=True)
    Hp, nV = U.shape
    for v in range(nV):
        U[0, v] = min(U[0, v], umax[v])
        U[0, v] = max(U[0, v], -umax[v])
        U[0, v] = min(U[0, v], u0[v] + du_lim)
        U[0, v] = max(U[0, v], u0[v] - du_lim)
        for j in range(1, Hp):
            U[j, v] = min(U[j, v], umax[v])
            U[j, v] = max(U[j, v], -umax[v])
            U[j, v] = min(U[j, v], U[j - 1, v] + du_lim)
            U[j, v] = max(U[j, v], U[j - 1, v] - du_lim)
    return U


def steering_limit(sc, speed, v):
    """main.py:105-108: min(mechanical limit, atan(a_lat,max * L / v^2))."""
    dyn = math.atan(LATERAL_ACC_LIMIT * (sc.Lf[v] + sc.Lr[v]) / speed ** 2)
    return min(sc.mechanicalSteeringLimit, dyn)


def control_tick_index(sc, t):
    """main.py:187: index of controlPathFullRes read for output time t."""
    return min(sc.ticks_total, math.ceil(t / sc.tick_length) + 1)


def evaluate_in_original_problem(sc, U, traj, ref_points, obst_future=None,
                                 tol=R.CONSTRAINT_TOL):
    """SCP_controller.py:343-400 (evaluateInOriginalProblem) without the QCQP
    re-check: U [Hp, nVeh] (controller output), traj [Hp, 2, nVeh], ref_points
    [Hp, 2, nVeh], obst_future [nObst, 2, Hp]."""
    nV, Hp = U.shape[1], U.shape[0]
    err2 = (ref_points - traj) ** 2
    objx = sum(sc.Q[v] * err2[:-1, :, v].sum() + sc.Q_final[v] * err2[-1, :, v].sum()
               for v in range(nV))
    obju = sum(sc.R[v] * (U[:, v] ** 2).sum() for v in range(nV))
    cv = np.zeros((nV, nV, Hp))
    nO = 0 if obst_future is None else obst_future.shape[0]
    co = np.zeros((nV, nO, Hp))
    feasible = True
    for k in range(Hp):
        for v in range(nV):
            for v2 in range(v + 1, nV):
                ci = sc.dsafeVehicles[v, v2] ** 2 - ((traj[k, :, v] - traj[k, :, v2]) ** 2).sum()
                cv[v, v2, k] = cv[v2, v, k] = ci
                feasible = feasible and not ci > tol
            for o in range(nO):
                ci = sc.dsafeObstacles[v, o] ** 2 - ((traj[k, :, v] - obst_future[o, :, k]) ** 2).sum()
                co[v, o, k] = ci
                feasible = feasible and not ci > tol
    return dict(predictionObjectiveValueX=objx, predictionObjectiveValueU=obju,
                predictionObjectiveValue=objx + obju, constraintValuesVehicle=cv,
                constraintValuesObstacle=co, predictionFeasible=feasible)


def obstacle_state(sc, tick):
    """obstaclePathFullRes[:, :, tick] (main.py:61-71): constant-velocity obstacles."""
    out = np.zeros((sc.nObst, 2))
    for o, ob in enumerate(sc.obstacles):
        out[o, 0] = (tick * sc.tick_length) * ob[3] * math.cos(ob[2]) + ob[0]
        out[o, 1] = (tick * sc.tick_length) * ob[3] * math.sin(ob[2]) + ob[1]
    return out


def obstacle_prediction(sc, tick_meas):
    """Iter.obstacleFutureTrajectories [nObst, 2, Hp] of an MPC step (MPC_Iter.py:45-51)
    from the obstacle state at the measurement tick (main.py:123)."""
    if not sc.nObst:
        return np.zeros((0, 2, sc.Hp))
    return R.obstacle_future(sc, obstacle_state(sc, tick_meas), sc.Hp)


class ClosedLoop:
    """Restatement of ``Simulation.runsimulation`` (main.py:98-206) for one
    realisation with the SCP controller of ``scp_reference`` (structured mode).
    ``x_init`` [nVeh, 6] replaces scenario.x0 (main.py:73-75)."""

    def __init__(self, sc, x_init=None, plant="scipy"):
        """``plant``: "scipy" — the reference's own integrator calls (odeint, dopri5);
        "rk4" — the device's fixed-step RK4 restated (delay_compensate_rk4, plant_step_rk4)."""
        self.sc = sc
        self.plant = plant
        nV = sc.nVeh
        self.du_lim = sc.mechanicalSteeringLimit * 2              # Scenarios.py:50
        self.path = np.full((NX, nV, sc.ticks_total + 1), np.nan)
        self.control = np.full((nV, sc.ticks_total + 1), np.nan)
        x_init = np.array([sc.x0[v] for v in range(nV)]) if x_init is None else x_init
        for v in range(nV):
            self.path[:, v, 0] = x_init[v]
            self.control[v, 0:sc.ticks_delay_u + sc.ticks_per_sim + 1] = sc.u0[v]
        self.u_prev = None
        self.records = []

    def step(self, i):
        sc = self.sc
        nV, tps = sc.nVeh, sc.ticks_per_sim
        tick_now = i * tps
        tick_meas = max(0, tick_now - sc.ticks_delay_x)
        tick_act = min(sc.ticks_total + 1, tick_now + 1 + sc.ticks_delay_u + tps)
        umax = np.array([steering_limit(sc, self.path[3, v, tick_now], v) for v in range(nV)])
        x_meas = self.path[:, :, tick_meas].T
        n_path = sc.ticks_delay_x + tps + sc.ticks_delay_u
        u_path = np.zeros((nV, n_path))
        lo = max(sc.ticks_delay_x - tick_now, 0)
        u_path[:, lo:lo + tick_act - 1 - tick_meas] = self.control[:, tick_meas + 1:tick_act]
        dc = delay_compensate_rk4 if self.plant == "rk4" else delay_compensate
        x0, u0, dtraj = dc(sc, x_meas, u_path[:, -1])
        obst = obstacle_prediction(sc, tick_meas)
        p = R.make_problem(sc, x0, u0, np.zeros((nV, 2)), Hp=sc.Hp, obst=obst)
        res = R.scp_solve(p, u_warm=self.u_prev, mode="structured")
        self.u_prev = res.u.copy()
        U = clip_controls(res.U, u0, umax, self.du_lim)
        for v in range(nV):
            sl = np.arange(i * tps + 1 + sc.ticks_delay_u + tps, (i + 1) * tps + 1 + sc.ticks_delay_u + tps)
            sl[sl >= self.control.shape[1] - 1] = self.control.shape[1] - 1
            self.control[v, sl] = U[0, v]
            timelist = np.linspace(i * sc.dt, (i + 1) * sc.dt, tps + 1)
            u_of_k = [self.control[v, control_tick_index(sc, t)] for t in timelist]
            ps = plant_step_rk4 if self.plant == "rk4" else plant_step
            ms = ps(sc, v, self.path[:, v, tick_now], i * sc.dt, u_of_k)
            self.path[:, v, tps * i + 1:tps * (i + 1) + 1] = ms[1:].T
        ev = evaluate_in_original_problem(sc, U, res.traj, p.ref_points,
                                          obst if sc.nObst else None)
        self.records.append(dict(x0=x0, u0=u0, delay_traj=dtraj, umax=umax, U=U, traj=res.traj,
                                 n_scp=res.n_scp, u=res.u, evaluation=ev, ref=p.ref_points))
        return self.records[-1]

    def result_for_plot(self):
        """``result_for_plot1`` of main.py:213-225 (the JSON draw_video.py:44-56 reads),
        as numpy arrays, over the steps run so far; timing fields are zero."""
        sc = self.sc
        nV, Hp, Nsim = sc.nVeh, sc.Hp, sc.Nsim
        out = dict(
            vehiclePathFullRes=self.path.copy(),
            obstaclePathFullRes=np.stack([obstacle_state(sc, t) for t in range(sc.ticks_total + 1)],
                                         axis=-1) if sc.nObst
            else np.zeros((0, 2, sc.ticks_total + 1)),
            controlPathFullRes=self.control.copy(),
            controlPredictions=np.zeros((Hp, nV, Nsim)),
            trajectoryPredictions=np.zeros((Hp, 2, nV, Nsim)),
            initial_pos=np.zeros((2, nV, Nsim)),
            ReferenceTrajectory=np.zeros((Hp, 2, nV, Nsim)),
            MPC_delay_compensation_trajectory=np.zeros((DELAY_STEPS, NX, nV, Nsim)),
            evaluations_obj_value=[float(r["evaluation"]["predictionObjectiveValue"])
                                   for r in self.records],
            controllerRuntime=np.zeros((Nsim, 1)),
            stepTime=np.zeros((Nsim, 1)))
        for i, r in enumerate(self.records):
            out["controlPredictions"][:, :, i] = r["U"]
            out["trajectoryPredictions"][:, :, :, i] = r["traj"]
            out["initial_pos"][:, :, i] = r["x0"][:, 0:2].T
            out["ReferenceTrajectory"][:, :, :, i] = r["ref"]
            out["MPC_delay_compensation_trajectory"][:, :, :, i] = r["delay_traj"]
        return out
