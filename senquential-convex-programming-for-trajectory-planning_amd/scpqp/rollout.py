"""Closed-loop Monte-Carlo rollouts on the GPU (main.py:98-206).

``ClosedLoopBatch`` runs ``Simulation.runsimulation`` with the SCP controller
for B independent realisations of one scenario at once.  Per MPC step i:

1. measurement, steering limits and the held command (main.py:101-117, 105-108)
2. delay compensation, ``IterClass`` (MPC_Iter.py:24-33)   -> scpqp_delay_compensate
3. the SCP solve, warm-started from the previous step's u  -> scpqp_solve
   (SCP_controller.py:42-43)
4. steering-limit enforcement (main.py:164-174)            -> scpqp_clip_controls
5. actuator-delayed control path and the plant over one step (main.py:176-191)
                                                            -> scpqp_plant_step
6. evaluateInOriginalProblem of the step (main.py:201-202, SCP_controller.py:343-400)
                                                            -> device tensor ops

All state lives on the device (torch-ROCm tensors); the per-step index
bookkeeping (which tick is measured, which control tick each plant output
reads) is the same for every realisation and is computed on the host once
per step, exactly as main.py computes it.  Realisations differ by their
initial state (and optional constant model-noise terms).
"""
from __future__ import annotations

import json
import math
import time

import numpy as np
import torch

from . import plant as PL
from .solver import ScpQpSolver

LATERAL_ACC_LIMIT = 9.81 / 2      # Scenarios.py:48
CONSTRAINT_TOL = 2 * 2.1 * 1e-3   # Config.py:18


def evaluate_in_original_problem(scenario, U, traj, ref_points, obst_future=None,
                                 tol=CONSTRAINT_TOL):
    """SCPcontroller.evaluateInOriginalProblem (SCP_controller.py:343-400) for a
    batch, on the device: U [B, Hp, nVeh] (the clipped controller output),
    traj [B, Hp, 2, nVeh] (trajectory prediction), ref_points [B, Hp, 2, nVeh],
    obst_future [B, nObst, 2, Hp] or None.  Returns tensors: the objective terms
    [B], constraint values [B, nVeh, nVeh, Hp] / [B, nVeh, nObst, Hp] and
    predictionFeasible [B] (from the predicted trajectory, as the reference)."""
    dev = U.device
    f = dict(dtype=torch.float64, device=dev)
    nV = U.shape[2]
    Q = torch.tensor([float(q) for q in scenario.Q], **f)
    Qf = torch.tensor([float(q) for q in scenario.Q_final], **f)
    Rw = torch.tensor([float(r) for r in scenario.R], **f)
    err2 = (ref_points - traj) ** 2                                  # [B, Hp, 2, nV]
    objx = (err2[:, :-1].sum(dim=(1, 2)) * Q).sum(-1) + (err2[:, -1].sum(dim=1) * Qf).sum(-1)
    obju = ((U ** 2).sum(dim=1) * Rw).sum(-1)
    ds2 = torch.as_tensor(np.asarray(scenario.dsafeVehicles, float) ** 2, **f)   # [nV, nV]
    p = traj.permute(0, 3, 2, 1)                                     # [B, nV, 2, Hp]
    d2 = ((p[:, :, None] - p[:, None, :]) ** 2).sum(3)               # [B, nV, nV, Hp]
    cv = ds2[None, :, :, None] - d2
    eye = torch.eye(nV, dtype=torch.bool, device=dev)[None, :, :, None]
    cv = torch.where(eye, torch.zeros_like(cv), cv)                  # diagonal stays 0
    viol = (cv > tol).flatten(1).any(1)
    out = dict(predictionObjectiveValueX=objx, predictionObjectiveValueU=obju,
               predictionObjectiveValue=objx + obju, constraintValuesVehicle=cv)
    if obst_future is not None and obst_future.shape[1] > 0:
        dso = torch.as_tensor(np.asarray(scenario.dsafeObstacles, float) ** 2, **f)  # [nV, nO]
        d2o = ((p[:, :, None] - obst_future[:, None]) ** 2).sum(3)   # [B, nV, nO, Hp]
        co = dso[None, :, :, None] - d2o
        viol = viol | (co > tol).flatten(1).any(1)
        out["constraintValuesObstacle"] = co
    out["predictionFeasible"] = ~viol
    return out


def held_command_tick(tick_now, tdx, tdu, tps, ticks_total):
    """u_path[:, -1] of main.py:101-117 (the command IterClass holds over the
    delay, MPC_Iter.py:29-32): the controlPathFullRes tick it copies, or None
    when the slice is truncated at the end of the simulation and u_path[:, -1]
    keeps its zero initialisation."""
    tick_meas = max(0, tick_now - tdx)
    tick_act = min(ticks_total + 1, tick_now + 1 + tdu + tps)
    n_path = tdx + tps + tdu
    lo = max(tdx - tick_now, 0)
    hi = lo + tick_act - 1 - tick_meas
    if hi < n_path:
        return None
    return tick_meas + 1 + (n_path - 1 - lo)


class ClosedLoopBatch:
    def __init__(self, scenario, B, device=None, h_max=PL.H_MAX, keep_path=False, evaluate=True,
                 timing=False, trace=False, **solver_kw):
        self.sc = scenario
        self.B = int(B)
        self.device = torch.device(device or "cuda")
        self.nV, self.Hp = int(scenario.nVeh), int(scenario.Hp)
        self.tps = int(scenario.ticks_per_sim)
        self.ticks_total = int(scenario.ticks_total)
        self.tdx, self.tdu = int(scenario.ticks_delay_x), int(scenario.ticks_delay_u)
        if self.tdx > self.tps:
            raise ValueError("measurement delay longer than one MPC step is not supported")
        self.h_max = h_max
        self.keep_path = keep_path
        self.evaluate = evaluate
        self.timing = timing
        self.nO = int(scenario.nObst)
        self.obstacles = np.asarray(scenario.obstacles, float).reshape(self.nO, -1) if self.nO \
            else np.zeros((0, 6))
        self.params = PL.plant_params(scenario.Lf, scenario.Lr)
        self.solver = ScpQpSolver(scenario, max_batch=self.B, device=self.device, **solver_kw)
        self.du_lim = float(scenario.mechanicalSteeringLimit) * 2          # Scenarios.py:50
        f = dict(dtype=torch.float64, device=self.device)
        self.L = torch.tensor([float(a) + float(b) for a, b in zip(scenario.Lf, scenario.Lr)], **f)
        self.control = torch.full((self.B, self.nV, self.ticks_total + 1), float("nan"), **f)
        self.state = torch.zeros((self.B, self.nV, 6), **f)
        self.last_path = None          # [B, nV, tps + 1, 6] of the previous step
        self.u_prev = None
        self.trace = trace      # keep every step's solve inputs and per-SCP-iteration trace
        self.out = self.solver.alloc_out(self.B, trace=trace)
        self.history = []

    def reset(self, x_init, noise=None):
        """main.py:73-75: vehiclePathFullRes[:, v, 0] = x0; the control path holds
        scenario.u0 for the first ticks_delay_u + ticks_per_sim + 1 ticks."""
        x = torch.as_tensor(np.asarray(x_init, float) if not isinstance(x_init, torch.Tensor)
                            else x_init, dtype=torch.float64, device=self.device)
        if tuple(x.shape) != (self.B, self.nV, 6):
            raise ValueError("x_init must be [B, nVeh, 6]")
        self.state.copy_(x)
        self.x_init = x.clone()
        self.control.fill_(float("nan"))
        u0 = torch.tensor([float(u) for u in self.sc.u0], dtype=torch.float64, device=self.device)
        self.control[:, :, 0:self.tdu + self.tps + 1] = u0[None, :, None]
        self.noise = None if noise is None else torch.as_tensor(noise, dtype=torch.float64,
                                                                device=self.device)
        self.last_path = None
        self.u_prev = None
        self.history = []
        self.i = 0

    def _obstacle_prediction(self, tick_meas):
        """Iter.obstacleFutureTrajectories (MPC_Iter.py:45-51) from the constant-velocity
        obstacle state at the measurement tick (main.py:61-71, 123); the same for every
        realisation.  Returns a device tensor [B, nObst, 2, Hp] or None."""
        if not self.nO:
            return None
        sc, ob = self.sc, self.obstacles
        t_meas = tick_meas * sc.tick_length
        x = t_meas * ob[:, 3] * np.cos(ob[:, 2]) + ob[:, 0]
        y = t_meas * ob[:, 3] * np.sin(ob[:, 2]) + ob[:, 1]
        lead = sc.delay_x + sc.dt + sc.delay_u
        step = ((np.arange(self.Hp) + 1) * sc.dt + lead)[None, :] * ob[:, 3:4]   # [nO, Hp]
        fut = np.zeros((self.nO, 2, self.Hp))
        fut[:, 0] = step * np.cos(ob[:, 2:3]) + x[:, None]
        fut[:, 1] = step * np.sin(ob[:, 2:3]) + y[:, None]
        t = torch.as_tensor(fut, dtype=torch.float64, device=self.device)
        return t[None].expand(self.B, -1, -1, -1).contiguous()

    def _held_command(self, tick_now):
        return held_command_tick(tick_now, self.tdx, self.tdu, self.tps, self.ticks_total)

    def step(self):
        i, sc, B, nV, Hp, tps = self.i, self.sc, self.B, self.nV, self.Hp, self.tps
        f = dict(dtype=torch.float64, device=self.device)
        if self.timing:
            torch.cuda.synchronize(self.device)
        t_step = time.perf_counter()
        tick_now = i * tps
        # measured state: tick_now - ticks_delay_x (inside the previous step's path)
        if self.tdx == 0 or self.last_path is None:
            x_meas = self.state
        else:
            x_meas = self.last_path[:, :, tps - min(self.tdx, tick_now), :].contiguous()
        speed = self.state[:, :, 3]
        umax = torch.minimum(torch.full_like(speed, float(sc.mechanicalSteeringLimit)),
                             torch.atan(LATERAL_ACC_LIMIT * self.L[None, :] / speed ** 2))
        src = self._held_command(tick_now)
        u_hold = torch.zeros((B, nV), **f) if src is None else self.control[:, :, src].contiguous()
        # IterClass delay compensation (MPC_Iter.py:24-33)
        horizon = sc.delay_x + sc.dt + sc.delay_u
        x0, dtraj = PL.delay_compensate(self.params, x_meas.contiguous(), u_hold, horizon,
                                        noise=self.noise, h_max=self.h_max, device=self.device)
        # SCP solve, warm-started from the previous controller output (SCP_controller.py:42-43)
        obst = self._obstacle_prediction(max(0, tick_now - self.tdx))
        u_warm = self.u_prev
        out = self.solver.solve(x0, u_hold, u_warm=u_warm, obst=obst, out=self.out)
        self.u_prev = out.u.clone()
        if self.timing:
            torch.cuda.synchronize(self.device)
        t_ctrl = time.perf_counter() - t_step
        U = out.u.clone()
        PL.clip_controls(U, u_hold, umax, nV, Hp, self.du_lim)
        # actuator-delayed control path (main.py:176-182)
        sl = np.arange(i * tps + 1 + self.tdu + tps, (i + 1) * tps + 1 + self.tdu + tps)
        sl[sl >= self.ticks_total] = self.ticks_total
        sl_t = torch.as_tensor(np.unique(sl), device=self.device)
        first = U.view(B, nV, -1)[:, :, 0]
        self.control[:, :, sl_t] = first[:, :, None].expand(B, nV, len(sl_t))
        # plant over [i dt, (i+1) dt]: output k reads control tick ceil(t_k / tick) + 1
        timelist = np.linspace(i * sc.dt, (i + 1) * sc.dt, tps + 1)
        idx = [min(self.ticks_total, math.ceil(t / sc.tick_length) + 1) for t in timelist]
        u_tick = self.control[:, :, torch.as_tensor(idx, device=self.device)].contiguous()
        path = PL.plant_step(self.params, self.state, u_tick, sc.tick_length, noise=self.noise,
                             h_max=self.h_max, device=self.device)
        self.last_path = path
        self.state = path[:, :, tps, :].contiguous()
        rec = dict(x0=x0, u0=u_hold, umax=umax, U=U, traj=out.traj.clone(),
                   n_scp=out.n_scp.clone(), status=out.status.clone())
        if self.evaluate:
            # main.py:201-202: evaluateInOriginalProblem on the clipped U and the prediction
            ref = self.solver.sample_reference(x0)
            rec["ref"] = ref
            rec["evaluation"] = evaluate_in_original_problem(
                sc, U.view(B, nV, Hp).transpose(1, 2), rec["traj"], ref, obst)
        if self.keep_path:
            rec["path"] = path
            rec["delay_traj"] = dtraj
            rec["u_tick"] = u_tick
            rec["x_start"] = path[:, :, 0, :]
        if self.trace:
            rec["u_warm"] = u_warm
            rec["obst"] = obst
            # kept on the host (a diagnostic mode: c2 at B = 1024 would hold ~106 MB per
            # step on the device), up to the largest SCP count of the step; iterations
            # past a problem's own n_scp stay NaN as on the device
            ns = int(out.n_scp.max().item())
            tr = torch.full((B,) + tuple(out.trace.shape[1:]), float("nan"), dtype=out.trace.dtype)
            tr[:, :ns] = out.trace[:, :ns].cpu()
            rec["trace"] = tr
            rec["u"] = out.u.clone()
        if self.timing:
            torch.cuda.synchronize(self.device)
        rec["controllerRuntime"] = t_ctrl               # batch latency: every realisation
        rec["stepTime"] = time.perf_counter() - t_step   # of the batch shares it
        self.history.append(rec)
        self.i += 1
        return rec

    def run(self, n_steps):
        for _ in range(n_steps):
            self.step()
        return self.history

    def result_for_plot(self, b):
        """``result_for_plot1`` of main.py:213-225 for realisation b, the dict
        draw_video.py:44-56 reads back, as numpy arrays over the steps run so far
        (needs keep_path=True and evaluate=True).  Unset path ticks stay NaN and
        unrun steps zero, as main.py initialises them (main.py:56-62).  Timing fields
        are the batch's per-step wall times (meaningful with timing=True)."""
        if not self.keep_path or not self.evaluate:
            raise ValueError("result_for_plot needs keep_path=True and evaluate=True")
        sc, nV, Hp, tps = self.sc, self.nV, self.Hp, self.tps
        Nsim, T = int(sc.Nsim), self.ticks_total
        veh = np.full((6, nV, T + 1), np.nan)
        veh[:, :, 0] = self.x_init[b].cpu().numpy().T
        obs = np.zeros((self.nO, 2, T + 1))
        if self.nO:
            t = np.arange(T + 1) * sc.tick_length                       # main.py:61-71
            ob = self.obstacles
            obs[:, 0] = t[None] * (ob[:, 3] * np.cos(ob[:, 2]))[:, None] + ob[:, 0:1]
            obs[:, 1] = t[None] * (ob[:, 3] * np.sin(ob[:, 2]))[:, None] + ob[:, 1:2]
        out = dict(
            vehiclePathFullRes=veh, obstaclePathFullRes=obs,
            controlPathFullRes=self.control[b].cpu().numpy(),
            controlPredictions=np.zeros((Hp, nV, Nsim)),
            trajectoryPredictions=np.zeros((Hp, 2, nV, Nsim)),
            initial_pos=np.zeros((2, nV, Nsim)),
            ReferenceTrajectory=np.zeros((Hp, 2, nV, Nsim)),
            MPC_delay_compensation_trajectory=np.zeros((PL.DELAY_STEPS, 6, nV, Nsim)),
            evaluations_obj_value=[float(r["evaluation"]["predictionObjectiveValue"][b])
                                   for r in self.history],
            controllerRuntime=np.zeros((Nsim, 1)), stepTime=np.zeros((Nsim, 1)))
        for i, r in enumerate(self.history[:Nsim]):
            lo = tps * i + 1
            hi = min(T + 1, tps * (i + 1) + 1)
            veh[:, :, lo:hi] = r["path"][b, :, 1:1 + hi - lo].cpu().numpy().transpose(2, 0, 1)
            out["controlPredictions"][:, :, i] = r["U"][b].view(nV, Hp).T.cpu().numpy()
            out["trajectoryPredictions"][:, :, :, i] = r["traj"][b].cpu().numpy()
            out["initial_pos"][:, :, i] = r["x0"][b, :, 0:2].T.cpu().numpy()
            out["ReferenceTrajectory"][:, :, :, i] = r["ref"][b].cpu().numpy()
            out["MPC_delay_compensation_trajectory"][:, :, :, i] = r["delay_traj"][b].cpu().numpy()
            out["controllerRuntime"][i, 0] = r["controllerRuntime"]
            out["stepTime"][i, 0] = r["stepTime"]
        return out

    def dump_result(self, fp, b):
        """json.dump of result_for_plot(b) with main.py:226-231's encoding (nested
        lists, NaN written as NaN)."""
        res = self.result_for_plot(b)
        json.dump({k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in res.items()}, fp)

    def close(self):
        self.solver.close()
