"""Drop-in for the reference's ``SCP_controller.py`` (SCP_controller.py:1-400).

``SCPcontroller(scenario, Iter, prevOutput).SCP_controller(Iter)`` runs the
whole sequential-convex-programming loop — constraint linearisation, the
convexified QP with slack, QCQP evaluation and the stopping rule
(SCP_controller.py:74-197) — in ONE launch of the HIP kernel through the
C-ABI (``scpqp_solve``).  ``QCQP_evaluate`` and ``forward_U`` run the device
evaluator (``scpqp_evaluate``).  There is no host solver: without the HIP
library these calls raise.

What differs from the reference, on purpose:

* the QP backend is the kernel's interior point method + active-set polish
  instead of cvxpy/GUROBI (the QP is strictly convex, so the minimiser is the
  same to solver tolerance);
* ``optimization_log`` holds every per-iteration list of the reference
  (SCP_controller.py:88-90, 169-189: 'P', 'q', 'Aineq', 'bineq', 'lb', 'ub',
  'x', 'slack', 'SCP_ObjVal', 'QCQP_ObjVal', 'delta_hat', 'delta', 'u',
  'feasible', 'prev_u', 'Traj', 'U', 'prevTraj', 'prevU'), rebuilt from the
  kernel's per-iteration trace, plus per-solve counters (SCP/IPM iterations,
  status flags).  The trace rows of the solve are copied to the host with the
  result; the lists are decoded from them on first access (``_LazyLog``), so
  the dense row rebuild stays out of ``optimizerTime``.  The decode holds host
  arrays only (no controller, no device tensors): a log can be copied or
  pickled (the copy is the decoded plain dict).  'Traj'/'prevTraj' are the
  predicted positions ``const_term + Mathcal_B u`` of forward_U, evaluated on
  the host from the same linearisation;
* the dense ``qcqp`` dictionary (QCQP_formulate, SCP_controller.py:278-341) is
  built lazily, only if a caller reads ``.qcqp``; the solve uses the
  factored forms on the device.
* nVeh == 1 and the last SCP iterate infeasible: the reference's retry
  (SCP_controller.py:51-66) builds an (n x n) warm start and cannot run
  (SURVEY B.9); here the result is flagged ``resultInvalid``.
"""
import functools
import time

import numpy as np

from Config import Config
from MPC_Iter import MPCclass

cfg = Config()

ST_INVALID = 2      # SCPQP_ST_INVALID


class _LazyLog(dict):
    """optimization_log whose per-iteration lists are decoded from the host copy of
    the device trace the first time any key beyond the counters is read (or the log is
    iterated, copied, compared, printed or pickled)."""

    def __init__(self, counters, decode):
        super().__init__(counters)
        self._decode = decode

    def copy(self):
        self._fill()
        return dict(self)

    def __reduce__(self):
        self._fill()
        return (dict, (dict(self),))

    def __repr__(self):
        self._fill()
        return super().__repr__()

    def __eq__(self, other):
        self._fill()
        return super().__eq__(other)

    def __ne__(self, other):
        self._fill()
        return super().__ne__(other)

    __hash__ = None

    def pop(self, k, *default):
        self._fill()
        return super().pop(k, *default)

    def popitem(self):
        self._fill()
        return super().popitem()

    def setdefault(self, k, default=None):
        self._fill()
        return super().setdefault(k, default)

    def update(self, *a, **kw):
        self._fill()
        return super().update(*a, **kw)

    def _fill(self):
        if self._decode is not None:
            dec, self._decode = self._decode, None
            super().update(dec())

    def __getitem__(self, k):
        if not super().__contains__(k):
            self._fill()
        return super().__getitem__(k)

    def __contains__(self, k):
        self._fill()
        return super().__contains__(k)

    def get(self, k, default=None):
        self._fill()
        return super().get(k, default)

    def __iter__(self):
        self._fill()
        return super().__iter__()

    def __len__(self):
        self._fill()
        return super().__len__()

    def keys(self):
        self._fill()
        return super().keys()

    def items(self):
        self._fill()
        return super().items()

    def values(self):
        self._fill()
        return super().values()


SLACK_WEIGHT = 1e5          # psi_omega_weight, SCP_controller.py:84
OMEGA_UB = 1e25             # upper_bound_omega, SCP_controller.py:85


def _iteration_log(trace, n_scp, nV, nO, Hp, hp_max, u_lim, Mb, const_term, Phi_0, Psi_0,
                   gamma0):
    """The reference's per-iteration optimization_log lists (SCP_controller.py:88-90,
    169-189) from the host copy of one problem's device trace.
    * P = blkdiag(2 Phi0, 0), q = [Psi0; 1e5], lb = [-uLim; 0], ub = [uLim; 1e25]
      (:117-127; the same arrays every iteration, as the reference appends them);
    * Aineq / bineq: dense rows from the factored ones and the Toeplitz blocks (:93-128);
    * x = [u; slack], SCP_ObjVal = fval = 1/2 x'Px + q'x + gamma0 (:146, :158);
    * slack = x[-1] as a shape-(1,) array, like the reference's u_var[-1] (:148);
    * delta_hat = (obj_0 + 1e5 maxviol_0) - fval (:159), with the merit obj_0 + 1e5
      maxviol_0 before the iteration as the kernel recorded it (trace header [8]);
    * Traj / U, prevTraj / prevU: forward_U of u and of the linearisation point (:183-187):
      positions const_term + Mathcal_B u, U = u per vehicle [Hp, nu, nVeh]."""
    from scpqp import trace as TR
    N = nV * Hp
    g = np.stack([Mb[0::2, 0, v] for v in range(nV)], 0)        # g_k x-components
    g = np.stack([g, np.stack([Mb[1::2, 0, v] for v in range(nV)], 0)], -1)
    its = TR.decode(trace, n_scp, nV, nO, Hp, hp_max, g=g, u_lim=u_lim)
    Phi0 = np.zeros((N, N))
    Psi0 = np.zeros(N)
    for v in range(nV):
        sl = slice(v * Hp, (v + 1) * Hp)
        Phi0[sl, sl] = Phi_0[:, :, v]
        Psi0[sl] = Psi_0[:, 0, v]
    P = np.zeros((N + 1, N + 1))
    P[:N, :N] = 2 * Phi0
    q = np.vstack([Psi0.reshape(-1, 1), [[SLACK_WEIGHT]]])
    lb = np.vstack([-np.ones((N, 1)) * u_lim, [[0.0]]])
    ub = np.vstack([np.ones((N, 1)) * u_lim, [[OMEGA_UB]]])

    def forward_U(uu):
        U = uu.reshape(nV, Hp).T[:, None, :].copy()                # [Hp, nu, nVeh]
        traj = np.stack([const_term[:, 0, v] + Mb[:, :, v] @ uu[v * Hp:(v + 1) * Hp]
                         for v in range(nV)], -1).reshape(Hp, 2, nV)
        return traj, U

    log = {k: [] for k in ('P', 'q', 'Aineq', 'bineq', 'lb', 'ub', 'x', 'slack', 'SCP_ObjVal',
                           'QCQP_ObjVal', 'delta_hat', 'delta', 'u', 'feasible', 'prev_u', 'Traj',
                           'U', 'prevTraj', 'prevU', 'ipm_iters')}
    for d in its:
        uu = d['z'][:-1]
        fval = float(uu @ Phi0 @ uu + Psi0 @ uu + SLACK_WEIGHT * d['slack'] + gamma0)
        log['P'].append(P)
        log['q'].append(q)
        log['Aineq'].append(d['A'])
        log['bineq'].append(d['b'].reshape(-1, 1))
        log['lb'].append(lb)
        log['ub'].append(ub)
        log['x'].append(d['z'].reshape(-1, 1))
        log['slack'].append(np.array([d['slack']]))
        log['SCP_ObjVal'].append(fval)
        log['QCQP_ObjVal'].append(np.array([[d['obj']]]))
        log['delta_hat'].append(d['merit0'] - fval)
        log['delta'].append(d['delta'])
        log['u'].append(uu.reshape(-1, 1))
        log['feasible'].append(d['feasible'])
        log['prev_u'].append(d['u_lin'].reshape(-1, 1))
        for key, vec in (('', uu), ('prev', d['u_lin'])):
            traj, U = forward_U(vec)
            log[key + 'Traj'].append(traj)
            log[key + 'U'].append(U)
        log['ipm_iters'].append(d['ipm_iters'])
    log['trace'] = its          # decoded kernel records (max_violation per iteration, rows)
    return log


class SCPcontroller:
    def __init__(self, scenario, Iter, prevOutput):
        from scpqp.dropin import solver_for
        self.scenario = scenario
        self.Iter = Iter
        self.prevOutput = prevOutput
        self.nu = scenario.model.nu
        self.ny = scenario.model.ny
        self.Hp = scenario.Hp
        self.nVeh = scenario.nVeh
        self.nObst = scenario.nObst
        self.dsafeExtra = scenario.dsafeExtra
        self.scenario_uLim = scenario.uLim
        self.solver = solver_for(scenario)
        self.mpc = MPCclass(scenario, Iter)
        self._qcqp = None
        self.u = np.zeros([self.nVeh * self.Hp, 1])

    # ------------------------------------------------------------------ device inputs
    def _inputs(self):
        it = self.Iter
        obst = None
        if self.nObst:
            obst = np.asarray(it.obstacleFutureTrajectories, dtype=float)[None]
        return dict(x0=it.x0[None], u0=it.u0.reshape(1, self.nVeh),
                    ec_noise=self.mpc.ec_noise[None], obst=obst,
                    ref_points=it.ReferenceTrajectoryPoints[None])

    # ------------------------------------------------------------------ SCP_controller.py:40-72
    def SCP_controller(self, Iter):
        self.Iter = Iter
        if self.prevOutput and ('u' in self.prevOutput):
            self.u = self.prevOutput['u'].reshape([self.Hp * self.nVeh, 1], order='F')
        controllerOutput = {'resultInvalid': False}
        timer = time.time()
        self.u, feasible, _, controllerOutput['optimization_log'] = self.SCP_optimizer(self.u)
        if self.nVeh == 1 and not feasible:
            controllerOutput['resultInvalid'] = True
        if controllerOutput['optimization_log']['status'] == ST_INVALID:
            controllerOutput['resultInvalid'] = True
        controllerOutput['u'] = self.u
        trajectoryPrediction, U = self.forward_U(self.u)
        U = np.squeeze(U[:, 0, :])
        controllerOutput['optimizerTime'] = time.time() - timer
        return U, trajectoryPrediction, controllerOutput

    def SCP_optimizer(self, u_approx):
        """The full SCP loop on the device (SCP_controller.py:74-197).
        Returns (u, feasible, objective, log)."""
        if abs(u_approx[0, 0]) < np.spacing(1):     # in place, like the reference (:75-76)
            u_approx[0] = np.spacing(1)
        res = self.solver.solve(u_warm=np.asarray(u_approx, float).reshape(1, -1), trace=True,
                                **self._inputs())
        u = res.u[0, :self.nVeh * self.Hp].cpu().numpy().reshape(-1, 1)
        status = int(res.status[0].item())
        n_scp = int(res.n_scp[0].item())
        # only the n_scp trace rows this solve wrote come to the host (the whole
        # trace_iters-row record, ~600 KB at 8 vehicles and Hp 30, went to a fresh pinned
        # buffer every solve); the decode runs only when the log is read
        tr_host = res.trace[0, :n_scp].cpu().numpy()
        m = self.mpc
        # the decode's inputs, host arrays only (the trace rows of this solve and the
        # linearisation): the log keeps neither the controller nor device tensors alive
        dec = functools.partial(_iteration_log, tr_host, n_scp,
                                self.nVeh, self.nObst, self.Hp, self.solver.hp_max,
                                self.scenario_uLim, m.Mathcal_B.copy(), m.const_term.copy(),
                                m.Phi_0.copy(), m.Psi_0.copy(), float(np.sum(m.gamma_0)))
        log = _LazyLog({'status': status & 0xff, 'flags': status & ~0xff,
                        'n_scp': n_scp, 'n_ipm': int(res.n_ipm[0].item()),
                        'obj': float(res.obj[0].item()),
                        'max_violation': float(res.max_violation[0].item()),
                        'sum_violations': float(res.sum_violations[0].item())}, dec)
        self._last_traj = res.traj[0, :self.Hp].cpu().numpy()
        return u, bool(res.feasible[0].item()), float(res.obj[0].item()), log

    # ------------------------------------------------------------------ SCP_controller.py:199-213
    def forward_U(self, u):
        """(Traj [Hp, ny, nVeh], U [Hp, nu, nVeh]) of a stacked control vector."""
        u = np.asarray(u, dtype=float).reshape(-1)
        U = u.reshape([self.nVeh, self.Hp]).T[:, None, :].copy()
        ev = self._evaluate(u)
        return ev['traj'], U

    # ------------------------------------------------------------------ SCP_controller.py:215-265
    def _evaluate(self, u):
        r = self.solver.evaluate(np.asarray(u, float).reshape(1, -1), **self._inputs())
        Hp = self.Hp
        return dict(obj=float(r['obj'][0].item()), maxv=float(r['max_violation'][0].item()),
                    sumv=float(r['sum_violations'][0].item()), feas=bool(r['feasible'][0].item()),
                    cveh=r['c_veh'][0, :, :, :Hp].cpu().numpy(),
                    cobs=r['c_obs'][0, :, :self.nObst, :Hp].cpu().numpy(),
                    traj=r['traj'][0, :Hp].cpu().numpy())

    def QCQP_evaluate(self, U):
        """(feasible, objValue, feasibilityScore, feasibilityScoreGradient,
        max_violation, sum_violations, constraintValuesVehicle, constraintValuesObstacle)."""
        u = np.asarray(U, dtype=float).reshape(-1)
        ev = self._evaluate(u)
        score, grad = self._feasibility_score(u, ev)
        return (ev['feas'], np.array([[ev['obj']]]), score, grad, ev['maxv'], ev['sumv'],
                ev['cveh'], ev['cobs'])

    def _feasibility_score(self, u, ev):
        """Penalty score c_quad * sum max(ci, 0)^2 and its gradient
        (SCP_controller.py:216-258), from the device constraint values and
        predicted positions; the obstacle terms repeat as the reference's
        nesting makes them."""
        c_quad = 1e9
        nV, Hp, nO = self.nVeh, self.Hp, self.nObst
        m = self.mpc
        Phi0 = np.zeros((nV * Hp, nV * Hp))
        Psi0 = np.zeros(nV * Hp)
        for v in range(nV):
            sl = slice(v * Hp, (v + 1) * Hp)
            Phi0[sl, sl] = m.Phi_0[:, :, v]
            Psi0[sl] = m.Psi_0[:, 0, v]
        score = np.array([[ev['obj']]])
        grad = (2 * Phi0 @ u + Psi0).reshape(-1, 1)
        pos = ev['traj']                                   # [Hp, 2, nV]
        Mb = m.Mathcal_B                                   # [2Hp, Hp, nV]

        def jac(v, k):                                     # d p_v,k / d u_v  -> [2, Hp]
            return Mb[2 * k:2 * k + 2, :, v]

        for v in range(nV):
            for k in range(Hp):
                for v2 in range(v + 1, nV):
                    ci = ev['cveh'][v, v2, k]
                    score = score + c_quad * max(ci, 0) ** 2
                    if ci > 0:
                        d = pos[k, :, v] - pos[k, :, v2]
                        grad[v * Hp:(v + 1) * Hp, 0] += 2 * c_quad * ci * (-2 * jac(v, k).T @ d)
                        grad[v2 * Hp:(v2 + 1) * Hp, 0] += 2 * c_quad * ci * (2 * jac(v2, k).T @ d)
                    for o in range(nO):
                        co = ev['cobs'][v, o, k]
                        score = score + c_quad * max(co, 0) ** 2
                        if co > 0:
                            d = pos[k, :, v] - self.Iter.obstacleFutureTrajectories[o, :, k]
                            grad[v * Hp:(v + 1) * Hp, 0] += 2 * c_quad * co * (-2 * jac(v, k).T @ d)
        return score, grad

    # ------------------------------------------------------------------ SCP_controller.py:278-341
    @property
    def qcqp(self):
        if self._qcqp is None:
            self._qcqp = self.QCQP_formulate(self.scenario)
        return self._qcqp

    def QCQP_formulate(self, scenario):
        """Dense quadratic-constraint tensors in the reference's layout, built
        from the device linearisation (compatibility only)."""
        nV, Hp, nO, ny = self.nVeh, self.Hp, self.nObst, self.ny
        n = nV * Hp
        m = self.mpc
        Phi0 = np.zeros([n, n])
        Psi0 = np.zeros([n, 1])
        gamma0 = 0
        Phi = np.zeros([nV - 1, nV, Hp, n, n])
        Psi = np.zeros([nV - 1, nV, Hp, n, 1])
        gamma = np.zeros([nV - 1, nV, Hp])
        Phi_o = np.zeros([nV, nO, Hp, n, n])
        Psi_o = np.zeros([nV, nO, Hp, n, 1])
        gamma_o = np.zeros([nV, nO, Hp])
        for v in range(nV):
            s1 = slice(v * Hp, (v + 1) * Hp)
            Phi0[s1, s1] = m.Phi_0[:, :, v]
            Psi0[s1, 0] = m.Psi_0[:, 0, v]
            gamma0 = gamma0 + m.gamma_0[:, v]
            for k in range(Hp):
                rows = slice(k * ny, (k + 1) * ny)
                J1 = m.Mathcal_B[rows, :, v]
                for v2 in range(v + 1, nV):
                    s2 = slice(v2 * Hp, (v2 + 1) * Hp)
                    J2 = m.Mathcal_B[rows, :, v2]
                    Phi[v, v2, k, s1, s1] = -J1.T @ J1
                    Phi[v, v2, k, s2, s2] = -J2.T @ J2
                    Phi[v, v2, k, s1, s2] = J1.T @ J2
                    Phi[v, v2, k, s2, s1] = J2.T @ J1
                    b = m.const_term[rows, 0, v] - m.const_term[rows, 0, v2]
                    Psi[v, v2, k, s1, 0] = -2 * J1.T @ b
                    Psi[v, v2, k, s2, 0] = 2 * J2.T @ b
                    gamma[v, v2, k] = (scenario.dsafeVehicles[v, v2] + self.dsafeExtra) ** 2 - b @ b
                for o in range(nO):
                    Phi_o[v, o, k, s1, s1] = -J1.T @ J1
                    b = m.const_term[rows, 0, v] - self.Iter.obstacleFutureTrajectories[o, :, k]
                    Psi_o[v, o, k, s1, 0] = -2 * J1.T @ b
                    gamma_o[v, o, k] = (scenario.dsafeObstacles[v, o] + self.dsafeExtra) ** 2 - b @ b
        Phi = 0.5 * (Phi + np.swapaxes(Phi, -1, -2))
        Phi_o = 0.5 * (Phi_o + np.swapaxes(Phi_o, -1, -2))
        Phi[np.abs(Phi) <= 1e-30] = 0
        Psi[np.abs(Psi) <= 1e-30] = 0
        return {'Phi0': Phi0, 'Psi0': Psi0, 'gamma0': gamma0, 'Phi': Phi, 'Psi': Psi,
                'gamma': gamma, 'Phi_o': Phi_o, 'Psi_o': Psi_o, 'gamma_o': gamma_o}

    # ------------------------------------------------------------------ SCP_controller.py:343-400
    def evaluateInOriginalProblem(self, controlPrediction, trajectoryPrediction, options):
        sc, it = self.scenario, self.Iter
        nV, Hp, nO = self.nVeh, self.Hp, self.nObst
        ev = {}
        err2 = (it.ReferenceTrajectoryPoints - trajectoryPrediction) ** 2
        ev['predictionObjectiveValueX'] = sum(
            sc.Q[v] * err2[:-1, :, v].sum() + sc.Q_final[v] * err2[-1, :, v].sum() for v in range(nV))
        ctrl = np.asarray(controlPrediction, dtype=float).reshape(Hp, -1)[:Hp, :]
        ev['predictionObjectiveValueU'] = sum(sc.R[v] * (ctrl[:, v] ** 2).sum() for v in range(nV))
        ev['predictionObjectiveValue'] = ev['predictionObjectiveValueX'] + ev['predictionObjectiveValueU']

        u = ctrl.reshape(-1, 1, order='F')
        (ev['predictionFeasibleQCQP'], _, _, _, _, _, ev['constraintValuesVehicleQCQP'],
         ev['constraintValuesObstacleQCQP']) = self.QCQP_evaluate(u)

        tol = cfg.QCQP.constraintTolerance
        cv = np.zeros([nV, nV, Hp])
        feasible = True
        if nO:
            co = np.zeros([nV, nO, Hp])
        for k in range(Hp):
            for v in range(nV):
                for v2 in range(v + 1, nV):
                    d2 = ((trajectoryPrediction[k, :, v] - trajectoryPrediction[k, :, v2]) ** 2).sum()
                    ci = sc.dsafeVehicles[v, v2] ** 2 - d2
                    cv[v, v2, k] = cv[v2, v, k] = ci
                    feasible = feasible and not ci > tol
                for o in range(nO):
                    d2 = ((trajectoryPrediction[k, :, v] - it.obstacleFutureTrajectories[o, :, k]) ** 2).sum()
                    ci = sc.dsafeObstacles[v, o] ** 2 - d2
                    co[v, o, k] = ci
                    feasible = feasible and not ci > tol
        ev['constraintValuesVehicle_trajPred'] = cv
        ev['predictionFeasible_trajPred'] = feasible
        if nO:
            ev['constraintValuesObstacle_trajPred'] = co
        # the reference tests hasattr() on a dict, which is always False (:391)
        if not hasattr(options, 'ignoreQCQPcheck'):
            if ev['predictionFeasibleQCQP'] != feasible:
                print('feasibility criteria disagree\n')
        ev['predictionFeasible'] = feasible
        ev['constraintValuesVehicle'] = cv
        if nO:
            ev['constraintValuesObstacle'] = co
        return ev
