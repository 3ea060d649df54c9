"""Drop-in for the reference's ``MPC_Iter.py`` (MPC_Iter.py:1-150).

``IterClass``  per-MPC-step preprocessing (MPC_Iter.py:13-55): delay
               compensation by integrating the plant over delay_x + dt + delay_u
               on the GPU (``scpqp_delay_compensate``, fixed-step RK4 in place
               of the reference's odeint), reference sampling on the GPU
               (``scpqp_sample_reference``), constant-velocity obstacle
               prediction.
``MPCclass``   discretisation + prediction + cost matrices (MPC_Iter.py:59-149).
               Ad, Bd, Ed, the Toeplitz blocks C A^m B, the constant term and
               Psi_0 come from one ``scpqp_linearize`` launch (8x8 Pade-13
               expm per vehicle on the GPU).  The remaining reference-format
               attributes (Mathcal_A, Mathcal_C, Phi_0, gamma_0) are
               reassembled on the host from those device outputs; the SCP
               solve itself never reads them.
"""
from math import sqrt

import numpy as np

from Scenarios import Indices

DELAY_STEPS = 10      # MPC_Iter.py:21
NOISE_STD = 0.000003  # Model.py:84-86


def delay_compensate(scenario, x_measured, u_path):
    """Integrate each vehicle from its measured state with the last commanded
    steering for delay_x + dt + delay_u (MPC_Iter.py:24-33).
    Returns x0 [nVeh, nx], u0 [nVeh, nu], trajectory [DELAY_STEPS, nx, nVeh]."""
    nV, nx, nu = scenario.nVeh, scenario.model.nx, scenario.model.nu
    horizon = scenario.delay_x + scenario.dt + scenario.delay_u
    assert u_path.shape[1] * scenario.tick_length - horizon < 1e-10
    from scpqp import plant
    params = plant.plant_params(scenario.Lf, scenario.Lr)
    x_meas = np.asarray(x_measured, float).reshape(1, nV, nx)
    u_hold = np.asarray(u_path, float)[:, -1].reshape(1, nV)
    x0d, trajd = plant.delay_compensate(params, x_meas, u_hold, horizon, n_out=DELAY_STEPS)
    u0 = u_hold.reshape(nV, nu).copy()
    return x0d[0].cpu().numpy(), u0, trajd[0].cpu().numpy()


def predict_obstacles(scenario, obstacleState):
    """Obstacle centres over the horizon, shifted by the delays (MPC_Iter.py:45-51).
    Returns [nObst, 2, Hp]."""
    idx = Indices()
    obs = np.asarray(scenario.obstacles, dtype=float).reshape(scenario.nObst, -1)
    speed, heading = obs[:, idx.speed], obs[:, idx.heading]
    lead = scenario.delay_x + scenario.dt + scenario.delay_u
    t = (np.arange(1, scenario.Hp + 1) * scenario.dt + lead)[None, :]
    out = np.zeros([scenario.nObst, 2, scenario.Hp])
    out[:, idx.x, :] = t * (speed * np.cos(heading))[:, None] + obstacleState[:, idx.x][:, None]
    out[:, idx.y, :] = t * (speed * np.sin(heading))[:, None] + obstacleState[:, idx.y][:, None]
    return out


class IterClass:
    def __init__(self, scenario, x_measured, u_path, obstacleState, uMax):
        from scpqp.dropin import solver_for
        self.x0, self.u0, self.MPC_delay_compensation_trajectory = delay_compensate(
            scenario, x_measured, u_path)
        # ReferenceTrajectoryPoints [Hp, 2, nVeh] from the device sampler
        solver = solver_for(scenario)
        ref = solver.sample_reference(self.x0[None], hp=np.array([scenario.Hp], np.int32))
        self.ReferenceTrajectoryPoints = ref[0, :scenario.Hp].cpu().numpy()
        if scenario.nObst:
            self.obstacleFutureTrajectories = predict_obstacles(scenario, obstacleState)
        self.uMax = uMax
        self.reset = 0


class MPCclass:
    """Discretisation and MPC matrices of all vehicles (MPC_Iter.py:59-97)."""

    def __init__(self, scenario, Iter):
        from scpqp.dropin import solver_for
        nx, nu, ny = scenario.model.nx, scenario.model.nu, scenario.model.ny
        nV, Hp, Hu = scenario.nVeh, scenario.Hp, scenario.Hu
        assert Hu <= Hp
        assert nu == 1 and Hu == Hp, "the device path implements nu = 1, Hu = Hp (main.py:47)"
        # process noise of Model.ode inside comp_jacobian (Model.py:84-86), drawn once per step
        if getattr(scenario.model, "is_noise", False):
            self.ec_noise = np.random.normal(0, NOISE_STD, (nV, 2))
        else:
            self.ec_noise = np.zeros((nV, 2))
        self._scenario = scenario
        self._Iter = Iter
        solver = solver_for(scenario)
        lin = solver.linearize(Iter.x0[None], Iter.u0.reshape(1, nV), self.ec_noise[None],
                               obst=self._obst(scenario, Iter),
                               ref_points=Iter.ReferenceTrajectoryPoints[None])
        lin = {k: v[0].cpu().numpy() for k, v in lin.items()}
        self.lin = lin
        Ad, Bd, Ed = lin["Ad"], lin["Bd"], lin["Ed"]        # [nV,6,6], [nV,6], [nV,6]
        g = lin["g"][:, :Hp]                                  # [nV, Hp, 2]  C A^m B
        ct = lin["const_term"][:, :Hp]                        # [nV, Hp, 2]

        self.A = np.repeat(np.transpose(Ad, (1, 2, 0))[:, :, None, :], Hp, axis=2)
        self.B = np.repeat(np.transpose(Bd, (1, 0))[:, None, None, :], Hp, axis=2)
        self.E = np.repeat(np.transpose(Ed, (1, 0))[:, None, :], Hp, axis=1)
        self.Mathcal_A = np.zeros([ny * Hp, nx, nV])
        self.Mathcal_B = np.zeros([ny * Hp, nu * Hu, nV])
        self.Mathcal_C = np.zeros([ny * Hp, 1, nV])
        self.Phi_0 = np.zeros([nu * Hu, nu * Hu, nV])
        self.Psi_0 = np.zeros([nu * Hu, 1, nV])
        self.gamma_0 = np.zeros([1, nV])
        self.const_term = np.zeros([ny * Hp, 1, nV])
        self.Reference = np.zeros([Hp * ny, nV])
        for v in range(nV):
            self.Reference[:, v] = Iter.ReferenceTrajectoryPoints[:, :ny, v].reshape(-1)
            self.const_term[:, 0, v] = ct[v].reshape(-1)
            for i in range(Hp):
                for j in range(i + 1):
                    self.Mathcal_B[ny * i:ny * (i + 1), j, v] = g[v, i - j]
            # C A^(i+1) and sum_{j<=i} C A^j E from the device Ad / Ed
            P = np.eye(nx)
            acc = np.zeros(ny)
            for i in range(Hp):
                acc = acc + (P @ Ed[v])[:ny]
                P = Ad[v] @ P
                self.Mathcal_A[ny * i:ny * (i + 1), :, v] = P[:ny]
                self.Mathcal_C[ny * i:ny * (i + 1), 0, v] = acc
            Qm = np.full(ny * Hp, float(scenario.Q[v]))
            Qm[ny * (Hp - 1):] = scenario.Q_final[v]
            Mb = self.Mathcal_B[:, :, v]
            H = Mb.T @ (Qm[:, None] * Mb) + scenario.R[v] * np.eye(nu * Hu)
            self.Phi_0[:, :, v] = 0.5 * (H + H.T)
            self.Psi_0[:, 0, v] = lin["psi0"][v, :Hp]
            err = self.Reference[:, v] - self.const_term[:, 0, v]
            self.gamma_0[0, v] = err @ (Qm * err)

    @staticmethod
    def _obst(scenario, Iter):
        if not scenario.nObst:
            return None
        return np.asarray(Iter.obstacleFutureTrajectories, dtype=float)[None]
