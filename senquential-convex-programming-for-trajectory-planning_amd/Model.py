"""Drop-in for the reference's ``Model.py``: vehicle defaults and the kinematic
bicycle model (Model.py:8-117).

``BicyleModel.ode`` / ``odes_`` are the plant right-hand side the reference
integrates on the host (delay compensation, MPC_Iter.py:25-33; plant
simulation, main.py:185) — they stay host functions here too.  The Jacobian
linearisation the SCP hot path needs runs on the GPU inside the solve kernel;
``comp_jacobian`` is kept for API compatibility and mirrors Model.py:45-59.
"""
from math import atan, cos, sin, sqrt, tan

import numpy as np


class DefaultVehicle:
    """Default geometry, speed and MPC weights of one vehicle (Model.py:8-30)."""

    def __init__(self):
        self.u0 = 0                      # initial steering angle [rad]
        self.x_start = 0                 # [m]
        self.y_start = 0                 # [m]
        self.heading = 0                 # [rad]
        # piecewise-linear desired path, rows (x, y) [m]
        self.referenceTrajectory = np.array([[0, 0], [1, 0], [3, 1]])
        self.speed = 4                   # [m/s]
        self.acceleration = 0            # [m/s^2]
        self.Length = .98                # bumper to bumper [m]
        self.Width = .88                 # [m]
        self.Lf = .34                    # centre to front axle [m]
        self.Lr = .34                    # centre to rear axle [m]
        self.Q = 1                       # trajectory deviation weight
        self.Q_final = 20                # weight of the last prediction step
        self.R = 4000                    # steering weight
        self.labelOffset = np.array([[0, 0]])


class BicyleModel:
    """Kinematic bicycle with first-order steering actuator, state
    [x, y, heading, v_rear, a, delta], input delta_ref (Model.py:33-117)."""

    def __init__(self, is_noise):
        self.nx = 6
        self.nu = 1
        self.ny = 2
        self.is_noise = is_noise

    def makeInitState(self, veh):
        self.makeInitStateVector = np.array(
            [veh.x_start, veh.y_start, veh.heading, veh.speed, veh.acceleration, 0],
            dtype=float).reshape(-1, 1)

    # -- right-hand side -------------------------------------------------------------
    def _rhs(self, x, u_ref, Lf, Lr):
        L = Lf + Lr
        rho = Lr / L
        t = tan(x[5])
        beta = atan(rho * t)
        vc = x[3] * sqrt(1 + (rho * t) ** 2)   # centre speed from rear-axle speed
        dx = np.array(x, dtype=float).copy()
        dx[0] = vc * cos(x[2] + beta)
        dx[1] = vc * sin(x[2] + beta)
        dx[2] = vc * t * cos(beta) / L
        dx[3] = x[4]
        dx[4] = 0
        dx[5] = (u_ref - x[5]) / 0.1            # steering actuator, T = 0.1 s
        if self.is_noise:
            dx[0] += np.random.normal(0, 0.000003)
            dx[1] += np.random.normal(0, 0.000003)
        return dx

    def ode(self, x, t, u_ref, Lf, Lr):
        """odeint signature f(x, t, ...) (Model.py:61-87)."""
        return self._rhs(x, float(np.asarray(u_ref).reshape(-1)[0]), Lf, Lr)

    def odes_(self, t, x, u_ref, Lf, Lr):
        """scipy ``ode`` signature f(t, x, ...) (Model.py:89-115)."""
        return self._rhs(x, float(np.asarray(u_ref).reshape(-1)[0]), Lf, Lr)

    def comp_jacobian(self, x, u, Lf, Lr):
        """Analytic (Ac, Bc, Cc, Ec) at (x, u) (Model.py:45-59)."""
        x = np.asarray(x, dtype=float).reshape(-1)
        L = Lf + Lr
        rho = Lr / L
        v, d = x[3], x[5]
        t = tan(d)
        sec2 = t * t + 1
        kap = sqrt(rho * rho * t * t + 1)
        th = x[2] + atan(rho * t)
        c, s = cos(th), sin(th)
        Ac = np.zeros((6, 6))
        Ac[0, 2] = -v * s * kap
        Ac[0, 3] = c * kap
        Ac[0, 5] = rho * rho * v * c * t * sec2 / kap - rho * v * s * sec2 / kap
        Ac[1, 2] = v * c * kap
        Ac[1, 3] = s * kap
        Ac[1, 5] = rho * v * c * sec2 / kap + rho * rho * v * s * t * sec2 / kap
        Ac[2, 3] = t / L
        Ac[2, 5] = v * sec2 / L
        Ac[3, 4] = 1
        Ac[5, 5] = -10
        Bc = np.array([[0], [0], [0], [0], [0], [10]], dtype=float)
        Cc = np.eye(self.ny, self.nx)
        uu = float(np.asarray(u).reshape(-1)[0])
        Ec = self.ode(x, 0, uu, Lf, Lr).reshape(-1, 1) - Ac @ x.reshape(-1, 1) - Bc * uu
        return Ac, Bc, Cc, Ec
