"""Drop-in for the reference's ``Scenarios.py`` (Scenarios.py:1-255):
time base, limits, vehicle/obstacle registries, the three scenario builders,
tick rounding and pairwise safety distances.  Host-side configuration; the
GPU solver reads the completed scenario once per handle.

Build choice: the reference reads ``scenario.uLim``
(SCP_controller.py:34) but never defines it; here ``uLim`` is the mechanical
steering limit 3 deg unless set explicitly.
"""
from math import cos, floor, pi, sin, sqrt

import numpy as np

from Model import BicyleModel, DefaultVehicle


def round_up(value):
    """Round half-up for tick arithmetic (Scenarios.py:7-9)."""
    return round(value + 0.00000001)


class DefaultObstacle:
    """Rotated rectangle moving with constant speed (Scenarios.py:12-22)."""

    def __init__(self):
        self.x = 0
        self.y = 0
        self.heading = 0
        self.speed = 0
        self.length = 2
        self.width = 2


class Indices:
    """State / obstacle row indices (Scenarios.py:24-37)."""

    def __init__(self):
        self.x = 0
        self.y = 1
        self.heading = 2
        self.speed = 3
        self.acceleration = 4
        self.length = 4
        self.width = 5


class Scenario:
    def __init__(self, is_noise):
        self.tick_length = 0.01          # [s]
        self.T_end = 20                  # [s]
        self.delay_x = 0                 # measurement delay [s]
        self.delay_u = .03               # actuation delay [s]
        self.dt = 0.4                    # MPC sample time [s]
        self.Hp = 10                     # prediction horizon
        self.Hu = 10                     # control horizon
        self.lateralAccelerationLimit = 9.81 / 2
        self.mechanicalSteeringLimit = pi / 180 * 3
        self.duLim = self.mechanicalSteeringLimit * 2
        self.model = BicyleModel(is_noise)
        self.nVeh = 0
        self.dsafeExtra = 1
        self.Q, self.Q_final, self.R = [], [], []
        self.Lf, self.Lr = [], []
        self.Length, self.Width, self.RVeh = [], [], []
        self.x0, self.u0 = [], []
        self.referenceTrajectories = []
        self.obstacles = []
        self.plotLimits = 5 * np.array([[-10, 10], [-10, 10]])
        self._uLim = None

    # build choice B.7 (see module docstring)
    @property
    def uLim(self):
        return self.mechanicalSteeringLimit if self._uLim is None else self._uLim

    @uLim.setter
    def uLim(self, value):
        self._uLim = value

    @property
    def nObst(self):
        return len(self.obstacles)

    @nObst.setter
    def nObst(self, value):
        # complete_scenario assigns nObst; the obstacle list stays authoritative
        pass

    def addVehicle(self, vehicle):
        self.model.makeInitState(vehicle)
        self.x0.append(self.model.makeInitStateVector)
        self.nVeh += 1
        self.Q.append(vehicle.Q)
        self.Q_final.append(vehicle.Q_final)
        self.R.append(vehicle.R)
        self.RVeh.append(np.linalg.norm(np.array([vehicle.Length, vehicle.Width]), 2) / 2)
        self.Lf.append(vehicle.Lf)
        self.Lr.append(vehicle.Lr)
        self.Width.append(vehicle.Width)
        self.Length.append(vehicle.Length)
        self.u0.append(vehicle.u0)
        self.referenceTrajectories.append(vehicle.referenceTrajectory)

    def addObstacle(self, obstacle):
        row = [obstacle.x, obstacle.y, obstacle.heading, obstacle.speed, obstacle.length,
               obstacle.width]
        self.obstacles.append(np.array(row, dtype=float).reshape(-1, 1))

    # -- scenario builders -------------------------------------------------------------
    def get_circle_scenario(self, angles):
        """Vehicles on a circle of radius 30 m driving through the centre (Scenarios.py:109-125)."""
        radius = 30
        for angle in angles:
            s, c = sin(angle), cos(angle)
            veh = DefaultVehicle()
            veh.labelOffset = np.array([[3, -3]]) @ np.array([[c, s], [-s, c]]) + np.array([[-2, 0]])
            veh.x_start = -c * radius
            veh.y_start = -s * radius
            veh.heading = angle
            veh.referenceTrajectory = np.array([[-c * radius, -s * radius], [c * radius, s * radius]])
            self.addVehicle(veh)
        self.plotLimits = 1.1 * radius * np.array([[-1, 1], [-1, 1]])
        if len(angles) == 2 and max(abs(sin(a)) for a in angles) < 0.1:
            self.plotLimits[1, :] = np.array([[-6, 6]])

    def get_frog_scenario(self):
        """One vehicle crossing two columns of moving obstacles (Scenarios.py:127-146)."""
        veh = DefaultVehicle()
        veh.x_start = -18
        veh.referenceTrajectory = np.array([[-100, 0], [100, 0]])
        self.addVehicle(veh)
        for o in range(-2, 9):
            for column_x in (7, 14):
                ob = DefaultObstacle()
                ob.x, ob.y = column_x, 9 * o - 15
                ob.speed, ob.heading = 2, pi / 2
                ob.length, ob.width = 4, 2
                self.addObstacle(ob)
        self.obstacles = np.array(self.obstacles)
        self.plotLimits = 35 * np.array([[-1, 1], [-1, 1]])

    def get_parallel_scenario(self, nVeh):
        """Vehicles in parallel lanes past four static obstacles (Scenarios.py:148-201)."""
        lane = np.arange(nVeh) - floor(nVeh / 2)
        evens = list(range(0, nVeh, 2))[::-1]
        order = evens + list(range(1, nVeh, 2))
        positions = np.zeros(nVeh)
        positions[order] = lane
        for i in range(nVeh):
            y = 3 * positions[i]
            veh = DefaultVehicle()
            veh.x_start, veh.y_start = -37, y
            veh.labelOffset = np.array([-6.1 - 4.5 * np.mod(positions[i] - 1, 2), 0])
            veh.referenceTrajectory = np.array([[-30, y], [30, y]])
            self.addVehicle(veh)
        for (x, y, ln, wd) in ((-15, 5, 2, 4), (-2, -7, 4, 2), (10, 5, 4, 2), (20, -7, 2, 2)):
            ob = DefaultObstacle()
            ob.x, ob.y, ob.length, ob.width = x, y, ln, wd
            self.addObstacle(ob)
        if nVeh == 2:
            self.CouplingAdjacencyMatrixPB = np.array([[0, 1], [0, 0]]) > 0
        elif nVeh > 2:
            self.CouplingAdjacencyMatrixPB = np.diag(range(nVeh - 1), 2) > 0
            self.CouplingAdjacencyMatrixPB[0, 1] = True
        self.plotLimits = np.array([[-50, 50], [-20, 20]])
        self.obstacles = np.array(self.obstacles)

    # -- completion ---------------------------------------------------------------------
    def complete_scenario(self):
        """Round time constants to ticks, fill safety distances (Scenarios.py:204-227)."""
        self.ticks_per_sim = round_up(self.dt / self.tick_length)
        self.dt = self.ticks_per_sim * self.tick_length
        self.Nsim = round_up(self.T_end / self.dt)
        self.T_end = self.Nsim * self.dt
        self.ticks_total = int(round_up(self.T_end / self.tick_length))
        self.ticks_delay_x = round_up(self.delay_x / self.tick_length)
        self.delay_x = self.ticks_delay_x * self.tick_length
        self.ticks_delay_u = round_up(self.delay_u / self.tick_length)
        self.delay_u = self.ticks_delay_u * self.tick_length
        self.calculate_All_Safety_Distances()
        n = self.nVeh
        if not hasattr(self, "CooperationCoefficientMatrix"):
            self.CooperationCoefficientMatrix = np.ones([n, n])
        lower = (np.triu(np.ones([n, n]), 0) == 0).astype(int)
        if not hasattr(self, "CouplingAdjacencyMatrixCoop"):
            self.CouplingAdjacencyMatrixCoop = lower
        if not hasattr(self, "CouplingAdjacencyMatrixPB"):
            self.CouplingAdjacencyMatrixPB = lower.copy()

    def calculate_All_Safety_Distances(self):
        """dsafe = sqrt((chord/2)^2 + (sum of half diagonals)^2) (Scenarios.py:229-252)."""
        idx = Indices()
        n, no = self.nVeh, self.nObst
        self.dsafeVehicles = np.zeros([n, n])
        self.dsafeObstacles = np.zeros([n, no])
        half_diag = [sqrt((self.Length[v] / 2) ** 2 + (self.Width[v] / 2) ** 2) for v in range(n)]
        for v in range(n):
            speed_v = float(np.asarray(self.x0[v]).reshape(-1)[idx.speed])
            for w in range(n):
                speed_w = float(np.asarray(self.x0[w]).reshape(-1)[idx.speed])
                chord = (speed_v + speed_w) * self.dt
                self.dsafeVehicles[v, w] = sqrt((chord / 2) ** 2 + (half_diag[v] + half_diag[w]) ** 2)
            for o in range(no):
                ob = np.asarray(self.obstacles[o], dtype=float).reshape(-1)
                chord = (speed_v + ob[idx.speed]) * self.dt
                r_ob = sqrt((ob[idx.length] / 2) ** 2 + (ob[idx.width] / 2) ** 2)
                self.dsafeObstacles[v, o] = sqrt((chord / 2) ** 2 + (half_diag[v] + r_ob) ** 2)
