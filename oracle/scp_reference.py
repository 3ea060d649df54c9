"""CPU restatement of the reference SCP-QP hot path.

TEST INFRASTRUCTURE ONLY.  The product (``scpqp`` + the drop-in modules) never
imports this file; only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may, and only as the checker / the timed
CPU baseline, never as the thing that is shipped.

Parity status
-------------
The reference (Zhang-Xiaoxue/Senquential-Convex-Programming-for-Trajectory-
Planning) is pure Python.  Importing or executing it was denied in this
environment and its QP backend (cvxpy + GUROBI) is not
installed, so this module restates its algorithm from the source text.  It is
pinned by:

* analytic known-answer tests taken from the source:
  exact Jacobian, closed-form discretisation, Toeplitz structure, sampler
  sequences, scenario constants (``tests/test_oracle_known_answers.py``);
* solver-independent KKT certificates: the convexified QP has a unique
  minimiser, so any sufficiently accurate solver reproduces the
  GUROBI answer; the QP here is a dense Mehrotra interior point method followed
  by an active-set polish that solves the optimality system exactly;
* a scipy cross-check of the QP on small instances.

Two modes are provided:

``faithful``   dense tensors exactly as ``SCP_controller.QCQP_formulate``
               (SCP_controller.py:278-341), ``scipy.linalg.expm`` discretisation
               (MPC_Iter.py:99-113) and ``np.linalg.matrix_power`` prediction
               matrices (MPC_Iter.py:129-149).  Used for golden fixtures and as
               the "reference CPU path" baseline.
``structured`` the same mathematics through the factored forms:
               Toeplitz blocks ``g_m = C A^m B`` and predicted positions.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.linalg

EPS = float(np.spacing(1))          # SCP_controller.py:75
CONSTRAINT_TOL = 2 * 2.1 * 1e-3     # Config.py:18
DELTA_TOL = 1e-3                    # SCP_controller.py:83
SLACK_WEIGHT = 1e5                  # SCP_controller.py:84
MAX_SCP_ITER = 20                   # SCP_controller.py:86


# ---------------------------------------------------------------------------
# Scenario restatement (Scenarios.py:40-252, Model.py:8-30)
# ---------------------------------------------------------------------------
def _round_up(v):
    """Scenarios.py:7-9."""
    return round(v + 0.00000001)


@dataclass
class OracleScenario:
    """Plain restatement of the fields of ``Scenarios.Scenario`` the path reads."""
    tick_length: float = 0.01
    T_end: float = 20.0
    delay_x: float = 0.0
    delay_u: float = 0.03
    dt: float = 0.4
    Hp: int = 10
    Hu: int = 10
    mechanicalSteeringLimit: float = math.pi / 180 * 3
    dsafeExtra: float = 1.0
    x0: list = field(default_factory=list)      # per vehicle (6,)
    Lf: list = field(default_factory=list)
    Lr: list = field(default_factory=list)
    Q: list = field(default_factory=list)
    Q_final: list = field(default_factory=list)
    R: list = field(default_factory=list)
    Length: list = field(default_factory=list)
    Width: list = field(default_factory=list)
    u0: list = field(default_factory=list)
    referenceTrajectories: list = field(default_factory=list)
    obstacles: list = field(default_factory=list)   # rows [x y heading speed length width]

    @property
    def nVeh(self):
        return len(self.x0)

    @property
    def nObst(self):
        return len(self.obstacles)

    @property
    def uLim(self):
        # Build choice: scenario.uLim is read by SCP_controller.py:34
        # but never defined by the reference; use the mechanical limit.
        return self.mechanicalSteeringLimit

    def add_vehicle(self, x_start, y_start, heading, ref):
        # DefaultVehicle (Model.py:8-30) + Scenario.addVehicle (Scenarios.py:89-103)
        self.x0.append(np.array([x_start, y_start, heading, 4.0, 0.0, 0.0]))
        self.Lf.append(0.34)
        self.Lr.append(0.34)
        self.Q.append(1.0)
        self.Q_final.append(20.0)
        self.R.append(4000.0)
        self.Length.append(0.98)
        self.Width.append(0.88)
        self.u0.append(0.0)
        self.referenceTrajectories.append(np.asarray(ref, dtype=float))

    def complete(self):
        """Scenarios.py:204-218 (tick rounding) + safety distances."""
        self.ticks_per_sim = _round_up(self.dt / self.tick_length)
        self.dt = self.ticks_per_sim * self.tick_length
        self.Nsim = _round_up(self.T_end / self.dt)
        self.T_end = self.Nsim * self.dt
        self.ticks_total = int(_round_up(self.T_end / self.tick_length))
        self.ticks_delay_x = _round_up(self.delay_x / self.tick_length)
        self.delay_x = self.ticks_delay_x * self.tick_length
        self.ticks_delay_u = _round_up(self.delay_u / self.tick_length)
        self.delay_u = self.ticks_delay_u * self.tick_length
        self.dsafeVehicles, self.dsafeObstacles = safety_distances(self)
        return self


def circle_scenario(n_veh, Hp=10):
    """Scenarios.py:109-121 with main.py:240 angles."""
    sc = OracleScenario(Hp=Hp, Hu=Hp)
    radius = 30.0
    for i in range(n_veh):
        a = 2 * math.pi / n_veh * (i + 1)
        s, c = math.sin(a), math.cos(a)
        sc.add_vehicle(-c * radius, -s * radius, a,
                       [[-c * radius, -s * radius], [c * radius, s * radius]])
    return sc.complete()


def frog_scenario(Hp=10):
    """Scenarios.py:127-146 (1 vehicle, 22 moving obstacles)."""
    sc = OracleScenario(Hp=Hp, Hu=Hp)
    sc.add_vehicle(-18.0, 0.0, 0.0, [[-100.0, 0.0], [100.0, 0.0]])
    for o in range(-2, 9):
        for xo in (7.0, 14.0):
            sc.obstacles.append(np.array([xo, 9.0 * o - 15, math.pi / 2, 2.0, 4.0, 2.0]))
    return sc.complete()


def parallel_scenario(n_veh, Hp=10, dsafe_extra=0.9):
    """Scenarios.py:148-201 (+ main.py:250 dsafeExtra override)."""
    sc = OracleScenario(Hp=Hp, Hu=Hp, dsafeExtra=dsafe_extra)
    base = np.arange(n_veh) - (n_veh // 2)
    evens = list(range(0, n_veh, 2))[::-1]
    order = evens + list(range(1, n_veh, 2))
    pos = np.zeros(n_veh)
    pos[order] = base
    for i in range(n_veh):
        y = 3 * pos[i]
        sc.add_vehicle(-37.0, y, 0.0, [[-30.0, y], [30.0, y]])
    for (x, y, ln, wd) in ((-15, 5, 2, 4), (-2, -7, 4, 2), (10, 5, 4, 2), (20, -7, 2, 2)):
        sc.obstacles.append(np.array([x, y, 0.0, 0.0, ln, wd], dtype=float))
    return sc.complete()


def safety_distances(sc):
    """Scenarios.py:229-252."""
    nV, nO = sc.nVeh, sc.nObst
    dv = np.zeros((nV, nV))
    do = np.zeros((nV, nO))
    for v in range(nV):
        hv = math.hypot(sc.Length[v] / 2, sc.Width[v] / 2)
        for w in range(nV):
            chord = (sc.x0[v][3] + sc.x0[w][3]) * sc.dt
            rr = hv + math.hypot(sc.Length[w] / 2, sc.Width[w] / 2)
            dv[v, w] = math.sqrt((chord / 2) ** 2 + rr ** 2)
        for o in range(nO):
            ob = sc.obstacles[o]
            chord = (sc.x0[v][3] + ob[3]) * sc.dt
            rr = math.sqrt((sc.Length[v] / 2) ** 2 + (sc.Width[v] / 2) ** 2) \
                + math.sqrt((ob[4] / 2) ** 2 + (ob[5] / 2) ** 2)
            do[v, o] = math.sqrt((chord / 2) ** 2 + rr ** 2)
    return dv, do


def obstacle_future(sc, obstacle_state, Hp):
    """MPC_Iter.py:45-51: obstacle positions [nObst, 2, Hp] (constant velocity)."""
    nO = sc.nObst
    out = np.zeros((nO, 2, Hp))
    for k in range(Hp):
        for o in range(nO):
            ob = sc.obstacles[o]
            step = ((k + 1) * sc.dt + sc.delay_x + sc.dt + sc.delay_u) * ob[3]
            out[o, 0, k] = step * math.cos(ob[2]) + obstacle_state[o, 0]
            out[o, 1, k] = step * math.sin(ob[2]) + obstacle_state[o, 1]
    return out


# ---------------------------------------------------------------------------
# Vehicle model (Model.py:45-87)
# ---------------------------------------------------------------------------
def bicycle_rhs(x, u_ref, Lf, Lr, noise=(0.0, 0.0)):
    """Model.py:61-87; ``noise`` replaces the two np.random.normal draws (:84-86)."""
    L = Lf + Lr
    rho = Lr / L
    t = math.tan(x[5])
    beta = math.atan(rho * t)
    vc = x[3] * math.sqrt(1 + (rho * t) ** 2)
    dx = np.empty(6)
    dx[0] = vc * math.cos(x[2] + beta) + noise[0]
    dx[1] = vc * math.sin(x[2] + beta) + noise[1]
    dx[2] = vc * t * math.cos(beta) / L
    dx[3] = x[4]
    dx[4] = 0.0
    dx[5] = (u_ref - x[5]) / 0.1
    return dx


def bicycle_jacobian(x, u, Lf, Lr, noise=(0.0, 0.0)):
    """Model.py:45-59: analytic Ac, Bc, Cc and affine residual Ec."""
    L = Lf + Lr
    rho = Lr / L
    v, psi, d = x[3], x[2], x[5]
    t = math.tan(d)
    sec2 = t * t + 1
    kap = math.sqrt(rho * rho * t * t + 1)
    th = psi + math.atan(rho * t)
    cth, sth = math.cos(th), math.sin(th)
    Ac = np.zeros((6, 6))
    Ac[0, 2] = -v * sth * kap
    Ac[0, 3] = cth * kap
    Ac[0, 5] = rho * rho * v * cth * t * sec2 / kap - rho * v * sth * sec2 / kap
    Ac[1, 2] = v * cth * kap
    Ac[1, 3] = sth * kap
    Ac[1, 5] = rho * v * cth * sec2 / kap + rho * rho * v * sth * t * sec2 / kap
    Ac[2, 3] = t / L
    Ac[2, 5] = v * sec2 / L
    Ac[3, 4] = 1.0
    Ac[5, 5] = -10.0
    Bc = np.zeros((6, 1))
    Bc[5, 0] = 10.0
    Cc = np.eye(2, 6)
    f = bicycle_rhs(x, float(u), Lf, Lr, noise)
    Ec = f.reshape(-1, 1) - Ac @ np.asarray(x, float).reshape(-1, 1) - Bc * float(u)
    return Ac, Bc, Cc, Ec


# ---------------------------------------------------------------------------
# Discretisation + prediction (MPC_Iter.py:59-149)
# ---------------------------------------------------------------------------
def discretize(x0, u0, Lf, Lr, dt, noise=(0.0, 0.0)):
    """MPC_Iter.py:99-113 (two 7x7 expm), then E[|E|<=1e-30] = 0 (:87)."""
    Ac, Bc, Cc, Ec = bicycle_jacobian(x0, u0, Lf, Lr, noise)
    M = np.zeros((7, 7))
    M[:6, :6] = Ac
    M[:6, 6:] = Bc
    T = scipy.linalg.expm(dt * M)
    Ad, Bd = T[:6, :6].copy(), T[:6, 6:7].copy()
    M[:6, 6:] = Ec
    Ed = scipy.linalg.expm(dt * M)[:6, 6:7].copy()
    Ed[np.abs(Ed) <= 1e-30] = 0.0
    return Ad, Bd, Cc, Ed


def prediction_matrices(A, B, C, E, Hp, Hu):
    """MPC_Iter.py:129-149: calA (2Hp x 6), calC (2Hp x 1), calB (2Hp x Hu)."""
    assert Hu <= Hp
    pw = [C @ np.eye(6)]
    acc = [C @ np.eye(6)]
    for i in range(1, Hp + 1):
        pw.append(C @ np.linalg.matrix_power(A, i))
        acc.append(pw[i] + acc[i - 1])
    calA = np.zeros((2 * Hp, 6))
    calC = np.zeros((2 * Hp, 1))
    calB = np.zeros((2 * Hp, Hu))
    for i in range(Hp):
        calA[2 * i:2 * i + 2] = pw[i + 1]
        calC[2 * i:2 * i + 2] = acc[i] @ E
        for j in range(i + 1):
            calB[2 * i:2 * i + 2, j:j + 1] = pw[i - j] @ B
    return calA, calC, calB


def cost_matrices(calB, const, reference, Qw, Rw, Qf, Hp, Hu):
    """MPC_Iter.py:116-127."""
    Q = Qw * np.eye(2 * Hp)
    Q[2 * Hp - 2, 2 * Hp - 2] = Qf
    Q[2 * Hp - 1, 2 * Hp - 1] = Qf
    R = Rw * np.eye(Hu)
    err = reference.reshape(-1, 1) - const
    M = calB.T @ Q @ calB + R
    Phi0 = 0.5 * (M + M.T)
    Psi0 = -2 * calB.T @ Q @ err
    gamma0 = float((err.T @ Q @ err)[0, 0])
    return Phi0, Psi0, gamma0


# ---------------------------------------------------------------------------
# Reference sampler (SampleReferTraj.py:8-122), quirks B.1-B.3 reproduced
# ---------------------------------------------------------------------------
def _project2d(x1, y1, x2, y2, x3, y3):
    """SampleReferTraj.py:81-122."""
    b = math.sqrt((x2 - x1) ** 2 + (y2 - y1) ** 2)
    if b != 0:
        xn, yn = (x2 - x1) / b, (y2 - y1) / b
        x31, y31 = x3 - x1, y3 - y1
        dot = xn * x31 + yn * y31
        dist = xn * y31 - yn * x31
        return x1 + dot * xn, y1 + dot * yn, dist, dot / b, b
    return x1, y1, math.sqrt((x3 - x1) ** 2 + (y3 - y1) ** 2), 0.0, b


def shortest_distance(cx, cy, x, y, strict_xor_quirk=True):
    """SampleReferTraj.py:34-79.  Returns (signed_dist, arclength, xp, yp, index).

    Quirk B.2: the minimum is seeded with curve point 1 and index 2.  The
    ``^`` at :70 raises TypeError on floats; with ``strict_xor_quirk`` we raise
    the same way, otherwise the intended ``**`` is used.
    """
    n = len(cx)
    assert n >= 2
    arc = 0.0
    xm, ym = cx[1], cy[1]
    arc_min = 0.0
    dmin = math.sqrt((x - cx[1]) ** 2 + (y - cy[1]) ** 2)
    imin = 2
    for j in range(1, n):
        xp, yp, sd, lam, plen = _project2d(cx[j - 1], cy[j - 1], cx[j], cy[j], x, y)
        if (0 < lam or j == 1) and (lam < 1 or j == n - 1):
            if abs(sd) < abs(dmin):
                xm, ym, dmin = xp, yp, sd
                arc_min = arc + lam * plen
                imin = j
        else:
            if strict_xor_quirk:
                raise TypeError("unsupported operand type(s) for ^: 'float' and 'int'")
            d_end = math.sqrt((x - cx[j]) ** 2 + (y - cy[j]) ** 2)
            if abs(d_end) < abs(dmin):
                xm, ym = cx[j], cy[j]
                dmin = math.copysign(d_end, sd) if sd != 0 else 0.0
                arc_min = arc + plen
                imin = j
        arc += plen
    return dmin, arc_min, xm, ym, imin


def sample_reference(n_samples, ref, vx, vy, step, strict_xor_quirk=True):
    """SampleReferTraj.py:8-32 (including the B.1 alternation past the end)."""
    ref = np.asarray(ref, dtype=float)
    out = np.zeros((n_samples, 2))
    _, _, x, y, idx = shortest_distance(ref[:, 0], ref[:, 1], float(vx), float(vy),
                                        strict_xor_quirk)
    npc = ref.shape[0]
    cur = np.array([x, y])
    for i in range(npc - 1):
        assert np.linalg.norm(ref[i + 1] - ref[i]) > step
    for i in range(n_samples):
        rem = np.linalg.norm(cur - ref[idx])
        if rem > step or idx == npc:
            d = ref[idx] - ref[idx - 1]
            cur = cur + step * d / np.linalg.norm(d)
        else:
            cur = ref[idx].copy()
            idx = min(idx, npc - 1)
            d = ref[idx] - ref[idx - 1]
            cur = cur + (step - rem) * d / np.linalg.norm(d)
        out[i] = cur
    return out


# ---------------------------------------------------------------------------
# Problem container
# ---------------------------------------------------------------------------
@dataclass
class Problem:
    """One joint SCP problem: what IterClass hands to SCPcontroller."""
    x0: np.ndarray            # [nVeh, 6]  delay-compensated state (Iter.x0)
    u0: np.ndarray            # [nVeh]     Iter.u0
    ref_points: np.ndarray    # [Hp, 2, nVeh] Iter.ReferenceTrajectoryPoints
    obst: np.ndarray          # [nObst, 2, Hp] Iter.obstacleFutureTrajectories
    ec_noise: np.ndarray      # [nVeh, 2] the two noise draws of Model.py:85-86
    Lf: np.ndarray
    Lr: np.ndarray
    Q: np.ndarray
    Q_final: np.ndarray
    R: np.ndarray
    dsafe_veh: np.ndarray     # [nVeh, nVeh]
    dsafe_obs: np.ndarray     # [nVeh, nObst]
    dsafe_extra: float
    u_lim: float
    dt: float
    Hp: int

    @property
    def nVeh(self):
        return self.x0.shape[0]

    @property
    def nObst(self):
        return self.obst.shape[0]


def reference_points(sc, x0, Hp, strict_xor_quirk=True):
    """MPC_Iter.py:35-43: RefPts[Hp, 2, nVeh] (stepSize = x0[v,3]*dt, quirk B.3)."""
    out = np.zeros((Hp, 2, sc.nVeh))
    for v in range(sc.nVeh):
        out[:, :, v] = sample_reference(Hp, sc.referenceTrajectories[v], x0[v, 0], x0[v, 1],
                                        x0[v, 3] * sc.dt, strict_xor_quirk)
    return out


def make_problem(sc, x0, u0=None, ec_noise=None, Hp=None, obst=None, ref_points=None):
    Hp = sc.Hp if Hp is None else Hp
    nV = sc.nVeh
    x0 = np.asarray(x0, float).reshape(nV, 6)
    u0 = np.zeros(nV) if u0 is None else np.asarray(u0, float).reshape(nV)
    ec = np.zeros((nV, 2)) if ec_noise is None else np.asarray(ec_noise, float).reshape(nV, 2)
    if obst is None:
        obst = np.zeros((sc.nObst, 2, Hp))
        if sc.nObst:
            st = np.array([[o[0], o[1]] for o in sc.obstacles])
            obst = obstacle_future(sc, st, Hp)
    if ref_points is None:
        ref_points = reference_points(sc, x0, Hp)
    return Problem(x0=x0, u0=u0, ref_points=np.asarray(ref_points, float), obst=np.asarray(obst, float),
                   ec_noise=ec, Lf=np.array(sc.Lf, float), Lr=np.array(sc.Lr, float),
                   Q=np.array(sc.Q, float), Q_final=np.array(sc.Q_final, float),
                   R=np.array(sc.R, float), dsafe_veh=np.asarray(sc.dsafeVehicles, float),
                   dsafe_obs=np.asarray(sc.dsafeObstacles, float).reshape(nV, sc.nObst),
                   dsafe_extra=float(sc.dsafeExtra), u_lim=float(sc.uLim), dt=float(sc.dt), Hp=int(Hp))


# ---------------------------------------------------------------------------
# Linearisation of one problem (MPCclass, MPC_Iter.py:59-97)
# ---------------------------------------------------------------------------
@dataclass
class Linearisation:
    Ad: np.ndarray       # [nVeh, 6, 6]
    Bd: np.ndarray       # [nVeh, 6]
    Ed: np.ndarray       # [nVeh, 6]
    calB: np.ndarray     # [nVeh, 2Hp, Hp]
    const: np.ndarray    # [nVeh, 2Hp]   const_term
    g: np.ndarray        # [nVeh, Hp, 2] Toeplitz generators g_m = C A^m B
    Phi0: np.ndarray     # [nVeh, Hp, Hp]
    Psi0: np.ndarray     # [nVeh, Hp]
    gamma0: np.ndarray   # [nVeh]


def linearise(p: Problem, mode="faithful"):
    nV, Hp = p.nVeh, p.Hp
    Ad = np.zeros((nV, 6, 6)); Bd = np.zeros((nV, 6)); Ed = np.zeros((nV, 6))
    calB = np.zeros((nV, 2 * Hp, Hp)); const = np.zeros((nV, 2 * Hp)); g = np.zeros((nV, Hp, 2))
    Phi0 = np.zeros((nV, Hp, Hp)); Psi0 = np.zeros((nV, Hp)); gamma0 = np.zeros(nV)
    for v in range(nV):
        A, B, C, E = discretize(p.x0[v], p.u0[v], p.Lf[v], p.Lr[v], p.dt, tuple(p.ec_noise[v]))
        Ad[v], Bd[v], Ed[v] = A, B[:, 0], E[:, 0]
        if mode == "faithful":
            cA, cC, cB = prediction_matrices(A, B, C, E, Hp, Hp)
            calB[v] = cB
            const[v] = (cA @ p.x0[v].reshape(-1, 1) + cC)[:, 0]
            for m in range(Hp):
                g[v, m] = cB[2 * m:2 * m + 2, 0]
        else:
            # state-space recursions: x_{k+1} = A x_k + E, g_m = C A^m B
            xs = p.x0[v].copy()
            b = B[:, 0].copy()
            for k in range(Hp):
                xs = A @ xs + E[:, 0]
                const[v, 2 * k:2 * k + 2] = xs[:2]
                g[v, k] = b[:2]
                b = A @ b
            for i in range(Hp):
                for j in range(i + 1):
                    calB[v, 2 * i:2 * i + 2, j] = g[v, i - j]
        ref = p.ref_points[:, :, v].reshape(-1)     # [x0 y0 x1 y1 ...] (MPC_Iter.py:83-84)
        Phi0[v], ps, gamma0[v] = cost_matrices(calB[v], const[v].reshape(-1, 1), ref,
                                               p.Q[v], p.R[v], p.Q_final[v], Hp, Hp)
        Psi0[v] = ps[:, 0]
    return Linearisation(Ad, Bd, Ed, calB, const, g, Phi0, Psi0, gamma0)


# ---------------------------------------------------------------------------
# Dense QCQP (SCP_controller.py:278-341) and its evaluation (:215-265)
# ---------------------------------------------------------------------------
@dataclass
class DenseQCQP:
    Phi0: np.ndarray
    Psi0: np.ndarray
    gamma0: float
    Phi: np.ndarray      # [nVeh-1, nVeh, Hp, N, N]
    Psi: np.ndarray      # [nVeh-1, nVeh, Hp, N]
    gamma: np.ndarray    # [nVeh-1, nVeh, Hp]
    Phi_o: np.ndarray    # [nVeh, nObst, Hp, N, N]
    Psi_o: np.ndarray
    gamma_o: np.ndarray


def qcqp_formulate(p: Problem, lin: Linearisation):
    nV, Hp, nO = p.nVeh, p.Hp, p.nObst
    N = nV * Hp
    Phi0 = np.zeros((N, N)); Psi0 = np.zeros(N); gamma0 = 0.0
    Phi = np.zeros((max(nV - 1, 0), nV, Hp, N, N))
    Psi = np.zeros((max(nV - 1, 0), nV, Hp, N))
    gam = np.zeros((max(nV - 1, 0), nV, Hp))
    Phio = np.zeros((nV, nO, Hp, N, N)); Psio = np.zeros((nV, nO, Hp, N)); gamo = np.zeros((nV, nO, Hp))
    for v in range(nV):
        s1 = slice(Hp * v, Hp * (v + 1))
        Phi0[s1, s1] = lin.Phi0[v]
        Psi0[s1] = lin.Psi0[v]
        gamma0 = gamma0 + lin.gamma0[v]
        for k in range(Hp):
            rows = slice(2 * k, 2 * k + 2)
            Bv = lin.calB[v][rows]
            for w in range(v + 1, nV):
                s2 = slice(Hp * w, Hp * (w + 1))
                Bw = lin.calB[w][rows]
                Phi[v, w, k, s1, s1] = -Bv.T @ Bv
                Phi[v, w, k, s2, s2] = -Bw.T @ Bw
                Phi[v, w, k, s1, s2] = Bv.T @ Bw
                Phi[v, w, k, s2, s1] = Bw.T @ Bv
                b = lin.const[v][rows] - lin.const[w][rows]
                Psi[v, w, k, s1] = -2 * Bv.T @ b
                Psi[v, w, k, s2] = 2 * Bw.T @ b
                gam[v, w, k] = (p.dsafe_veh[v, w] + p.dsafe_extra) ** 2 - b @ b
            for o in range(nO):
                Phio[v, o, k, s1, s1] = -Bv.T @ Bv
                b = lin.const[v][rows] - p.obst[o, :, k]
                Psio[v, o, k, s1] = -2 * Bv.T @ b
                gamo[v, o, k] = (p.dsafe_obs[v, o] + p.dsafe_extra) ** 2 - b @ b
    for v in range(nV):
        for k in range(Hp):
            for w in range(v + 1, nV):
                Phi[v, w, k] = 0.5 * (Phi[v, w, k] + Phi[v, w, k].T)
            for o in range(nO):
                Phio[v, o, k] = 0.5 * (Phio[v, o, k] + Phio[v, o, k].T)
    Phi[np.abs(Phi) <= 1e-30] = 0.0
    Psi[np.abs(Psi) <= 1e-30] = 0.0
    return DenseQCQP(Phi0, Psi0, gamma0, Phi, Psi, gam, Phio, Psio, gamo)


@dataclass
class Evaluation:
    feasible: bool
    obj: float
    max_violation: float
    sum_violations: float
    c_veh: np.ndarray    # [nVeh, nVeh, Hp] (-inf where not evaluated)
    c_obs: np.ndarray    # [nVeh, nObst, Hp]


def qcqp_evaluate_dense(q: DenseQCQP, U, nV, Hp, nO, tol=CONSTRAINT_TOL):
    """SCP_controller.py:215-265, obstacle block nested inside the v2 loop (B.4)."""
    U = np.asarray(U, float).reshape(-1)
    obj = float(U @ q.Phi0 @ U + q.Psi0 @ U + q.gamma0)
    feasible, sv, mv = True, 0.0, 0.0
    cv = np.full((nV, nV, Hp), -np.inf)
    co = np.full((nV, nO, Hp), -np.inf)
    for v in range(nV):
        for k in range(Hp):
            for w in range(v + 1, nV):
                ci = float(U @ q.Phi[v, w, k] @ U + q.Psi[v, w, k] @ U + q.gamma[v, w, k])
                cv[v, w, k] = cv[w, v, k] = ci
                if ci > tol:
                    feasible = False
                    sv += ci
                    mv = max(mv, ci)
                for o in range(nO):
                    ci = float(U @ q.Phi_o[v, o, k] @ U + q.Psi_o[v, o, k] @ U + q.gamma_o[v, o, k])
                    co[v, o, k] = ci
                    if ci > tol:
                        feasible = False
                        sv += ci
                        mv = max(mv, ci)
    return Evaluation(feasible, obj, mv, sv, cv, co)


def linearised_rows_dense(q: DenseQCQP, u, nV, Hp, nO):
    """SCP_controller.py:93-128: Aineq (m x N+1), bineq (m)."""
    N = nV * Hp
    m = nV * (nV - 1) // 2 * Hp + nV * nO * Hp
    A = np.zeros((m, N + 1)); b = np.zeros(m)
    r = 0
    for i in range(nV - 1):
        for j in range(i + 1, nV):
            for k in range(Hp):
                Ph = q.Phi[i, j, k]
                A[r, :N] = q.Psi[i, j, k] + 2 * u @ Ph
                b[r] = -(q.gamma[i, j, k] - u @ Ph @ u)
                r += 1
    for i in range(nV):
        for o in range(nO):
            for k in range(Hp):
                Ph = q.Phi_o[i, o, k]
                A[r, :N] = q.Psi_o[i, o, k] + 2 * u @ Ph
                b[r] = -(q.gamma_o[i, o, k] - u @ Ph @ u)
                r += 1
    A[:, N] = -1.0
    A[np.abs(A) <= 1e-20] = 0.0
    return A, b


# ---------------------------------------------------------------------------
# Structured forms
# ---------------------------------------------------------------------------
def positions(lin: Linearisation, u, nV, Hp):
    """Predicted positions p[v, k, :] = const + calB u (SCP_controller.py:199-213)."""
    u = np.asarray(u, float).reshape(nV, Hp)
    P = np.zeros((nV, Hp, 2))
    for v in range(nV):
        P[v] = (lin.const[v] + lin.calB[v] @ u[v]).reshape(Hp, 2)
    return P


def row_list(nV, Hp, nO):
    """Row order of SCP_controller.py:97-114: pairs (i<j) with k innermost, then (v,o,k)."""
    rows = []
    for i in range(nV - 1):
        for j in range(i + 1, nV):
            for k in range(Hp):
                rows.append((i, j, -1, k))
    for i in range(nV):
        for o in range(nO):
            for k in range(Hp):
                rows.append((i, -1, o, k))
    return rows


def linearised_rows_structured(p: Problem, lin: Linearisation, u):
    nV, Hp, nO = p.nVeh, p.Hp, p.nObst
    N = nV * Hp
    pos = positions(lin, u, nV, Hp)
    rows = row_list(nV, Hp, nO)
    A = np.zeros((len(rows), N + 1)); b = np.zeros(len(rows))
    uu = np.asarray(u, float).reshape(nV, Hp)
    for r, (i, j, o, k) in enumerate(rows):
        if j >= 0:
            d = pos[i, k] - pos[j, k]
            D = p.dsafe_veh[i, j] + p.dsafe_extra
        else:
            d = pos[i, k] - p.obst[o, :, k]
            D = p.dsafe_obs[i, o] + p.dsafe_extra
        Bi = lin.calB[i][2 * k:2 * k + 2]
        A[r, Hp * i:Hp * (i + 1)] = -2 * d @ Bi
        if j >= 0:
            Bj = lin.calB[j][2 * k:2 * k + 2]
            A[r, Hp * j:Hp * (j + 1)] = 2 * d @ Bj
        c = D * D - d @ d
        b[r] = -c + A[r, :N] @ uu.reshape(-1)
    A[:, N] = -1.0
    return A, b


def evaluate_structured(p: Problem, lin: Linearisation, u, tol=CONSTRAINT_TOL, obst_quirk=True):
    """Same outputs as qcqp_evaluate_dense, through positions (A.4/A.5)."""
    nV, Hp, nO = p.nVeh, p.Hp, p.nObst
    uu = np.asarray(u, float).reshape(nV, Hp)
    pos = positions(lin, u, nV, Hp)
    obj = 0.0
    for v in range(nV):
        e = pos[v] - p.ref_points[:, :, v]
        w = np.full(Hp, p.Q[v]); w[-1] = p.Q_final[v]
        obj += float(np.sum(w[:, None] * e * e) + p.R[v] * uu[v] @ uu[v])
    feasible, sv, mv = True, 0.0, 0.0
    cv = np.full((nV, nV, Hp), -np.inf)
    co = np.full((nV, nO, Hp), -np.inf)
    for v in range(nV):
        for k in range(Hp):
            for w in range(v + 1, nV):
                d = pos[v, k] - pos[w, k]
                ci = (p.dsafe_veh[v, w] + p.dsafe_extra) ** 2 - d @ d
                cv[v, w, k] = cv[w, v, k] = ci
                if ci > tol:
                    feasible = False; sv += ci; mv = max(mv, ci)
            reps = (nV - 1 - v) if obst_quirk else 1
            for _ in range(reps):
                for o in range(nO):
                    d = pos[v, k] - p.obst[o, :, k]
                    ci = (p.dsafe_obs[v, o] + p.dsafe_extra) ** 2 - d @ d
                    co[v, o, k] = ci
                    if ci > tol:
                        feasible = False; sv += ci; mv = max(mv, ci)
    return Evaluation(feasible, obj, mv, sv, cv, co)


# ---------------------------------------------------------------------------
# QP: min 1/2 z'Pz + q'z  s.t.  G z <= h
#
# The reference hands this QP to cvxpy + GUROBI (SCP_controller.py:135-141).
# Its minimiser is unique, so any solver that certifies the KKT
# conditions returns the reference's answer.  Here: a Mehrotra predictor-
# corrector interior point method on the scaled problem (controls in units of
# uLim, unit-norm constraint rows), then an active-set polish that solves the
# equality-constrained optimality system on the identified active set.
# ---------------------------------------------------------------------------
IPM_TOL = 1e-10
POLISH_DELTA = 3e-7
POLISH_RHO = 1e-12
POLISH_REFINE = 40          # cap on multiplier-iteration solves per polish round
POLISH_TOL = 1e-9           # the iteration stops once max|x_k - x_{k-1}| <= tol max(1, |x_k|)


@dataclass
class QPResult:
    z: np.ndarray
    lam: np.ndarray
    iters: int
    converged: bool
    polished: bool
    certificate: dict = None          # unscaled KKT residuals (kkt_residuals)
    certified: bool = False           # certificate_scaled within the CERT_* bounds
    certificate_scaled: dict = None
    escalations: int = 0              # fallback stages qp_solve needed (0: the first polish)


def qp_matrices(Phi0, Psi0, A, b, u_lim):
    """SCP_controller.py:118-128 in inequality form.

    Rows: [Aineq (m); u <= uLim (N); -u <= uLim (N); -omega <= 0 (1)].
    The omega upper bound 1e25 (:85,127) is treated as +inf (GUROBI treats
    bounds >= 1e20 as infinite).
    """
    N = Phi0.shape[0]
    n = N + 1
    P = np.zeros((n, n)); P[:N, :N] = 2 * Phi0
    q = np.zeros(n); q[:N] = Psi0; q[N] = SLACK_WEIGHT
    I = np.eye(N)
    G = np.vstack([A, np.hstack([I, np.zeros((N, 1))]), np.hstack([-I, np.zeros((N, 1))]),
                   np.eye(1, n, N) * -1.0])
    h = np.concatenate([b, np.full(N, u_lim), np.full(N, u_lim), [0.0]])
    return P, q, G, h


def qp_scale(P, q, G, h, u_lim, N):
    """Controls in units of uLim, every constraint row scaled to unit 2-norm."""
    n = len(q)
    sv = np.ones(n); sv[:N] = u_lim
    Ps = P * sv[:, None] * sv[None, :]
    qs = q * sv
    Gs = G * sv[None, :]
    rn = np.sqrt((Gs ** 2).sum(1))
    rn[rn == 0] = 1.0
    return Ps, qs, Gs / rn[:, None], h / rn, sv, rn


def _max_step(s, ds, l, dl):
    a = np.inf
    neg = ds < 0
    if neg.any():
        a = min(a, float(np.min(-s[neg] / ds[neg])))
    neg = dl < 0
    if neg.any():
        a = min(a, float(np.min(-l[neg] / dl[neg])))
    return min(a, 1.0)


def ipm_start_omega(P, q, G, h):
    """The HIP kernel's IPM starting point (scpqp.hip ph_init_b, round 3), for the
    scaled QP of qp_matrices/qp_scale (last column omega, last row -omega <= 0):
    controls from the omega-free normal system, omega = the smallest value that
    satisfies every collision row, plus one; s = h - G x shifted positive and
    floored at a tenth of its largest entry; lam = 0.3 q_omega / mc, q_omega on
    the omega bound.  Any interior start leads the IPM to the same QP; this one
    saves 20-25 % of the cold iterations (tools/ipm_corrector_study.py)."""
    N = len(q) - 1
    Gu = G[:, :N]
    xu = np.linalg.solve(P[:N, :N] + Gu.T @ Gu, -q[:N] + Gu.T @ h)
    r = Gu @ xu - h
    col = G[:, N]
    coll = col[:-1] < 0
    om = max(0.0, float(np.max(r[:-1][coll] / -col[:-1][coll])) if coll.any() else 0.0) + 1.0
    x = np.append(xu, om)
    s = h - G @ x
    s = s + max(-1.5 * s.min(), 0.0)
    s = np.maximum(s, 0.1 * max(1.0, s.max()))
    lam = np.full(len(h), 0.3 * abs(q[N]) / len(h))
    lam[-1] = abs(q[N]) / -col[-1]
    return x, s, lam


def qp_ipm(P, q, G, h, tol=IPM_TOL, maxit=60, init="cvxopt"):
    """Mehrotra predictor-corrector IPM for inequality QPs (CVXOPT coneqp class).

    ``init``: 'cvxopt' (coneqp's default starting point and step rule) or 'omega'
    (the HIP kernel's: ipm_start_omega, the step factor max(0.99, 1 - mu) and separate
    primal and dual step lengths).  Returns (x, s, lam, iterations, status) with
    status 1 = converged, 2 = normal-matrix Cholesky broke down (end of the
    central path reached numerically), 0 = iteration cap.
    """
    mc = len(h)
    if init == "omega":
        x, s, lam = ipm_start_omega(P, q, G, h)
    else:
        x = np.linalg.solve(P + G.T @ G, -q + G.T @ h)
        s = h - G @ x
        lam = -s.copy()
        ts = -s.min()
        if ts >= -1e-8 * max(np.linalg.norm(s), 1.0):
            s = s + (1 + ts)
        tz = -lam.min()
        if tz >= -1e-8 * max(np.linalg.norm(lam), 1.0):
            lam = lam + (1 + tz)
    qn = max(1.0, np.abs(q).max()); hn = max(1.0, np.abs(h).max())
    for it in range(maxit):
        rd = P @ x + q + G.T @ lam
        rp = G @ x + s - h
        gap = s @ lam
        pobj = 0.5 * x @ P @ x + q @ x
        if (np.abs(rp).max() <= tol * hn and np.abs(rd).max() <= tol * qn
                and gap <= tol * max(1.0, abs(pobj))):
            return x, s, lam, it, 1
        mu = gap / mc
        d = lam / s
        try:
            L = np.linalg.cholesky(P + G.T @ (d[:, None] * G))
        except np.linalg.LinAlgError:
            return x, s, lam, it, 2

        def solve(rc):
            dx = scipy.linalg.cho_solve((L, True), -rd - G.T @ (d * rp - rc / s))
            ds = -rp - G @ dx
            return dx, ds, -(rc + lam * ds) / s

        dx, ds, dl = solve(s * lam)
        a = _max_step(s, ds, lam, dl)
        sigma = ((s + a * ds) @ (lam + a * dl) / mc / mu) ** 3
        dx, ds, dl = solve(s * lam + ds * dl - sigma * mu)
        # fraction to the boundary: 0.99 (coneqp); the kernel's round-3 rule max(0.99, 1 - mu)
        # goes with its starting point (scpqp.hip step_factor)
        eta = max(0.99, 1.0 - mu) if init == "omega" else 0.99
        if init == "omega":   # the kernel: separate primal and dual step lengths (update_body)
            ap = min(1.0, eta * _max_step(s, ds, np.ones_like(lam), np.zeros_like(dl)))
            ad = min(1.0, eta * _max_step(np.ones_like(s), np.zeros_like(ds), lam, dl))
            x = x + ap * dx; s = s + ap * ds; lam = lam + ad * dl
            continue
        a = min(1.0, eta * _max_step(s, ds, lam, dl))
        x = x + a * dx; s = s + a * ds; lam = lam + a * dl
    return x, s, lam, maxit, 0


POLISH_ROUNDS = 6           # active-set corrections of the polish (primal-dual active set)
POLISH_SINGLE = 80          # single-row corrections of the exact polish's safeguard (below)


def _pdas_update(G, h, act, xp, lam_act, tol=1e-9):
    """One primal-dual active-set correction: add violated inactive rows, drop
    active rows with negative multipliers.  Returns (certified, new active set).

    The IPM may stop early (normal-matrix breakdown near the end of the central
    path, or its iteration cap) with rows still undecided; {lam > s} is then a
    guess and the polish corrects it in a few rounds (Hintermueller, Ito &
    Kunisch 2002 semismooth-Newton view of active-set updates).
    """
    r = G @ xp - h
    hn = max(1.0, np.abs(h).max())
    lam_full = np.zeros(len(h)); lam_full[act] = lam_act
    viol = r > tol * hn
    neg = act & (lam_full < -tol * max(1.0, np.abs(lam_act).max() if lam_act.size else 1.0))
    if not viol.any() and not neg.any():
        return True, act
    return False, (act & ~neg) | viol


def _kkt_active(P, q, G, h, act):
    """[P G_A'; G_A 0][x; y] = [-q; h_A] (least squares if the active rows are dependent)."""
    n = len(q)
    Ga, ha = G[act], h[act]
    na = int(act.sum())
    K = np.zeros((n + na, n + na))
    K[:n, :n] = P; K[:n, n:] = Ga.T; K[n:, :n] = Ga
    rhs = np.concatenate([-q, ha])
    try:
        sol = np.linalg.solve(K, rhs)
    except np.linalg.LinAlgError:
        sol = np.linalg.lstsq(K, rhs, rcond=None)[0]
    return sol[:n], sol[n:]


def qp_polish_exact(P, q, G, h, x, s, lam, rounds=POLISH_ROUNDS, single=POLISH_SINGLE):
    """Solve [P G_A'; G_A 0][x; y] = [-q; h_A] on the active set A = {lam > s},
    correcting A until the point certifies (primal feasible, y >= 0).

    Full-swap corrections first (_pdas_update).  A plain primal-dual active-set
    iteration is not globally convergent: from a poor guess it can cycle or diverge
    (c2 problem 323, QP 1: the coneqp-start IPM broke down with one row wrongly
    active, and the swaps grew the infeasible set 14 -> 8 -> 148 rows; verdict r05).
    Safeguard: once a swap would change no fewer rows than the best state so far, go
    back to that state and correct one row at a time, the most negative multiplier
    first, else the most violated row."""
    act = lam > s
    hn = max(1.0, np.abs(h).max())
    best_n, best_act = None, act
    one_row = False
    for k in range(rounds + single):
        xp, la = _kkt_active(P, q, G, h, act)
        if not (np.all(np.isfinite(xp)) and np.all(np.isfinite(la))):
            return None
        ok, nxt = _pdas_update(G, h, act, xp, la)
        if ok:
            lam_full = np.zeros_like(lam); lam_full[act] = la
            return xp, lam_full
        n_bad = int((nxt != act).sum())
        if not one_row:
            if best_n is not None and (n_bad >= best_n or k >= rounds):
                one_row = True
                act = best_act
                continue
            if best_n is None or n_bad < best_n:
                best_n, best_act = n_bad, act
            act = nxt
            continue
        lam_full = np.zeros(len(h)); lam_full[act] = la
        act = act.copy()
        if (act & (lam_full < 0)).any() and lam_full[act].min() < -1e-9 * max(1.0, np.abs(la).max()):
            act[np.flatnonzero(act)[np.argmin(lam_full[act])]] = False
        else:
            r = G @ xp - h
            r[act] = -np.inf
            act[int(np.argmax(r))] = True
    return None


def qp_polish_regularised(P, q, G, h, x, s, lam, delta=POLISH_DELTA, rho=POLISH_RHO,
                          nref=POLISH_REFINE, rounds=POLISH_ROUNDS):
    """Proximal method-of-multipliers polish on the active set, with the same
    primal-dual active-set corrections (what the HIP kernel does).  Each round
    iterates until x stops moving (POLISH_TOL) or ``nref`` solves; only a
    converged point can certify."""
    act = lam > s
    y_all = np.where(act, lam, 0.0)
    xk = x.copy()
    L = None
    extended = False
    for _ in range(rounds):
        Ga, ha = G[act], h[act]
        y = y_all[act].copy()
        if L is None:
            try:
                L = np.linalg.cholesky(P + rho * np.eye(len(q)) + Ga.T @ Ga / delta)
            except np.linalg.LinAlgError:
                return None
        conv = False
        for k in range(nref):
            xn = scipy.linalg.cho_solve((L, True), -q - Ga.T @ y + Ga.T @ ha / delta + rho * xk)
            y = y + (Ga @ xn - ha) / delta
            step = np.abs(xn - xk).max()
            xk = xn
            if k >= 1 and step <= POLISH_TOL * max(1.0, np.abs(xk).max()):
                conv = True
                break
        if not np.all(np.isfinite(xk)):
            return None
        ok, nxt = _pdas_update(G, h, act, xk, y)
        if ok and conv:
            lam_full = np.zeros_like(lam); lam_full[act] = y
            return xk, lam_full
        y_all = np.zeros(len(h)); y_all[act] = y
        if np.array_equal(nxt, act):
            if conv or extended:
                return None          # converged on this active set but not certified: stuck
            extended = True          # same active set, still moving: one more batch (same factor)
            continue
        y_all[~nxt] = 0.0            # dropped rows leave, added rows start at y = 0
        act = nxt
        L = None
    return None


def kkt_residuals(P, q, G, h, x, lam):
    """Solver-independent certificate: stationarity, primal/dual feasibility, complementarity."""
    r = G @ x - h
    return dict(stationarity=float(np.abs(P @ x + q + G.T @ lam).max()),
                primal=float(max(r.max(), 0.0)),
                dual=float(max(-lam.min(), 0.0)),
                complementarity=float(np.abs(lam * r).max()))


# The oracle's acceptance bounds, on the scaled QP (controls in units of uLim, every
# row of unit norm; qp_scale): stationarity absolute (the slack weight 1e5 sits in q,
# so 1e-7 is 1e-12 of the largest gradient entry), primal feasibility relative to
# max(1, |h|), dual feasibility and complementarity relative to max(1, |lam|).
CERT_STATIONARITY = 1e-7
CERT_PRIMAL = 1e-9
CERT_DUAL = 1e-9
CERT_COMPLEMENTARITY = 1e-9


class UncertifiedQP(RuntimeError):
    """The oracle could not certify a QP's KKT point (qp_solve raises it rather than
    hand an uncertified answer to a parity check)."""


def certificate_scaled(Ps, qs, Gs, hs, x, lam):
    r = Gs @ x - hs
    lm = max(1.0, float(np.abs(lam).max()))
    c = dict(stationarity=float(np.abs(Ps @ x + qs + Gs.T @ lam).max()),
             primal=float(max(r.max(), 0.0)) / max(1.0, float(np.abs(hs).max())),
             dual=float(max(-lam.min(), 0.0)) / lm,
             complementarity=float(np.abs(lam * r).max()) / lm)
    c["certified"] = bool(c["stationarity"] <= CERT_STATIONARITY and c["primal"] <= CERT_PRIMAL
                          and c["dual"] <= CERT_DUAL
                          and c["complementarity"] <= CERT_COMPLEMENTARITY)
    return c


def qp_solve(P, q, G, h, u_lim, N, polish="exact", tol=IPM_TOL, require_certificate=None):
    """Scaled IPM + polish.  ``polish``: 'exact' (oracle), 'regularised' (HIP mirror), None.

    'exact' escalates until the point certifies (certificate_scaled): the coneqp-start
    IPM and the exact KKT polish; the same IPM 100x tighter; the kernel's starting point
    (ipm_start_omega) at both tolerances; the regularised polish from each of these
    points.  If none certifies it raises UncertifiedQP (``require_certificate``, default
    on for 'exact'): the parity checker never accepts an uncertified QP (verdict r05).
    'regularised' mirrors the device, including its resumed IPM, and records whether it
    certified (the device can end a QP uncertified too: SCPQP_FL_POLISH_REJECTED)."""
    Ps, qs, Gs, hs, sv, rn = qp_scale(P, q, G, h, u_lim, N)
    if require_certificate is None:
        require_certificate = polish == "exact"
    x, s, lam, it, st = qp_ipm(Ps, qs, Gs, hs, tol=tol,
                               init="omega" if polish == "regularised" else "cvxopt")
    pol = None
    escalation = 0
    if polish == "exact":
        pol = qp_polish_exact(Ps, qs, Gs, hs, x, s, lam)
        starts = [("cvxopt", 0.01 * tol), ("omega", tol), ("omega", 0.01 * tol)]
        for init, t in starts:
            if pol is not None and certificate_scaled(Ps, qs, Gs, hs, *pol)["certified"]:
                break
            escalation += 1
            x2, s2, lam2, it2, st2 = qp_ipm(Ps, qs, Gs, hs, tol=t, init=init)
            pol = qp_polish_exact(Ps, qs, Gs, hs, x2, s2, lam2)
            if pol is not None:
                x, s, lam, it, st = x2, s2, lam2, it2, st2
        if pol is None or not certificate_scaled(Ps, qs, Gs, hs, *pol)["certified"]:
            for init, t in [("cvxopt", tol)] + starts:
                escalation += 1
                x2, s2, lam2, it2, st2 = qp_ipm(Ps, qs, Gs, hs, tol=t, init=init)
                pol = qp_polish_regularised(Ps, qs, Gs, hs, x2, s2, lam2, nref=200)
                if pol is not None and certificate_scaled(Ps, qs, Gs, hs, *pol)["certified"]:
                    x, s, lam, it, st = x2, s2, lam2, it2, st2
                    break
    elif polish == "regularised":
        pol = qp_polish_regularised(Ps, qs, Gs, hs, x, s, lam)
        if pol is None and st == 1:
            # the kernel resumes a converged IPM 100x tighter when its polish does not
            # certify (scpqp.hip qp_solve_body); qp_ipm is deterministic, so a rerun
            # from the same start continues the same trajectory
            x, s, lam, it, st = qp_ipm(Ps, qs, Gs, hs, tol=0.01 * tol, init="omega")
            pol = qp_polish_regularised(Ps, qs, Gs, hs, x, s, lam)
    if pol is not None:
        x, lam = pol
    cs = certificate_scaled(Ps, qs, Gs, hs, x, lam)
    if require_certificate and not cs["certified"]:
        raise UncertifiedQP(f"QP not certified after {escalation} escalations: "
                            + ", ".join(f"{k} {v:.2e}" for k, v in cs.items() if k != "certified"))
    z = x * sv
    lam_u = lam / rn          # multipliers of the unscaled rows
    cert = kkt_residuals(P, q, G, h, z, lam_u)
    return QPResult(z, lam_u, it, st == 1, pol is not None, cert, cs["certified"], cs, escalation)


# ---------------------------------------------------------------------------
# SCP loop (SCP_controller.py:40-197)
# ---------------------------------------------------------------------------
@dataclass
class SCPResult:
    u: np.ndarray            # [nVeh*Hp] vehicle-major
    traj: np.ndarray         # [Hp, 2, nVeh]
    U: np.ndarray            # [Hp, nVeh]
    feasible: bool
    obj: float
    max_violation: float
    sum_violations: float
    n_scp: int
    n_ipm: int
    converged: bool          # stopping rule met (vs cap of 20)
    history: list            # per SCP iteration dict(u_lin, A, b, z, obj, maxviol, delta)
    lin: Linearisation = None


def forward_u(lin: Linearisation, u, nV, Hp):
    """SCP_controller.py:199-213: Traj [Hp, 2, nVeh], U [Hp, nVeh]."""
    pos = positions(lin, u, nV, Hp)
    traj = np.transpose(pos, (1, 2, 0)).copy()
    U = np.asarray(u, float).reshape(nV, Hp).T.copy()
    return traj, U


def scp_solve(p: Problem, u_warm=None, mode="faithful", max_scp=MAX_SCP_ITER,
              keep_history=False, polish="exact", obst_quirk=True):
    nV, Hp, nO = p.nVeh, p.Hp, p.nObst
    N = nV * Hp
    lin = linearise(p, mode)
    dense = qcqp_formulate(p, lin) if mode == "faithful" else None

    def evaluate(u):
        if dense is not None:
            return qcqp_evaluate_dense(dense, u, nV, Hp, nO)
        return evaluate_structured(p, lin, u, obst_quirk=obst_quirk)

    def rows(u):
        if dense is not None:
            return linearised_rows_dense(dense, u, nV, Hp, nO)
        return linearised_rows_structured(p, lin, u)

    Phi0 = np.zeros((N, N)); Psi0 = np.zeros(N)
    for v in range(nV):
        Phi0[Hp * v:Hp * (v + 1), Hp * v:Hp * (v + 1)] = lin.Phi0[v]
        Psi0[Hp * v:Hp * (v + 1)] = lin.Psi0[v]
    u = np.zeros(N) if u_warm is None else np.array(u_warm, float).reshape(N).copy()
    if abs(u[0]) < EPS:           # SCP_controller.py:75-76 (B.5)
        u[0] = EPS
    ev = evaluate(u)
    obj0, mv0 = ev.obj, ev.max_violation
    hist = []
    n_ipm = 0
    it = 0
    conv = False
    for it in range(max_scp):
        A, b = rows(u)
        P, q, G, h = qp_matrices(Phi0, Psi0, A, b, p.u_lim)
        res = qp_solve(P, q, G, h, p.u_lim, N, polish=polish)
        n_ipm += res.iters
        u_lin = u
        u = res.z[:N].copy()
        ev = evaluate(u)
        delta = (obj0 + SLACK_WEIGHT * mv0) - (ev.obj + SLACK_WEIGHT * ev.max_violation)
        obj0, mv0 = ev.obj, ev.max_violation
        if keep_history:
            hist.append(dict(u_lin=u_lin, A=A, b=b, z=res.z.copy(), obj=ev.obj,
                             maxviol=ev.max_violation, delta=delta, ipm_iters=res.iters,
                             polished=res.polished, certificate=res.certificate,
                             certified=res.certified, certificate_scaled=res.certificate_scaled,
                             escalations=res.escalations))
        if nV == 1 and abs(delta) < DELTA_TOL and ev.max_violation > CONSTRAINT_TOL:
            conv = True
            break
        if abs(delta) < DELTA_TOL and ev.max_violation <= CONSTRAINT_TOL:
            conv = True
            break
    traj, U = forward_u(lin, u, nV, Hp)
    return SCPResult(u=u, traj=traj, U=U, feasible=ev.feasible, obj=ev.obj,
                     max_violation=ev.max_violation, sum_violations=ev.sum_violations,
                     n_scp=it + 1, n_ipm=n_ipm, converged=conv, history=hist, lin=lin)
