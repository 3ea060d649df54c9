"""Known-answer tests that pin the CPU restatement.

The reference has no tests and could not be executed here, so
these analytic answers, derived from the source text, are what ties
``oracle/scp_reference.py`` to the reference's behaviour.
"""
import math

import numpy as np
import pytest

from oracle import scp_reference as R

LF = LR = 0.34


def _rand_states(n, seed=0):
    g = np.random.default_rng(seed)
    X = np.zeros((n, 6))
    X[:, 0:2] = g.uniform(-30, 30, (n, 2))
    X[:, 2] = g.uniform(-math.pi, math.pi, n)
    X[:, 3] = g.uniform(0.5, 8, n)
    X[:, 4] = g.uniform(-1, 1, n)
    X[:, 5] = g.uniform(-0.3, 0.3, n)
    return X, g.uniform(-0.05, 0.05, n)


# C.1 ------------------------------------------------------------------------------------
def test_jacobian_matches_central_differences():
    X, U = _rand_states(50)
    for x, u in zip(X, U):
        Ac, Bc, Cc, Ec = R.bicycle_jacobian(x, u, LF, LR)
        J = np.zeros((6, 6))
        for j in range(6):
            h = 1e-6 * max(1.0, abs(x[j]))
            xp, xm = x.copy(), x.copy()
            xp[j] += h
            xm[j] -= h
            J[:, j] = (R.bicycle_rhs(xp, u, LF, LR) - R.bicycle_rhs(xm, u, LF, LR)) / (2 * h)
        assert np.allclose(Ac, J, rtol=1e-7, atol=1e-7)
        # row 2 simplifies to v tan(delta) / L
        f = R.bicycle_rhs(x, u, LF, LR)
        assert f[2] == pytest.approx(x[3] * math.tan(x[5]) / (LF + LR), rel=1e-12)
        assert np.array_equal(Bc[:, 0], [0, 0, 0, 0, 0, 10.0])
        assert np.array_equal(Cc, np.eye(2, 6))


# C.2 ------------------------------------------------------------------------------------
def test_ec_structure():
    X, U = _rand_states(50, seed=1)
    for x, u in zip(X, U):
        _, _, _, Ec = R.bicycle_jacobian(x, u, LF, LR)
        Ec = Ec[:, 0]
        assert Ec[3] == 0.0 and Ec[4] == 0.0
        assert abs(Ec[5]) < 1e-14
        L = LF + LR
        assert Ec[2] == pytest.approx(-x[3] * (1 + math.tan(x[5]) ** 2) * x[5] / L, rel=1e-9, abs=1e-13)
        _, _, _, Ec2 = R.bicycle_jacobian(x, u + 0.01, LF, LR)
        assert np.allclose(Ec[:5], Ec2[:5, 0], atol=1e-13)      # independent of u0
    x = np.array([1.0, 2.0, 0.7, 4.0, 0.0, 0.0])
    _, _, _, Ec = R.bicycle_jacobian(x, 0.0, LF, LR)
    assert Ec[0, 0] == pytest.approx(4.0 * 0.7 * math.sin(0.7), rel=1e-12)
    assert Ec[1, 0] == pytest.approx(-4.0 * 0.7 * math.cos(0.7), rel=1e-12)


# C.3 ------------------------------------------------------------------------------------
def test_closed_form_discretisation():
    Ad, Bd, Cd, Ed = R.discretize(np.array([0, 0, 0, 4.0, 0, 0]), 0.0, LF, LR, 0.4)
    assert np.allclose(Bd[:, 0], [0, 1.7758241539215744, 1.7754797875816084, 0, 0,
                                  0.98168436111126578], rtol=1e-13, atol=1e-15)
    assert Ad[5, 5] == pytest.approx(0.018315638888734179, rel=1e-13)
    assert Ad[2, 5] == pytest.approx(0.57746138888897991, rel=1e-13)
    assert Ad[1, 5] == pytest.approx(0.90652878725489638, rel=1e-13)
    assert Ad[1, 2] == pytest.approx(1.6, rel=1e-13)
    assert Ad[0, 3] == pytest.approx(0.4, rel=1e-13)
    assert Ad[0, 4] == pytest.approx(0.08, rel=1e-13)
    assert np.all(Ed == 0.0)


# C.4 ------------------------------------------------------------------------------------
def test_toeplitz_structure():
    sc = R.circle_scenario(2, Hp=12)
    p = R.make_problem(sc, np.array(sc.x0), ec_noise=np.full((2, 2), 1e-6))
    for mode in ("faithful", "structured"):
        L = R.linearise(p, mode)
        for v in range(2):
            A = L.Ad[v]
            C = np.eye(2, 6)
            for i in range(12):
                for j in range(12):
                    blk = L.calB[v][2 * i:2 * i + 2, j]
                    if j <= i:
                        assert np.allclose(blk, L.g[v, i - j], rtol=1e-12, atol=1e-15)
                    else:
                        assert np.all(blk == 0)
        if mode == "faithful":
            cA, _, _ = R.prediction_matrices(L.Ad[0], L.Bd[0][:, None], np.eye(2, 6),
                                             L.Ed[0][:, None], 12, 12)
            for i in range(12):
                assert np.allclose(cA[2 * i:2 * i + 2], C @ np.linalg.matrix_power(L.Ad[0], i + 1))
    Lf = R.linearise(p, "faithful")
    Ls = R.linearise(p, "structured")
    for f in ("g", "const", "Phi0", "Psi0", "gamma0"):
        a, b = getattr(Lf, f), getattr(Ls, f)
        assert np.max(np.abs(a - b)) <= 1e-10 * max(1.0, np.max(np.abs(a)))


# C.5 ------------------------------------------------------------------------------------
def test_scenario_constants():
    sc = R.circle_scenario(4, Hp=20)
    assert (sc.ticks_per_sim, sc.Nsim, sc.ticks_total, sc.ticks_delay_u, sc.ticks_delay_x) == \
        (40, 50, 2000, 3, 0)
    assert sc.dsafeVehicles[0, 1] == pytest.approx(2.0723899247004653, rel=1e-15)
    assert (sc.dsafeVehicles[0, 1] + 1) ** 2 == pytest.approx(9.43957984940093, rel=1e-14)
    assert R.CONSTRAINT_TOL == pytest.approx(0.0042, rel=1e-15)
    assert sc.uLim == pytest.approx(0.05235987755982989, rel=1e-15)
    assert math.hypot(0.98, 0.88) / 2 == pytest.approx(0.6585590330410782, rel=1e-15)
    assert math.atan(4.905 * 0.68 / 16) > sc.uLim        # dynamic limit not binding


# C.6 ------------------------------------------------------------------------------------
def test_sampler_on_line_and_overshoot_alternation():
    ref = np.array([[-30.0, 0.0], [30.0, 0.0]])
    pts = R.sample_reference(10, ref, -20.0, 0.3, 1.6)
    assert np.allclose(pts, [[-20 + 1.6 * (i + 1), 0.0] for i in range(10)], atol=1e-12)
    # overshoot (B.1): r0 = 0.5 < s = 1.6 -> E + (s - r0) d, then E + r0 d, alternating
    pts = R.sample_reference(6, ref, 29.5, 0.0, 1.6)
    assert np.allclose(pts[:, 0], [31.1, 30.5, 31.1, 30.5, 31.1, 30.5], atol=1e-12)
    assert np.all(np.abs(pts[:, 1]) < 1e-12)


def test_sampler_seeded_with_second_vertex_and_xor_quirk():
    # 3-point polyline where the vehicle projects beyond segment 1: the '^' branch
    ref = np.array([[0.0, 0.0], [10.0, 0.0], [20.0, 10.0]])
    with pytest.raises(TypeError):
        R.shortest_distance(ref[:, 0], ref[:, 1], 25.0, 20.0, strict_xor_quirk=True)
    d, arc, xm, ym, idx = R.shortest_distance(ref[:, 0], ref[:, 1], 5.0, 1.0, strict_xor_quirk=False)
    assert (xm, ym, idx) == (5.0, 0.0, 1) and d == pytest.approx(1.0) and arc == pytest.approx(5.0)


# C.7 ------------------------------------------------------------------------------------
def test_single_vehicle_box_qp_closed_form():
    sc = R.circle_scenario(1, Hp=10)
    x0 = np.array(sc.x0)
    x0[0, 0] += 4.0 * 0.43 * math.cos(x0[0, 2])
    x0[0, 1] += 4.0 * 0.43 * math.sin(x0[0, 2])
    p = R.make_problem(sc, x0)
    r = R.scp_solve(p, mode="faithful")
    assert r.n_scp == 1                                  # m = 0: one QP at cold start
    assert np.max(np.abs(r.u)) < 1e-6                    # on the line: Psi0 ~ 0 -> u* ~ 0
    # off the line: box-constrained minimiser, checked against projected gradient fixed point
    x1 = x0.copy()
    x1[0, 1] += 0.8
    p = R.make_problem(sc, x1)
    r = R.scp_solve(p, mode="faithful")
    L = r.lin
    H, g = 2 * L.Phi0[0], L.Psi0[0]
    u = r.u
    proj = np.clip(u - 1e-5 * (H @ u + g), -sc.uLim, sc.uLim)
    assert np.max(np.abs(proj - u)) < 1e-10
    assert r.n_scp <= 2


# C.8 ------------------------------------------------------------------------------------
@pytest.mark.parametrize("n_veh,hp", [(3, 8), (4, 20)])
def test_linearisation_identity_and_concavity(n_veh, hp):
    sc = R.circle_scenario(n_veh, Hp=hp)
    g = np.random.default_rng(3)
    x0 = np.array(sc.x0) + g.normal(0, 0.05, (n_veh, 6)) * [1, 1, 0.1, 0.3, 0, 0.04]
    p = R.make_problem(sc, x0, ec_noise=g.normal(0, 3e-6, (n_veh, 2)))
    L = R.linearise(p, "faithful")
    q = R.qcqp_formulate(p, L)
    for trial in range(3):
        ub = g.uniform(-sc.uLim, sc.uLim, n_veh * hp)
        Ad, bd = R.linearised_rows_dense(q, ub, n_veh, hp, 0)
        As, bs = R.linearised_rows_structured(p, L, ub)
        assert np.max(np.abs(Ad - As)) <= 1e-8
        assert np.max(np.abs(bd - bs)) <= 1e-8 * max(1.0, np.max(np.abs(bd)))
        # concavity: c(u) <= c(ub) + grad(ub)'(u - ub)  ->  lin-feasible => feasible
        u = g.uniform(-sc.uLim, sc.uLim, n_veh * hp)
        ev = R.evaluate_structured(p, L, u)
        rows = R.row_list(n_veh, hp, 0)
        lin = As[:, :-1] @ u - bs
        for r_, (i, j, o, k) in enumerate(rows):
            assert ev.c_veh[i, j, k] <= lin[r_] + 1e-9


# C.9 ------------------------------------------------------------------------------------
def test_qp_certificate_and_slack_identity():
    sc = R.circle_scenario(4, Hp=20)
    x0 = np.array(sc.x0)
    for v in range(4):
        x0[v, 0] += 1.72 * math.cos(x0[v, 2])
        x0[v, 1] += 1.72 * math.sin(x0[v, 2])
    p = R.make_problem(sc, x0)
    r = R.scp_solve(p, mode="structured", keep_history=True)
    assert r.converged
    N = 80
    for h in r.history:
        c = h["certificate"]
        assert c["stationarity"] <= 1e-6 and c["primal"] <= 1e-9 and c["dual"] <= 1e-9
        assert c["complementarity"] <= 1e-7
        z, A, b = h["z"], h["A"], h["b"]
        omega = max(0.0, float(np.max(A[:, :N] @ z[:N] - b)))
        assert abs(z[N] - omega) <= 1e-9


# C.10 -----------------------------------------------------------------------------------
@pytest.mark.parametrize("n_veh,hp,want,total", [(4, 20, 16, 120), (8, 30, 88, 840), (4, 10, 0, 60)])
def test_cold_start_activity(n_veh, hp, want, total):
    sc = R.circle_scenario(n_veh, Hp=hp)
    x0 = np.array(sc.x0)
    for v in range(n_veh):
        x0[v, 0] += 1.72 * math.cos(x0[v, 2])
        x0[v, 1] += 1.72 * math.sin(x0[v, 2])
    p = R.make_problem(sc, x0)
    L = R.linearise(p, "structured")
    ev = R.evaluate_structured(p, L, np.zeros(n_veh * hp))
    iu = np.triu_indices(n_veh, 1)
    vals = ev.c_veh[iu[0], iu[1], :]
    assert vals.size == total
    assert int((vals > 0).sum()) == want
