"""Known answers derived from the reference's source text,
applied directly to the HIP outputs through the C-ABI.

The reference has no tests and cannot be run here, so these closed
forms are the reference-anchored evidence that does not go through the CPU
restatement.  Each test cites the Appendix C item and the reference lines.
"""
import math

import numpy as np
import pytest
import torch

from oracle import scp_reference as R      # scenario builders only (Scenarios.py restated)
from scpqp import trace as TR
from scpqp.solver import ScpQpSolver

pytestmark = pytest.mark.gpu


def _straight(sc, travel=1.72):
    """Cold-start geometry of SURVEY §8d: each vehicle moved `travel` m along its heading
    (the delay-compensated state with u = a = delta = 0)."""
    x0 = np.array(sc.x0, float)
    for v in range(sc.nVeh):
        x0[v, 0] += travel * math.cos(x0[v, 2])
        x0[v, 1] += travel * math.sin(x0[v, 2])
    return x0


# C.3: closed-form ZOH discretisation at psi = delta = a = 0, v = 4 (MPC_Iter.py:99-113,
# Model.py:45-59); Lf = Lr = 0.34, dt = 0.4
def test_c3_closed_form_discretisation(gpu):
    sc = R.circle_scenario(1, Hp=10)
    S = ScpQpSolver(sc, max_batch=1)
    x0 = np.array([[[0.0, 0.0, 0.0, 4.0, 0.0, 0.0]]])
    lin = S.linearize(x0, np.zeros((1, 1)), np.zeros((1, 1, 2)))
    Ad = lin["Ad"][0, 0].cpu().numpy()
    Bd = lin["Bd"][0, 0].cpu().numpy()
    Ed = lin["Ed"][0, 0].cpu().numpy()
    assert np.allclose(Bd, [0, 1.7758241539215744, 1.7754797875816084, 0, 0,
                            0.98168436111126578], rtol=1e-13, atol=1e-15)
    assert Ad[5, 5] == pytest.approx(0.018315638888734179, rel=1e-13)   # e^-4
    assert Ad[2, 5] == pytest.approx(0.57746138888897991, rel=1e-13)
    assert Ad[1, 5] == pytest.approx(0.90652878725489638, rel=1e-13)
    assert Ad[1, 2] == pytest.approx(1.6, rel=1e-13)                     # v dt
    assert Ad[0, 3] == pytest.approx(0.4, rel=1e-13)                     # dt
    assert Ad[0, 4] == pytest.approx(0.08, rel=1e-13)                    # dt^2 / 2
    assert np.all(np.abs(Ed) <= 1e-15)                                   # Ec = 0 here
    # C.4 on the same outputs: g_m = C Ad^m Bd (MPC_Iter.py:139-147)
    g = lin["g"][0, 0].cpu().numpy()
    A = np.eye(6)
    for m in range(10):
        assert np.allclose(g[m], (A @ Bd)[:2], rtol=1e-12, atol=1e-15), m
        A = Ad @ A
    S.close()


# C.2 through the device discretisation: at delta = 0, Ec = [v psi sin psi, -v psi cos psi,
# 0, 0, 0, 0] (Model.py:58), so Ed = (int_0^dt e^{Ac s} ds) Ec; with Ec[2:] = 0 and
# Ac's rows 0..1 feeding nothing back, Ed[0:2] = dt Ec[0:2] exactly in exact arithmetic.
def test_c2_ec_structure_through_ed(gpu):
    sc = R.circle_scenario(1, Hp=10)
    S = ScpQpSolver(sc, max_batch=3)
    x0 = np.zeros((3, 1, 6))
    for b, psi in enumerate((0.7, -1.3, 2.4)):
        x0[b, 0] = [1.0, 2.0, psi, 4.0, 0.0, 0.0]
    lin = S.linearize(x0, np.zeros((3, 1)), np.zeros((3, 1, 2)))
    Ed = lin["Ed"][:, 0].cpu().numpy()
    for b, psi in enumerate((0.7, -1.3, 2.4)):
        want = 0.4 * np.array([4.0 * psi * math.sin(psi), -4.0 * psi * math.cos(psi)])
        assert np.allclose(Ed[b, :2], want, rtol=1e-12, atol=1e-14)
        assert np.all(Ed[b, 2:] == 0.0)
    # Ec does not depend on u0 (Model.py:58): Ed unchanged by u0
    lin2 = S.linearize(x0, np.full((3, 1), 0.03), np.zeros((3, 1, 2)))
    assert np.allclose(lin2["Ed"][:, 0, :5].cpu().numpy(), Ed[:, :5], rtol=0, atol=1e-15)
    S.close()


# C.5: dsafe = 2.0723899247004653 for two default vehicles at 4 m/s (Scenarios.py:229-243):
# the device constraint values satisfy c + |p_i - p_j|^2 = (dsafe + dsafeExtra)^2
def test_c5_safety_distance_in_device_constraints(gpu):
    sc = R.circle_scenario(4, Hp=20)
    S = ScpQpSolver(sc, max_batch=2)
    x0 = np.repeat(_straight(sc)[None], 2, 0)
    g = np.random.default_rng(4)
    U = g.uniform(-sc.uLim, sc.uLim, (2, 80))
    ev = S.evaluate(U, x0, np.zeros((2, 4)), np.zeros((2, 4, 2)))
    cv = ev["c_veh"].cpu().numpy()
    tr = ev["traj"].cpu().numpy()                    # [B, Hp, 2, nVeh]
    D2 = (2.0723899247004653 + 1.0) ** 2
    assert D2 == pytest.approx(9.43957984940093, rel=1e-15)
    for b in range(2):
        for i in range(4):
            for j in range(i + 1, 4):
                d2 = np.sum((tr[b, :, :, i] - tr[b, :, :, j]) ** 2, axis=1)
                assert np.allclose(cv[b, i, j] + d2, D2, rtol=1e-12, atol=0)
                assert np.array_equal(cv[b, i, j], cv[b, j, i])
            assert np.all(np.isneginf(cv[b, i, i]))   # diagonal never set (SCP_controller.py:224)
    S.close()


# C.7: one vehicle, no obstacles: m = 0, so the QP is the box QP
# min u'Phi0 u + Psi0'u, |u| <= uLim (SCP_controller.py:118-128); on the line u* ~ 0 and
# SCP stops after one QP; off the line u* is the projected-gradient fixed point.
def test_c7_single_vehicle_box_qp(gpu):
    sc = R.circle_scenario(1, Hp=10)
    x_on = _straight(sc, 4.0 * 0.43)
    x_off = x_on.copy()
    x_off[0, 1] += 0.8
    x0 = np.stack([x_on, x_off])
    S = ScpQpSolver(sc, max_batch=2)
    out = S.solve(x0, np.zeros((2, 1)), np.zeros((2, 1, 2)))
    lin = S.linearize(x0, np.zeros((2, 1)), np.zeros((2, 1, 2)))
    torch.cuda.synchronize()
    assert int(out.n_scp[0]) == 1
    assert float(out.u[0].abs().max()) < 1e-6
    assert int(out.n_scp[1]) <= 2
    # Phi0 = calB' Q calB + R I from the device Toeplitz blocks (MPC_Iter.py:116-127)
    g = lin["g"][1, 0].cpu().numpy()
    Hp = 10
    calB = np.zeros((2 * Hp, Hp))
    for i in range(Hp):
        for j in range(i + 1):
            calB[2 * i:2 * i + 2, j] = g[i - j]
    q = np.full(2 * Hp, float(sc.Q[0]))
    q[-2:] = float(sc.Q_final[0])
    Phi0 = calB.T @ (q[:, None] * calB) + float(sc.R[0]) * np.eye(Hp)
    Psi0 = lin["psi0"][1, 0].cpu().numpy()
    u = out.u[1].cpu().numpy()
    proj = np.clip(u - 1e-5 * (2 * Phi0 @ u + Psi0), -sc.uLim, sc.uLim)
    assert np.max(np.abs(proj - u)) < 1e-10
    S.close()


# C.9 on the device trace: omega* = max(0, max_r(a_r u* - b_r)) and every
# QP iterate inside the box (SCP_controller.py:118-127)
def test_c9_slack_identity_on_device_trace(gpu):
    sc = R.circle_scenario(4, Hp=20)
    S = ScpQpSolver(sc, max_batch=1)
    x0 = _straight(sc)[None]
    out = S.solve(x0, np.zeros((1, 4)), np.zeros((1, 4, 2)), trace=True)
    lin = S.linearize(x0, np.zeros((1, 4)), np.zeros((1, 4, 2)))
    torch.cuda.synchronize()
    n = int(out.n_scp[0])
    g = lin["g"][0].cpu().numpy()
    its = TR.decode(out.trace[0].cpu().numpy(), n, 4, 0, 20, 20, g=g, u_lim=S.u_lim)
    assert (out.status[0].item() & 0xff) == 0          # converged
    for d in its:
        u = d["z"][:80]
        assert np.all(np.abs(u) <= sc.uLim * (1 + 1e-12))
        omega = max(0.0, float(np.max(d["A"][:, :80] @ u - d["b"])))
        assert abs(d["slack"] - omega) <= 1e-9 * max(1.0, abs(omega))
    S.close()


# C.10: cold-start activity (straight-line geometry, u = 0): 16 of 120 pair rows violated
# for 4 vehicles at Hp 20, 88 of 840 for 8 vehicles at Hp 30, none at Hp 10
@pytest.mark.parametrize("n_veh,hp,want,total", [(4, 20, 16, 120), (8, 30, 88, 840), (4, 10, 0, 60)])
def test_c10_cold_start_activity(gpu, n_veh, hp, want, total):
    sc = R.circle_scenario(n_veh, Hp=hp)
    S = ScpQpSolver(sc, max_batch=1)
    x0 = _straight(sc)[None]
    ev = S.evaluate(np.zeros((1, n_veh * hp)), x0, np.zeros((1, n_veh)), np.zeros((1, n_veh, 2)))
    cv = ev["c_veh"][0].cpu().numpy()
    iu = np.triu_indices(n_veh, 1)
    vals = cv[iu[0], iu[1], :]
    assert vals.size == total
    assert int((vals > 0).sum()) == want
    S.close()
