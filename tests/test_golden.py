"""The CPU restatement reproduces the committed golden fixtures (regression pin
of the oracle), and the fixtures are self-consistent: every recorded QP carries
a KKT certificate and the recorded rows are the reference's linearisation
(SCP_controller.py:93-128) of the recorded iterate."""
import glob
import os

import numpy as np
import pytest

from oracle import scp_reference as R

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BUILDERS = {
    "c1_circle1_hp10": lambda: R.circle_scenario(1, Hp=10),
    "c2_circle4_hp20": lambda: R.circle_scenario(4, Hp=20),
    "c3_circle8_hp30": lambda: R.circle_scenario(8, Hp=30),
    "c5_circle4_mixed": lambda: R.circle_scenario(4, Hp=30),
    "frog_hp10": lambda: R.frog_scenario(Hp=10),
    "parallel5_hp10": lambda: R.parallel_scenario(5, Hp=10),
    "c3_circle8_hp30_hist": lambda: R.circle_scenario(8, Hp=30),
    "c5_circle4_mixed_hist": lambda: R.circle_scenario(4, Hp=30),
}
# (fixture, problem) pairs with a per-iteration history; problem b > 0 under "hist{b}_*"
HISTORIES = [("c1_circle1_hp10", 0), ("c2_circle4_hp20", 0), ("frog_hp10", 0),
             ("parallel5_hp10", 0), ("c3_circle8_hp30_hist", 0), ("c5_circle4_mixed_hist", 0),
             ("c5_circle4_mixed_hist", 1), ("c5_circle4_mixed_hist", 2)]


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def problem(sc, f, b):
    H = int(f["hp"][b])
    nO, nV = sc.nObst, sc.nVeh
    ob = f["obst"][b].reshape(-1)[:nO * 2 * H].reshape(nO, 2, H)
    return R.make_problem(sc, f["x0"][b], f["u0"][b], f["ec_noise"][b], Hp=H, obst=ob), H


def test_all_fixtures_present():
    have = {os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz"))}
    assert set(BUILDERS) <= have


@pytest.mark.parametrize("name", ["c1_circle1_hp10", "c2_circle4_hp20", "c5_circle4_mixed",
                                  "frog_hp10", "parallel5_hp10"])
def test_oracle_reproduces_fixture(name):
    f = load(name)
    sc = BUILDERS[name]()
    nV = sc.nVeh
    mode = str(f["mode"])
    B = f["x0"].shape[0]
    for b in range(min(B, 3)):
        p, H = problem(sc, f, b)
        r = R.scp_solve(p, mode=mode)
        assert r.n_scp == f["n_scp"][b]
        assert np.max(np.abs(r.u - f["u"][b, :nV * H])) <= 1e-9
        assert np.max(np.abs(r.traj.reshape(-1) - f["traj"][b, :H * 2 * nV])) <= 1e-8
        assert np.max(np.abs(p.ref_points.reshape(-1) - f["ref_points"][b, :H * 2 * nV])) == 0.0


@pytest.mark.parametrize("name,pb", HISTORIES)
def test_fixture_history_is_consistent(name, pb):
    f = load(name)
    sc = BUILDERS[name]()
    p, H = problem(sc, f, pb)
    L = R.linearise(p, "structured")
    nV = sc.nVeh
    N = nV * H
    pre = "hist" if pb == 0 else f"hist{pb}"
    hz = f[pre + "_z"]
    assert len(hz) == f["n_scp"][pb]
    for it in range(len(hz)):
        A, b = R.linearised_rows_structured(p, L, f[pre + "_u_lin"][it])
        assert np.max(np.abs(A - f[pre + "_A"][it]), initial=0.0) <= 1e-8
        assert np.max(np.abs(b - f[pre + "_b"][it]), initial=0.0) <= 1e-8 * max(1, np.abs(b).max(initial=0))
        kkt = f[pre + "_kkt"][it]
        assert kkt[1] <= 1e-9 and kkt[2] <= 1e-9
        # stationarity and complementarity in unscaled units (multipliers up to the
        # slack weight 1e5): 1e-6 absolute; c3 and c5 (Hp 30) reach 1.0e-6 and 1.5e-7
        assert kkt[0] <= 1e-6 and kkt[3] <= (1e-7 if N <= 80 else 2e-6)
        z = hz[it]
        assert np.all(np.abs(z[:N]) <= sc.uLim * (1 + 1e-9))
    assert np.array_equal(hz[-1][:N], f["u"][pb, :N])


def test_c3_fixture_structured():
    f = load("c3_circle8_hp30")
    sc = BUILDERS["c3_circle8_hp30"]()
    p, H = problem(sc, f, 0)
    L = R.linearise(p, "structured")
    assert np.allclose(L.g, f["lin_g"], rtol=0, atol=1e-14)
    ev = R.evaluate_structured(p, L, f["u"][0, :8 * H])
    assert ev.obj == pytest.approx(float(f["obj"][0]), rel=1e-12)
    assert bool(ev.feasible) == bool(f["feasible"][0])
