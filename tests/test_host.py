"""Host-side logic of the drop-in modules and helpers, against the restatement.

Only host code is exercised here (scenario builders, plant model, geometry
helpers, delay compensation, obstacle prediction, batch generation, FLOP
model); every solve/linearise/evaluate/sample call needs the GPU and lives in
the -m gpu tests.
"""
import math
import os
import sys

import numpy as np
import pytest

import Config
import MIQP
import Model
import MPC_Iter
import SampleReferTraj
import Scenarios
from oracle import scp_reference as R
from scpqp import batch as BT
from scpqp import flops as FL


def _circle(n, hp=10):
    sc = Scenarios.Scenario(False)
    sc.Hp = sc.Hu = hp
    sc.get_circle_scenario([2 * math.pi / n * (i + 1) for i in range(n)])
    sc.complete_scenario()
    return sc


@pytest.mark.parametrize("kind", ["circle4", "circle8", "frog", "parallel5", "parallel11"])
def test_scenarios_match_restatement(kind):
    sc = Scenarios.Scenario(False)
    if kind.startswith("circle"):
        n = int(kind[6:])
        sc.get_circle_scenario([2 * math.pi / n * (i + 1) for i in range(n)])
        o = R.circle_scenario(n)
    elif kind == "frog":
        sc.get_frog_scenario()
        o = R.frog_scenario()
    else:
        n = int(kind[8:])
        sc.get_parallel_scenario(n)
        sc.dsafeExtra = 0.9
        o = R.parallel_scenario(n)
    sc.complete_scenario()
    assert sc.nVeh == o.nVeh and sc.nObst == o.nObst
    assert np.array_equal(np.array(sc.x0).reshape(sc.nVeh, 6), np.array(o.x0))
    assert np.array_equal(sc.dsafeVehicles, o.dsafeVehicles)
    if sc.nObst:
        assert np.array_equal(sc.dsafeObstacles, o.dsafeObstacles)
        assert np.array_equal(np.asarray(sc.obstacles).reshape(sc.nObst, 6), np.array(o.obstacles))
        assert np.asarray(sc.obstacles).shape == (sc.nObst, 6, 1)     # main.py:70 indexing
    for a, b in zip(sc.referenceTrajectories, o.referenceTrajectories):
        assert np.array_equal(np.asarray(a, float), b)
    assert (sc.ticks_per_sim, sc.Nsim, sc.ticks_total, sc.ticks_delay_u) == (40, 50, 2000, 3)
    assert sc.uLim == pytest.approx(math.pi / 60)
    assert sc.dsafeExtra == o.dsafeExtra
    if kind.startswith("circle"):
        assert sc.CouplingAdjacencyMatrixPB.shape == (sc.nVeh, sc.nVeh)
    elif kind.startswith("parallel"):
        # Scenarios.py:197 builds np.diag(range(nVeh-1), 2): (nVeh+1) square, kept as is
        assert sc.CouplingAdjacencyMatrixPB.shape == (sc.nVeh + 1, sc.nVeh + 1)


def test_uLim_build_choice_and_override():
    sc = _circle(2)
    assert sc.uLim == sc.mechanicalSteeringLimit
    sc.uLim = 0.1
    assert sc.uLim == 0.1


def test_model_matches_restatement():
    m = Model.BicyleModel(False)
    g = np.random.default_rng(2)
    for _ in range(20):
        x = np.array([*g.uniform(-5, 5, 2), g.uniform(-3, 3), g.uniform(1, 6), 0.0, g.uniform(-.2, .2)])
        u = g.uniform(-0.05, 0.05)
        assert np.array_equal(m.ode(x, 0.0, u, .34, .34), R.bicycle_rhs(x, u, .34, .34))
        assert np.array_equal(m.odes_(0.0, x, u, .34, .34), R.bicycle_rhs(x, u, .34, .34))
        a = m.comp_jacobian(x, np.array([u]), .34, .34)
        b = R.bicycle_jacobian(x, u, .34, .34)
        for p, q in zip(a, b):
            assert np.array_equal(p, q)
    veh = Model.DefaultVehicle()
    m.makeInitState(veh)
    assert m.makeInitStateVector.shape == (6, 1)
    assert (veh.Q, veh.Q_final, veh.R, veh.Lf, veh.Lr) == (1, 20, 4000, .34, .34)


def test_geometry_helpers_match_restatement():
    g = np.random.default_rng(4)
    for _ in range(50):
        ref = g.uniform(-30, 30, (2, 2))
        x, y = (float(v) for v in g.uniform(-30, 30, 2))
        a = SampleReferTraj.getShortestDistance(ref[:, 0], ref[:, 1], x, y)
        b = R.shortest_distance(ref[:, 0], ref[:, 1], x, y)
        assert np.allclose(a, b, rtol=0, atol=0)
    ref3 = np.array([[0.0, 0.0], [10.0, 0.0], [20.0, 10.0]])
    a = SampleReferTraj.getShortestDistance(ref3[:, 0], ref3[:, 1], 25.0, 20.0)
    b = R.shortest_distance(ref3[:, 0], ref3[:, 1], 25.0, 20.0, strict_xor_quirk=False)
    assert np.allclose(a, b, rtol=0, atol=1e-15)
    p = SampleReferTraj.Projection2D(0.0, 0.0, 0.0, 0.0, 3.0, 4.0)
    assert p == (0.0, 0.0, 5.0, 0, 0.0)


def test_sampler_argument_check_raises_before_launch():
    with pytest.raises(AssertionError):
        SampleReferTraj.sampleReferenceTrajectory(5, np.array([[0, 0], [1, 0]]), 0.0, 0.0, 1.6)


def test_obstacle_prediction_matches_restatement():
    sc = Scenarios.Scenario(False)
    sc.Hp = sc.Hu = 12
    sc.get_frog_scenario()
    sc.complete_scenario()
    o = R.frog_scenario(Hp=12)
    st = np.asarray(sc.obstacles).reshape(sc.nObst, 6)[:, :2] + 0.5
    a = MPC_Iter.predict_obstacles(sc, st)
    b = R.obstacle_future(o, st, 12)
    assert np.allclose(a, b, rtol=1e-15, atol=1e-13)
    c = BT.obstacle_prediction(sc, 12, st)
    assert np.allclose(c, b, rtol=1e-15, atol=1e-13)


def test_batch_generation_is_deterministic_and_shard_independent():
    sc = _circle(4, hp=20)
    a = BT.make_batch(sc, 8, base_seed=3)
    b = BT.make_batch(sc, 4, base_seed=3, offset=4)
    assert np.array_equal(a.x0[4:], b.x0) and np.array_equal(a.ec_noise[4:], b.ec_noise)
    assert a.x0.shape == (8, 4, 6) and a.ec_noise.shape == (8, 4, 2) and a.hp.dtype == np.int32
    d = a.x0 - BT.delay_compensated_nominal(sc)[None]
    assert np.all(d[:, :, 4] == 0)
    assert abs(d[:, :, 0].std() - 0.05) < 0.03
    m = BT.make_batch(sc, 6, mixed_hp=(10, 20, 30))
    assert m.hp.tolist() == [10, 20, 30, 10, 20, 30] and m.hp_max == 30


def test_mixed_horizon_obstacle_slots_are_packed():
    sc = Scenarios.Scenario(False)
    sc.Hp = sc.Hu = 30
    sc.get_parallel_scenario(3)
    sc.complete_scenario()
    bt = BT.make_batch(sc, 3, mixed_hp=(10, 20, 30))
    for b, H in enumerate((10, 20, 30)):
        want = BT.obstacle_prediction(sc, H).reshape(-1)
        slot = bt.obst[b].reshape(-1)
        assert np.array_equal(slot[:want.size], want)
        assert np.all(slot[want.size:] == 0)


def test_flop_model_sizes():
    assert FL._sizes(4, 20, 0) == (80, 81, 120, 281)
    assert FL._sizes(8, 30, 0) == (240, 241, 840, 1321)
    assert FL.factor(81) == 81 ** 3 // 3
    # 7 QPs, 109 IPM iterations, 8 polish rounds with 40 solves, 0 warm-certified QPs
    f = FL.problem_flops(4, 20, 0, 7, 109, 8, 40, 0)
    assert 5e7 < f < 1e8
    assert FL.batch_flops(4, [20, 20], 0, [7, 7], [109, 109], [8, 8], [40, 40], [0, 0]) == 2 * f
    # a warm-certified QP skips the IPM initial point
    assert FL.problem_flops(4, 20, 0, 7, 109, 8, 40, 3) < f
    assert FL.compulsory_bytes(4, 20, 0) > 0


def test_config_and_miqp_stub():
    assert Config.Config().QCQP.constraintTolerance == pytest.approx(0.0042)
    with pytest.raises(NotImplementedError):
        MIQP.MIQPcontroller(None, None, None)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_traffic_and_bound_from_committed_records():
    """bench.py reads the committed PMC summaries: raw = FETCH_SIZE (KiB) + WRITE_SIZE,
    corrected = 2 FETCH_SIZE + WRITE_SIZE; the roofline bound follows the measured MFMA
    share (the raw key and the hard-coded "mfma" label were wrong)."""
    import glob
    import json
    sys.path.insert(0, ROOT)
    import bench
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r0[3-9]_pmc_traffic_c*.json")))
    assert paths
    for path in paths:
        with open(path) as fh:
            tj = json.load(fh)
        corr, raw = bench.pmc_traffic(tj)
        assert raw == pytest.approx(tj["fetch_size_kib_raw"] * 1024 + tj["write_size_kib"] * 1024)
        assert corr == pytest.approx(2 * tj["fetch_size_kib_raw"] * 1024 + tj["write_size_kib"] * 1024)
        assert raw < corr
    with pytest.raises(KeyError):
        bench.pmc_traffic({"hbm_bytes_per_launch": 1.0})
    assert bench.roofline_bound({"mfma_f64_flops": 0.0}, 1e9)[0] == "fp64-valu"
    assert bench.roofline_bound({"mfma_f64_flops": 0.6e9}, 1e9)[0] == "mfma"
    assert bench.roofline_bound(None, 1e9)[0] == "fp64-valu"


def test_bench_cpu_leg_round_trip(tmp_path):
    """The CPU leg the launching process hands to rank 0 survives the JSON round trip."""
    sys.path.insert(0, ROOT)
    import bench
    cpu = dict(wall=1.5, cpu_s=3.0, cores=2, sample=2,
               modes={"faithful": dict(wall=1.5, cpu_s=3.0), "structured": dict(wall=1.0, cpu_s=2.0)},
               trajs=[(np.arange(6.0).reshape(3, 2), 5, True), (np.ones((3, 2)), 20, False)])
    path = str(tmp_path / "cpu.json")
    bench.cpu_leg_dump(cpu, path)
    back = bench.cpu_leg_load(path)
    assert back["wall"] == 1.5 and back["cores"] == 2 and back["sample"] == 2
    assert back["modes"]["structured"]["cpu_s"] == 2.0
    for (t0, n0, c0), (t1, n1, c1) in zip(cpu["trajs"], back["trajs"]):
        assert np.array_equal(t0, t1) and n0 == n1 and c0 == c1


def test_bench_cpu_baseline_fields_on_a_sample():
    """SURVEY 8(d)'s CPU leg on a 4-problem c2 sample: the reference CPU path (faithful
    mode) and the structured mode, each at the all-core and the 1-core rate, on the same
    problems, and the faithful trajectories are the parity sample."""
    sys.path.insert(0, ROOT)
    import bench
    from scpqp import shard
    sc = _circle(4, hp=20)
    bt = shard.shard_batch(sc, 8, 0, base_seed=0)
    cpu = bench.cpu_leg(bt, 4, 4, 8, cores=2)
    assert cpu["sample"] == 4 and cpu["cores"] == 2 and len(cpu["trajs"]) == 4
    assert set(cpu["modes"]) == {"faithful", "structured"}
    blk = bench.cpu_baseline_block(cpu, "c2", 4)
    for k in ("value", "value_1core", "value_structured", "value_structured_1core"):
        assert np.isfinite(blk[k]) and blk[k] > 0, k
    m = cpu["modes"]
    assert blk["value"] == pytest.approx(4 / m["faithful"]["wall"])
    assert blk["value_1core"] == pytest.approx(4 / m["faithful"]["cpu_s"])
    assert blk["value_structured_1core"] == pytest.approx(4 / m["structured"]["cpu_s"])
    assert blk["mode"] == "faithful" and blk["cores"] == 2 and blk["kind"] == "port"
    # two workers: the all-core rate exceeds the 1-core rate (up to start-up noise)
    assert blk["value"] > 0.8 * blk["value_1core"]
    for t, ns, conv in cpu["trajs"]:
        assert t.shape == (20, 2, 4) and 1 <= ns <= 20
    assert bench.cpu_modes(8) == ("structured",)


def _lazy_log_counter():
    calls = []

    def dec():
        calls.append(1)
        return {"x": [np.ones((3, 1))], "delta": [0.5]}
    return calls, dec


def test_lazy_log_copy_and_pickle_decode_first():
    """optimization_log: copy / pickle / pop see the decoded lists, and the
    decode runs once."""
    import copy
    import pickle
    import SCP_controller as SC
    calls, dec = _lazy_log_counter()
    log = SC._LazyLog({"status": 0, "n_scp": 1}, dec)
    assert dict.__contains__(log, "status") and not calls
    c = log.copy()
    assert c["delta"] == [0.5] and len(calls) == 1
    back = pickle.loads(pickle.dumps(log))
    assert back["x"][0].shape == (3, 1) and back["status"] == 0
    assert copy.copy(log)["delta"] == [0.5] and copy.deepcopy(log)["n_scp"] == 1
    assert log.pop("delta") == [0.5] and len(calls) == 1
    # != decodes first as well: it agrees with not ==
    calls2 = []

    def dec2():
        calls2.append(1)
        return {"delta": [0.5]}
    log2 = SC._LazyLog({"status": 0, "n_scp": 1}, dec2)
    assert (log2 != {"status": 0, "n_scp": 1}) and len(calls2) == 1
    full = {"status": 0, "n_scp": 1, "delta": [0.5]}
    log3 = SC._LazyLog({"status": 0, "n_scp": 1}, lambda: {"delta": [0.5]})
    assert not (log3 != full) and log3 == full


def test_iteration_log_keys_and_formulas():
    """The drop-in's per-iteration log has every key of SCP_controller.py:88-90 with the
    reference's shapes; delta_hat, fval and forward_U follow their formulas (:146-187)."""
    import SCP_controller as SC
    from scpqp import trace as TR
    rng = np.random.default_rng(3)
    nV, nO, Hp, u_lim = 3, 1, 5, 0.4
    N = nV * Hp
    m = len(TR.row_list(nV, Hp, nO))
    stride = TR.HDR + 2 * N + 4 * m
    n_scp = 2
    tr = rng.standard_normal((n_scp, stride))
    tr[:, 5] = 7.0                       # ipm iterations
    tr[:, 6] = 1.0
    tr[:, 7] = 1.0
    tr[:, TR.HDR + 2 * N + 2::4] = -np.abs(tr[:, TR.HDR + 2 * N + 2::4]) - 0.5   # w_r < 0
    Mb = rng.standard_normal((2 * Hp, Hp, nV))
    const_term = rng.standard_normal((2 * Hp, 1, nV))
    Phi_0 = np.stack([np.eye(Hp) * (v + 1) for v in range(nV)], -1)
    Psi_0 = rng.standard_normal((Hp, 1, nV))
    log = SC._iteration_log(tr, n_scp, nV, nO, Hp, Hp, u_lim, Mb, const_term, Phi_0, Psi_0, 2.5)
    for k in ("P", "q", "Aineq", "bineq", "lb", "ub", "x", "slack", "SCP_ObjVal", "QCQP_ObjVal",
              "delta_hat", "delta", "u", "feasible", "prev_u", "Traj", "U", "prevTraj", "prevU"):
        assert len(log[k]) == n_scp, k
    assert log["P"][0].shape == (N + 1, N + 1) and log["P"][0][N, N] == 0.0
    assert log["q"][0][-1, 0] == 1e5 and log["ub"][0][-1, 0] == 1e25 and log["lb"][0][-1, 0] == 0
    assert np.all(log["ub"][0][:N] == u_lim) and np.all(log["lb"][0][:N] == -u_lim)
    assert log["Aineq"][0].shape == (m, N + 1) and log["Traj"][0].shape == (Hp, 2, nV)
    assert log["U"][0].shape == (Hp, 1, nV)
    for it in range(n_scp):
        x = log["x"][it].reshape(-1)
        fval = 0.5 * x @ log["P"][it] @ x + log["q"][it].reshape(-1) @ x + 2.5
        assert log["SCP_ObjVal"][it] == pytest.approx(fval, rel=1e-12)
        assert log["delta_hat"][it] == pytest.approx(tr[it, 8] - fval, rel=1e-12)
        assert log["slack"][it].shape == (1,) and log["slack"][it][0] == tr[it, 4]
        u = log["u"][it].reshape(-1)
        for v in range(nV):
            X = (const_term[:, :, v] + Mb[:, :, v] @ u[v * Hp:(v + 1) * Hp, None]).reshape(2, Hp, order="F")
            assert np.allclose(log["Traj"][it][:, :, v], X.T)
            assert np.allclose(log["U"][it][:, 0, v], u[v * Hp:(v + 1) * Hp])
        pu = log["prev_u"][it].reshape(-1)
        assert np.allclose(log["prevU"][it][:, 0, 0], pu[:Hp])


@pytest.mark.parametrize("config", ["c2", "c3", "c4", "c5"])
def test_round6_bench_records_carry_cpu_baseline_and_parity(config):
    """Verdict r05 item 6: every configuration's committed bench line carries the CPU
    baseline, the trajectory parity sample, the median step time beside the mean
     and the iteration maxima."""
    import json
    with open(os.path.join(ROOT, "profiles", f"r06_bench_{config}.json")) as fh:
        d = json.load(fh)
    blk = d["cpu_baseline"]
    assert blk["value"] > 0 and blk["cores"] >= 1 and blk["kind"] == "port" and blk["sample"]
    assert d["traj_linf_err"] is not None and d["traj_linf_err"] <= 1e-6
    assert d["ms_per_step_median"] > 0 and d["ms_per_step"] > 0
    assert 1 <= d["max_scp_iters"] <= 20 and d["max_ipm_iters_per_problem"] >= 1
    assert d["roofline"]["frac"] > 0 and d["value"] > 0


def test_traffic_record_registers_from_the_code_object():
    """Verdict r05 item 3: the c2 traffic record carries the descriptor's VGPR count and
    stack size (tools/kernel_resources.py), and the stack is back at <= 260 B per lane."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    path = bench.pmc_record("traffic", "c2")
    assert os.path.basename(path).startswith("r06_")
    with open(path) as fh:
        tj = json.load(fh)
    co = tj["code_object"]
    assert co["vgpr_count"] > 128 and co["private_segment_fixed_size"] <= 260
    assert tj["hbm_bytes_per_launch"] <= 4.3e9
