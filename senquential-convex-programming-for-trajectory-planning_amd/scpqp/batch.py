"""Synthetic problem batches.

A *problem* is one joint SCP solve of all vehicles of a scenario: what the
reference's ``main.py`` hands to ``SCPcontroller`` at one MPC step
(main.py:123-134).  A batch is many such problems of ONE scenario (same vehicle
geometry, weights and reference polylines), each with its own measured state
and noise draws.  Inputs are generated on the host from per-problem seeds
(``base_seed + global_index``), so a problem's data does not depend on how the
batch is sharded over ranks.

Layout (all float64, C-contiguous, problem-major so each workgroup reads one
contiguous slab):

=============  ======================  =========================================
array          shape                   meaning (reference field)
=============  ======================  =========================================
``x0``         [B, nVeh, 6]            Iter.x0 (MPC_Iter.py:30)
``u0``         [B, nVeh]               Iter.u0 (MPC_Iter.py:31)
``ec_noise``   [B, nVeh, 2]            the two N(0, 3e-6) draws Model.py:85-86
                                       adds to dx[0], dx[1] inside comp_jacobian
``hp``         [B] int32               per-problem horizon (mixed-horizon c5)
``obst``       [B, nObst, 2, Hp_max]   Iter.obstacleFutureTrajectories; each
                                       slot holds [nObst][2][hp_b] packed
=============  ======================  =========================================
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# x0 perturbation std: x, y, heading, speed, accel, steering
X0_SIGMA = np.array([0.05, 0.05, 0.005, 0.02, 0.0, 0.002])
EC_SIGMA = 3e-6          # Model.py:85-86: np.random.normal(0, 0.000003)


@dataclass
class Batch:
    x0: np.ndarray
    u0: np.ndarray
    ec_noise: np.ndarray
    hp: np.ndarray
    obst: np.ndarray
    hp_max: int
    seeds: np.ndarray

    @property
    def size(self):
        return self.x0.shape[0]

    def slice(self, lo, hi):
        return Batch(self.x0[lo:hi], self.u0[lo:hi], self.ec_noise[lo:hi], self.hp[lo:hi],
                     self.obst[lo:hi], self.hp_max, self.seeds[lo:hi])


def delay_compensated_nominal(scenario):
    """Nominal Iter.x0 at MPC step 0: with u = 0, a = 0, delta = 0 the bicycle
    drives straight for delay_x + dt + delay_u seconds (MPC_Iter.py:25-33)."""
    T = scenario.delay_x + scenario.dt + scenario.delay_u
    out = np.zeros((scenario.nVeh, 6))
    for v in range(scenario.nVeh):
        x = np.asarray(scenario.x0[v], float).reshape(-1)
        travel = x[3] * T
        out[v] = x
        out[v, 0] += travel * math.cos(x[2])
        out[v, 1] += travel * math.sin(x[2])
    return out


def obstacle_prediction(scenario, hp, obstacle_xy=None):
    """MPC_Iter.py:45-51: constant-velocity obstacle positions [nObst, 2, hp]."""
    obs = np.asarray(scenario.obstacles, float).reshape(-1, 6) if scenario.nObst else np.zeros((0, 6))
    nO = obs.shape[0]
    xy = obs[:, :2] if obstacle_xy is None else np.asarray(obstacle_xy, float).reshape(nO, 2)
    out = np.zeros((nO, 2, hp))
    lead = scenario.delay_x + scenario.dt + scenario.delay_u
    for k in range(hp):
        step = ((k + 1) * scenario.dt + lead) * obs[:, 3]
        out[:, 0, k] = step * np.cos(obs[:, 2]) + xy[:, 0]
        out[:, 1, k] = step * np.sin(obs[:, 2]) + xy[:, 1]
    return out


def make_batch(scenario, B, base_seed=0, offset=0, perturb=True, noise=True, hp=None,
               mixed_hp=None):
    """Problems ``offset .. offset+B-1`` of the synthetic stream for ``scenario``.

    ``mixed_hp``: a sequence of horizons; problem g gets ``mixed_hp[g % len]``
    (config c5).  Otherwise every problem uses ``hp`` (default scenario.Hp).
    """
    nV, nO = scenario.nVeh, scenario.nObst
    hps = np.full(B, scenario.Hp if hp is None else hp, dtype=np.int32)
    if mixed_hp is not None:
        hps = np.array([mixed_hp[(offset + b) % len(mixed_hp)] for b in range(B)], dtype=np.int32)
    hp_max = int(hps.max()) if B else int(scenario.Hp if hp is None else hp)
    if mixed_hp is not None:
        hp_max = int(max(mixed_hp))
    nominal = delay_compensated_nominal(scenario)
    x0 = np.repeat(nominal[None], B, axis=0)
    ec = np.zeros((B, nV, 2))
    seeds = base_seed + offset + np.arange(B, dtype=np.int64)
    if perturb or noise:
        for b in range(B):
            g = np.random.Generator(np.random.PCG64(int(seeds[b])))
            dx = g.standard_normal((nV, 6)) * X0_SIGMA
            en = g.standard_normal((nV, 2)) * EC_SIGMA
            if perturb:
                x0[b] += dx
            if noise:
                ec[b] = en
    u0 = np.zeros((B, nV))
    # per-problem slot of nObst*2*hp_max doubles holding [nObst][2][hp_b] packed
    # (include/scpqp.h: per-problem arrays use their own horizon inside the slot)
    obst = np.zeros((B, nO, 2, hp_max))
    if nO:
        flat = obst.reshape(B, -1)
        for H in np.unique(hps):
            base = obstacle_prediction(scenario, int(H)).reshape(-1)
            flat[hps == H, :base.size] = base
    return Batch(np.ascontiguousarray(x0), u0, ec, hps, obst, hp_max, seeds)


def pack_slots(natural, hp, trailing_hp_axis):
    """Natural per-problem arrays -> the packed per-slot layout the C-ABI reads.

    ``natural`` is [B, ..., hp_max] with the horizon on axis ``trailing_hp_axis``
    (counted within one problem: obst [nObst, 2, hp_max] -> axis 2, ref_points
    [hp_max, 2, nVeh] -> axis 0, u_warm [nVeh, hp_max] -> axis 1).  Problem b's
    slot receives its first hp[b] steps as one contiguous prefix, i.e. the
    array [..., hp_b] C-contiguous, zero-padded to the slot size.  For hp_b ==
    hp_max this is the identity."""
    nat = np.asarray(natural, float)
    B = nat.shape[0]
    out = np.zeros((B, int(np.prod(nat.shape[1:]))))
    for b in range(B):
        H = int(hp[b])
        sl = [slice(None)] * (nat.ndim - 1)
        sl[trailing_hp_axis] = slice(0, H)
        blk = np.ascontiguousarray(nat[b][tuple(sl)]).reshape(-1)
        out[b, :blk.size] = blk
    return out.reshape(nat.shape)
