"""Handle cache behind the drop-in modules (MPC_Iter, SCP_controller, SampleReferTraj).

The reference rebuilds its solver state every MPC step (``SCPcontroller``
construction, main.py:131-133).  Here the scenario constants are uploaded once:
one ``ScpQpSolver`` (max_batch 1) is cached on the scenario object and reused
as long as the fields the device copy depends on are unchanged.  Polyline
samplers for the free function ``sampleReferenceTrajectory`` are cached by
polyline content.
"""
from __future__ import annotations

import hashlib
from types import SimpleNamespace

import numpy as np

_SAMPLERS: dict = {}
SAMPLER_HP = 64          # SCPQP_MAX_HP


def _digest(*arrays):
    h = hashlib.sha1()
    for a in arrays:
        h.update(np.ascontiguousarray(np.asarray(a, dtype=np.float64)).tobytes())
        h.update(b"|")
    return h.hexdigest()


def scenario_signature(sc):
    refs = [np.asarray(t, float) for t in sc.referenceTrajectories]
    return (int(sc.nVeh), int(sc.nObst), int(sc.Hp), float(sc.dt), float(sc.dsafeExtra),
            float(sc.uLim),
            _digest(sc.Lf, sc.Lr, sc.Q, sc.Q_final, sc.R, sc.dsafeVehicles,
                    np.asarray(sc.dsafeObstacles).reshape(-1), *refs))


def solver_for(sc):
    """The cached single-problem device solver of scenario ``sc``."""
    from .solver import ScpQpSolver
    sig = scenario_signature(sc)
    cached = getattr(sc, "_scpqp_cache", None)
    if cached is not None and cached[0] == sig:
        return cached[1]
    if cached is not None:
        cached[1].close()
    solver = ScpQpSolver(sc, max_batch=1)
    sc._scpqp_cache = (sig, solver)
    return solver


def sampler_for(polyline):
    """A one-vehicle handle whose only job is the reference sampler on ``polyline``.

    dt = 1 so that the device step size (speed * dt) equals the caller's stepSize.
    """
    from .solver import ScpQpSolver
    poly = np.asarray(polyline, dtype=float).reshape(-1, 2)
    key = _digest(poly)
    s = _SAMPLERS.get(key)
    if s is None:
        ns = SimpleNamespace(nVeh=1, nObst=0, Hp=SAMPLER_HP, Lf=[.34], Lr=[.34], Q=[1.0],
                             Q_final=[1.0], R=[1.0], dsafeVehicles=np.zeros((1, 1)),
                             dsafeObstacles=np.zeros((1, 0)), referenceTrajectories=[poly],
                             uLim=1.0, dt=1.0, dsafeExtra=0.0)
        s = ScpQpSolver(ns, max_batch=1)
        _SAMPLERS[key] = s
    return s
