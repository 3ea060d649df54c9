"""Drop-in for the reference's ``SampleReferTraj.py`` (SampleReferTraj.py:1-122).

``sampleReferenceTrajectory`` runs the GPU sampler (``scpqp_sample_reference``)
on a handle cached per polyline; the argument checks of the reference
(segment longer than the step, SampleReferTraj.py:18-19) are raised on the
host before the launch.  ``getShortestDistance`` / ``Projection2D`` are the
reference's public geometry helpers, kept as host functions for callers that
use them directly; the sampling path itself never calls them (the kernel
carries its own projection, B.1/B.2 quirks included).
"""
from math import sqrt

import numpy as np


def normalize(x):
    return x / np.linalg.norm(x, 2)


def sampleReferenceTrajectory(nSamples, referenceTrajectory, vehicle_x, vehicle_y, stepSize):
    """``nSamples`` points spaced ``stepSize`` along the polyline from the
    projection of (vehicle_x, vehicle_y) (SampleReferTraj.py:8-32)."""
    from scpqp.dropin import SAMPLER_HP, sampler_for
    poly = np.asarray(referenceTrajectory, dtype=float).reshape(-1, 2)
    for i in range(poly.shape[0] - 1):
        assert np.linalg.norm(poly[i + 1] - poly[i], 2) > stepSize
    n = int(nSamples)
    if not 0 < n <= SAMPLER_HP:
        raise ValueError(f"nSamples must be in 1..{SAMPLER_HP}")
    s = sampler_for(poly)
    x0 = np.array([[[float(vehicle_x), float(vehicle_y), 0.0, float(stepSize), 0.0, 0.0]]])
    ref = s.sample_reference(x0, hp=np.array([n], np.int32))
    return ref[0, :n, :, 0].cpu().numpy()


def getShortestDistance(curve_x, curve_y, x, y):
    """Closest point of a polyline to (x, y): (signed distance, arc length,
    x_min, y_min, segment index) (SampleReferTraj.py:34-79)."""
    assert isinstance(x, (int, float))
    assert isinstance(y, (int, float))
    assert len(curve_x) == len(curve_y)
    assert len(curve_x) >= 2
    # the reference seeds its search with the second vertex and index 2
    best = [sqrt((x - curve_x[1]) ** 2 + (y - curve_y[1]) ** 2), 0, curve_x[1], curve_y[1], 2]
    travelled = 0
    last = len(curve_x) - 1
    for j in range(1, len(curve_x)):
        xp, yp, sd, lam, seg = Projection2D(curve_x[j - 1], curve_y[j - 1], curve_x[j], curve_y[j],
                                            x, y)
        inside = (lam > 0 or j == 1) and (lam < 1 or j == last)
        if inside:
            if abs(sd) < abs(best[0]):
                best = [sd, travelled + lam * seg, xp, yp, j]
        else:
            # the reference writes '^' here (a TypeError on floats); '**' is used
            d_end = sqrt((x - curve_x[j]) ** 2 + (y - curve_y[j]) ** 2)
            if d_end < abs(best[0]):
                best = [np.sign(sd) * d_end, travelled + seg, curve_x[j], curve_y[j], j]
        travelled += seg
    return tuple(best)


def Projection2D(x1, y1, x2, y2, x3, y3):
    """Projection of (x3, y3) on the line through (x1, y1), (x2, y2):
    (xp, yp, signed distance, line parameter, segment length) (SampleReferTraj.py:81-122)."""
    seg = sqrt((x2 - x1) ** 2 + (y2 - y1) ** 2)
    if seg == 0:
        return x1, y1, sqrt((x3 - x1) ** 2 + (y3 - y1) ** 2), 0, seg
    ux, uy = (x2 - x1) / seg, (y2 - y1) / seg
    rx, ry = x3 - x1, y3 - y1
    along = ux * rx + uy * ry
    across = ux * ry - uy * rx
    return x1 + along * ux, y1 + along * uy, across, along / seg, seg
