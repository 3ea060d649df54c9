"""Decode the per-SCP-iteration trace of ``ScpQpSolver.solve(..., trace=True)``.

The kernel records, for every SCP iteration of every problem, what the
reference keeps in ``controllerOutput['optimization_log']`` and in its loop
state (SCP_controller.py:148-189): the iterate the constraints are linearised
at, the linearised rows, the QP's solution with its slack, and the stopping-rule
terms (obj, max violation, delta).  Layout: include/scpqp.h, scpqp_batch_out.trace.

Rows are stored in the kernel's factored, scaled form:
``e_r = 2 d uLim / nrm``, ``w_r = -1 / nrm``, ``h_r = b_r / nrm``.  The dense
``Aineq`` / ``bineq`` of SCP_controller.py:100-101,125 follow from them and the
Toeplitz blocks g_m of ``scpqp_linearize``: row (i, j, k) has
``A[i-block, l] = -2 d' g_{k-l}``, ``A[j-block, l] = +2 d' g_{k-l}`` (l <= k),
``A[omega] = -1`` and ``b = h nrm``.  This is host-side bookkeeping for tests
and logs; nothing here is on the solve path.
"""
from __future__ import annotations

import numpy as np

HDR = 10   # header doubles of one iteration record (include/scpqp.h)


def row_list(nV, H, nO):
    """Row order of SCP_controller.py:97-114: pairs (i<j), k innermost, then (v, o, k)."""
    rows = [(i, j, -1, k) for i in range(nV - 1) for j in range(i + 1, nV) for k in range(H)]
    rows += [(i, -1, o, k) for i in range(nV) for o in range(nO) for k in range(H)]
    return rows


def decode(trace_b, n_iter, nV, nO, H, hp_max, g=None, u_lim=None):
    """Problem b's trace [iters, stride] (numpy) -> list of per-iteration dicts with
    the oracle's history keys (u_lin, z, obj, maxviol, delta, ...) and, when the
    Toeplitz blocks ``g`` [nV, H, 2] and ``u_lim`` are given, the dense rows A [m, N+1]
    and b [m] of SCP_controller.py:93-128."""
    N, Nm = nV * H, nV * hp_max
    m = len(row_list(nV, H, nO))
    out = []
    for it in range(n_iter):
        t = np.asarray(trace_b[it], float)
        rows = t[HDR + 2 * Nm:HDR + 2 * Nm + 4 * m].reshape(m, 4)
        d = dict(delta=t[0], obj=t[1], maxviol=t[2], sumviol=t[3], slack=t[4],
                 ipm_iters=int(t[5]), certified=bool(int(t[6]) & 1), warm=bool(int(t[6]) & 2),
                 feasible=bool(t[7]), merit0=t[8], polish_rounds=int(t[9]) % 4096,
                 polish_solves=int(t[9]) // 4096, u_lin=t[HDR:HDR + N].copy(),
                 z=np.concatenate([t[HDR + Nm:HDR + Nm + N], t[4:5]]), rows=rows.copy())
        if g is not None:
            d["A"], d["b"] = dense_rows(rows, np.asarray(g, float).reshape(nV, H, 2), nV, nO, H,
                                        u_lim)
        out.append(d)
    return out


def dense_rows(rows, g, nV, nO, H, u_lim):
    """Factored scaled rows [m, 4] -> Aineq [m, N+1], bineq [m] (SCP_controller.py:100-101,125)."""
    N = nV * H
    m = rows.shape[0]
    A = np.zeros((m, N + 1))
    b = np.zeros(m)
    for r, (i, j, o, k) in enumerate(row_list(nV, H, nO)):
        e0, e1, w, h = rows[r]
        nrm = -1.0 / w
        dx, dy = e0 * nrm / (2 * u_lim), e1 * nrm / (2 * u_lim)
        gk = g[:, k::-1, :]                          # g_{k-l} for l = 0..k, [nV, k+1, 2]
        A[r, H * i:H * i + k + 1] = -2 * (dx * gk[i, :, 0] + dy * gk[i, :, 1])
        if j >= 0:
            A[r, H * j:H * j + k + 1] = 2 * (dx * gk[j, :, 0] + dy * gk[j, :, 1])
        A[r, N] = -1.0
        b[r] = h * nrm
    return A, b
