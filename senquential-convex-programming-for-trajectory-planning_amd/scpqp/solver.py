"""Batched solver object over the C-ABI (device buffers are torch-ROCm tensors).

``ScpQpSolver(scenario, ...)`` plays the role of the construction-time state of
``SCPcontroller`` (SCP_controller.py:19-38) for a whole batch: it holds the
scenario constants on the device.  ``solve`` runs the reference's
``SCP_controller`` (SCP_controller.py:40-197) for every problem of the batch in
one kernel launch; ``linearize``, ``evaluate`` and ``sample_reference`` expose
``MPCclass`` (MPC_Iter.py:59-149), ``QCQP_evaluate`` + ``forward_U``
(SCP_controller.py:199-265) and ``sampleReferenceTrajectory``
(SampleReferTraj.py:8-32).

PyTorch is only plumbing here: device memory and the stream.  Every array goes
through the HIP kernels; there is no host compute path.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib as LB

CONSTRAINT_TOL = 2 * 2.1 * 1e-3      # Config.py:18
DELTA_TOL = 1e-3                     # SCP_controller.py:83
SLACK_WEIGHT = 1e5                   # SCP_controller.py:84
MAX_SCP_ITER = 20                    # SCP_controller.py:86


def _dptr(arr):
    return arr.ctypes.data_as(C.POINTER(C.c_double))


def _vptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


@dataclass
class SolveResult:
    u: torch.Tensor          # [B, nVeh*Hp]  (vehicle-major; problem b uses its first nVeh*hp_b)
    traj: torch.Tensor       # [B, Hp, 2, nVeh]
    status: torch.Tensor     # [B] int32
    n_scp: torch.Tensor
    n_ipm: torch.Tensor
    obj: torch.Tensor
    max_violation: torch.Tensor
    sum_violations: torch.Tensor
    feasible: torch.Tensor
    n_polish: torch.Tensor   # active-set polish rounds (all QPs of the problem)
    n_refine: torch.Tensor   # multiplier-iteration solves (all QPs)
    n_warm: torch.Tensor     # QPs certified from the previous QP's active set
    trace: torch.Tensor = None   # [B, trace_iters, trace_stride] per-SCP-iteration record, or None


class ScpQpSolver:
    """Scenario-bound batched SCP-QP solver on one GPU."""

    def __init__(self, scenario, max_batch, device=None, hp_max=None, u_lim=None,
                 max_scp_iter=MAX_SCP_ITER, max_ipm_iter=60, ipm_tol=1e-9, polish_delta=3e-7,
                 polish_rho=1e-12, polish_refine=0, obstacle_quirk=True, warm_start=True):
        if not torch.cuda.is_available():
            raise RuntimeError("scpqp: no GPU visible; the HIP path has no CPU fallback")
        self.lib = LB.load()
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None \
            else torch.device(device)
        if self.device.index is None:          # "cuda" -> the current device, explicitly
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.nV = int(scenario.nVeh)
        self.nO = int(scenario.nObst)
        self.hp_max = int(hp_max or scenario.Hp)
        self.max_batch = int(max_batch)
        nV, nO = self.nV, self.nO
        self._keep = []

        def arr(x, shape=None, dtype=np.float64):
            a = np.ascontiguousarray(np.asarray(x, dtype=dtype).reshape(shape if shape else -1))
            self._keep.append(a)
            return a

        lf, lr = arr(scenario.Lf), arr(scenario.Lr)
        q, qf, r = arr(scenario.Q), arr(scenario.Q_final), arr(scenario.R)
        dv = arr(scenario.dsafeVehicles, (nV * nV,))
        do = arr(np.asarray(scenario.dsafeObstacles).reshape(-1) if nO else np.zeros(1))
        refs = [np.asarray(t, float).reshape(-1, 2) for t in scenario.referenceTrajectories]
        mp = max(2, max(len(t) for t in refs))
        if mp > LB.MAX_REFPTS:
            raise ValueError("reference polyline has too many points")
        poly = np.zeros((nV, mp, 2))
        npts = np.zeros(nV, np.int32)
        for v, t in enumerate(refs):
            poly[v, :len(t)] = t
            npts[v] = len(t)
        poly = arr(poly)
        npts = arr(npts, dtype=np.int32)
        self.u_lim = float(scenario.uLim if u_lim is None else u_lim)
        self.dt = float(scenario.dt)
        P = LB.Params(dt=self.dt, u_lim=self.u_lim, dsafe_extra=float(scenario.dsafeExtra),
                      constraint_tol=CONSTRAINT_TOL, delta_tol=DELTA_TOL, slack_weight=SLACK_WEIGHT,
                      max_scp_iter=max_scp_iter, max_ipm_iter=max_ipm_iter,
                      polish_refine=polish_refine,
                      flags=(LB.FLAG_OBST_QUIRK if obstacle_quirk else 0) |
                      (0 if warm_start else LB.FLAG_COLD_QP), ipm_tol=ipm_tol,
                      polish_delta=polish_delta, polish_rho=polish_rho,
                      lf=_dptr(lf), lr=_dptr(lr), q=_dptr(q), q_final=_dptr(qf), r=_dptr(r),
                      dsafe_veh=_dptr(dv), dsafe_obs=_dptr(do) if nO else None,
                      ref_polyline=_dptr(poly), ref_npts=npts.ctypes.data_as(C.POINTER(C.c_int32)),
                      ref_max_pts=mp)
        D = LB.Dims(n_veh=nV, hp_max=self.hp_max, n_obst=nO, max_batch=self.max_batch)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            LB.check(self.lib.scpqp_create(C.byref(D), C.byref(P), self.device.index or 0,
                                           C.byref(h)), self.lib)
        self.h = h
        self._keep = []

    def close(self):
        if getattr(self, "h", None):
            self.lib.scpqp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ utils
    def resources(self):
        lds, ws = C.c_int64(), C.c_int64()
        big, grid = C.c_int32(), C.c_int32()
        LB.check(self.lib.scpqp_resources(self.h, C.byref(lds), C.byref(ws), C.byref(big),
                                          C.byref(grid)), self.lib)
        return dict(lds_bytes=lds.value, ws_bytes_per_wg=ws.value, plan=big.value, grid=grid.value)

    def _dev(self, x, dtype=torch.float64):
        if x is None:
            return None
        if isinstance(x, torch.Tensor):
            return x.to(self.device, dtype).contiguous()
        return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=self.device)

    def _inputs(self, x0, u0=None, ec_noise=None, hp=None, obst=None, ref_points=None,
                u_warm=None, max_scp_iter=0, need_obst=True):
        """Move the inputs to the device and check every size against (B, nVeh, nObst,
        hp_max) before anything is launched: the kernel indexes each per-problem slot
        with hp_max strides.  Per-problem slots are sized for hp_max; a problem of
        horizon hp_b reads the PACKED prefix of its slot (obst [nObst][2][hp_b],
        ref_points [hp_b][2][nVeh], u_warm [nVeh*hp_b]), which equals the natural
        layout whenever hp_b == hp_max (scpqp.batch.pack_slots packs natural arrays)."""
        x0 = self._dev(x0)
        B = x0.shape[0] if x0.dim() > 0 else 0
        if B > self.max_batch:
            raise ValueError("batch larger than max_batch")
        nV, nO, Hm = self.nV, self.nO, self.hp_max
        _need(x0, B * nV * 6, "x0 [B, nVeh, 6]")
        u0 = self._dev(u0) if u0 is not None else torch.zeros(B, nV, dtype=torch.float64,
                                                             device=self.device)
        _need(u0, B * nV, "u0 [B, nVeh]")
        ec = self._dev(ec_noise)
        _need(ec, B * nV * 2, "ec_noise [B, nVeh, 2]")
        if hp is not None and not isinstance(hp, torch.Tensor):
            h = np.asarray(hp).reshape(-1)
            if h.size == B and B and bool(np.all(h == Hm)):
                # every problem at hp_max is the no-hp form: the kernel may then run the
                # launch on its compiled-shape instantiation (csrc shape_c)
                hp = None
        hpt = self._dev(hp, torch.int32)
        _need(hpt, B, "hp [B]")
        if need_obst and nO and obst is None:
            raise ValueError("scenario has obstacles: pass obst [B, nObst, 2, Hp]")
        ob = self._dev(obst) if nO else None
        _need(ob, B * nO * 2 * Hm, "obst [B, nObst, 2, hp_max] (packed per slot)")
        rp = self._dev(ref_points)
        _need(rp, B * Hm * 2 * nV, "ref_points [B, hp_max, 2, nVeh] (packed per slot)")
        uw = self._dev(u_warm)
        _need(uw, B * nV * Hm, "u_warm [B, nVeh*hp_max] (packed per slot)")
        bufs = (x0, u0, ec, hpt, ob, rp, uw)
        bi = LB.BatchIn(x0=_vptr(x0), u0=_vptr(u0), ec_noise=_vptr(ec), hp=_vptr(hpt),
                        obst=_vptr(ob), ref_points=_vptr(rp), u_warm=_vptr(uw),
                        max_scp_iter=int(max_scp_iter), reserved=0)
        return B, bi, bufs

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ entry points
    def solve(self, x0, u0=None, ec_noise=None, hp=None, obst=None, ref_points=None, u_warm=None,
              max_scp_iter=0, out=None, trace=False):
        """SCP_controller for a batch.  Arrays: x0 [B,nVeh,6], u0 [B,nVeh], ec_noise [B,nVeh,2],
        hp [B] int, obst [B,nObst,2,hp_max], ref_points [B,hp_max,2,nVeh], u_warm
        [B,nVeh*hp_max]; per-problem slots are read as packed prefixes for hp_b < hp_max
        (see _inputs).  ``trace=True`` also records every SCP iteration (the reference's
        optimization_log, SCP_controller.py:169-189) into ``out.trace``; decode it with
        scpqp.trace.decode."""
        B, bi, bufs = self._inputs(x0, u0, ec_noise, hp, obst, ref_points, u_warm, max_scp_iter)
        if out is None:
            out = self.alloc_out(B, trace=trace)
        self._check_out(out, B)
        bo = LB.BatchOut(u=_vptr(out.u), traj=_vptr(out.traj), status=_vptr(out.status),
                         n_scp=_vptr(out.n_scp), n_ipm=_vptr(out.n_ipm), obj=_vptr(out.obj),
                         max_violation=_vptr(out.max_violation),
                         sum_violations=_vptr(out.sum_violations), feasible=_vptr(out.feasible),
                         n_polish=_vptr(out.n_polish), n_refine=_vptr(out.n_refine),
                         n_warm=_vptr(out.n_warm), trace=_vptr(out.trace))
        LB.check(self.lib.scpqp_solve(self.h, B, C.byref(bi), C.byref(bo), self._stream()),
                 self.lib)
        self._last_inputs = bufs   # keep device inputs alive until the stream consumes them
        return out

    def trace_layout(self):
        """(doubles per SCP iteration, iterations per problem) of SolveResult.trace."""
        st, it = C.c_int32(), C.c_int32()
        LB.check(self.lib.scpqp_trace_layout(self.h, C.byref(st), C.byref(it)), self.lib)
        return st.value, it.value

    def alloc_out(self, B, trace=False):
        dev, Hm, nV = self.device, self.hp_max, self.nV
        f = dict(dtype=torch.float64, device=dev)
        i = dict(dtype=torch.int32, device=dev)
        tr = None
        if trace:
            st, it = self.trace_layout()
            tr = torch.full((B, it, st), float("nan"), **f)
        return SolveResult(u=torch.zeros(B, nV * Hm, **f), traj=torch.zeros(B, Hm, 2, nV, **f),
                           status=torch.zeros(B, **i), n_scp=torch.zeros(B, **i),
                           n_ipm=torch.zeros(B, **i), obj=torch.zeros(B, **f),
                           max_violation=torch.zeros(B, **f), sum_violations=torch.zeros(B, **f),
                           feasible=torch.zeros(B, **i), n_polish=torch.zeros(B, **i),
                           n_refine=torch.zeros(B, **i), n_warm=torch.zeros(B, **i), trace=tr)

    def _check_out(self, out, B):
        """Every output buffer must hold B problems' slots on this device (the kernel
        writes b * slot strides without bounds), contiguous, of the right dtype."""
        nV, Hm = self.nV, self.hp_max
        sizes = dict(u=B * nV * Hm, traj=B * Hm * 2 * nV, status=B, n_scp=B, n_ipm=B, obj=B,
                     max_violation=B, sum_violations=B, feasible=B, n_polish=B, n_refine=B,
                     n_warm=B)
        if out.trace is not None:
            st, it = self.trace_layout()
            sizes["trace"] = B * st * it
        for k, n in sizes.items():
            t = getattr(out, k)
            want = torch.int32 if k in ("status", "n_scp", "n_ipm", "feasible", "n_polish",
                                        "n_refine", "n_warm") else torch.float64
            if t is None:
                raise ValueError(f"output {k} is missing")
            if t.device != self.device or t.dtype != want or not t.is_contiguous() or t.numel() < n:
                raise ValueError(f"output {k}: need a contiguous {want} tensor of >= {n} "
                                 f"elements on {self.device}")

    def linearize(self, x0, u0=None, ec_noise=None, hp=None, obst=None, ref_points=None):
        B, bi, bufs = self._inputs(x0, u0, ec_noise, hp, obst, ref_points, need_obst=False)
        nV, Hm, dev = self.nV, self.hp_max, self.device
        f = dict(dtype=torch.float64, device=dev)
        res = dict(Ad=torch.zeros(B, nV, 6, 6, **f), Bd=torch.zeros(B, nV, 6, **f),
                   Ed=torch.zeros(B, nV, 6, **f), g=torch.zeros(B, nV, Hm, 2, **f),
                   const_term=torch.zeros(B, nV, Hm, 2, **f), psi0=torch.zeros(B, nV, Hm, **f),
                   ref_points=torch.zeros(B, Hm, 2, nV, **f))
        lo = LB.LinOut(**{k: _vptr(v) for k, v in res.items()})
        LB.check(self.lib.scpqp_linearize(self.h, B, C.byref(bi), C.byref(lo), self._stream()),
                 self.lib)
        torch.cuda.current_stream(dev).synchronize()
        return res

    def evaluate(self, u, x0, u0=None, ec_noise=None, hp=None, obst=None, ref_points=None):
        B, bi, bufs = self._inputs(x0, u0, ec_noise, hp, obst, ref_points)
        nV, nO, Hm, dev = self.nV, self.nO, self.hp_max, self.device
        ut = self._dev(u).reshape(B, -1)
        if ut.shape[1] < nV * Hm:
            ut = torch.nn.functional.pad(ut, (0, nV * Hm - ut.shape[1]))
        ut = ut.contiguous()
        f = dict(dtype=torch.float64, device=dev)
        res = dict(obj=torch.zeros(B, **f), max_violation=torch.zeros(B, **f),
                   sum_violations=torch.zeros(B, **f),
                   feasible=torch.zeros(B, dtype=torch.int32, device=dev),
                   c_veh=torch.zeros(B, nV, nV, Hm, **f), c_obs=torch.zeros(B, nV, max(nO, 1), Hm, **f),
                   traj=torch.zeros(B, Hm, 2, nV, **f))
        eo = LB.EvalOut(**{k: _vptr(v) for k, v in res.items()})
        LB.check(self.lib.scpqp_evaluate(self.h, B, C.byref(bi), C.c_void_p(ut.data_ptr()),
                                         C.byref(eo), self._stream()), self.lib)
        torch.cuda.current_stream(dev).synchronize()
        return res

    def sample_reference(self, x0, hp=None):
        B, bi, bufs = self._inputs(x0, hp=hp, need_obst=False)
        ref = torch.zeros(B, self.hp_max, 2, self.nV, dtype=torch.float64, device=self.device)
        LB.check(self.lib.scpqp_sample_reference(self.h, B, C.byref(bi),
                                                 C.c_void_p(ref.data_ptr()), self._stream()),
                 self.lib)
        torch.cuda.current_stream(self.device).synchronize()
        return ref


def _need(t, n, what):
    """Exact element count of an optional device input (None passes)."""
    if t is not None and t.numel() != n:
        raise ValueError(f"{what}: expected {n} elements, got {t.numel()} (shape "
                         f"{tuple(t.shape)})")


def unpack_problem(res, b, nV, hp):
    """Slice problem b of a batched result into the reference's shapes for its horizon."""
    u = res.u[b, :nV * hp]
    traj = res.traj[b].reshape(-1)[:hp * 2 * nV].reshape(hp, 2, nV)
    return u, traj
