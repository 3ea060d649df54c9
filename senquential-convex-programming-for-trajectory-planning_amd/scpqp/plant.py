"""The bicycle plant around the solve, batched on the GPU (csrc/plant.hip).

``delay_compensate``  IterClass delay compensation (MPC_Iter.py:24-33)
``plant_step``        closed-loop plant simulation of one MPC step (main.py:176-191)
``clip_controls``     steering-limit enforcement (main.py:164-174)

Arrays are torch-ROCm float64 tensors on the GPU; PyTorch only provides the
memory and the stream.  The reference integrates with scipy (odeint / dopri5);
the kernels use fixed-step RK4 with steps of at most ``h_max`` seconds (default
2.5 ms: ~1e-11 from the exact flow, below the reference's 1e-8 tolerances).
There is no CPU path: without the HIP library or a GPU these raise.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as LB

H_MAX = 2.5e-3
STEER_TAU = 0.1       # Model.py:83: dx[5] = (u_ref - u) / 0.1
DELAY_STEPS = 10      # MPC_Iter.py:21: outputs of the delay-compensation trajectory


def plant_params(lf, lr):
    """scpqp_plant_params for per-vehicle axle distances (Model.py:26-27)."""
    lf = [float(v) for v in lf]
    lr = [float(v) for v in lr]
    if not 1 <= len(lf) <= LB.MAX_VEH or len(lr) != len(lf):
        raise ValueError("need 1..16 vehicles with lf and lr each")
    p = LB.PlantParams()
    p.n_veh = len(lf)
    for v in range(len(lf)):
        p.lf[v] = lf[v]
        p.lr[v] = lr[v]
    return p


def _dev(t, device):
    return torch.as_tensor(t, dtype=torch.float64, device=device).contiguous()


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def delay_compensate(params, x_meas, u_hold, horizon, n_out=DELAY_STEPS, noise=None, h_max=H_MAX,
                     device=None, want_traj=True):
    """x_meas [B, nVeh, 6], u_hold [B, nVeh] -> (x0 [B, nVeh, 6],
    traj [B, n_out, 6, nVeh] or None): MPC_Iter.py:24-33 for every problem."""
    device = torch.device(device or "cuda")
    lib = LB.load()
    x = _dev(x_meas, device)
    u = _dev(u_hold, device)
    B, V = int(x.shape[0]), params.n_veh
    if tuple(x.shape) != (B, V, 6) or tuple(u.shape) != (B, V):
        raise ValueError("x_meas must be [B, nVeh, 6] and u_hold [B, nVeh]")
    nz = None if noise is None else _dev(noise, device)
    if nz is not None and tuple(nz.shape) != (B, V, 2):
        raise ValueError("noise must be [B, nVeh, 2]")
    x0 = torch.empty((B, V, 6), dtype=torch.float64, device=device)
    traj = torch.empty((B, n_out, 6, V), dtype=torch.float64, device=device) if want_traj else None
    LB.check(lib.scpqp_delay_compensate(C.byref(params), B, float(horizon), int(n_out), _ptr(x),
                                        _ptr(u), _ptr(nz), _ptr(x0), _ptr(traj), float(h_max),
                                        _stream(device)), lib)
    return x0, traj


def plant_step(params, x_start, u_tick, tick, noise=None, h_max=H_MAX, device=None):
    """x_start [B, nVeh, 6], u_tick [B, nVeh, K] (K = ticks_per_sim + 1) ->
    x_path [B, nVeh, K, 6]: main.py:184-191 (output k integrated from t0 over
    k ticks with the constant control u_tick[..., k])."""
    device = torch.device(device or "cuda")
    lib = LB.load()
    x = _dev(x_start, device)
    u = _dev(u_tick, device)
    B, V = int(x.shape[0]), params.n_veh
    K = int(u.shape[-1])
    if tuple(x.shape) != (B, V, 6) or tuple(u.shape) != (B, V, K) or K < 1:
        raise ValueError("x_start must be [B, nVeh, 6] and u_tick [B, nVeh, K]")
    nz = None if noise is None else _dev(noise, device)
    out = torch.empty((B, V, K, 6), dtype=torch.float64, device=device)
    LB.check(lib.scpqp_plant_step(C.byref(params), B, K - 1, float(tick), _ptr(x), _ptr(u),
                                  _ptr(nz), _ptr(out), float(h_max), _stream(device)), lib)
    return out


def clip_controls(u, u0, umax, n_veh, hp, du_lim):
    """In place on the solver's vehicle-major controls u [B, >= nVeh*hp]
    (main.py:164-174).  u0, umax: [B, nVeh] device tensors."""
    lib = LB.load()
    if u.dtype != torch.float64 or not u.is_contiguous() or u.dim() != 2:
        raise ValueError("u must be a contiguous float64 [B, ld] tensor")
    u0 = _dev(u0, u.device)
    um = _dev(umax, u.device)
    B, ld = int(u.shape[0]), int(u.shape[1])
    LB.check(lib.scpqp_clip_controls(B, int(n_veh), int(hp), ld, float(du_lim), _ptr(u), _ptr(u0),
                                     _ptr(um), _stream(u.device)), lib)
    return u
