"""ctypes binding of ``include/scpqp.h`` (the C-ABI of the HIP library).

The shared library ``libscpqp.so`` is built in-tree (``__graft_entry__.build()``
or ``python -m scpqp.build``).  There is no CPU fallback: if the library or a
GPU is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libscpqp.so")

MAX_VEH = 16
MAX_OBST = 32
MAX_REFPTS = 8
MAX_HP = 64

ST_CONVERGED = 0
ST_MAX_SCP = 1
ST_INVALID = 2
ST_NUMERIC = 3
FL_POLISH_REJECTED = 0x100
FL_IPM_MAXIT = 0x200
FL_SAMPLER = 0x400
FLAG_OBST_QUIRK = 1
FLAG_COLD_QP = 2

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class Dims(C.Structure):
    _fields_ = [("n_veh", C.c_int32), ("hp_max", C.c_int32), ("n_obst", C.c_int32),
                ("max_batch", C.c_int32)]


class Params(C.Structure):
    _fields_ = [("dt", C.c_double), ("u_lim", C.c_double), ("dsafe_extra", C.c_double),
                ("constraint_tol", C.c_double), ("delta_tol", C.c_double),
                ("slack_weight", C.c_double), ("max_scp_iter", C.c_int32),
                ("max_ipm_iter", C.c_int32), ("polish_refine", C.c_int32), ("flags", C.c_int32),
                ("ipm_tol", C.c_double), ("polish_delta", C.c_double), ("polish_rho", C.c_double),
                ("lf", _dp), ("lr", _dp), ("q", _dp), ("q_final", _dp), ("r", _dp),
                ("dsafe_veh", _dp), ("dsafe_obs", _dp), ("ref_polyline", _dp),
                ("ref_npts", _ip), ("ref_max_pts", C.c_int32)]


class BatchIn(C.Structure):
    _fields_ = [("x0", C.c_void_p), ("u0", C.c_void_p), ("ec_noise", C.c_void_p),
                ("hp", C.c_void_p), ("obst", C.c_void_p), ("ref_points", C.c_void_p),
                ("u_warm", C.c_void_p), ("max_scp_iter", C.c_int32), ("reserved", C.c_int32)]


class BatchOut(C.Structure):
    _fields_ = [("u", C.c_void_p), ("traj", C.c_void_p), ("status", C.c_void_p),
                ("n_scp", C.c_void_p), ("n_ipm", C.c_void_p), ("obj", C.c_void_p),
                ("max_violation", C.c_void_p), ("sum_violations", C.c_void_p),
                ("feasible", C.c_void_p), ("n_polish", C.c_void_p), ("n_refine", C.c_void_p),
                ("n_warm", C.c_void_p), ("trace", C.c_void_p)]


class LinOut(C.Structure):
    _fields_ = [("Ad", C.c_void_p), ("Bd", C.c_void_p), ("Ed", C.c_void_p), ("g", C.c_void_p),
                ("const_term", C.c_void_p), ("psi0", C.c_void_p), ("ref_points", C.c_void_p)]


class EvalOut(C.Structure):
    _fields_ = [("obj", C.c_void_p), ("max_violation", C.c_void_p),
                ("sum_violations", C.c_void_p), ("feasible", C.c_void_p), ("c_veh", C.c_void_p),
                ("c_obs", C.c_void_p), ("traj", C.c_void_p)]


class PlantParams(C.Structure):
    _fields_ = [("n_veh", C.c_int32), ("pad0", C.c_int32), ("lf", C.c_double * MAX_VEH),
                ("lr", C.c_double * MAX_VEH)]


# every symbol include/scpqp.h declares (checked by tests/test_abi.py)
EXPORTS = ("scpqp_create", "scpqp_destroy", "scpqp_last_error", "scpqp_version", "scpqp_solve",
           "scpqp_linearize", "scpqp_evaluate", "scpqp_sample_reference", "scpqp_resources",
           "scpqp_trace_layout",
           "scpqp_delay_compensate", "scpqp_plant_step", "scpqp_clip_controls")

_lib = None


def load(path=None):
    """Load the in-tree HIP library (raises OSError if it was not built).  The product
    path reads no environment variable: another build is loaded only by an explicit
    ``path`` or by ``use_build`` (benchmark and tools A/B runs)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise OSError(f"scpqp: HIP library not built ({p}); run __graft_entry__.build()")
    lib = C.CDLL(p)
    H = C.c_void_p
    lib.scpqp_create.argtypes = [C.POINTER(Dims), C.POINTER(Params), C.c_int, C.POINTER(H)]
    lib.scpqp_create.restype = C.c_int
    lib.scpqp_destroy.argtypes = [H]
    lib.scpqp_destroy.restype = C.c_int
    lib.scpqp_last_error.argtypes = []
    lib.scpqp_last_error.restype = C.c_char_p
    lib.scpqp_version.argtypes = []
    lib.scpqp_version.restype = C.c_char_p
    lib.scpqp_solve.argtypes = [H, C.c_int32, C.POINTER(BatchIn), C.POINTER(BatchOut), C.c_void_p]
    lib.scpqp_solve.restype = C.c_int
    lib.scpqp_linearize.argtypes = [H, C.c_int32, C.POINTER(BatchIn), C.POINTER(LinOut), C.c_void_p]
    lib.scpqp_linearize.restype = C.c_int
    lib.scpqp_evaluate.argtypes = [H, C.c_int32, C.POINTER(BatchIn), C.c_void_p,
                                   C.POINTER(EvalOut), C.c_void_p]
    lib.scpqp_evaluate.restype = C.c_int
    lib.scpqp_sample_reference.argtypes = [H, C.c_int32, C.POINTER(BatchIn), C.c_void_p, C.c_void_p]
    lib.scpqp_sample_reference.restype = C.c_int
    lib.scpqp_resources.argtypes = [H, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                    C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    lib.scpqp_resources.restype = C.c_int
    lib.scpqp_trace_layout.argtypes = [H, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    lib.scpqp_trace_layout.restype = C.c_int
    PP = C.POINTER(PlantParams)
    V = C.c_void_p
    lib.scpqp_delay_compensate.argtypes = [PP, C.c_int32, C.c_double, C.c_int32, V, V, V, V, V,
                                           C.c_double, V]
    lib.scpqp_delay_compensate.restype = C.c_int
    lib.scpqp_plant_step.argtypes = [PP, C.c_int32, C.c_int32, C.c_double, V, V, V, V, C.c_double, V]
    lib.scpqp_plant_step.restype = C.c_int
    lib.scpqp_clip_controls.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_double,
                                        V, V, V, V]
    lib.scpqp_clip_controls.restype = C.c_int
    if path is None:
        _lib = lib
    return lib


def use_build(path):
    """Tools / tests only (bench.py --lib, tools/bitwise_ab.py): make every later
    ``load()`` of this process return another build of the same C-ABI (an A/B variant or
    a diagnostic build), loaded before any solver is created."""
    global _lib
    _lib = load(os.path.abspath(path))
    return _lib


def check(rc, lib=None):
    if rc != 0:
        lib = lib or load()
        raise RuntimeError(f"scpqp error {rc}: {lib.scpqp_last_error().decode()}")
