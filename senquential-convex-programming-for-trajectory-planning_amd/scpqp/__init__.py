"""scpqp — MI355X-native batched SCP-QP trajectory planner (HIP/CDNA4, fp64).

Public API:
  ScpQpSolver   batched solver bound to one scenario (C-ABI in include/scpqp.h)
  batch         synthetic problem batches
  build_library compile csrc/scpqp.hip for gfx950 into scpqp/libscpqp.so
"""
from .build import build_library, LIB_PATH  # noqa: F401
from . import batch  # noqa: F401


def __getattr__(name):
    # torch is imported lazily so that host-only tools (build, ABI checks) stay light
    if name in ("ScpQpSolver", "SolveResult", "unpack_problem"):
        from . import solver
        return getattr(solver, name)
    raise AttributeError(name)
