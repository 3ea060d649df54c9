"""Build the HIP library in-tree: csrc/*.hip -> scpqp/libscpqp.so (gfx950).

The library is linked from separate translation units compiled in parallel:
``scpqp.hip`` (the C-ABI host side), ``plant.hip``, and ``kernels.hip`` once per kernel
group (``-DSCPQP_KGROUP=1..10``: the kernel instantiations of ``scpqp_kernel.h``).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

_PKG = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG)
_REPO = os.path.dirname(_ROOT)
CSRC = os.path.join(_ROOT, "csrc")
SRC = os.path.join(CSRC, "scpqp.hip")
KERNEL_SRC = os.path.join(CSRC, "kernels.hip")
HEADER = os.path.join(CSRC, "scpqp_kernel.h")
SRCS = [SRC, os.path.join(CSRC, "plant.hip")]
KERNEL_GROUPS = 10
INCLUDE = os.path.join(_REPO, "include")
LIB_PATH = os.path.join(_PKG, "libscpqp.so")
ARCH = os.environ.get("SCPQP_ARCH", "gfx950")


def _jobs():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, int(os.environ.get("MAX_JOBS", n)), n))


def build_library(force=False, verbose=False, defines=(), out=None, csrc=None):
    """Compile with hipcc unless the .so is newer than its sources.

    ``defines``/``out`` build a diagnostic variant (e.g. ``("SCPQP_PROF",)`` ->
    ``libscpqp_prof.so``); the shipped library is built with neither.  ``csrc``: another
    copy of the source directory (tools/build_variant.py: a patched A/B variant)."""
    out = out or LIB_PATH
    src_dir = csrc or CSRC
    srcs = [os.path.join(src_dir, os.path.basename(x)) for x in SRCS]
    ksrc = os.path.join(src_dir, os.path.basename(KERNEL_SRC))
    hdr = os.path.join(src_dir, os.path.basename(HEADER))
    deps = srcs + [ksrc, hdr, os.path.join(INCLUDE, "scpqp.h"), __file__]
    if not force and os.path.exists(out):
        t = os.path.getmtime(out)
        if all(os.path.getmtime(d) <= t for d in deps):
            return out
    flags = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
             f"-I{INCLUDE}"] + [f"-D{d}" for d in defines]
    tmp = tempfile.mkdtemp(prefix="scpqp_build_")
    try:
        units = [(s, os.path.join(tmp, os.path.basename(s) + ".o"), []) for s in srcs]
        units += [(ksrc, os.path.join(tmp, f"kernels_{g}.o"), [f"-DSCPQP_KGROUP={g}"])
                  for g in range(1, KERNEL_GROUPS + 1)]

        def compile_unit(u):
            src, obj, extra = u
            cmd = ["hipcc", "-c"] + flags + extra + [src, "-o", obj]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
            return obj

        # the heaviest groups (c5, c3) first
        order = sorted(units, key=lambda u: 0 if u[2] and u[2][0].endswith(("=3", "=2", "=4")) else 1)
        with ThreadPoolExecutor(_jobs()) as ex:
            objs = list(ex.map(compile_unit, order))
        cmd = ["hipcc", "-shared", "-fPIC", "--offload-arch=" + ARCH] + objs + ["-o", out + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return out


if __name__ == "__main__":
    if "--prof" in sys.argv:
        # --fine adds the factorisation sub-phase stamps (perturbs whole-batch timelines)
        defs = ("SCPQP_PROF", "SCPQP_PROF_FINE") if "--fine" in sys.argv else ("SCPQP_PROF",)
        print(build_library(force="--force" in sys.argv, verbose=True, defines=defs,
                            out=os.path.join(_PKG, "libscpqp_prof.so")))
    elif "--check" in sys.argv:
        # the reduction-buffer check (scpqp_diag_reduce_check) and its bitwise reference
        print(build_library(force="--force" in sys.argv, verbose=True,
                            defines=("SCPQP_DIAG_REDUCE_CHECK",),
                            out=os.path.join(_PKG, "libscpqp_check.so")))
        print(build_library(force="--force" in sys.argv, verbose=True,
                            defines=("SCPQP_DIAG_REDUCE2",),
                            out=os.path.join(_PKG, "libscpqp_reduce2.so")))
    else:
        print(build_library(force="--force" in sys.argv, verbose=True))
