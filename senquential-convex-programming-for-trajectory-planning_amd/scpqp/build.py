"""Build the HIP library in-tree: csrc/scpqp.hip + csrc/plant.hip -> scpqp/libscpqp.so (gfx950)."""
from __future__ import annotations

import os
import subprocess
import sys

_PKG = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG)
_REPO = os.path.dirname(_ROOT)
SRC = os.path.join(_ROOT, "csrc", "scpqp.hip")
SRCS = [SRC, os.path.join(_ROOT, "csrc", "plant.hip")]
INCLUDE = os.path.join(_REPO, "include")
LIB_PATH = os.path.join(_PKG, "libscpqp.so")
ARCH = os.environ.get("SCPQP_ARCH", "gfx950")


def build_library(force=False, verbose=False, defines=(), out=None):
    """Compile with hipcc unless the .so is newer than its sources.

    ``defines``/``out`` build a diagnostic variant (e.g. ``("SCPQP_PROF",)`` ->
    ``libscpqp_prof.so``); the shipped library is built with neither."""
    out = out or LIB_PATH
    deps = SRCS + [os.path.join(INCLUDE, "scpqp.h"), __file__]
    if not force and os.path.exists(out):
        t = os.path.getmtime(out)
        if all(os.path.getmtime(d) <= t for d in deps):
            return out
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", f"-I{INCLUDE}"] + [f"-D{d}" for d in defines] + \
          SRCS + ["-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    if "--prof" in sys.argv:
        # --fine adds the factorisation sub-phase stamps (perturbs whole-batch timelines)
        defs = ("SCPQP_PROF", "SCPQP_PROF_FINE") if "--fine" in sys.argv else ("SCPQP_PROF",)
        print(build_library(force="--force" in sys.argv, verbose=True, defines=defs,
                            out=os.path.join(_PKG, "libscpqp_prof.so")))
    else:
        print(build_library(force="--force" in sys.argv, verbose=True))
