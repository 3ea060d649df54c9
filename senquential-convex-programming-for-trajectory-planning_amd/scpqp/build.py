"""Build the HIP library in-tree: csrc/scpqp.hip -> scpqp/libscpqp.so (gfx950)."""
from __future__ import annotations

import os
import subprocess
import sys

_PKG = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG)
_REPO = os.path.dirname(_ROOT)
SRC = os.path.join(_ROOT, "csrc", "scpqp.hip")
INCLUDE = os.path.join(_REPO, "include")
LIB_PATH = os.path.join(_PKG, "libscpqp.so")
ARCH = os.environ.get("SCPQP_ARCH", "gfx950")


def build_library(force=False, verbose=False):
    """Compile with hipcc unless the .so is newer than its sources."""
    deps = [SRC, os.path.join(INCLUDE, "scpqp.h"), __file__]
    if not force and os.path.exists(LIB_PATH):
        t = os.path.getmtime(LIB_PATH)
        if all(os.path.getmtime(d) <= t for d in deps):
            return LIB_PATH
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", f"-I{INCLUDE}", SRC, "-o", LIB_PATH + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True))
