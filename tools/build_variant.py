"""Build an A/B variant of the library from patch files (tools/patches/*.patch) applied to
a temporary copy of csrc/, with optional -D defines; the shipped source is untouched.

    python tools/build_variant.py <out.so> [patch ...] [-DNAME ...]

e.g. the round-5 reduction buffers (the races of ADVICE r05) under the check build:
    python tools/build_variant.py ab/check_r05.so tools/patches/r05_reduce_buffers.patch \\
        -DSCPQP_DIAG_REDUCE_CHECK
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")
sys.path.insert(0, PKG)
from scpqp.build import CSRC, build_library  # noqa: E402


def main():
    out = os.path.abspath(sys.argv[1])
    patches = [a for a in sys.argv[2:] if not a.startswith("-D")]
    defines = [a[2:] for a in sys.argv[2:] if a.startswith("-D")]
    tmp = tempfile.mkdtemp(prefix="scpqp_variant_")
    try:
        rel = os.path.relpath(CSRC, ROOT)
        dst = os.path.join(tmp, rel)
        shutil.copytree(CSRC, dst)
        for p in patches:
            subprocess.run(["patch", "-p1", "-d", tmp, "-i", os.path.abspath(p)], check=True)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        print(build_library(force=True, defines=defines, out=out, csrc=dst))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
