"""Kernel resources from the code objects of a built library (no GPU needed).

Extracts the gfx950 code objects from the library's ``.hip_fatbin`` section (clang
offload bundles, one per translation unit) and reads each kernel's AMDGPU metadata
notes with ``llvm-readelf --notes``: VGPRs, AGPRs, SGPRs, spills, private segment
(stack) bytes per lane, static LDS.  These are the kernel descriptor's numbers — the
register counts that occupancy reasoning needs (a rocprofv3 CSV's VGPR_Count column is
in allocation granules, not registers).

    python tools/kernel_resources.py [lib.so] [name-filter]   # JSON lines, one per kernel
"""
from __future__ import annotations

import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd", "scpqp",
                   "libscpqp.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
FIELDS = (".agpr_count", ".name", ".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count",
          ".sgpr_spill_count", ".private_segment_fixed_size", ".group_segment_fixed_size",
          ".max_flat_workgroup_size")


def _section(lib, name):
    """(file offset, size) of an ELF section, from llvm-readelf -S."""
    out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-S", "-W", lib], check=True,
                         capture_output=True, text=True).stdout
    for line in out.splitlines():
        parts = line.replace("[", " ").replace("]", " ").split()
        if name in parts:
            i = parts.index(name)
            return int(parts[i + 3], 16), int(parts[i + 4], 16)
    raise ValueError(f"{lib}: no section {name}")


def code_objects(lib, arch="gfx950"):
    off, size = _section(lib, ".hip_fatbin")
    with open(lib, "rb") as fh:
        fh.seek(off)
        blob = fh.read(size)
    objs = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", blob, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if arch in triple and esize:
                objs.append(blob[pos + eoff:pos + eoff + esize])
        pos = blob.find(MAGIC, pos + 1)
    return objs


def kernels(lib=LIB, arch="gfx950"):
    """Metadata of every kernel in the library's code objects (list of dicts)."""
    res = []
    with tempfile.TemporaryDirectory() as tmp:
        for i, co in enumerate(code_objects(lib, arch)):
            path = os.path.join(tmp, f"co{i}.elf")
            with open(path, "wb") as fh:
                fh.write(co)
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", path],
                                   check=True, capture_output=True, text=True).stdout
            cur = None
            for line in notes.splitlines():
                s = line.strip().lstrip("- ").strip()
                key = s.split(":", 1)[0]
                if key not in FIELDS and key != ".agpr_count":
                    continue
                val = s.split(":", 1)[1].strip()
                if key == ".agpr_count":
                    # a kernel's entry starts with .agpr_count (msgpack keys are sorted)
                    cur = {"unit": i}
                    res.append(cur)
                if cur is None:
                    continue
                cur[key.lstrip(".")] = val if key == ".name" else int(val)
    return res


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names),
                         capture_output=True, text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else LIB
    flt = sys.argv[2] if len(sys.argv) > 2 else "scp_kernel"
    ks = [k for k in kernels(lib) if flt in k["name"] or flt in demangle([k["name"]])[0]]
    names = demangle([k["name"] for k in ks])
    for k, d in zip(ks, names):
        m = re.search(r"scp_kernel<(.*)>", d)
        k["template"] = m.group(1) if m else d
        k["stack_bytes_per_lane"] = k.get("private_segment_fixed_size")
        print(json.dumps(k))


if __name__ == "__main__":
    main()
