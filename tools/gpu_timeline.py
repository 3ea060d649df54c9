"""Per-problem start/end timeline of one c2 launch (diagnostic build libscpqp_prof.so).

Shows how the makespan of a batch splits into problem latency and queueing:
which problems finish last, when they started, how many SCP iterations they took.
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")
sys.path[:0] = [ROOT, PKG]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import scp_reference as R  # noqa: E402
from scpqp import _lib as LB  # noqa: E402
from scpqp import batch as BT  # noqa: E402
from scpqp.solver import ScpQpSolver  # noqa: E402

lib = LB.load(os.environ.get("SCPQP_PROF_LIB") or os.path.join(PKG, "scpqp", "libscpqp_prof.so"))
LB._lib = lib
lib.scpqp_prof_times.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
sc = R.circle_scenario(4, Hp=20)
bt = BT.make_batch(sc, B, base_seed=0)
S = ScpQpSolver(sc, max_batch=B)
S.solve(bt.x0, bt.u0, bt.ec_noise)
torch.cuda.synchronize()
out = S.solve(bt.x0, bt.u0, bt.ec_noise)
torch.cuda.synchronize()
buf = (C.c_ulonglong * (2 * B))()
lib.scpqp_prof_times(buf, B)
t = np.array(buf[:], dtype=np.float64).reshape(B, 2) / 100.0   # 100 MHz -> microseconds
t -= t[:, 0].min()
lat = t[:, 1] - t[:, 0]
nscp = out.n_scp.cpu().numpy()
nipm = out.n_ipm.cpu().numpy()
print(f"B={B} resources {S.resources()}  makespan {t[:, 1].max() / 1e3:.2f} ms")
print(f"latency ms: mean {lat.mean() / 1e3:.2f} p50 {np.median(lat) / 1e3:.2f} "
      f"p90 {np.percentile(lat, 90) / 1e3:.2f} max {lat.max() / 1e3:.2f}")
print(f"start ms: p50 {np.median(t[:, 0]) / 1e3:.2f} max {t[:, 0].max() / 1e3:.2f}")
for k in range(1, 21):
    sel = nscp == k
    if sel.any():
        print(f"  nscp {k:2d}: {sel.sum():4d} problems, latency mean {lat[sel].mean() / 1e3:6.2f} ms "
              f"max {lat[sel].max() / 1e3:6.2f}, ipm/problem {nipm[sel].mean():6.1f}")
order = np.argsort(-t[:, 1])[:12]
print("last to finish: idx start end latency nscp nipm")
for i in order:
    print(f"  {i:5d} {t[i, 0] / 1e3:6.2f} {t[i, 1] / 1e3:6.2f} {lat[i] / 1e3:6.2f} {nscp[i]:3d} {nipm[i]:4d}")

# does a cheap pre-pass predict the cost?  QCQP_evaluate at u = 0 (the kernel's own first step)
ev = S.evaluate(np.zeros((B, 4 * 20)), bt.x0, bt.u0, bt.ec_noise)
feat = {"maxviol(u=0)": ev["max_violation"].cpu().numpy(), "sumviol(u=0)": ev["sum_violations"].cpu().numpy(),
        "obj(u=0)": ev["obj"].cpu().numpy()}
def spearman(a, b):
    ra = np.argsort(np.argsort(a)); rb = np.argsort(np.argsort(b))
    return float(np.corrcoef(ra, rb)[0, 1])
for k, f in feat.items():
    print(f"spearman({k}, latency) = {spearman(f, lat):+.3f}   (nipm) {spearman(f, nipm):+.3f}   (nscp) {spearman(f, nscp):+.3f}")
