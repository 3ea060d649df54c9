"""Where the IPM iterations of a c2 batch go (GPU, per-iteration trace): per QP index,
the problems reaching it, warm attempts / certified, cold IPM iterations; and the QP
sequence (ipm iterations, flags) of the slowest problems.  Header fields of the trace
record: [5] IPM iterations, [6] flags (1 certified, 2 warm attempted).
    python tools/qp_trace_stats.py [B] [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import scp_reference as R  # noqa: E402
from scpqp import batch as BT  # noqa: E402
from scpqp.solver import ScpQpSolver  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
sc = R.circle_scenario(4, Hp=20)
bt = BT.make_batch(sc, B, base_seed=0)
S = ScpQpSolver(sc, max_batch=B)
out = S.solve(bt.x0, bt.u0, bt.ec_noise, trace=True)
torch.cuda.synchronize()
tr = out.trace.cpu().numpy()          # [B, maxScp, stride]
nscp = out.n_scp.cpu().numpy()
nipm = out.n_ipm.cpu().numpy()
ipm = tr[:, :, 5]
fl = np.nan_to_num(tr[:, :, 6]).astype(int)
pr = np.nan_to_num(tr[:, :, 9]).astype(np.int64)
rounds, solves = pr % 4096, pr // 4096
print(f"B={B}: SCP iterations {nscp.sum()}, IPM iterations {nipm.sum()}, mean {nipm.mean():.1f}/problem")
print(" qp  reach  warm_try  warm_ok  cold  ipm/cold  max_ipm  ipm_share  rounds(ok/failed warm)  solves(ok/failed warm)")
tot = nipm.sum()
for k in range(int(nscp.max())):
    m = nscp > k
    w = (fl[m, k] & 2) != 0
    ok = w & ((fl[m, k] & 1) != 0) & (ipm[m, k] == 0)
    cold = ~ok
    ci = ipm[m, k][cold]
    fw = w & ~ok
    rk, sk = rounds[m, k], solves[m, k]
    print(f" {k:2d} {m.sum():6d} {w.sum():8d} {ok.sum():8d} {cold.sum():5d} {ci.mean() if len(ci) else 0:9.2f}"
          f" {ci.max() if len(ci) else 0:8.0f} {ipm[m, k].sum() / tot:9.3f}"
          f"   {rk[ok].mean() if ok.any() else 0:5.2f}/{rk[fw].mean() if fw.any() else 0:5.2f}"
          f"   {sk[ok].mean() if ok.any() else 0:6.2f}/{sk[fw].mean() if fw.any() else 0:6.2f}")
order = np.argsort(-nipm)
print("slowest problems (by IPM iterations): idx nscp nipm | per QP: ipm[flags:polish rounds/solves]")
for b in order[:12]:
    seq = " ".join(f"{int(ipm[b, k])}[{fl[b, k]}:{rounds[b, k]}/{solves[b, k]}]" for k in range(nscp[b]))
    print(f"  {b:5d} {nscp[b]:3d} {nipm[b]:4d} | {seq}")
S.close()
