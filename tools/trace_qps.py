"""Per-QP record of selected problems of the c2 batch from the device trace (header slots:
IPM iterations, QP flags 1 certified / 2 warm, polish rounds + 4096 x refinement solves).
    python tools/trace_qps.py [problem ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]


def main():
    import torch
    from oracle import scp_reference as R
    from scpqp import shard
    from scpqp.solver import ScpQpSolver
    probs = [int(a) for a in sys.argv[1:]] or [271, 158, 1012, 1008, 0, 1]
    sc = R.circle_scenario(4, Hp=20)
    bt = shard.shard_batch(sc, 1024, 0, base_seed=0)
    S = ScpQpSolver(sc, max_batch=1024)
    out = S.solve(bt.x0, bt.u0, bt.ec_noise, trace=True)
    torch.cuda.synchronize()
    tr = out.trace.cpu().numpy()
    ns = out.n_scp.cpu().numpy()
    nipm = out.n_ipm.cpu().numpy()
    tot = {"cold": 0, "warm_ok": 0, "warm_fail": 0}
    ipm_by = {"cold": 0, "warm_fail": 0}
    for b in range(1024):
        for it in range(int(ns[b])):
            h = tr[b, it]
            fl, ipm = int(h[6]), int(h[5])
            kind = "warm_ok" if fl & 2 and ipm == 0 else ("warm_fail" if fl & 2 else "cold")
            tot[kind] += 1
            if kind in ipm_by:
                ipm_by[kind] += ipm
    print("batch QPs:", tot, "IPM iterations:", ipm_by, "total", int(nipm.sum()))
    # warm-start outcome by QP index (the kernel tries it from the third QP on)
    import collections
    by = collections.defaultdict(lambda: [0, 0, 0, 0])   # ok, fail, ipm after fail, rounds of fails
    for b in range(1024):
        for it in range(int(ns[b])):
            h = tr[b, it]
            fl, ipm, rr = int(h[6]), int(h[5]), int(h[9])
            if fl & 2:
                k = by[it]
                if ipm == 0:
                    k[0] += 1
                else:
                    k[1] += 1
                    k[2] += ipm
    for it in sorted(by):
        ok, fail, ipf, _ = by[it]
        print(f"QP index {it:2d}: warm tried {ok + fail:4d}, certified {ok:4d} ({ok / max(ok + fail, 1):.0%}), "
              f"failed {fail:4d} (IPM after failing: {ipf / max(fail, 1):.1f} per QP)")
    for b in probs:
        print(f"problem {b}: n_scp {int(ns[b])} n_ipm {int(nipm[b])}")
        for it in range(int(ns[b])):
            h = tr[b, it]
            rr = int(h[9])
            print(f"   QP {it:2d}: ipm {int(h[5]):3d} flags {int(h[6])} polish rounds {rr % 4096:2d} "
                  f"solves {rr // 4096:3d} delta {h[0]: .3e} maxviol {h[2]:.3e}")
    S.close()


if __name__ == "__main__":
    main()
