"""Certification sweep of the CPU restatement (verdict r05 item 1): run the oracle's
exact mode (and the device-mirror regularised mode) over a sample of a configuration's
batch and count, per QP, the certificate (certificate_scaled) and the escalation stages
qp_solve needed.  The exact mode raises UncertifiedQP on a QP it cannot certify.

    python tools/oracle_certify_sweep.py c2 [stride] [workers]
"""
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]
import numpy as np  # noqa: E402

CFG = {"c2": (4, 20, 1024, None), "c3": (8, 30, 4096, None), "c5": (4, 30, 3072, (10, 20, 30))}


def job(args):
    cfg, b = args
    from oracle import scp_reference as R
    from scpqp import shard
    nv, hp, B, mixed = CFG[cfg]
    sc = R.circle_scenario(nv, Hp=hp)
    bt = shard.shard_batch(sc, B, 0, base_seed=0, mixed_hp=mixed)
    H = int(bt.hp[b])
    p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=H)
    out = []
    modes = ("exact", "regularised") if cfg != "c3" else ("exact",)
    rs = {}
    for pol in modes:
        r = R.scp_solve(p, mode="structured", keep_history=True, polish=pol)
        rs[pol] = r
        out.append([(h["certified"], h["escalations"], h["certificate_scaled"]["stationarity"])
                    for h in r.history])
    spread = None
    if "regularised" in rs:
        n = min(rs["exact"].n_scp, rs["regularised"].n_scp)
        N = nv * H
        spread = max(float(np.abs(rs["exact"].history[i]["z"][:N] - rs["regularised"].history[i]["z"][:N]).max())
                     for i in range(n))
    return b, out, spread


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    workers = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    B = CFG[cfg][2] if cfg != "c3" else 32
    jobs = [(cfg, b) for b in range(0, B, stride)]
    with mp.get_context("spawn").Pool(workers) as pool:
        res = pool.map(job, jobs)
    for mi, mode in enumerate(("exact", "regularised")):
        qs = [q for _, out, _ in res if mi < len(out) for q in out[mi]]
        if not qs:
            continue
        unc = sum(1 for q in qs if not q[0])
        esc = sum(1 for q in qs if q[1] > 0)
        print(f"{cfg} {mode}: {len(res)} problems, {len(qs)} QPs, uncertified {unc}, "
              f"escalated {esc}, max scaled stationarity {max(q[2] for q in qs):.2e}")
    sp = [s for _, _, s in res if s is not None]
    if sp:
        worst = int(np.argmax(sp))
        print(f"{cfg}: max exact-vs-regularised spread per iteration {max(sp):.2e} "
              f"(problem {res[worst][0]})")


if __name__ == "__main__":
    main()
