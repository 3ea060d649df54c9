#!/usr/bin/env python3
"""Benchmark: batched SCP-QP solves/sec on MI355X (BASELINE.json metric).

One *step* = one full SCP solve (linearise dynamics, then the <=20 convexified
QPs under the reference's stopping rule, SCP_controller.py:40-197) of every
problem of a batch of synthetic problems, in ONE kernel launch.  Workload at
N=1 is BASELINE config c2: the 4-vehicle circle ("crossing") scenario,
Hp = 20, batch = 1024 noise seeds.  With N GPUs each rank solves its own 1024
problems (global problem indices rank*1024 ...), no collective on the data
path ("weak" scaling); only a barrier and a max-reduction of the time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Without a launcher (no WORLD_SIZE in the environment), ``--gpus N`` with N > 1
starts the N rank processes itself, one per GPU, before anything touches a GPU
(spawn_ranks), and exits with the worst rank's return code.

Prints ONE JSON line (rank 0).  ``roofline`` prices the dominant (only)
kernel against the FP64 peak with the algorithmic FLOP count of the executed
algorithm (scpqp/flops.py); ``cpu_baseline`` times the in-repo CPU
restatement of the reference path (oracle/: faithful mode = the reference CPU
path, and structured mode = the optimised CPU path, each at the all-core and the
1-core rate) on a bounded sample of the same problems on the host cores, and
``traj_linf_err`` is the GPU-vs-oracle trajectory error on that sample.
"""
from __future__ import annotations

import argparse
import json
import math
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

FP64_PEAK_TFLOPS = 78.6   # MI355X dense FP64 (vector == MFMA on gfx950), AMD datasheet
HBM_PEAK_GBS = 8000.0
METRIC = "SCP-QP solves/sec/GPU (4 veh, Hp=20); traj ℓ∞ err vs CVXOPT"
# committed rocprofv3 PMC summaries of the shipped kernel (tools/gpu.sh pmc + pmc_summary.py):
# the newest round's record of each configuration
PMC_ROUNDS = ("r06", "r05")


def pmc_record(kind, config):
    """profiles/<round>_pmc_<kind>_<config>.json of the newest round that has one."""
    for rnd in PMC_ROUNDS:
        p = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{kind}_{config}.json")
        if os.path.exists(p):
            return p
    return os.path.join(ROOT, "profiles", f"{PMC_ROUNDS[0]}_pmc_{kind}_{config}.json")


# ----------------------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    """Spawned worker: the oracle's restatement of the reference path in one mode,
    single-threaded.  faithful = the dense QCQP_formulate tensors of
    SCP_controller.py:278-341 (the named "reference CPU path"); structured = the
    factored rows of SURVEY A.5 (the optimised CPU path)."""
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    sys.path.insert(0, ROOT)
    from oracle import scp_reference as R
    n_veh, mode, hps, x0s, u0s, ecs = args
    sc = R.circle_scenario(n_veh, Hp=int(max(hps)))
    out = []
    t0 = time.perf_counter()
    for x0, u0, ec, hp in zip(x0s, u0s, ecs, hps):
        p = R.make_problem(sc, x0, u0, ec, Hp=int(hp))
        r = R.scp_solve(p, mode=mode)
        out.append((r.traj, r.n_scp, r.converged))
    return time.perf_counter() - t0, out


def cpu_modes(n_veh):
    """Oracle modes timed by the CPU leg, the reference CPU path first.  At 8 vehicles,
    Hp 30 the dense Phi of the faithful mode is 774 MB per problem, so only the
    structured mode is timed there."""
    return ("faithful", "structured") if n_veh <= 4 else ("structured",)


def cpu_baseline(bt, n_veh, sample, workers, mode):
    """All-core leg: `sample` problems over `workers` spawned single-threaded processes.
    Returns (wall seconds, summed worker seconds, per-problem results)."""
    idx = np.arange(sample)
    chunks = [c for c in np.array_split(idx, workers) if len(c)]
    jobs = [(n_veh, mode, bt.hp[c], bt.x0[c], bt.u0[c], bt.ec_noise[c]) for c in chunks]
    ctx = mp.get_context("spawn")
    env_keep = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    with ctx.Pool(len(jobs)) as pool:
        pool.map(_noop, range(len(jobs)))   # interpreter start-up outside the timed region
        t0 = time.perf_counter()
        res = pool.map(_cpu_worker, jobs)
        wall = time.perf_counter() - t0
    if env_keep is not None:
        os.environ["OMP_NUM_THREADS"] = env_keep
    cpu_s = sum(r[0] for r in res)
    trajs = [t for r in res for t in r[1]]
    return wall, cpu_s, trajs


def _noop(_):
    return 0


def pmc_traffic(tj):
    """(corrected, raw) HBM bytes per launch from a committed traffic summary
    (tools/pmc_summary.py): corrected = FETCH_SIZE x2 + WRITE_SIZE, raw = FETCH_SIZE +
    WRITE_SIZE, both converted from KiB.  A summary without these keys is an error."""
    for k in ("hbm_bytes_per_launch", "fetch_size_kib_raw", "hbm_write_bytes_per_launch"):
        if k not in tj:
            raise KeyError(f"traffic summary lacks {k!r}")
    return float(tj["hbm_bytes_per_launch"]), \
        float(tj["fetch_size_kib_raw"]) * 1024.0 + float(tj["hbm_write_bytes_per_launch"])


def roofline_bound(sq, flops):
    """The unit that carries the kernel's FP64 work: "mfma" when the measured MFMA
    FLOPs (SQ_INSTS_VALU_MFMA_F64 x 2048) are at least half of the executed FLOPs,
    else "fp64-valu" (the VALU FMA pipe; the kernel is latency-bound either way)."""
    if not sq or not flops:
        return "fp64-valu", "no counter record for this workload: the VALU path is assumed"
    share = float(sq.get("mfma_f64_flops", 0.0)) / flops
    if share >= 0.5:
        return "mfma", f"MFMA carries {share:.0%} of the executed FP64 FLOPs"
    return "fp64-valu", f"MFMA carries {share:.0%} of the executed FP64 FLOPs (VALU FMA pipe)"


def cpu_leg(bt, n_veh, cpu_sample, B, cores=None):
    """Time every oracle mode of cpu_modes() on the same bounded sample.  Per mode:
    wall (all cores) and cpu_s (summed single-thread worker seconds, so sample / cpu_s
    is the 1-core rate).  The first mode's trajectories are the parity sample."""
    cores = cores or host_cores()
    sample = min(cpu_sample, B)
    modes = {}
    trajs = None
    for mode in cpu_modes(n_veh):
        wall, cpu_s, tr = cpu_baseline(bt, n_veh, sample, cores, mode)
        modes[mode] = dict(wall=wall, cpu_s=cpu_s)
        trajs = tr if trajs is None else trajs
    first = modes[cpu_modes(n_veh)[0]]
    return dict(wall=first["wall"], cpu_s=first["cpu_s"], modes=modes, trajs=trajs, cores=cores,
                sample=sample)


def cpu_baseline_block(cpu, config, n_veh):
    """The bench line's cpu_baseline: `value` is the reference CPU path (the first mode)
    on all cores; the structured (optimised CPU) mode and the 1-core rates beside it."""
    modes = cpu["modes"]
    ref = cpu_modes(n_veh)[0]
    n = cpu["sample"]
    blk = {
        "value": n / modes[ref]["wall"], "unit": "SCP solves/s", "cores": cpu["cores"],
        "kind": "port",
        "mode": ref,
        "value_1core": n / modes[ref]["cpu_s"],
        "value_structured": n / modes["structured"]["wall"],
        "value_structured_1core": n / modes["structured"]["cpu_s"],
        "sample": f"first {n} problems of the same {config} batch, oracle "
                  + ("faithful mode (dense QCQP_formulate tensors" if ref == "faithful"
                     else "structured mode (factored rows; the dense Phi is 774 MB per problem")
                  + f", scipy expm, dense IPM + exact polish), {cpu['cores']} spawned "
                  f"single-threaded workers; " + ", ".join(
                      f"{m}: {v['cpu_s']:.1f} s of CPU work, {v['wall']:.2f} s wall"
                      for m, v in modes.items()),
        "note": "value / value_structured: all cores (sample / wall); *_1core: one core "
                "(sample / summed single-thread worker seconds); structured = factored "
                "constraint rows (SURVEY A.5), the optimised CPU path",
    }
    return blk


def cpu_leg_dump(cpu, path):
    """The parent's CPU leg for the ranks it spawns (rank 0 reads it back)."""
    d = dict(cpu, trajs=[(np.asarray(t).tolist(), int(ns), bool(cv)) for t, ns, cv in cpu["trajs"]])
    with open(path, "w") as fh:
        json.dump(d, fh)


def cpu_leg_load(path):
    with open(path) as fh:
        d = json.load(fh)
    d["trajs"] = [(np.asarray(t), ns, cv) for t, ns, cv in d["trajs"]]
    return d


def host_cores():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    # the GPU box exposes the whole machine's CPUs; its share is 16 (gpurun docs)
    return max(1, min(n, int(os.environ.get("SCPQP_CPU_WORKERS", "16"))))


# ----------------------------------------------------------------------------- ranks
def spawn_ranks(n, cpu_path=None):
    """``bench.py --gpus N`` run directly: start the N ranks as child processes of
    this one (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rank r on GPU r) and
    wait for them.  Nothing here initialises the GPU (device_count() does not on
    this ROCm build).  More ranks than devices is a single-box rehearsal of the
    sharded path: the ranks share devices and the collectives run on gloo (RCCL
    refuses two ranks on one device).  If a rank fails, the others are stopped."""
    import socket
    import subprocess
    import torch
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env0 = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n))
    if cpu_path:
        env0["SCPQP_CPU_RESULT"] = cpu_path
    ndev = torch.cuda.device_count()
    if ndev < n:
        print(f"bench: {n} ranks on {ndev} device(s): ranks share devices, gloo collectives",
              file=sys.stderr, flush=True)
        env0.setdefault("SCPQP_DIST_BACKEND", "gloo")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                              env=dict(env0, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0:
                rc = rc or (code if code > 0 else 1)
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="problems per GPU (config c2: 1024)")
    ap.add_argument("--n-veh", type=int, default=4)
    ap.add_argument("--hp", type=int, default=20)
    ap.add_argument("--cpu-sample", type=int, default=512)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--config", choices=("c2", "c3", "c4", "c5"), default="c2",
                    help="BASELINE config: c2 4 veh Hp 20 B 1024 (the metric's workload, default); "
                         "c3 8 veh Hp 30 B 4096; c4 4 veh Hp 20, 65536 problems as 8192 per "
                         "rank (8 GPUs); c5 4 veh mixed Hp {10,20,30} B 3072")
    ap.add_argument("--lib", default=None,
                    help="tools only: another build of the library (A/B runs, tools/gpu.sh ab)")
    args = ap.parse_args()
    mixed = None
    if args.config == "c4":
        # BASELINE configs[3]: 4 vehicles x 65536 Monte-Carlo realisations, Hp 20, sharded
        # over 8 GPUs -> 8192 problems per rank
        args.n_veh, args.hp, args.batch = 4, 20, args.batch if args.batch != 1024 else 8192
    if args.config == "c3":
        args.n_veh, args.hp, args.batch = 8, 30, args.batch if args.batch != 1024 else 4096
        args.cpu_sample = min(args.cpu_sample, 32)
    elif args.config == "c5":
        args.n_veh, args.hp, args.batch = 4, 30, args.batch if args.batch != 1024 else 3072
        mixed = (10, 20, 30)

    spawner = args.gpus > 1 and "WORLD_SIZE" not in os.environ
    world = args.gpus if spawner else int(os.environ.get("WORLD_SIZE", "1"))
    rank = 0 if spawner else int(os.environ.get("RANK", "0"))
    local = 0 if spawner else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {args.gpus}", file=sys.stderr)

    from scpqp import flops as FL
    from scpqp import shard
    import Scenarios  # the drop-in scenario module (host logic)

    sc = Scenarios.Scenario(False)
    sc.Hp = sc.Hu = args.hp
    sc.get_circle_scenario([2 * math.pi / args.n_veh * (i + 1) for i in range(args.n_veh)])
    sc.complete_scenario()
    B = args.batch
    bt = shard.shard_batch(sc, B, rank, base_seed=0, mixed_hp=mixed)

    # CPU baseline first, at every N, before any process of the run touches the GPU:
    # bench.py --gpus N run directly times it in the parent (which never initialises the
    # GPU) on rank 0's shard and hands it to rank 0; under an external launcher rank 0
    # times it itself before its first GPU call (the other ranks wait in the rendezvous)
    cpu = None
    if spawner:
        path = None
        if not args.no_cpu:
            import tempfile
            cpu = cpu_leg(bt, args.n_veh, args.cpu_sample, B)
            fd, path = tempfile.mkstemp(prefix="scpqp_cpu_", suffix=".json")
            os.close(fd)
            cpu_leg_dump(cpu, path)
        try:
            rc = spawn_ranks(args.gpus, path)
        finally:
            if path:
                os.unlink(path)
        sys.exit(rc)
    if rank == 0 and not args.no_cpu:
        if os.environ.get("SCPQP_CPU_RESULT"):
            cpu = cpu_leg_load(os.environ["SCPQP_CPU_RESULT"])
        else:
            cpu = cpu_leg(bt, args.n_veh, args.cpu_sample, B)

    import torch
    if world > 1:
        import torch.distributed as dist
        # one rank per GPU; more ranks than GPUs only in a single-box rehearsal of the
        # sharded path (ranks share a device; SCPQP_DIST_BACKEND=gloo if RCCL refuses it)
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(os.environ.get("SCPQP_DIST_BACKEND", "nccl"))
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.lib:
        from scpqp import _lib
        _lib.use_build(args.lib)
    from scpqp.solver import ScpQpSolver

    S = ScpQpSolver(sc, max_batch=B, device=dev)
    x0 = torch.as_tensor(bt.x0, device=dev)
    u0 = torch.as_tensor(bt.u0, device=dev)
    ec = torch.as_tensor(bt.ec_noise, device=dev)
    out = S.alloc_out(B)
    stream = torch.cuda.current_stream(dev)

    hpt = torch.as_tensor(bt.hp, device=dev) if mixed else None
    if rank == 0:
        print(f"bench: {args.config} B={B}/rank x {world} ranks, warmup {args.warmup}, "
              f"steps {args.steps}", file=sys.stderr, flush=True)
    for _ in range(args.warmup):
        S.solve(x0, u0, ec, hp=hpt, out=out)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # one event per step boundary on the launch stream (no extra synchronisation in the
    # timed region): the mean over the K steps prices the roofline, the median is the
    # per-step statistic of SURVEY 8(d)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for k in range(args.steps):
        S.solve(x0, u0, ec, hp=hpt, out=out)
        evs[k + 1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    step_ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)]
    kern_ms = evs[0].elapsed_time(evs[-1]) / max(args.steps, 1)   # one launch per step
    kern_ms_median = float(np.median(step_ms)) if step_ms else kern_ms
    elapsed = shard.max_over_ranks(elapsed, dist, dev)

    # end-to-end leg: host (pinned) inputs -> H2D -> solve -> D2H of the result
    # arrays main.py consumes (u, traj, status, obj, max_violation); reported beside `value`,
    # never as it
    ins = (x0, u0, ec) + ((hpt,) if mixed else ())
    h_in = [t.cpu().pin_memory() for t in ins]
    d_in = [torch.empty_like(t) for t in ins]
    outs = (out.u, out.traj, out.status, out.obj, out.max_violation)
    h_out = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in outs]
    e2e_steps = max(min(args.steps, 5), 1)
    torch.cuda.synchronize()
    te = time.perf_counter()
    for _ in range(e2e_steps):
        for d, h in zip(d_in, h_in):
            d.copy_(h, non_blocking=True)
        S.solve(d_in[0], d_in[1], d_in[2], hp=d_in[3] if mixed else None, out=out)
        for h, d in zip(h_out, outs):
            h.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
    e2e_s = shard.max_over_ranks(time.perf_counter() - te, dist, dev)
    e2e_value = world * B * e2e_steps / e2e_s

    n_scp = out.n_scp.cpu().numpy()
    n_ipm = out.n_ipm.cpu().numpy()
    status = out.status.cpu().numpy()
    n_pol = out.n_polish.cpu().numpy()
    n_ref = out.n_refine.cpu().numpy()
    n_warm = out.n_warm.cpu().numpy()
    flops = FL.batch_flops(args.n_veh, bt.hp, 0, n_scp, n_ipm, n_pol, n_ref, n_warm)
    achieved_tf = flops / (kern_ms * 1e-3) / 1e12
    dense = FL.survey_dense_batch(args.n_veh, bt.hp, 0, n_scp, n_ipm)
    dense_tf = dense / (kern_ms * 1e-3) / 1e12
    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed

    # HBM bytes per launch from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this
    # workload at its default batch (tools/gpu.sh pmc + tools/pmc_summary.py)
    traffic, traffic_raw, sq = None, None, None
    default_b = {"c2": 1024, "c3": 4096, "c4": 8192, "c5": 3072}[args.config]
    tpath = pmc_record("traffic", args.config)
    spath = pmc_record("sq", args.config)
    if B == default_b and os.path.exists(tpath):
        try:
            with open(tpath) as fh:
                tj = json.load(fh)
        except (OSError, ValueError):
            tj = None
        if tj is not None:
            traffic, traffic_raw = pmc_traffic(tj)
    if B == default_b and os.path.exists(spath):
        try:
            with open(spath) as fh:
                sq = json.load(fh)
        except (OSError, ValueError):
            sq = None
    res = S.resources()
    bound, bound_note = roofline_bound(sq, flops)

    line = {
        "metric": METRIC,
        "value": value,
        "unit": "SCP solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "ms_per_step_median": shard.max_over_ranks(kern_ms_median * 1e-3, dist, dev) * 1e3,
        "ms_per_step_note": "ms_per_step: the K timed steps' wall time / K (max over ranks); "
                            "ms_per_step_median: median of the per-step HIP-event times on the "
                            "launch stream (max over ranks)",
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (circle scenario x0 + N(0,diag(.05,.05,.005,.02,0,.002)^2), Ec noise N(0,3e-6^2))",
        "config": {"workload": f"{args.config}: {args.n_veh}-vehicle circle/crossing, "
                               f"Hp={'{10,20,30} mixed' if mixed else args.hp}, "
                               f"batch={B} noise seeds per GPU, full SCP solve per problem",
                   "n_veh": args.n_veh, "hp": list(mixed) if mixed else args.hp, "batch_per_gpu": B,
                   "parallelism": (f"{world} of 8 shards of c4's 65536 problems (8192 per rank, "
                                   f"no collective)" if args.config == "c4" else
                                   f"{world} independent shards (no collective)")},
        "roofline": {"bound": bound, "bound_note": bound_note, "achieved": achieved_tf, "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved_tf / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "kernel": "scp_kernel", "kernel_ms": kern_ms,
                     "traffic_source": f"profiles/{os.path.basename(tpath)} (FETCH_SIZE x2 + WRITE_SIZE)"
                     if traffic is not None else None,
                     "traffic_raw_fetch": traffic_raw,
                     "traffic_raw_note": "raw FETCH_SIZE + WRITE_SIZE in bytes (no x2 read correction; "
                                         "the true HBM bytes lie between traffic_raw_fetch and traffic)"
                     if traffic_raw is not None else None,
                     "hbm_achieved_GBps": traffic / (kern_ms * 1e-3) / 1e9 if traffic else None,
                     "hbm_frac": traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None,
                     "lds_bank_conflict_ratio": sq["lds_bank_conflict_ratio"] if sq else None,
                     "sq_wait_any_frac": sq["wait_any_frac"] if sq else None,
                     "mfma_f64_insts_per_launch": sq.get("mfma_f64_insts") if sq else None,
                     "mfma_flop_share": (sq.get("mfma_f64_flops", 0.0) / flops) if sq and flops else None,
                     "sq_source": f"profiles/{os.path.basename(spath)} (SQ_LDS_BANK_CONFLICT / "
                                  f"SQ_LDS_IDX_ACTIVE, SQ_WAIT_ANY / SQ_WAVE_CYCLES, "
                                  f"SQ_INSTS_VALU_MFMA_F64 x 2048 FLOP)" if sq else None,
                     "memory_plan": res["plan"], "lds_bytes": res["lds_bytes"],
                     "workgroups": res["grid"],
                     "flops_per_launch": flops,
                     "flops_note": "executed algorithm (scpqp/flops.py) at the measured counters",
                     "survey_dense_flops_per_launch": dense,
                     "survey_dense_achieved": dense_tf,
                     "survey_dense_frac": dense_tf / FP64_PEAK_TFLOPS,
                     "survey_dense_note": "SURVEY 8(d) dense-KKT F_ipm at the measured IPM "
                                          "iteration counts (solver-independent numerator)",
                     "peak_note": "FP64 dense peak (vector = MFMA rate on gfx950, AMD spec)"},
        "qp_solves_per_s": world * float(n_scp.sum()) * args.steps / elapsed,
        "mean_scp_iters": float(n_scp.mean()),
        "max_scp_iters": int(n_scp.max()),
        "mean_ipm_iters_per_qp": float(n_ipm.sum() / max(n_scp.sum(), 1)),
        "mean_ipm_iters_per_problem": float(n_ipm.mean()),
        "max_ipm_iters_per_problem": int(n_ipm.max()),
        "warm_certified_qp_frac": float(n_warm.sum() / max(n_scp.sum(), 1)),
        "mean_polish_solves_per_qp": float(n_ref.sum() / max(n_scp.sum(), 1)),
        "status_converged_frac": float(np.mean((status & 0xff) == 0)),
        "e2e_solves_per_s": e2e_value,
        "e2e_note": f"host pinned inputs, H2D + solve + D2H of u/traj/status/obj/max_violation, "
                    f"synchronised per step, {e2e_steps} steps",
    }
    if cpu is not None:
        trajs = out.traj.cpu().numpy()
        # parity on problems where both sides met the stopping rule with the same SCP count;
        # problems that run into the 20-QP cap without converging oscillate, and their
        # final iterate is reported separately (it depends chaotically on QP rounding)
        errs, capped = [], []
        for b, (tr, ns, conv) in enumerate(cpu["trajs"]):
            if ns == n_scp[b]:
                H = int(bt.hp[b])
                mine = trajs[b].reshape(-1)[:H * 2 * args.n_veh].reshape(H, 2, args.n_veh)
                e = float(np.abs(mine - tr).max())
                (errs if conv and (status[b] & 0xff) == 0 else capped).append(e)
        line["cpu_baseline"] = cpu_baseline_block(cpu, args.config, args.n_veh)
        line["traj_linf_err"] = max(errs) if errs else None
        line["traj_err_reference"] = ("in-repo CPU restatement of the reference path (oracle/; "
                                      "CVXOPT/GUROBI absent, parity unpinned: SURVEY 8c)")
        line["traj_err_sample"] = (f"{len(errs)}/{cpu['sample']} problems converged on both sides "
                                   f"with equal SCP iteration count")
        line["traj_linf_err_capped"] = max(capped) if capped else None
        line["capped_sample"] = f"{len(capped)} problems at the 20-QP cap (not converged)"
    if rank == 0:
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()
    S.close()


if __name__ == "__main__":
    main()
