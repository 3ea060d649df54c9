"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo).

Each rank takes its shard of the global problem stream (scpqp.shard), solves
it (here with the CPU restatement as a stand-in worker — this test is about
sharding and timing logic, the GPU path is covered by the -m gpu tests), and
rank 0 checks that the gathered results equal a single-process run over the
whole range and that the max-over-ranks timing reduction works.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import scp_reference as R
from scpqp import batch as BT
from scpqp import shard

PER_RANK = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _solve(sc, bt):
    out = []
    for b in range(bt.size):
        p = R.make_problem(sc, bt.x0[b], bt.u0[b], bt.ec_noise[b], Hp=int(bt.hp[b]))
        r = R.scp_solve(p, mode="structured")
        out.append((r.u, r.n_scp))
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = R.circle_scenario(4, Hp=20)
        bt = shard.shard_batch(sc, PER_RANK, rank, base_seed=77)
        res = _solve(sc, bt)
        gathered = [None] * world
        dist.all_gather_object(gathered, (rank, bt.seeds.tolist(), res))
        tmax = shard.max_over_ranks(1.0 + rank, dist)
        dist.barrier()
        if rank == 0:
            q.put((gathered, tmax))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, port, q), nprocs=world, join=True,
                       start_method="spawn")
    gathered, tmax = q.get()
    assert tmax == 2.0
    sc = R.circle_scenario(4, Hp=20)
    full = BT.make_batch(sc, world * PER_RANK, base_seed=77)
    ref = _solve(sc, full)
    seeds = []
    results = []
    for rank, s, res in sorted(gathered, key=lambda t: t[0]):
        seeds += s
        results += res
    assert seeds == full.seeds.tolist()
    for (u, n), (ur, nr) in zip(results, ref):
        assert n == nr
        assert np.array_equal(u, ur)


def test_shard_ranges_are_disjoint_and_cover():
    cov = []
    for r in range(8):
        lo, hi = shard.global_range(1024, r)
        cov += list(range(lo, hi))
    assert cov == list(range(8 * 1024))


def test_shard_inputs_independent_of_world_size():
    sc = R.circle_scenario(4, Hp=20)
    a = shard.shard_batch(sc, 4, 1, base_seed=5)       # global 4..7 at world 2 x 4
    b = shard.shard_batch(sc, 2, 2, base_seed=5)       # global 4..5 at world 4 x 2
    assert np.array_equal(a.x0[:2], b.x0) and np.array_equal(a.ec_noise[:2], b.ec_noise)


def test_max_over_ranks_single_process():
    assert shard.max_over_ranks(3.5) == 3.5
