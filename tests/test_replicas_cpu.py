"""SURVEY §8(e) replica path on CPU (gloo, world size 2): envs sharded over
ranks with seeds 4 * global_index, no data-path collective, then one counter
all-reduce and one returns all-gather (vmp.replicas). The per-rank env is the C
oracle's batched rollout (the checker standing in for the HIP env, which needs
a GPU); the GPU form of this test is tests/test_gpu_replicas.py.
Reference: the process fan-out of exp.py:1-2 / exp_performance.py:63-83."""
import multiprocessing as mp
import os
import socket

import numpy as np
import torch

from oracle import oracle as O
from vmp.replicas import reduce_replicas, shard_seeds

CFG = dict(pms=100, vms=300, arrival_rate=1.8182, service_length=200, training_steps=10000,
           eval_steps=100000, seed=0, reward_function="wr", allow_null_action=True)
N, STEPS = 8, 120


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_local = N // world
        seeds = shard_seeds(rank, n_local)
        # one oracle rollout per local env with its shard seed (stride 4 inside
        # the oracle: seed0 + 4 * j == shard seed j)
        rs, ctr = O.rollout(CFG, n_local, int(seeds[0]), 4, STEPS, policy=0, eval_mode=False)
        csum, rets = reduce_replicas(torch.from_numpy(ctr), torch.from_numpy(rs), dist)
        q.put((rank, csum.numpy().copy(), rets.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_shard_seeds_are_global_index_seeds():
    allseeds = np.concatenate([shard_seeds(r, 3) for r in range(4)])
    assert np.array_equal(allseeds, 4 * np.arange(12))


def test_two_ranks_equal_one_rank():
    rs1, ctr1 = O.rollout(CFG, N, 0, 4, STEPS, policy=0, eval_mode=False)
    csum1, rets1 = reduce_replicas(torch.from_numpy(ctr1), torch.from_numpy(rs1), None)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (c, x)) for r, c, x in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert np.array_equal(res[r][0], csum1.numpy()), r
        assert np.array_equal(res[r][1], rets1.numpy()), r  # bit-identical, global env order
