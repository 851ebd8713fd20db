"""SURVEY §8(e) replica path on the HIP env: 2 ranks x N/2 envs (gloo, both on
cuda:0, seeds 4 * global_index) must give the same counter sums and the same
per-env returns, in global env order, as 1 rank x N envs. Reference: the
process fan-out of exp.py:1-2 / exp_performance.py:63-83."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = dict(pms=100, vms=1000, arrival_rate=1.8182, service_length=300, training_steps=10000,
           eval_steps=100000, seed=0, reward_function="wr", allow_null_action=True)
N, K = 64, 150


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, n_local, dist=None):
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.replicas import reduce_replicas, shard_seeds, step_returns
    env = BatchedVmEnv(Config(**CFG), n_local, seeds=shard_seeds(rank, n_local), device="cuda:0")
    rs, _ = env.rollout("firstfit", K)
    out = reduce_replicas(env.counters().cpu(), step_returns(rs).cpu(), dist)
    env.close()
    return out


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c, r = _run(rank, N // world, dist)
        q.put((rank, c.numpy().copy(), r.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_two_ranks_equal_one_rank_on_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    c1, r1 = _run(0, N)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (c, x)) for r, c, x in (q.get(timeout=100) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert np.array_equal(res[r][0], c1.numpy()), r
        assert np.array_equal(res[r][1], r1.numpy()), r
