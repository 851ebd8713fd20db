"""Env-shard replicas over the GPUs of a node.

The reference's only parallelism is process fan-out of independent runs
(exp.py:1-2 `cores = 8`, exp_performance.py:63-83: one OS process per seed).
Here every rank (one process per GPU) owns a contiguous block of envs; env i of
the job has seed `base + stride * i` with i = rank * n_local + local index, so
a result never depends on how many GPUs share the job. Heuristic rollouts need
no data-path collective; at the end the integer counters are summed and the
per-env returns gathered in global env order (two RCCL collectives over xGMI
when the process group is NCCL = RCCL on ROCm; gloo works the same on CPU).
"""
import numpy as np
import torch


def shard_seeds(rank, n_local, base=0, stride=4):
    """Seeds of this rank's envs: base + stride * (rank * n_local + j)."""
    return base + stride * (int(rank) * int(n_local) + np.arange(int(n_local), dtype=np.int64))


def step_returns(rewards):
    """Per-env sum of a [K, n] reward block in step order (k = 0, 1, ...):
    elementwise adds, so an env's return does not depend on how many envs share
    its launch (a torch reduction over dim 0 may block differently per shape)."""
    ret = rewards[0].clone()
    for k in range(1, rewards.shape[0]):
        ret += rewards[k]
    return ret


def reduce_replicas(counters, returns, dist=None):
    """counters int64 [n_local, C], returns float [n_local] (this rank's envs) ->
    (counter sums int64 [C] over all envs of the job, returns [world * n_local]
    in global env order). `dist` is torch.distributed (initialised) or None."""
    ctr = counters.to(torch.int64).sum(0)
    ret = returns.contiguous()
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return ctr, ret
    dist.all_reduce(ctr, op=dist.ReduceOp.SUM)
    out = torch.empty(dist.get_world_size() * ret.numel(), dtype=ret.dtype, device=ret.device)
    dist.all_gather_into_tensor(out, ret)
    return ctr, out
