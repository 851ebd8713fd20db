"""bench.py — batched env-steps/s of the VmEnv hot path on MI355X.

Workload (BASELINE.json north_star, SURVEY §8(d) C-main): config/100.yml with
vms=1000 (P100 V1000, arrival_rate 1.8182 as shipped, service_length 1000,
reward wr, allow_null_action), FirstFit act + VmEnv.step fused in one launch per
step for every env (the Base.test loop body, base.py:71-86) in training mode
(info = {} as in env.py:168; the eval-mode info metrics are derived on demand
by vmp_get_stats), obs/reward/done written to HBM each step. Envs per GPU fixed (weak scaling); env i of the job
has seed 4*i. Before timing, every env is fast-forwarded to the
steady-state fill (~200 running / ~800 waiting VMs) with the fused rollout.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E]
       (N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "vm-placement-migration-gym_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "env-steps/sec (batched) at 100-PM config, 1/2/4/8 GPUs; reward MAE vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)

CFG = dict(pms=100, vms=1000, arrival_rate=1.8182, service_length=1000, training_steps=10000,
           eval_steps=100000, seed=0, reward_function="wr", sequence="uniform",
           cap_target_util=True, beta=0.5, allow_null_action=True)


def step_bytes(P, V):
    """Algorithmic HBM bytes per env-step of the per-step kernel:
    state read + write (8 B/VM word, 16 B/PM, 256 B header), obs f32[3V+2P],
    reward f64, done u8."""
    state = 8 * V + 16 * P + 256
    return 2 * state + 4 * (3 * V + 2 * P) + 8 + 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=32768, help="envs per GPU")
    ap.add_argument("--ff-steps", type=int, default=2500, help="steady-state fast-forward")
    ap.add_argument("--rollout-k", type=int, default=100, help="steps per fused rollout launch")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from vmp import _lib
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config

    N = args.envs
    P, V = CFG["pms"], CFG["vms"]
    D = 3 * V + 2 * P
    seeds = 4 * (rank * N + np.arange(N, dtype=np.int64))
    env = BatchedVmEnv(Config(**CFG), N, seeds=seeds, device=dev)
    env.eval(False)
    L = _lib.lib()
    stream = torch.cuda.current_stream(dev)
    h = env._bind()

    # ---- fast-forward to steady state (untimed) ----
    ff = args.ff_steps
    k = args.rollout_k
    while ff > 0:
        kk = min(k, ff)
        env.rollout("firstfit", kk)
        ff -= kk
    torch.cuda.synchronize(dev)

    obs = torch.empty((N, D), dtype=torch.float32, device=dev)
    rew = torch.empty((N,), dtype=torch.float64, device=dev)
    done = torch.empty((N,), dtype=torch.uint8, device=dev)
    p_obs, p_rew, p_done = _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(done)

    def one_step():
        _lib.check(L.vmp_heuristic_step(h, 0, None, p_obs, p_rew, p_done, None))

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize(dev)

    # ---- timed region: exactly K steps, barrier + sync on both sides ----
    K = args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(K):
        ev[i][0].record(stream)
        one_step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    value = world * N * K / elapsed

    # ---- fused K-step rollout (state resident on chip), same envs ----
    kr = args.rollout_k
    rbuf = torch.empty((kr, N), dtype=torch.float64, device=dev)
    env.rollout("firstfit", kr, rewards=rbuf)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    r0 = time.perf_counter()
    nrep = 3
    for _ in range(nrep):
        env.rollout("firstfit", kr, rewards=rbuf)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    r_el = time.perf_counter() - r0
    if dist:
        t = torch.tensor([r_el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        r_el = float(t[0])
    fused_value = world * N * kr * nrep / r_el
    steps_done = args.ff_steps + args.warmup + K + kr * (nrep + 1)

    # ---- reward MAE / counter equality vs the CPU oracle on sampled envs ----
    parity = None
    cpu = None
    if rank == 0:
        from oracle import oracle as O
        n_chk = 2
        r_gpu = rbuf[:, :n_chk].double().cpu().numpy()
        ctr_gpu = env.counters()[:n_chk].cpu().numpy()
        errs, ctr_ok = [], True
        for i in range(n_chk):
            e = O.OracleEnv(dict(CFG, seed=int(seeds[i])))
            e.eval(False)
            e.reset(int(seeds[i]))
            for s in range(steps_done - kr):
                e.step(e.firstfit())
            for s in range(kr):
                _, r, _, _ = e.step(e.firstfit())
                errs.append(abs(r - r_gpu[s, i]))
            ctr_ok &= bool(np.array_equal(e.counters()[0], ctr_gpu[i]))
        parity = {"reward_mae": float(np.mean(errs)), "counters_equal": ctr_ok,
                  "envs_checked": n_chk, "steps_checked": steps_done}

        if world == 1 and not args.no_cpu:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            n_cpu, warm_cpu, steps_cpu = 4 * threads, 1500, 4000
            sec, _ = O.rollout_timed(CFG, n_cpu, 0, 4, warm_cpu, steps_cpu, 0, threads)
            cpu = {"value": n_cpu * steps_cpu / sec, "unit": "env-steps/s", "cores": threads,
                   "kind": "port",
                   "sample": f"{n_cpu} envs x {steps_cpu} FirstFit act+step after {warm_cpu} "
                             f"warm-up steps, OpenMP {threads} threads (C oracle, same config)"}

    bpe = step_bytes(P, V)
    achieved = bpe * N / (kern_ms * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("envs") == N and tj.get("bytes_per_launch"):
                traffic = float(tj["bytes_per_launch"])
        except Exception:
            traffic = None
    out = {
        "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": K,
        "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / K, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "config/100.yml with vms=1000 (P100 V1000), FirstFit act + "
                               "VmEnv.step fused, one launch per step", "envs_per_gpu": N,
                   "global_envs": world * N, "pms": P, "vms": V,
                   "arrival_rate": CFG["arrival_rate"], "service_length": CFG["service_length"],
                   "reward_function": "wr", "policy": "firstfit", "mode": "train",
                   "parallelism": f"env-shard x{world}", "steady_state_ff_steps": args.ff_steps},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "vmp::k_env<16, true> (heuristic act+step, one step per launch)", "kernel_ms": kern_ms,
                     "bytes_per_env_step": bpe},
        "cpu_baseline": cpu,
        "fused_rollout": {"value": fused_value, "unit": "env-steps/s", "k_steps": kr},
        "parity": parity,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    env.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
