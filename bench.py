"""bench.py — batched env-steps/s of the VmEnv hot path on MI355X.

Workload (BASELINE.json north_star, SURVEY §8(d) C-main): config/100.yml with
vms=1000 (P100 V1000, arrival_rate 1.8182 as shipped, service_length 1000,
reward wr, allow_null_action), FirstFit act + VmEnv.step fused in one launch per
step for every env (the Base.test loop body, base.py:71-86) in training mode
(info = {} as in env.py:168; the eval-mode info metrics are derived on demand
by vmp_get_stats), obs/reward/done written to HBM each step. Envs per GPU fixed (weak scaling); env i of the job
has seed 4*i. Before timing, every env is fast-forwarded to the
steady-state fill (~200 running / ~800 waiting VMs) with the fused rollout, with
its phase staggered: the fill -> finish -> refill cycle of this workload
repeats every ~L = 1000 steps (service ~ Poisson(1000) + 1), so the envs are
reset in G = 10 groups 100 steps apart and are 2 600-3 500 steps old when the
timed window starts, i.e. spread over one whole service period (a window in
which every env sits in the same phase would time only that phase; the
`period` leg times 1 000 consecutive launches of phase-aligned envs instead).

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


def step_bytes(P, V, words, pms):
    """Algorithmic HBM bytes per env-step of the per-step kernel:
    state read (8 B/VM word, 16 B/PM, 256 B header), obs f32[3V+2P], header
    write, reward f64, done u8, the VM words that changed (`words` per
    env-step: a running VM's word holds its finish key and is not rewritten
    while it runs) and the PMs that changed (`pms` per env-step, cpu + memory
    f64: only the PM words a place / suspend / free wrote are stored back)."""
    state = 8 * V + 16 * P + 256
    return state + 4 * (3 * V + 2 * P) + 256 + 8 + 1 + 8 * words + 16 * pms


def changed_words(c0, c1, env_steps):
    """(VM words, PMs) written per env-step between two counter snapshots
    ([total_requests, served, suspend, place, dropped, timestep] per env):
    words = accepted arrivals + finishers + placements + suspensions, PMs =
    finishers + placements + suspensions (each event writes one PM's cpu and
    memory). Upper bounds: a slot freed and refilled in the same step is
    written once, and several events on one PM write it once."""
    d = (c1 - c0).double().sum(0)
    return (float((d[0] - d[4] + d[1] + d[2] + d[3]) / env_steps),
            float((d[1] + d[2] + d[3]) / env_steps))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=32768, help="envs per GPU")
    ap.add_argument("--ff-steps", type=int, default=2500, help="steady-state fast-forward")
    ap.add_argument("--phase-groups", type=int, default=10,
                    help="env groups reset --phase-delta steps apart before timing")
    ap.add_argument("--phase-delta", type=int, default=100)
    ap.add_argument("--period-steps", type=int, default=1000,
                    help="period leg: consecutive launches of phase-aligned envs (0: skip)")
    ap.add_argument("--period-ff", type=int, default=2000)
    ap.add_argument("--period-groups", type=int, default=1,
                    help="period leg phase groups (1: phase-aligned; > 1: staggered as "
                         "the headline, --phase-delta apart, to price the mixing itself)")
    ap.add_argument("--period-dump", default="", help="period leg: save the per-launch ms (.npy)")
    ap.add_argument("--period-only", action="store_true",
                    help="run only the period leg (rocprofv3 of that window)")
    ap.add_argument("--nominal-steps", type=int, default=50,
                    help="C-main at nominal load (lambda 0.182) timed launches (0: skip)")
    ap.add_argument("--rollout-k", type=int, default=100, help="steps per fused rollout launch")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ppo", action="store_true", help="skip the PPO train / eval legs")
    ap.add_argument("--ppo-envs", type=int, default=8192, help="PPO training envs per GPU")
    ap.add_argument("--ppo-eval-envs", type=int, default=4096)
    ap.add_argument("--ppo-updates", type=int, default=5,
                    help="timed collect + update cycles per PPO training leg (median reported)")
    ap.add_argument("--ext-steps", type=int, default=50, help="external-action leg steps")
    ap.add_argument("--stress-ff", type=int, default=2000, help="C5 fast-forward (2*L)")
    ap.add_argument("--stress-steps", type=int, default=20)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        import datetime
        # a rank that fails a leg must not leave the others waiting forever
        backend = os.environ.get("VMP_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    timeout=datetime.timedelta(seconds=300))
        else:  # rehearsal of the N > 1 path with several ranks on one GPU
            dist.init_process_group(backend, timeout=datetime.timedelta(seconds=300))
            local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from vmp import _lib
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config

    N = args.envs
    P, V = CFG["pms"], CFG["vms"]
    D = 3 * V + 2 * P
    from vmp.replicas import shard_seeds
    seeds = shard_seeds(rank, N)  # 4 * global env index
    env = BatchedVmEnv(Config(**CFG), N, seeds=seeds, device=dev)
    env.eval(False)
    L = _lib.lib()
    stream = torch.cuda.current_stream(dev)
    h = env._bind()

    if args.period_only:
        env.close()
        per = bench_period(args, dev, rank, world, dist, CFG)
        if rank == 0:
            print(json.dumps({"period": per}), flush=True)
        if dist:
            dist.destroy_process_group()
        return

    # ---- fast-forward to steady state, phases staggered (untimed) ----
    reset_at, ff_total = fast_forward(env, "firstfit", seeds, args.ff_steps, args.phase_groups,
                                      args.phase_delta, args.rollout_k, offset=rank * N)
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
    # (one HIP event pair on the launch stream brackets the K launches: the
    # average launch duration includes the gaps between back-to-back kernels,
    # so it is an upper bound of rocprofv3's per-dispatch average)
    K = args.steps
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    c_before = env.counters()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(K):
        one_step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    words, pmw = changed_words(c_before, env.counters(), N * K)  # after the clock stops
    kern_ms = ev0.elapsed_time(ev1) / K
    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    value = world * N * K / elapsed

    # ---- external-action mode (the PPO path): vmp_step on i32[N, V] actions ----
    ext = _guard(bench_external, args, env, dev, stream, dist, world, P, V)
    ext_steps = args.ext_steps + 2 if isinstance(ext, dict) and "error" not in ext else 0

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
    steps_done = ff_total + args.warmup + K + ext_steps + kr * (nrep + 1)

    # ---- replica reduction: counters summed, per-env returns of the
    # last fused rollout gathered over ranks (RCCL at N > 1) ----
    from vmp.replicas import reduce_replicas, step_returns
    ctr_sum, ret_all = reduce_replicas(env.counters(), step_returns(rbuf), dist)
    replicas = {"counters_sum": [int(x) for x in ctr_sum.cpu().tolist()],
                "counters": ["total_requests", "served", "suspend_action", "place_action",
                             "dropped", "timestep"],
                "returns_gathered": int(ret_all.numel()),
                "return_mean": float(ret_all.mean()),
                "return_steps": kr,
                "collectives": ("all_reduce(int64 counters, SUM) + all_gather(f64 returns) "
                                f"over {'RCCL' if world > 1 else 'none (1 rank)'}")}

    # ---- reward MAE / counter equality vs the CPU oracle on sampled envs ----
    parity = None
    cpu = None
    if rank == 0:
        from oracle import oracle as O
        # one env of every phase group (env i is in group i mod G), spread over
        # the batch, replayed through the oracle over its whole age; the last
        # fused rollout's rewards and the final counters are compared
        G = max(1, int(args.phase_groups))
        chk = sorted({g + G * ((g * 977) % max(1, N // G)) for g in range(G)} & set(range(N)))
        r_gpu = rbuf[:, chk].double().cpu().numpy()
        ctr_gpu = env.counters()[chk].cpu().numpy()
        errs, ctr_ok = [], True
        for j, i in enumerate(chk):
            e = O.OracleEnv(dict(CFG, seed=int(seeds[i])))
            e.eval(False)
            e.reset(int(seeds[i]))
            for s in range(steps_done - int(reset_at[i]) - kr):  # env i's age
                e.step(e.firstfit())
            for s in range(kr):
                _, r, _, _ = e.step(e.firstfit())
                errs.append(abs(r - r_gpu[s, j]))
            ctr_ok &= bool(np.array_equal(e.counters()[0], ctr_gpu[j]))
        parity = {"reward_mae": float(np.mean(errs)), "reward_max_abs_err": float(np.max(errs)),
                  "counters_equal": ctr_ok, "envs_checked": len(chk), "env_indices": chk,
                  "phase_groups": sorted({i % G for i in chk}),
                  "ages_checked": [steps_done - int(reset_at[i]) for i in chk],
                  "rewards_compared": len(errs)}

        if world == 1 and not args.no_cpu:
            # 48 envs per thread: ~1.5 s passes (16 per thread gave ~0.5 s
            # passes and up to 6 % spread under the box's CPU quota)
            cpu = cpu_baseline(CFG, args.cpu_threads, "same config", envs_per_thread=48)

    bpe = step_bytes(P, V, words, pmw)
    achieved = bpe * N / (kern_ms * 1e-3) / 1e9
    traffic = None
    issue = None
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("envs") == N and tj.get("bytes_per_launch"):
                traffic = float(tj["bytes_per_launch"])
            if tj.get("envs") == N and tj.get("SQ_INSTS_VALU"):
                issue = issue_roofline(tj, N, kern_ms)
        except Exception:
            traffic = None
    env.close()
    period = None if args.period_steps <= 0 else _guard(bench_period, args, dev, rank, world,
                                                       dist, CFG)
    nominal = None if args.nominal_steps <= 0 else _guard(bench_nominal, args, dev, rank, world,
                                                         dist)
    ppo_train = ppo_train_bf16 = ppo_eval = None
    if not args.no_ppo:
        ppo_train = _guard(bench_ppo_train, args, dev, rank, world, dist)
        ppo_train_bf16 = _guard(bench_ppo_train, args, dev, rank, world, dist, "bf16")
        ppo_eval = _guard(bench_ppo_eval, args, dev, rank, world, dist)
    stress = None if args.no_ppo else _guard(bench_stress, args, dev, rank, world, dist)
    stress2k = None if args.no_ppo else _guard(bench_stress, args, dev, rank, world, dist, 2048)
    out = {
        "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": K,
        "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / K, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "config/100.yml with vms=1000 (P100 V1000), FirstFit act + "
                               "VmEnv.step fused, one launch per step", "envs_per_gpu": N,
                   "global_envs": world * N, "pms": P, "vms": V,
                   "arrival_rate": CFG["arrival_rate"], "service_length": CFG["service_length"],
                   "reward_function": "wr", "policy": "firstfit", "mode": "train",
                   "parallelism": f"env-shard x{world}", "steady_state_ff_steps": args.ff_steps,
                   "phase_stagger": f"{args.phase_groups} groups x {args.phase_delta} steps: "
                                    f"env ages {ff_total - (args.phase_groups - 1) * args.phase_delta}"
                                    f"-{ff_total} at the window"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "vmp::k_env<16, true> (heuristic act+step, one step per launch)", "kernel_ms": kern_ms,
                     "bytes_per_env_step": bpe, "vm_words_written_per_env_step": words,
                     "pms_written_per_env_step": pmw, "issue": issue},
        "cpu_baseline": cpu,
        "reference_cpu": _reference_cpu(),
        "fused_rollout": {"value": fused_value, "unit": "env-steps/s", "k_steps": kr},
        "period": period,
        "nominal_load": nominal,
        "external_actions": ext,
        "replicas": replicas,
        "parity": parity,
        "ppo_train": ppo_train,
        "ppo_train_bf16": ppo_train_bf16,
        "ppo_eval": ppo_eval,
        "stress_p1000_v10000": stress,
        "stress_p1000_v10000_2048envs": stress2k,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


N_SIMDS = 1024  # MI355X: 256 CUs x 4 SIMD-32


def issue_roofline(pmc, N, kern_ms):
    """The headline kernel's instruction-issue ceiling beside its HBM one
    (VERDICT r4 item 5): instructions per launch from the committed PMC pass
    (profiles/traffic.json, the same window's SQ_INSTS_* counters) against the
    issue capacity of the live launch time at the PMC pass's measured clock.
    VALU: a wave64 VALU instruction occupies a SIMD-32 for 2 cycles
    (MI355X_MICROARCH.md §Wave scheduling), so busy = 2 x VALU / (1 024 SIMDs x
    cycles); `valu_frac_single_wave` prices 4 cycles, the rate one wave alone
    sustains (the figure an issue-bound wave with no co-resident partner
    would see). The HBM `frac` and this one together bound the kernel."""
    clk = float(pmc.get("eff_clock_GHz") or 2.4) * 1e9
    cyc = clk * kern_ms * 1e-3
    cyc_prof = clk * float(pmc["avg_ns"]) * 1e-9
    valu, salu = float(pmc["SQ_INSTS_VALU"]), float(pmc.get("SQ_INSTS_SALU", 0.0))
    lds = float(pmc.get("SQ_INSTS_LDS", 0.0))
    busy = pmc.get("valu_busy")  # rocprofv3's VALUBusy of the same pass, if collected
    return {"bound": "valu-issue", "unit": "SIMD issue cycles",
            "valu_insts_per_env_step": valu / N, "salu_insts_per_env_step": salu / N,
            "lds_insts_per_env_step": lds / N,
            "frac": 2.0 * valu / (N_SIMDS * cyc),
            "frac_at_profile_time": 2.0 * valu / (N_SIMDS * cyc_prof),
            "valu_busy_pmc": busy,
            "valu_busy_pmc_at_live_time": None if busy is None else busy * cyc_prof / cyc,
            "valu_frac_single_wave": 4.0 * valu / (N_SIMDS * cyc),
            "clock_GHz": clk / 1e9, "profile_kernel_ms": float(pmc["avg_ns"]) * 1e-6,
            "source": "profiles/traffic.json (rocprofv3 --pmc SQ_INSTS_VALU/SALU/LDS, "
                      "GRBM_GUI_ACTIVE of the headline window)"}


def fast_forward(env, policy, seeds, ff, groups, delta, k, offset=0):
    """Fused-rollout fast-forward with staggered phases: env i (global index
    offset + i, group (offset + i) mod `groups`) is reset with its own seed at
    step group * delta, so after ff + (groups - 1) * delta steps the envs'
    ages are spread over (groups - 1) * delta steps; an env's phase depends on
    its global index only, so results do not depend on the rank count.
    Returns (reset step per env, total steps)."""
    N = env.n_envs
    groups = max(1, int(groups))
    grp = (int(offset) + np.arange(N)) % groups
    reset_at = grp * delta
    total = ff + (groups - 1) * delta
    events = [g * delta for g in range(1, groups)]
    t = 0
    while t < total:
        if t in events:
            env.reset(seeds, mask=torch.from_numpy(grp == t // delta), obs=False)
        nxt = min([x for x in events if x > t] + [total])
        kk = min(k, nxt - t)
        env.rollout(policy, kk)
        t += kk
    return reset_at, total


def bench_period(args, dev, rank, world, dist, cfg):
    """the headline workload over a whole service period.
    Phase-aligned envs (all reset together, as at the start of an episode)
    fast-forwarded --period-ff = 2 000 steps, then --period-steps = 1 000
    consecutive per-step launches (steps 2 001-3 000: the refill burst after
    the first VMs finish, and the quiet phase after it). Per-launch kernel
    time from a HIP event pair around every launch on the launch stream;
    mean / max and 100-launch bins, changed VM words and the roofline of the
    window's mean launch."""
    from vmp import _lib
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.replicas import shard_seeds
    N = args.envs
    P, V = cfg["pms"], cfg["vms"]
    env = BatchedVmEnv(Config(**cfg), N, seeds=shard_seeds(rank, N), device=dev)
    env.eval(False)
    G = max(1, args.period_groups)
    if G > 1:  # same window position, envs' ages spread as in the headline leg
        fast_forward(env, "firstfit", shard_seeds(rank, N), args.period_ff - (G - 1) * args.phase_delta,
                     G, args.phase_delta, args.rollout_k, offset=rank * N)
    left = args.period_ff if G == 1 else 0
    while left > 0:
        env.rollout("firstfit", min(args.rollout_k, left))
        left -= args.rollout_k
    L, h = _lib.lib(), env._bind()
    stream = torch.cuda.current_stream(dev)
    obs = torch.empty((N, 3 * V + 2 * P), dtype=torch.float32, device=dev)
    rew = torch.empty((N,), dtype=torch.float64, device=dev)
    done = torch.empty((N,), dtype=torch.uint8, device=dev)
    p_obs, p_rew, p_done = _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(done)
    K = args.period_steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K)]
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    c0 = env.counters()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        _lib.check(L.vmp_heuristic_step(h, 0, None, p_obs, p_rew, p_done, None))
        b.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = _max_over_ranks(time.perf_counter() - t0, dev, dist)
    c1 = env.counters()
    words, pmw = changed_words(c0, c1, N * K)
    ms = np.array([a.elapsed_time(b) for a, b in ev])
    if args.period_dump and rank == 0:
        np.save(args.period_dump, ms)
    env.close()
    mean_ms = _max_over_ranks(float(ms.mean()), dev, dist)
    bins = [round(float(ms[i:i + 100].mean()), 4) for i in range(0, K, 100)]
    bpe = step_bytes(P, V, words, pmw)
    ach = bpe * N / (mean_ms * 1e-3) / 1e9
    return {"value": world * N / (mean_ms * 1e-3), "unit": "env-steps/s",
            "value_kind": "mean per-launch kernel time over the window",
            "wall_value": world * N * K / el,
            "window": f"steps {args.period_ff + 1}-{args.period_ff + K} of "
                      + ("phase-aligned envs" if G == 1 else
                         f"envs in {G} phase groups {args.phase_delta} steps apart"),
            "steps": K, "mean_ms": mean_ms, "max_ms": float(ms.max()),
            "min_ms": float(ms.min()), "ms_by_100_steps": bins,
            "bytes_per_env_step": bpe, "vm_words_written_per_env_step": words,
            "pms_written_per_env_step": pmw,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS,
                         "kernel": "vmp::k_env<16, true> (heuristic act+step)"}}


def bench_nominal(args, dev, rank, world, dist):
    """SURVEY §8(d) C-main at nominal load: config/100.yml with vms = 1000 at
    lambda = 0.182 (100 % load, exp_suspension.py:19; ~724 NULL slots and ~121
    waiting VMs per env), L = 1000, reward wr, FirstFit act + step per launch,
    phases staggered as the headline's; its own roofline (same byte model) and
    its own CPU baseline (the C oracle, OpenMP, rank 0 at N = 1)."""
    from vmp import _lib
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.replicas import shard_seeds
    cfg = dict(CFG, arrival_rate=0.182)
    N = args.envs
    P, V = cfg["pms"], cfg["vms"]
    seeds = shard_seeds(rank, N)
    env = BatchedVmEnv(Config(**cfg), N, seeds=seeds, device=dev)
    env.eval(False)
    _, ff_total = fast_forward(env, "firstfit", seeds, 2000, args.phase_groups, args.phase_delta,
                               args.rollout_k, offset=rank * N)
    L, h = _lib.lib(), env._bind()
    stream = torch.cuda.current_stream(dev)
    obs = torch.empty((N, 3 * V + 2 * P), dtype=torch.float32, device=dev)
    rew = torch.empty((N,), dtype=torch.float64, device=dev)
    done = torch.empty((N,), dtype=torch.uint8, device=dev)
    p_obs, p_rew, p_done = _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(done)
    for _ in range(5):
        _lib.check(L.vmp_heuristic_step(h, 0, None, p_obs, p_rew, p_done, None))
    pl = env.state()["vm_placement"]
    running = float((pl < P).sum(1).double().mean())
    waiting = float((pl == P).sum(1).double().mean())
    del pl
    K = args.nominal_steps
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    c0 = env.counters()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(K):
        _lib.check(L.vmp_heuristic_step(h, 0, None, p_obs, p_rew, p_done, None))
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = _max_over_ranks(time.perf_counter() - t0, dev, dist)
    words, pmw = changed_words(c0, env.counters(), N * K)
    kern_ms = _max_over_ranks(ev0.elapsed_time(ev1) / K, dev, dist)
    env.close()
    bpe = step_bytes(P, V, words, pmw)
    ach = bpe * N / (kern_ms * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # 160 envs per thread: a pass of ~1 s (16 envs per thread pass in
        # ~0.1 s, where the cgroup's 100 ms CPU-quota periods make the spread)
        cpu = cpu_baseline(cfg, args.cpu_threads, "lambda 0.182", envs_per_thread=160)
    return {"value": world * N * K / el, "unit": "env-steps/s", "dtype": "f64",
            "workload": "config/100.yml with vms=1000, lambda 0.182 (100 % load), L 1000, "
                        "reward wr, FirstFit act + step, one launch per step",
            "envs_per_gpu": N, "ff_steps": ff_total, "steps": K, "mean_running": running,
            "mean_waiting": waiting, "ms_per_step": 1e3 * el / K, "kernel_ms": kern_ms,
            "bytes_per_env_step": bpe, "vm_words_written_per_env_step": words,
            "pms_written_per_env_step": pmw,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS,
                         "kernel": "vmp::k_env<16, true> (heuristic act+step)"},
            "cpu_baseline": cpu}


def host_cpus():
    """The host this run sees: nproc, the affinity set, the cgroup CPU quota (in
    cores, None when unlimited) and the CPU model string."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cores": quota,
            "cpu_model": model}


def cpu_baseline(cfg, threads=0, what="", envs_per_thread=16):
    """SURVEY §8(d) / BASELINE.md §4 CPU baseline: the C oracle (FirstFit act +
    VmEnv.step, training mode as the GPU leg) over OpenMP on every core this
    process may run on (the affinity set, capped by the cgroup's CPU quota when
    one is set: threads beyond the quota only time-slice), 16 envs per thread
    (envs_per_thread),
    warmed up 2 500 steps (the GPU window's env ages), then 7 timed passes of
    1 000 steps (one service period each) after an untimed one; value = the
    median pass, spread = (max - min) / median, spread_trimmed the same
    without the extreme passes."""
    from oracle import oracle as O
    host = host_cpus()
    if not threads:
        threads = host["affinity"]
        if host["cgroup_quota_cores"]:
            threads = max(1, min(threads, int(host["cgroup_quota_cores"])))
    n_env, warm, steps, reps = envs_per_thread * threads, 2500, 1000, 7
    # one more pass than reported: the first pass after the warm-up steps is
    # untimed warm-up of its own (it ran up to 7 % slow on a shared host)
    secs, _ = O.rollout_timed(cfg, n_env, 0, 4, warm, steps, 0, threads, eval_mode=False,
                              reps=reps + 1)
    rates = n_env * steps / secs[1:]
    med = float(np.median(rates))
    srt = np.sort(rates)
    return {"value": med, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "repeats": [float(x) for x in rates], "spread": float((rates.max() - rates.min()) / med),
            # the same without the slowest and the fastest pass: one pass
            # caught by a neighbour's load on the shared host moves `spread`
            # alone (tools/cpu_spread.py on the GPU box: 1-2 % at 16 threads)
            "spread_trimmed": float((srt[-2] - srt[1]) / med),
            "warmup_pass": float(n_env * steps / secs[0]),
            **host,
            "sample": f"{n_env} envs x {steps} FirstFit act+step per pass, {reps} passes (median) "
                      f"after one untimed pass and {warm} warm-up steps, OpenMP {threads} "
                      f"threads (C oracle, {what})"}


def _guard(fn, *a):
    """A secondary leg reports its failure in the JSON instead of ending the run."""
    try:
        return fn(*a)
    except Exception as ex:  # noqa: BLE001
        return {"error": f"{type(ex).__name__}: {ex}"}


def _max_over_ranks(x, dev, dist):
    if dist:
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        x = float(t[0])
    return x


F32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md chip table (f32 matrix = vector peak)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (spec, no sparsity)


def mlp_flops(dims):
    """Forward multiply-add FLOPs of a Linear stack per sample: 2 sum(in * out)."""
    return 2.0 * sum(a * b for a, b in zip(dims[:-1], dims[1:]))


def ppo_update_flops(D, H, VA, T, E, mb_evaluated, mbs):
    """Algorithmic FLOPs of one PPOTrainer collect + update (ppo.py:172-295)
    from the GEMM shapes: the rollout's actor forward for T x E
    samples; the update's critic forward of the T x E + E values; per
    evaluated minibatch (mbs x E samples) the actor and critic forward and
    backward (3x forward, less the first layers' unneeded input gradient).
    Recomputation (the fused bf16 head's backward) is not counted."""
    actor, critic = [D, H, H, VA], [D, H, H, 1]
    fa, fc = mlp_flops(actor), mlp_flops(critic)
    first = 2.0 * D * H
    collect = T * E * fa
    values = (T * E + E) * fc
    per_sample = 3 * fa - first + 3 * fc - first
    update = values + mb_evaluated * mbs * E * per_sample
    return collect, update


def mfma_roofline(flops, seconds, precision, what):
    peak = F32_MFMA_PEAK_TFLOPS if precision == "f32" else BF16_MFMA_PEAK_TFLOPS
    ach = flops / seconds / 1e12
    return {"bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
            "flops": flops, "what": what}


def bench_ppo_train(args, dev, rank, world, dist, precision="f32"):
    """BASELINE config 3 (config/100.yml, PPO from scratch, reward wr, 8192 envs per
    GPU): one untimed collect + update, then --ppo-updates (5) timed cycles of
    batch_size rollout steps of every env + PPOAgent.update (4 epochs x 4
    minibatches), data-parallel over ranks (one RCCL all-reduce
    of the flat gradient per optimizer step). Median and spread reported."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    torch.manual_seed(0)
    N = args.ppo_envs
    cfg = Config(pms=100, vms=300, service_length=1000, arrival_rate=1.8182,
                 training_steps=10000, eval_steps=100000, seed=0, reward_function="wr",
                 sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True)
    env = BatchedVmEnv(cfg, N, seeds=4 * (rank * N + np.arange(N, dtype=np.int64)), device=dev)
    ag = PPOAgent(env, PPOConfig(hidden_size=512, batch_size=100, minibatch_size=25,
                                 migration_ratio=0.002, masked=True, precision=precision))
    tr = ag.trainer()
    tr.collect()
    tr.update()
    torch.cuda.synchronize(dev)
    H = ag.config.hidden_size
    fused = precision == "bf16" and ag.model.bf16_fused()
    # per timed update: (collect s, update s, evaluated minibatches, minibatch steps, kl
    # breaks, executed minibatches). With the KL look-ahead a break also runs and
    # discards the next minibatch (stats["rollbacks"] counts the broken one and
    # that one): executed = steps + rollbacks >= evaluated = steps + breaks
    runs = []
    for _ in range(max(1, int(args.ppo_updates))):
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        tr.collect()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        st = tr.update()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        t2 = time.perf_counter()
        runs.append((_max_over_ranks(t1 - t0, dev, dist), _max_over_ranks(t2 - t1, dev, dist),
                     st["minibatches"] + st["kl_breaks"], st["minibatches"], st["kl_breaks"],
                     st["minibatches"] + max(st.get("rollbacks", 0), st["kl_breaks"])))
    col = np.array([r[0] for r in runs])
    upd = np.array([r[1] for r in runs])
    tot = col + upd
    steps = world * N * tr.T
    # algorithmic FLOPs of each timed update (the KL early stop may skip minibatches)
    fus = np.array([ppo_update_flops(env.D, H, env.V * env.A, tr.T, N, r[2],
                                     ag.config.minibatch_size)[1] for r in runs])
    fc = ppo_update_flops(env.D, H, env.V * env.A, tr.T, N, 0, ag.config.minibatch_size)[0]
    # executed: the look-ahead's discarded minibatches, and the fused head's
    # backward recomputing the last layer's logits: matrix-core work beyond the
    # algorithmic count (what a PMC MFMA-busy pass sees)
    fex = np.array([ppo_update_flops(env.D, H, env.V * env.A, tr.T, N, r[5],
                                     ag.config.minibatch_size)[1] for r in runs])
    recompute = np.array([r[5] * ag.config.minibatch_size * N * 2.0 * H * env.V * env.A
                          for r in runs]) if fused else np.zeros(len(runs))
    med = int(np.argsort(upd)[len(upd) // 2])  # the median update
    upd_s, col_s, total = float(upd[med]), float(col[med]), float(np.median(tot))
    env.close()
    return {"value": steps / total, "unit": "env-steps/s",
            "value_kind": f"median over {len(runs)} timed collect + update cycles",
            "roofline": dict(mfma_roofline(float(fus[med]), upd_s, precision,
                                           "PPOAgent.update (all GEMMs, per GPU) / update wall "
                                           "time, median update"),
                             executed_flops=float(fex[med] + recompute[med])),
            "collect_roofline": mfma_roofline(fc, col_s, precision,
                                              "rollout actor forward / collect wall time"),
            "updates_timed": len(runs), "update_s_all": [float(x) for x in upd],
            "collect_s_all": [float(x) for x in col],
            "update_s_spread": float((upd.max() - upd.min()) / np.median(upd)),
            "head": ("fused bf16 matrix-core actor head (vmp_actor_head_bf16_fwd/_bwd)" if fused
                     else "f32 logits + HIP head" if precision == "f32"
                     else "bf16 GEMM -> f32 logits + HIP head"),
            "dtype": "f32" if precision == "f32" else "bf16 GEMM inputs, f32 accumulate/params",
            "workload": "config/100.yml (P100 V300), PPO train from scratch, reward wr, "
                        "hidden 512, batch 100 / minibatch 25, 4 epochs",
            "envs_per_gpu": N, "global_envs": world * N,
            "s_per_update": total, "collect_s": float(np.median(col)),
            "update_s": float(np.median(upd)), "update_s_min": float(upd.min()),
            "minibatch_steps": [r[3] for r in runs], "kl_breaks": [r[4] for r in runs],
            "minibatches_executed": [r[5] for r in runs],
            "parallelism": f"data-parallel x{world} (RCCL grad all-reduce)" if world > 1
            else "single GPU"}


def bench_stress(args, dev, rank, world, dist, N=512):
    """BASELINE config 5: P1000 / V10000 at 100 % load
    (lambda = 1000/0.55/1000), L = 1000, reward kl, BestFit act + step, N envs
    per GPU (512; the 2048-env line shows the kernel at a batch that fills
    every CU's two workgroup slots several times) on the block-per-env kernel
    k_env_big. Fast-forwarded 2*L = 2000
    steps with the fused rollout (steady state: ~1600 running / ~380 waiting VMs
    per env), then K timed per-step launches; kernel time from HIP events on
    the launch stream."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp import _lib
    P, V = 1000, 10000
    cfg = Config(pms=P, vms=V, arrival_rate=round(1000 / 0.55 / 1000, 3), service_length=1000,
                 training_steps=10000, eval_steps=100000, seed=0, reward_function="kl",
                 sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True)
    env = BatchedVmEnv(cfg, N, seeds=4 * (rank * N + np.arange(N, dtype=np.int64)), device=dev)
    left = args.stress_ff
    while left > 0:
        env.rollout("bestfit", min(250, left))
        left -= 250
    obs = torch.empty((N, env.D), dtype=torch.float32, device=dev)
    rew = torch.empty((N,), dtype=torch.float64, device=dev)
    done = torch.empty((N,), dtype=torch.uint8, device=dev)
    L, h = _lib.lib(), env._bind()
    stream = torch.cuda.current_stream(dev)
    pl = env.state()["vm_placement"]
    running, waiting = float((pl < P).sum(1).double().mean()), float((pl == P).sum(1).double().mean())
    del pl
    _lib.check(L.vmp_heuristic_step(h, 1, None, _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(done), None))
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    K = args.stress_steps
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c_before = env.counters()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(K):
        _lib.check(L.vmp_heuristic_step(h, 1, None, _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(done),
                                        None))
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = _max_over_ranks(time.perf_counter() - t0, dev, dist)
    words, pmw = changed_words(c_before, env.counters(), N * K)
    kern_ms = _max_over_ranks(ev0.elapsed_time(ev1) / K, dev, dist)
    env.close()
    bpe = step_bytes(P, V, words, pmw)
    ach = bpe * N / (kern_ms * 1e-3) / 1e9
    return {"value": world * N * K / el, "unit": "env-steps/s", "dtype": "f64",
            "workload": "P1000 V10000, lambda 1.818, L 1000, reward kl, BestFit act + step "
                        "(k_env_big: one 256-thread workgroup per env, two per CU)", "envs_per_gpu": N,
            "ff_steps": args.stress_ff, "steps": K, "mean_running": running,
            "mean_waiting": waiting, "ms_per_step": 1e3 * el / K, "kernel_ms": kern_ms,
            "bytes_per_env_step": bpe, "vm_words_written_per_env_step": words,
            "pms_written_per_env_step": pmw,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "kernel": "vmp::k_env_big<40, true>"}}


def bench_external(args, env, dev, stream, dist, world, P, V):
    """SURVEY §8(d) C-main, external-action mode (the path PPO drives): per step
    the FirstFit action of every env is produced by an act-only launch
    (vmp_heuristic_act, untimed by the events) into an i32[N, V] buffer, then
    vmp_step (VmEnv.step, env.py:66-103) consumes it, writing obs / reward /
    done. Kernel time = HIP events around vmp_step only; the wall rate counts
    both launches."""
    if args.ext_steps <= 0:  # leg skipped (profiling runs of the headline kernel)
        return None
    from vmp import _lib
    N = env.n_envs
    L, h = _lib.lib(), env._bind()
    D = 3 * V + 2 * P
    act = torch.empty((N, V), dtype=torch.int32, device=dev)
    obs = torch.empty((N, D), dtype=torch.float32, device=dev)
    rew = torch.empty((N,), dtype=torch.float64, device=dev)
    done = torch.empty((N,), dtype=torch.uint8, device=dev)
    pa, po, pr, pd = _lib.ptr(act), _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(done)

    def one(e0=None, e1=None):
        _lib.check(L.vmp_heuristic_act(h, 0, pa))
        if e0 is not None:
            e0.record(stream)
        _lib.check(L.vmp_step(h, pa, po, pr, pd, None))
        if e1 is not None:
            e1.record(stream)
    for _ in range(2):
        one()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    K = args.ext_steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K)]
    c_before = env.counters()
    t0 = time.perf_counter()
    for a, b in ev:
        one(a, b)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = _max_over_ranks(time.perf_counter() - t0, dev, dist)
    words, pmw = changed_words(c_before, env.counters(), N * K)
    kern_ms = _max_over_ranks(float(np.mean([a.elapsed_time(b) for a, b in ev])), dev, dist)
    bpe = step_bytes(P, V, words, pmw) + 4 * V
    ach = bpe * N / (kern_ms * 1e-3) / 1e9
    return {"value": world * N / (kern_ms * 1e-3), "unit": "env-steps/s",
            "value_kind": "step kernel alone (events around vmp_step)",
            "act_plus_step_wall": world * N * K / el, "steps": K, "kernel_ms": kern_ms,
            "bytes_per_env_step": bpe, "vm_words_written_per_env_step": words,
            "pms_written_per_env_step": pmw,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS,
                         "kernel": "vmp::k_env_ext<16> (external actions)"}}


def _reference_cpu():
    """The unmodified reference VmEnv.step timed in the build container
    (tools/time_reference.py -> tests/golden/ref_cpu_timing.json): a different
    box from this run's; carried for context beside cpu_baseline."""
    pth = os.path.join(ROOT, "tests", "golden", "ref_cpu_timing.json")
    if not os.path.exists(pth):
        return None
    d = json.load(open(pth))
    r = d["results"].get("p100v1000", {})
    return {"value": r.get("single_core_steps_per_s"), "unit": "env-steps/s", "cores": 1,
            "kind": "reference (unmodified Python VmEnv.step)",
            "procs_8_aggregate": r.get("procs_8_aggregate_steps_per_s"),
            "box": "build container, not the GPU box: " + str(d["box"].get("model")),
            "sample": d["what"]}


def bench_ppo_eval(args, dev, rank, world, dist):
    """BASELINE config 2: config/10.yml PPO eval with weights-10/ppo-wr.pt (the
    reference's own weights, tests/golden/ppo10_wr_weights.npz), 4096 batched envs,
    masked, migration_ratio 0.5 WAIT coin flips: per step mask + actor forward +
    masked sample + env.step for every env."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    N = args.ppo_eval_envs
    cfg = Config(pms=10, vms=30, service_length=1000, arrival_rate=0.0182, training_steps=10000,
                 eval_steps=100000, seed=1, reward_function="wr", sequence="uniform",
                 cap_target_util=True, beta=0.5, allow_null_action=True)
    env = BatchedVmEnv(cfg, N, seeds=1 + 4 * (rank * N + np.arange(N, dtype=np.int64)),
                       device=dev)
    env.eval(True)
    ag = PPOAgent(env, PPOConfig(hidden_size=512, masked=True, migration_ratio=0.5))
    w = np.load(os.path.join(ROOT, "tests", "golden", "ppo10_wr_weights.npz"))
    ag.model.load_state_dict({k: torch.tensor(w[k]) for k in w.files})
    ag.eval(True)
    from vmp.ppo import ActStepGraph
    G = 4  # steps per graph: actor + head + step of every env, 4 times per replay
    g = ActStepGraph(ag, steps=G)
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    K = 200
    t0 = time.perf_counter()
    for _ in range(K // G):
        g.replay()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = _max_over_ranks(time.perf_counter() - t0, dev, dist)
    flops = N * K * mlp_flops([env.D, 512, 512, env.V * env.A])
    env.close()
    return {"value": world * N * K / el, "unit": "env-steps/s", "dtype": "f32",
            "roofline": mfma_roofline(flops, el, "f32",
                                      "actor forward (Network.get_action) / replayed step wall time"),
            "workload": "config/10.yml (P10 V30), PPO eval, weights-10/ppo-wr.pt, masked, "
                        "migration_ratio 0.5, one HIP graph per 4 batched steps (every step complete)",
            "envs_per_gpu": N, "steps": K,
            "ms_per_step": 1e3 * el / K}


if __name__ == "__main__":
    main()
