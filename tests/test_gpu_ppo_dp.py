"""BASELINE config 4's code path on the MI355X (SURVEY §8(e),
src/agents/ppo.py:172-295): data-parallel PPOTrainer on 2 gloo ranks sharing
cuda:0, each rank holding 32 of 64 config/100.yml envs (P100 / V300 / A102,
hidden 512, batch 100 / minibatch 25, 4 epochs), one collect + one update
through the HIP env, the HIP head and the HIP GAE, compared with ONE process
holding all 64 envs:

  - each rank's rollout, replayed through a 64-env single-process env in
    global env order, reproduces the ranks' observations and rewards
    bit-for-bit (the env shards are the global envs: seeds 4 * global index);
  - every sampled action is valid under its mask;
  - the ranks' sampling streams are folded with the rank (HeadRng.fold), so
    rank 1 does not redraw rank 0's uniforms;
  - the first AdamW step's all-reduced gradient equals the single-process
    gradient to f32 rounding (3e-5 relative L2), both ranks identical;
  - after the update (16 AdamW steps), both ranks hold bit-identical
    parameters, equal to the single-process update on the concatenated
    rollout within 1e-3 relative L2 of the change and 5e-5 absolute (the
    update moves them by ~7e-4; the two differ only in the f32 summation
    order of the sharded gradient, which AdamW's per-element normalisation
    passes on at full step size where a gradient element nearly cancels).
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
CFG100 = dict(pms=100, vms=300, service_length=1000, arrival_rate=1.8182, training_steps=10000,
              eval_steps=100000, seed=0, reward_function="wr", sequence="uniform",
              cap_target_util=True, beta=0.5, allow_null_action=True)
PCFG = dict(hidden_size=512, batch_size=100, minibatch_size=25, migration_ratio=0.002,
            masked=True, k_epochs=4)
N_GLOBAL, WORLD = 64, 2
BUFS = ("obs", "bits", "act", "logp", "rew", "done", "last_obs")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _agent(n_envs):
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    torch.manual_seed(0)  # every rank alike, as bench.py / vmp.main do
    env = BatchedVmEnv(Config(**CFG100), n_envs, device=DEV)
    return env, PPOAgent(env, PPOConfig(**PCFG))


def _first_step_grads(ag, n_keep=1 << 20):
    """Capture the (all-reduced, clipped) flat gradient of the update's first
    AdamW step at fixed positions: AdamW normalises the gradient per element,
    so comparing gradients is the sharp test of the sharded loss and the
    all-reduce (a scale error would vanish in the parameters)."""
    out = {}
    st = ag.optimizer.step
    idx = None

    def step(*a, **k):
        nonlocal idx
        if "g" not in out:
            g = torch.cat([p.grad.flatten() for p in ag.model.parameters()]).double()
            if idx is None:
                idx = torch.randperm(g.numel(), generator=torch.Generator().manual_seed(3))[
                    :n_keep].to(g.device)
            out["g"] = g[idx].cpu().numpy()
        return st(*a, **k)
    ag.optimizer.step = step
    return out


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        env, ag = _agent(N_GLOBAL // world)
        p0 = {k: v.detach().cpu().numpy().copy() for k, v in ag.model.state_dict().items()}
        tr = ag.trainer()
        tr.collect()
        roll = {k: getattr(tr, k).cpu().numpy().copy() for k in BUFS}
        g1 = _first_step_grads(ag)
        st = tr.update()
        params = {k: v.detach().cpu().numpy().copy() for k, v in ag.model.state_dict().items()}
        q.put((rank, p0, roll, params, int(ag.model.rng.seed), st["minibatches"],
               st["kl_breaks"], g1["g"]))
        env.close()
    finally:
        dist.destroy_process_group()


def test_data_parallel_trainer_two_ranks_on_gpu_equals_one_process():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    from tests.torch_ref import unpack_bits
    from vmp.ppo import PPOTrainer
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, p0, roll, params, seed, n_mb, n_kl, g1 = q.get(timeout=240)
        res[r] = dict(p0=p0, roll=roll, params=params, seed=seed, n_mb=n_mb, n_kl=n_kl, g1=g1)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # rank-folded sampling streams; same initial parameters everywhere
    assert res[0]["seed"] != res[1]["seed"]
    for k in res[0]["p0"]:
        assert np.array_equal(res[0]["p0"][k], res[1]["p0"][k]), k
    # the global rollout, env order = rank-major (PPOTrainer._episode_seeds)
    cat = {k: np.concatenate([res[r]["roll"][k] for r in range(WORLD)],
                             axis=0 if k == "last_obs" else 1) for k in BUFS}
    env, ag = _agent(N_GLOBAL)
    for k, v in ag.model.state_dict().items():
        assert np.array_equal(v.cpu().numpy(), res[0]["p0"][k]), k
    V, A = env.V, env.A
    T = cat["rew"].shape[0]
    bits = torch.from_numpy(cat["bits"]).to(DEV)
    act = torch.from_numpy(cat["act"]).to(DEV)
    full = unpack_bits(bits.reshape(T * N_GLOBAL, V, -1), A).reshape(T, N_GLOBAL, V, A)
    assert not full.gather(-1, act.long()[..., None]).any(), "a sampled action is masked"
    # replay the ranks' actions through one 64-env env: same obs, masks, rewards
    tr = PPOTrainer(ag, distributed=False)
    tr._start_episode(tr.obs[0])
    obs_g = torch.from_numpy(cat["obs"]).to(DEV)
    r64 = torch.empty((N_GLOBAL,), dtype=torch.float64, device=DEV)
    d8 = torch.empty((N_GLOBAL,), dtype=torch.uint8, device=DEV)
    nxt = torch.empty_like(tr.last_obs)
    for t in range(T):
        cur = tr.obs[0] if t == 0 else nxt
        assert torch.equal(cur, obs_g[t]), t
        assert torch.equal(env.mask_bits(), bits[t]), t
        env.step(act[t], obs=nxt, reward=r64, done=d8, want_valid=False)
        assert torch.equal(r64.float().cpu(), torch.from_numpy(cat["rew"][t])), t
    assert np.array_equal(nxt.cpu().numpy(), cat["last_obs"])
    # the single-process update on the concatenated rollout
    for k in ("obs", "bits", "act", "logp", "rew", "done", "last_obs"):
        getattr(tr, k).copy_(torch.from_numpy(cat[k]).to(DEV))
    g1 = _first_step_grads(ag)
    st = tr.update()
    assert st["minibatches"] == res[0]["n_mb"] == res[1]["n_mb"]
    assert st["kl_breaks"] == res[0]["n_kl"] == res[1]["n_kl"]
    # the first step's gradient: the sharded loss + one all-reduce = the global one
    assert np.array_equal(res[0]["g1"], res[1]["g1"])
    g_rel = np.linalg.norm(res[0]["g1"] - g1["g"]) / np.linalg.norm(g1["g"])
    worst = moved = num = den = 0.0
    for k, v in ag.model.state_dict().items():
        ref = v.cpu().numpy()
        assert np.array_equal(res[0]["params"][k], res[1]["params"][k]), k  # ranks identical
        d = res[0]["params"][k].astype(np.float64) - ref
        c = ref.astype(np.float64) - res[0]["p0"][k]
        worst = max(worst, float(np.abs(d).max()))
        moved = max(moved, float(np.abs(c).max()))
        num += float((d * d).sum())
        den += float((c * c).sum())
    rel = (num / den) ** 0.5
    print(f"2-rank DP vs 1 process: first-step gradient rel L2 {g_rel:.2e}; parameters after "
          f"16 AdamW steps: rel L2 of the change {rel:.2e}, max |diff| {worst:.2e}, "
          f"max |change| {moved:.2e}")
    assert moved > 1e-4
    # f32 summation order only (two 3 200-row shards + a sum vs one 6 400-row
    # GEMM / reduction): the gradient agrees to f32 rounding; AdamW divides
    # every element by its own RMS, so elements whose gradient is a near-
    # cancelling sum carry that rounding into full-size steps (measured max
    # |diff| 1.2e-5 against a 7e-4 change on the first run of this test)
    assert g_rel <= 3e-5, g_rel
    assert rel <= 1e-3, rel
    assert worst <= 5e-5, worst
    env.close()


# ---------------------------------------------------------------------------
# BASELINE config 4 at one GPU's full share: 32 768 envs
# over 8 MI355X is 4 096 envs per GPU; here two gloo ranks of 2 048 envs each
# share cuda:0 (config/100.yml, hidden 512, batch 100 / minibatch 25, 4 epochs).
N_SHARE, SHARE_WORLD = 2048, 2
TRACE_POS = 1 << 16  # gradient positions compared step by step


def _flat_params(m):
    return torch.cat([p.detach().flatten() for p in m.parameters()])


def _install_dp_trace(ag, idx, out, force=None):
    """Wrap the optimizer step: before each step record the (all-reduced,
    clipped) flat gradient at `idx`; after it the full parameter vector
    (`out["p"]`). With `force` (a list of full parameter vectors) the step is
    replaced by loading force[k] instead, so every minibatch of this run is
    evaluated at exactly the parameters the other run had there (teacher
    forcing: the gradients then compare at equal parameters at every step,
    free of AdamW's amplification of rounding in near-zero gradient elements)."""
    st = ag.optimizer.step
    params = list(ag.model.parameters())

    def step(*a, **k):
        g = torch.cat([p.grad.flatten() for p in params]).double()[idx].cpu().numpy()
        out.setdefault("g", []).append(g)
        if force is None:
            r = st(*a, **k)
            out.setdefault("p", []).append(_flat_params(ag.model).cpu().numpy())
            return r
        src = torch.from_numpy(force[len(out["g"]) - 1]).to(params[0].device)
        with torch.no_grad():
            o = 0
            for p in params:
                p.copy_(src[o:o + p.numel()].view_as(p))
                o += p.numel()
        return None
    ag.optimizer.step = step


def _share_worker(rank, world, port, tmp, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        env, ag = _agent(N_SHARE)
        p0 = _flat_params(ag.model)
        idx = torch.randperm(p0.numel(), generator=torch.Generator().manual_seed(11))[
            :TRACE_POS].to(p0.device)
        tr = ag.trainer()
        tr.collect()
        np.savez(os.path.join(tmp, f"roll{rank}.npz"),
                 counters=env.counters().cpu().numpy(),
                 **{k: getattr(tr, k).cpu().numpy() for k in BUFS})
        trace = {}
        _install_dp_trace(ag, idx, trace)
        st = tr.update()
        np.savez(os.path.join(tmp, f"res{rank}.npz"), p0_full=p0.cpu().numpy(),
                 p1_full=_flat_params(ag.model).cpu().numpy(), g=np.stack(trace["g"]),
                 p_steps=np.stack(trace["p"]) if rank == 0 else np.zeros(1, np.float32),
                 idx=idx.cpu().numpy())
        q.put((rank, int(ag.model.rng.seed), st["minibatches"], st["kl_breaks"]))
        env.close()
    finally:
        dist.destroy_process_group()


def test_config4_full_share_two_ranks_vs_oracle_and_one_process(tmp_path):
    """Two ranks x 2 048 envs (one GPU's share of config 4) on the HIP path:
      - 2 sampled envs of EACH rank replayed through the C oracle: masks,
        observations, f32 rewards and counters bit-exact;
      - every sampled action of both ranks valid under its mask;
      - ranks' parameters bit-identical before and after the update (and
        every step's all-reduced gradient identical on both ranks);
      - every AdamW step's all-reduced gradient within 3e-5 relative L2 of ONE
        process holding all 4 096 envs and the concatenated rollout, that
        process evaluated at the data-parallel run's parameters before every
        step (teacher forcing; 65 536 fixed positions)."""
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    from oracle import oracle as O
    from tests.torch_ref import unpack_bits
    from vmp.ppo import PPOTrainer
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    tmp = str(tmp_path)
    procs = [ctx.Process(target=_share_worker, args=(r, SHARE_WORLD, port, tmp, q))
             for r in range(SHARE_WORLD)]
    for p in procs:
        p.start()
    meta = {}
    for _ in procs:
        r, seed, n_mb, n_kl = q.get(timeout=400)
        meta[r] = (seed, n_mb, n_kl)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert meta[0][0] != meta[1][0]  # rank-folded sampling streams
    roll = [dict(np.load(os.path.join(tmp, f"roll{r}.npz"))) for r in range(SHARE_WORLD)]
    res = [dict(np.load(os.path.join(tmp, f"res{r}.npz"))) for r in range(SHARE_WORLD)]
    assert np.array_equal(res[0]["p0_full"], res[1]["p0_full"])
    assert np.array_equal(res[0]["p1_full"], res[1]["p1_full"])  # ranks identical after 16 steps
    assert np.array_equal(res[0]["g"], res[1]["g"])  # every step's all-reduced gradient
    V, A, T = 300, 102, roll[0]["rew"].shape[0]
    # every sampled action is valid
    for r in range(SHARE_WORLD):
        bits = torch.from_numpy(roll[r]["bits"]).to(DEV)
        act = torch.from_numpy(roll[r]["act"]).to(DEV).long()
        for t in range(T):
            full = unpack_bits(bits[t], A)
            assert not full.gather(-1, act[t][..., None]).any(), (r, t)
    # 2 envs of each rank through the C oracle (global index r * 2048 + i, seed 4 * gi)
    for r in range(SHARE_WORLD):
        for i in (0, N_SHARE - 1 - 17 * r):
            gi = r * N_SHARE + i
            e = O.OracleEnv(dict(CFG100, seed=4 * gi))
            e.eval(False)
            e.reset(4 * gi)
            full = unpack_bits(torch.from_numpy(roll[r]["bits"][:, i]), A).numpy()
            for t in range(T):
                assert np.array_equal(e.obs(), roll[r]["obs"][t, i]), (r, i, t)
                assert np.array_equal(e.mask(), full[t]), (r, i, t)
                o, rew, _, _ = e.step(roll[r]["act"][t, i].astype(np.int64))
                assert np.float32(rew) == roll[r]["rew"][t, i], (r, i, t)
            assert np.array_equal(o, roll[r]["last_obs"][i]), (r, i)
            assert np.array_equal(e.counters()[0], roll[r]["counters"][i]), (r, i)
    # one process holding all 4 096 envs, the concatenated rollout
    n_glob = SHARE_WORLD * N_SHARE
    env, ag = _agent(n_glob)
    assert np.array_equal(_flat_params(ag.model).cpu().numpy(), res[0]["p0_full"])
    tr = PPOTrainer(ag, distributed=False)
    for k in BUFS:
        cat = np.concatenate([roll[r][k] for r in range(SHARE_WORLD)],
                             axis=0 if k == "last_obs" else 1)
        getattr(tr, k).copy_(torch.from_numpy(cat).to(DEV))
        del cat
    del roll
    idx = torch.from_numpy(res[0]["idx"]).to(DEV)
    trace = {}
    _install_dp_trace(ag, idx, trace, force=res[0]["p_steps"])
    st = tr.update()
    env.close()
    assert st["minibatches"] == meta[0][1] and st["kl_breaks"] == meta[0][2]
    ours, ref = res[0]["g"], np.stack(trace["g"])
    assert ours.shape == ref.shape and len(ref) == st["minibatches"]
    rel = [float(np.linalg.norm(ours[k] - ref[k]) / np.linalg.norm(ref[k])) for k in range(len(ref))]
    moved = float(np.abs(res[0]["p1_full"].astype(np.float64) - res[0]["p0_full"]).max())
    print(f"config 4 at 2 x 2048 envs: all-reduced gradient vs one process at equal parameters, "
          f"rel L2 per step: first {rel[0]:.2e}, max {max(rel):.2e} over {len(rel)} AdamW steps; "
          f"max |parameter change| {moved:.2e}")
    assert moved > 1e-4
    assert max(rel) <= 3e-5, rel


def _bf16_share_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vmp.batched import BatchedVmEnv
        from vmp.config import Config
        from vmp.ppo import PPOAgent, PPOConfig
        torch.manual_seed(0)
        env = BatchedVmEnv(Config(**CFG100), N_SHARE, device=DEV)
        ag = PPOAgent(env, PPOConfig(**PCFG, precision="bf16"))
        assert ag.model.bf16_fused()
        tr = ag.trainer()
        tr.collect()
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        st = tr.update()
        torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated() - base
        total = torch.cuda.get_device_properties(0).total_memory
        q.put((rank, tr._device_sharers(tr.dev), tr._dl_budget, tr._budget, peak, total,
               st["minibatches"], _flat_params(ag.model).cpu().numpy()))
        env.close()
    finally:
        dist.destroy_process_group()


def test_bf16_update_two_ranks_one_gpu_budgets_dlogits():
    """VERDICT r5 item 7 / ADVICE r5: the fused bf16 head's dlogits chunk is
    budgeted from free HBM and the ranks sharing the device (not a fixed
    16 GiB): two gloo ranks x 2 048 config/100.yml envs on cuda:0 each run a
    bf16 update without running out of memory, detect their co-tenant, keep
    their dlogits budget within half the device split between them and the
    activation budget within an eighth split likewise, and end bit-identical."""
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bf16_share_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, *rest = q.get(timeout=300)
        res[r] = rest
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        sharers, dl, act_budget, peak, total, n_mb, _ = res[r]
        assert sharers == 2, sharers
        assert (1 << 26) <= dl <= min(1 << 34, total // 4), dl
        assert act_budget <= total // 16, act_budget
        assert n_mb >= 1
        # the update's own peak stays inside the two budgets it was given
        # (+ parameters, AdamW state and look-ahead copies: < 1 GB here)
        assert peak <= dl + act_budget + (1 << 30), (peak, dl, act_budget)
        print(f"rank {r}: dlogits budget {dl / 2**30:.2f} GiB, activation budget "
              f"{act_budget / 2**30:.2f} GiB, update peak {peak / 2**30:.2f} GiB")
    assert res[0][0:3] == res[1][0:3]  # budgets min-reduced: every rank chunks alike
    assert np.array_equal(res[0][6], res[1][6])
