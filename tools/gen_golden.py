"""Generate golden fixtures from the UNMODIFIED reference (container only).

Run:  python tools/gen_golden.py          (re-execs itself once with the env
      below; the reference never ships, only the .npz/.json it writes do)

Environment (set by the launcher below):
  PYTHONPATH=tools/oracle_stubs:/root/reference   gymnasium/tensorboard/cvxpy stubs
  NPY_DISABLE_CPU_FEATURES=...                    scalar argsort + scalar log, the
                                                  numpy build that produced the
                                                  published BestFit data
Outputs (tests/golden/):
  rng_kat.npz              numpy SeedSequence/PCG64/uniform/around/poisson KATs
  traj_<name>.npz          lock-step trajectories (sparse actions in, per-step
                           rewards/counters/state hashes out) for wr/ut/kl
  ppo10_wr_weights.npz     weights-10/ppo-wr.pt state dict (prefix stripped)
  ppo10_fwd.npz            reference Network outputs on recorded observations
  ppo_update.npz           one reference PPOAgent.update() on a fixed batch
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
SCALAR = ("AVX512F AVX512CD AVX512_SKX AVX512_CLX AVX512_CNL AVX512_ICL "
          "AVX2 FMA3 F16C AVX")

if os.environ.get("VMP_GEN_CHILD") != "1":
    env = dict(os.environ)
    env.update(VMP_GEN_CHILD="1", PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg",
               NPY_DISABLE_CPU_FEATURES=SCALAR, OMP_NUM_THREADS="1",
               PYTHONPATH=os.path.join(HERE, "oracle_stubs") + ":" + REF)
    sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                             env=env, cwd=REF))

import oracle_boot  # noqa: E402,F401  (tensorboard stub)
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.compile = lambda m, *a, **k: m  # eager == compiled outputs

import gymnasium as gym  # noqa: E402
import vmenv  # noqa: E402,F401
from vmenv.envs.config import Config  # noqa: E402
from src.agents.firstfit import FirstFitAgent  # noqa: E402
from src.agents.bestfit import BestFitAgent  # noqa: E402

sys.path.insert(0, REPO)
from tests.golden_hash import state_hash, obs_hash  # noqa: E402

os.makedirs(OUT, exist_ok=True)


def u128_split(x):
    return [(x >> 64) & 0xFFFFFFFFFFFFFFFF, x & 0xFFFFFFFFFFFFFFFF]


def gen_rng_kat():
    seeds = [0, 1, 2, 3, 5, 42, 1234567, 2**32 - 1, 2**32, 2**32 + 5, 2**40 + 7, 2**63 - 1]
    lams = [0.0182, 0.182, 1.8182, 9.9, 10.0, 100.0, 1000.0, 4100.0]
    st, raw, dbl, around, pois, after = [], [], [], [], [], []
    for s in seeds:
        g = np.random.default_rng(s)
        d = g.bit_generator.state["state"]
        st.append(u128_split(d["state"]) + u128_split(d["inc"]))
        raw.append(g.bit_generator.random_raw(8))
        g = np.random.default_rng(s)
        dbl.append(g.random(8))
        g = np.random.default_rng(s)
        around.append(np.around(g.uniform(0.1, 1, 16), 2))
        prow, arow = [], []
        for lam in lams:
            g = np.random.default_rng(s)
            prow.append(g.poisson(lam, size=40))
            arow.append(g.bit_generator.random_raw())
        pois.append(prow)
        after.append(arow)
    np.savez_compressed(os.path.join(OUT, "rng_kat.npz"),
                        seeds=np.array(seeds, dtype=np.uint64),
                        lams=np.array(lams), state_inc=np.array(st, dtype=np.uint64),
                        raw=np.array(raw, dtype=np.uint64), dbl=np.array(dbl),
                        around=np.array(around), poisson=np.array(pois, dtype=np.int64),
                        raw_after=np.array(after, dtype=np.uint64))


def make_env(cfg, reward):
    c = dict(cfg)
    c["reward_function"] = reward
    return gym.make("VmEnv-v1", config=Config(**c))


def run_traj(name, cfg, policy, T, p_susp=0.0, p_rand=0.0, eval_mode=True,
             reset_none_at=None, mask_steps=(), pert_seed=1234, rewards=("wr", "ut", "kl"),
             record_rank=False):
    """Step one reference env per reward function in lock-step on the same action
    stream (the state evolution does not depend on the reward, env.py:108-156)."""
    envs = [make_env(cfg, r) for r in rewards]
    for e in envs:
        if eval_mode:
            e.eval()
        e.reset(seed=cfg["seed"])
    e0 = envs[0]
    agent = (FirstFitAgent if policy == "ff" else BestFitAgent)(e0)
    prng = np.random.default_rng(pert_seed)
    P, V = cfg["pms"], cfg["vms"]
    A = e0.action_dim
    obs = e0._get_obs()
    a_step, a_vm, a_tgt, a_valid = [], [], [], []
    rew = np.zeros((len(rewards), T))
    ctr = np.zeros((T, 6), dtype=np.int64)
    misc = np.zeros((T, 5))  # waiting_ratio, tcm, tmm, total_cpu_req, total_mem_req
    shash = np.zeros(T, dtype=np.uint64)
    ohash = np.zeros(T, dtype=np.uint64)
    done = np.zeros(T, dtype=np.uint8)
    rank = np.zeros(T, dtype=np.int64)
    masks, mask_at = [], []
    for t in range(T):
        if reset_none_at is not None and t == reset_none_at:
            for e in envs:
                e.reset()  # seed=None: streams continue (env.py:181-182)
            obs = e0._get_obs()
        if t in mask_steps:
            masks.append(np.packbits(e0.get_invalid_action_mask(True)))
            mask_at.append(t)
        act = np.asarray(agent.act(obs)).astype(np.int64)
        pl = e0.vm_placement.copy()
        if p_susp > 0:
            run = np.flatnonzero((pl < P) & (prng.random(V) < p_susp))
            act[run] = P
        if p_rand > 0:
            sel = np.flatnonzero(prng.random(V) < p_rand)
            act[sel] = prng.integers(0, A, size=sel.size)
        outs = [e.step(act.copy()) for e in envs]
        obs, _, d0, _, info = outs[0]
        for e in envs[1:]:
            assert np.array_equal(e.vm_placement, e0.vm_placement)
        valid = np.asarray(info["valid"])
        nz = np.flatnonzero(act != pl)
        assert np.all(valid[act == pl] == 1)  # stays are always valid (env.py:36-37)
        a_step.extend([t] * nz.size)
        a_vm.extend(nz.tolist())
        a_tgt.extend(act[nz].tolist())
        a_valid.extend(valid[nz].tolist())
        for k in range(len(rewards)):
            rew[k, t] = outs[k][1]
        ctr[t] = [e0.total_requests, e0.served_requests, e0.suspend_action,
                  e0.place_action, e0.dropped_requests, e0.timestep]
        misc[t] = [e0.waiting_ratio, e0.target_cpu_mean, e0.target_memory_mean,
                   e0.total_cpu_requested, e0.total_memory_requested]
        shash[t] = state_hash(e0.vm_placement, e0.vm_cpu, e0.vm_memory, e0.cpu,
                              e0.memory, e0.vm_remaining_runtime)
        ohash[t] = obs_hash(obs)
        done[t] = int(d0)
        if record_rank:
            rank[t] = e0._get_rank()
    out = dict(
        config=json.dumps(cfg), policy=policy, eval_mode=int(eval_mode), T=T,
        reset_none_at=-1 if reset_none_at is None else reset_none_at,
        rewards=json.dumps(list(rewards)),
        act_step=np.array(a_step, dtype=np.int32), act_vm=np.array(a_vm, dtype=np.int32),
        act_tgt=np.array(a_tgt, dtype=np.int32), act_valid=np.array(a_valid, dtype=np.uint8),
        reward=rew, counters=ctr, misc=misc, state_hash=shash, obs_hash=ohash, done=done,
        mask_at=np.array(mask_at, dtype=np.int32),
        masks=np.array(masks, dtype=np.uint8) if masks else np.zeros((0, 0), np.uint8),
        final_placement=e0.vm_placement.astype(np.int64), final_cpu=e0.cpu.copy(),
        final_mem=e0.memory.copy(), final_vm_cpu=e0.vm_cpu.copy(),
        final_vm_mem=e0.vm_memory.copy(), final_remaining=e0.vm_remaining_runtime.astype(np.int64),
    )
    if record_rank:
        out["rank"] = rank
    np.savez_compressed(os.path.join(OUT, "traj_%s.npz" % name), **out)
    print("traj", name, "T", T, "actions", len(a_step), "sum", rew.sum(axis=1), "ctr", ctr[-1])
    return e0


BASE = dict(arrival_rate=0.182, service_length=100, pms=10, vms=30, training_steps=10000,
            eval_steps=100000, seed=1, reward_function="wr", sequence="uniform",
            cap_target_util=True, beta=0.5, allow_null_action=True)


def cfg(**kw):
    c = dict(BASE)
    c.update(kw)
    return c


def gen_trajs():
    run_traj("p10_ff", cfg(eval_steps=800), "ff", 800, p_susp=0.02, p_rand=0.02,
             mask_steps=(0, 100, 400, 799), record_rank=True)
    run_traj("p10_bf", cfg(seed=7, arrival_rate=0.3, service_length=60, eval_steps=600), "bf",
             600, p_susp=0.01, p_rand=0.01, mask_steps=(50, 300))
    run_traj("p100_ff", cfg(pms=100, vms=300, arrival_rate=0.909, service_length=200, seed=0,
                            eval_steps=500), "ff", 500, p_susp=0.005, p_rand=0.003,
             mask_steps=(499,))
    run_traj("p100_bf", cfg(pms=100, vms=300, arrival_rate=1.8182, service_length=100, seed=3,
                            eval_steps=400), "bf", 400, p_susp=0.003, p_rand=0.002,
             mask_steps=(399,))
    run_traj("p100v1000_ff", cfg(pms=100, vms=1000, arrival_rate=1.8182, service_length=300,
                                 seed=11, eval_steps=300), "ff", 300, p_susp=0.002,
             p_rand=0.001)
    run_traj("p10_drop_low", cfg(arrival_rate=1.8, service_length=50, seed=2,
                                 sequence="lowuniform", eval_steps=300), "ff", 300,
             p_susp=0.01, p_rand=0.01, mask_steps=(299,))
    # A = P+1, training-mode termination, reset(seed=None) stream continuation
    run_traj("p10_high_train", cfg(arrival_rate=0.5, service_length=30, seed=5,
                                   sequence="highuniform", allow_null_action=False,
                                   cap_target_util=False, beta=0.3, training_steps=200,
                                   eval_steps=100), "ff", 300, p_susp=0.02, p_rand=0.03,
             eval_mode=False, reset_none_at=150, mask_steps=(10, 290))
    # BASELINE config 1: config/10.yml, firstfit, 1 env, eval_steps=1000, seed 1
    c1 = cfg(arrival_rate=0.0182, service_length=1000, eval_steps=1000, training_steps=10000)
    run_traj("c1_10yml_ff", c1, "ff", 1000)
    # unperturbed heuristic streams: every sparse action IS the heuristic's proposal
    run_traj("p100_ffpure", cfg(pms=100, vms=300, arrival_rate=1.8182, service_length=150,
                                seed=21, eval_steps=400), "ff", 400)
    run_traj("p100_bfpure", cfg(pms=100, vms=300, arrival_rate=1.8182, service_length=150,
                                seed=22, eval_steps=400), "bf", 400)
    run_traj("p20_bfpure", cfg(pms=20, vms=60, arrival_rate=0.9, service_length=40,
                               seed=23, eval_steps=400), "bf", 400)


def load_ref_weights():
    sd = torch.load(os.path.join(REF, "weights-10", "ppo-wr.pt"), map_location="cpu",
                    weights_only=True)
    return {k.replace("_orig_mod.", ""): v for k, v in sd.items()}


def gen_ppo():
    from src.agents.ppo import Network, PPOAgent, PPOConfig
    sd = load_ref_weights()
    np.savez_compressed(os.path.join(OUT, "ppo10_wr_weights.npz"),
                        **{k: v.numpy() for k, v in sd.items()})
    c = cfg(arrival_rate=0.182, service_length=100, eval_steps=200)
    env = make_env(c, "wr")
    env.eval()
    env.reset(seed=c["seed"])
    net = Network(env.observation_space.shape[0], env.action_space, 512, torch.float32)
    net.load_state_dict(sd)
    ff = FirstFitAgent(env)
    obs_l, mask_l = [], []
    obs = env._get_obs()
    for t in range(200):
        if t % 12 == 5:
            obs_l.append(obs.copy())
            mask_l.append(env.get_invalid_action_mask(True))
        obs, *_ = env.step(ff.act(obs))
    obs_b = torch.tensor(np.array(obs_l))
    mask_b = torch.tensor(np.array(mask_l))
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        logits = net.actor(obs_b)
        value = net.critic(obs_b)
        det = torch.stack([net.get_det_action(o[None]) for o in obs_b])
        # given actions: random valid ones drawn from the mask
        acts = []
        for m in mask_l:
            row = []
            for v in range(m.shape[0]):
                ok = np.flatnonzero(~m[v])
                row.append(ok[torch.randint(len(ok), (1,), generator=g).item()] if len(ok) else 0)
            acts.append(row)
        acts = torch.tensor(acts)
        _, lp, ent = net.get_action(obs_b, action=acts, invalid_mask=mask_b.clone())
        _, lp_u, ent_u = net.get_action(obs_b, action=acts)
    np.savez_compressed(os.path.join(OUT, "ppo10_fwd.npz"), obs=obs_b.numpy(),
                        mask=mask_b.numpy(), logits=logits.numpy(), value=value.numpy(),
                        det=det.numpy(), action=acts.numpy(), logprob=lp.numpy(),
                        entropy=ent.numpy(), logprob_nomask=lp_u.numpy(),
                        entropy_nomask=ent_u.numpy())
    print("ppo fwd", logits.shape, lp[:3])

    # one reference update() on a fixed batch at hidden 64
    torch.manual_seed(0)
    np.random.seed(0)
    env = make_env(cfg(eval_steps=200), "wr")
    agent = PPOAgent(env, PPOConfig(hidden_size=64, episodes=1, training_progress_bar=False))
    model = agent.model
    before = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    B = agent.config.batch_size
    V, A, D = env.config.vms, env.action_dim, agent.obs_dim
    masks = torch.zeros((B, V, A), dtype=bool)
    acts = torch.zeros((B, V), dtype=int)
    obs_b = torch.zeros(B, D)
    nobs_b = torch.zeros(B, D)
    lp_b = torch.zeros(B)
    r_b = torch.zeros(B)
    d_b = torch.zeros(B, dtype=int)
    obs, _ = env.reset(seed=3)
    obs = torch.tensor(obs)
    for i in range(B):
        m = torch.tensor(env.get_invalid_action_mask(True))
        with torch.no_grad():
            a, lp, _ = model.get_action(obs[None], invalid_mask=m)
        a = a.flatten()
        nobs, r, d, _, _ = env.step(a.numpy())
        nobs = torch.tensor(nobs)
        masks[i], acts[i], obs_b[i], nobs_b[i] = m, a, obs, nobs
        lp_b[i], r_b[i], d_b[i] = lp.item(), r, int(i == 60)  # one synthetic episode cut
        obs = nobs
    batch = dict(mask=masks.numpy(), action=acts.numpy(), obs=obs_b.numpy(),
                 next_obs=nobs_b.numpy(), logprob=lp_b.numpy(), reward=r_b.numpy(),
                 done=d_b.numpy())
    agent.update(masks, acts, obs_b, nobs_b, lp_b, r_b, d_b)
    after = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    out = {"b_" + k: v for k, v in batch.items()}
    out.update({"p0_" + k: v for k, v in before.items()})
    out.update({"p1_" + k: v for k, v in after.items()})
    np.savez_compressed(os.path.join(OUT, "ppo_update.npz"), **out)
    print("ppo update done; max |dp| =",
          max(float(np.abs(after[k] - before[k]).max()) for k in before))


def gen_ppo100():
    """One reference PPOAgent.update() at the config/100.yml shape (P100 / V300,
    A 102, D 1100; BASELINE config 3) on a 100-step batch the reference's own
    model sampled from its env, at hidden size 8 so the fixture stays small.
    Masks are stored bit-packed (np.packbits over the [V, A] rows)."""
    from src.agents.ppo import PPOAgent, PPOConfig
    torch.manual_seed(0)
    np.random.seed(0)
    c = dict(BASE, pms=100, vms=300, service_length=1000, arrival_rate=1.8182,
             training_steps=10000, eval_steps=100000, seed=0, reward_function="wr",
             cap_target_util=True, allow_null_action=True)
    env = make_env(c, "wr")
    agent = PPOAgent(env, PPOConfig(hidden_size=8, episodes=1, batch_size=100,
                                    minibatch_size=25, migration_ratio=0.002,
                                    training_progress_bar=False))
    model = agent.model
    before = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    B = agent.config.batch_size
    V, A, D = env.config.vms, env.action_dim, agent.obs_dim
    masks = torch.zeros((B, V, A), dtype=bool)
    acts = torch.zeros((B, V), dtype=int)
    obs_b, nobs_b = torch.zeros(B, D), torch.zeros(B, D)
    lp_b, r_b = torch.zeros(B), torch.zeros(B)
    d_b = torch.zeros(B, dtype=int)
    obs, _ = env.reset(seed=3)
    obs = torch.tensor(obs)
    for i in range(B):
        m = torch.tensor(env.get_invalid_action_mask(True))
        with torch.no_grad():
            a, lp, _ = model.get_action(obs[None], invalid_mask=m)
        a = a.flatten()
        nobs, r, d, _, _ = env.step(a.numpy())
        nobs = torch.tensor(nobs)
        masks[i], acts[i], obs_b[i], nobs_b[i] = m, a, obs, nobs
        lp_b[i], r_b[i], d_b[i] = lp.item(), r, int(i == 60)
        obs = nobs
    out = {"b_mask_bits": np.packbits(masks.numpy().reshape(B, -1), axis=1),
           "b_action": acts.numpy().astype(np.int16), "b_obs": obs_b.numpy(),
           "b_next_obs": nobs_b.numpy(), "b_logprob": lp_b.numpy(), "b_reward": r_b.numpy(),
           "b_done": d_b.numpy(), "shape": np.array([B, V, A, D])}
    # k_epochs = 2 (8 AdamW steps, every ratio stays inside the clip range) and
    # the config's 4 epochs (the reference breaks on KL in epoch 4): counted
    # head calls and optimizer steps record where its minibatch loop stopped
    args = (masks, acts, obs_b, nobs_b, lp_b, r_b, d_b)
    for tag, ke in (("e2_", 2), ("", 4)):
        model.load_state_dict({k: torch.tensor(v) for k, v in before.items()})
        agent.config.k_epochs = ke
        agent.optimizer = torch.optim.AdamW(model.parameters(), lr=agent.config.lr)
        n = {"head": 0, "step": 0}
        ga, st = model.get_action, agent.optimizer.step

        def get_action(*a, **k):
            n["head"] += 1
            return ga(*a, **k)

        def step(*a, **k):
            n["step"] += 1
            return st(*a, **k)
        model.get_action, agent.optimizer.step = get_action, step
        agent.update(*[x.clone() for x in args])
        model.get_action = ga
        after = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
        out.update({"p1_" + tag + k: v for k, v in after.items()})
        out[tag + "ref_calls"] = np.array([n["head"], n["step"]])
    out.update({"p0_" + k: v for k, v in before.items()})
    np.savez_compressed(os.path.join(OUT, "ppo100_update.npz"), **out)
    print("ppo100 update done; max |dp| =",
          max(float(np.abs(after[k] - before[k]).max()) for k in before))


def gen_ppo100_steps():
    """Per-step trace of the reference's 4-epoch update at the config/100.yml
    shape (same model, batch and seeds as gen_ppo100, whose fixture it reads):
    after every AdamW step, the flat parameter vector (state_dict keys sorted)
    at 8192 fixed random positions; for every minibatch the reference
    evaluates, its new log-probabilities and new values (ppo.py:258, 266),
    from which the test finds the first minibatch whose clip branches differ
    (ppo.py:267-280). Pins the update step by step where the final-parameter
    check (5 % after a clip-branch flip) cannot."""
    from src.agents.ppo import PPOAgent, PPOConfig
    d = np.load(os.path.join(OUT, "ppo100_update.npz"))
    B, V, A, D = (int(x) for x in d["shape"])
    torch.manual_seed(0)
    np.random.seed(0)
    c = dict(BASE, pms=100, vms=300, service_length=1000, arrival_rate=1.8182,
             training_steps=10000, eval_steps=100000, seed=0, reward_function="wr",
             cap_target_util=True, allow_null_action=True)
    env = make_env(c, "wr")
    agent = PPOAgent(env, PPOConfig(hidden_size=8, episodes=1, batch_size=100,
                                    minibatch_size=25, migration_ratio=0.002, k_epochs=4,
                                    training_progress_bar=False))
    model = agent.model
    model.load_state_dict({k[3:]: torch.tensor(d[k]) for k in d.files if k.startswith("p0_")})
    agent.optimizer = torch.optim.AdamW(model.parameters(), lr=agent.config.lr)
    keys = sorted(model.state_dict())
    n = sum(model.state_dict()[k].numel() for k in keys)
    idx = np.sort(np.random.default_rng(20261017).choice(n, 8192, replace=False))

    def flat():
        sd = model.state_dict()
        return torch.cat([sd[k].detach().flatten() for k in keys]).numpy()[idx].copy()
    trace = {"p": [flat()], "lp": [], "v": []}
    ga, gv, st = model.get_action, model.get_value, agent.optimizer.step

    def get_action(*a, **k):
        out = ga(*a, **k)
        trace["lp"].append(out[1].detach().numpy().copy())
        return out

    def get_value(*a, **k):
        out = gv(*a, **k)
        trace["v"].append(out.detach().numpy().reshape(-1).copy())
        return out

    def step(*a, **k):
        r = st(*a, **k)
        trace["p"].append(flat())
        return r
    model.get_action, model.get_value, agent.optimizer.step = get_action, get_value, step
    mask = np.unpackbits(d["b_mask_bits"], axis=1)[:, :V * A].reshape(B, V, A).astype(bool)
    agent.update(torch.tensor(mask), torch.tensor(d["b_action"].astype(np.int64)),
                 *[torch.tensor(d[k]) for k in ("b_obs", "b_next_obs", "b_logprob",
                                                "b_reward", "b_done")])
    # the two leading get_value calls are values / next_values (ppo.py:235-236)
    out = {"idx": idx.astype(np.int64), "p": np.stack(trace["p"]),
           "lp": np.stack(trace["lp"]), "v": np.stack(trace["v"][2:]),
           "values": trace["v"][0], "next_values": trace["v"][1]}
    np.savez_compressed(os.path.join(OUT, "ppo100_steps.npz"), **out)
    print("ppo100 steps done:", out["p"].shape, out["lp"].shape, out["v"].shape)


if __name__ == "__main__":
    what = sys.argv[1:] or ["rng", "traj", "ppo", "ppo100"]
    if "ppo100" in what:
        gen_ppo100()
    if "ppo100" in what or "ppo100_steps" in what:
        gen_ppo100_steps()
    if "rng" in what:
        gen_rng_kat()
    if "traj" in what:
        gen_trajs()
    if "ppo" in what:
        gen_ppo()
