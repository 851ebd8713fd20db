"""FirstFitAgent.act / BestFitAgent.act take the observation they are passed
(src/agents/firstfit.py:21-38, bestfit.py:21-40 read nothing else), on the
MI355X through vmp_heuristic_act_obs:

  - on the envs' own observations along a trajectory, the action equals the
    env-state path (vmp_heuristic_act, which Base.test's fused step uses and
    tests/test_gpu_env.py pins against the oracle);
  - on EDITED observations (sizes and loads that are not hundredths, stale
    placements, PMs set to tie on cpu + memory) it equals a literal
    restatement of firstfit.py / bestfit.py over the f32 obs, with numpy's
    scalar introsort argsort from the oracle (oracle_argsort_f32, pinned by
    the BestFit goldens), and differs from the env-state action;
  - the agents' act() follows the obs: VmEnv (N = 1) and BatchedVmEnv.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
CFGS = {
    "p100v1000": dict(pms=100, vms=1000, arrival_rate=1.8182, service_length=300,
                      training_steps=10000, eval_steps=100000, seed=0, reward_function="wr",
                      allow_null_action=True),
    "p10v30": dict(pms=10, vms=30, arrival_rate=0.6, service_length=40, training_steps=10000,
                   eval_steps=100000, seed=0, reward_function="kl", allow_null_action=True),
    "p200v600": dict(pms=200, vms=600, arrival_rate=3.0, service_length=150,
                     training_steps=10000, eval_steps=100000, seed=0, reward_function="ut",
                     allow_null_action=True),
}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")


def _argsort(v):
    v = np.ascontiguousarray(v, dtype=np.float32)
    out = np.zeros(v.size, np.int64)
    O.lib().oracle_argsort_f32(O._p(v), v.size, O._p(out))
    return out


def literal_act(obs, P, V, policy):
    """firstfit.py:21-38 / bestfit.py:21-40 over one f32 observation."""
    obs = np.asarray(obs, dtype=np.float32)
    placement = obs[:V].astype(np.int64)  # convert_obs_to_dict's astype(int), utils.py:41
    vm_cpu, vm_mem = obs[V:2 * V], obs[2 * V:3 * V]
    cpu, mem = obs[3 * V:3 * V + P].copy(), obs[3 * V + P:].copy()
    action = placement.copy()
    one = np.float32(1)
    for v in range(V):
        if placement[v] != P:
            continue
        order = range(P) if policy == "firstfit" else np.flip(_argsort(cpu + mem))
        for p in order:
            if cpu[p] + vm_cpu[v] <= one and mem[p] + vm_mem[v] <= one:
                action[v] = p
                cpu[p] += vm_cpu[v]
                if policy == "bestfit":
                    mem[p] += vm_mem[v]
                break
    return action


def _edit(obs, P, V, g, ties):
    """Perturb observations: PM loads and waiting sizes off the hundredths
    grid, some running / NULL slots turned WAIT, and (ties) groups of PMs set
    to equal cpu + memory so BestFit's visiting order decides."""
    o = obs.copy()
    N = o.shape[0]
    for i in range(N):
        pl = o[i, :V]
        pl[g.random(V) < 0.05] = P  # stale: running / NULL slots shown as waiting
        # off-integer placements: astype(int) truncates, so P + 0.4 waits and
        # p + 0.3 stays on PM p
        frac = g.random(V) < 0.05
        pl[frac] += np.float32(0.4)
        w = pl.astype(np.int64) == P
        o[i, V:2 * V][w] = g.uniform(0.05, 0.6, int(w.sum())).astype(np.float32)
        o[i, 2 * V:3 * V][w] = g.uniform(0.05, 0.6, int(w.sum())).astype(np.float32)
        cpu = o[i, 3 * V:3 * V + P]
        mem = o[i, 3 * V + P:]
        cpu[:] = np.clip(cpu + g.normal(0, 0.02, P).astype(np.float32), 0, 1)
        mem[:] = np.clip(mem + g.normal(0, 0.02, P).astype(np.float32), 0, 1)
        if ties:
            grp = g.choice(P, size=min(P, 24), replace=False)
            cpu[grp] = np.float32(0.25)
            mem[grp] = np.float32(0.25)
    return o


@pytest.mark.parametrize("name", list(CFGS))
@pytest.mark.parametrize("policy", ["firstfit", "bestfit"])
def test_act_obs_equals_state_path_on_own_obs(name, policy):
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    cfg = CFGS[name]
    N = 16
    env = BatchedVmEnv(Config(**cfg), N, seeds=np.arange(N) * 4, device=DEV)
    obs = env.obs()
    for t in range(120):
        a_obs = env.heuristic_act_obs(obs, policy)
        a_st = env.heuristic_act(policy)
        assert torch.equal(a_obs, a_st), (name, policy, t)
        obs, _, _, _ = env.step(a_st)
    env.close()


@pytest.mark.parametrize("name", list(CFGS))
@pytest.mark.parametrize("policy", ["firstfit", "bestfit"])
def test_act_obs_on_edited_obs_equals_literal_agent(name, policy):
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    cfg = CFGS[name]
    P, V, N = cfg["pms"], cfg["vms"], 6
    env = BatchedVmEnv(Config(**cfg), N, seeds=np.arange(N) * 4, device=DEV)
    env.rollout("firstfit", 200)
    g = np.random.default_rng(7)
    differs = 0
    for ties in (False, True):
        obs = _edit(env.obs().cpu().numpy(), P, V, g, ties)
        got = env.heuristic_act_obs(torch.from_numpy(obs).to(DEV), policy).cpu().numpy()
        st = env.heuristic_act(policy).cpu().numpy()
        for i in range(N):
            want = literal_act(obs[i], P, V, policy)
            assert np.array_equal(got[i], want), (name, policy, ties, i,
                                                  np.flatnonzero(got[i] != want)[:8])
            differs += int(not np.array_equal(got[i], st[i]))
    assert differs > 0, "the edits should change the action"
    env.close()


def test_act_obs_large_p():
    """P = 4000 / V = 1100 (the block kernel's env; k_act_obs keeps the PM view
    in up to 160 KB of LDS, 73 KB here): edited observations against the
    literal agents."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    P, V, N = 4000, 1100, 2
    cfg = dict(pms=P, vms=V, arrival_rate=20.0, service_length=30, training_steps=10000,
               eval_steps=100000, seed=0, reward_function="wr", allow_null_action=True)
    env = BatchedVmEnv(Config(**cfg), N, seeds=np.arange(N) * 4, device=DEV)
    env.rollout("firstfit", 40)
    g = np.random.default_rng(3)
    obs = _edit(env.obs().cpu().numpy(), P, V, g, True)
    for policy in ("firstfit", "bestfit"):
        got = env.heuristic_act_obs(torch.from_numpy(obs).to(DEV), policy).cpu().numpy()
        for i in range(N):
            assert np.array_equal(got[i], literal_act(obs[i], P, V, policy)), (policy, i)
    env.close()


def test_agents_act_follows_the_passed_obs():
    from vmp.agents import BestFitAgent, FirstFitAgent
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.env import VmEnv
    cfg = CFGS["p10v30"]
    P, V = cfg["pms"], cfg["vms"]
    env = VmEnv(Config(**cfg), device=DEV)
    obs, _ = env.reset(seed=3)
    g = np.random.default_rng(1)
    for Agent, pol in ((FirstFitAgent, "firstfit"), (BestFitAgent, "bestfit")):
        ag = Agent(env)
        for _ in range(30):
            edited = _edit(obs[None], P, V, g, True)[0]
            assert np.array_equal(ag.act(edited), literal_act(edited, P, V, pol))
            a = ag.act(obs)
            assert np.array_equal(a, literal_act(obs, P, V, pol))
            obs, _, _, _, _ = env.step(a)
    env.close()
    benv = BatchedVmEnv(Config(**cfg), 4, seeds=np.arange(4) * 4, device=DEV)
    benv.rollout("firstfit", 50)
    o = _edit(benv.obs().cpu().numpy(), P, V, g, True)
    a = BestFitAgent(benv).act(torch.from_numpy(o).to(DEV))
    for i in range(4):
        assert np.array_equal(a[i], literal_act(o[i], P, V, "bestfit"))
    benv.close()
