"""PPO path on the MI355X: the HIP actor head (vmp_policy_head / _backward)
against the reference Network's recorded outputs and a plain-PyTorch fp32
reference of the same op, sampling law and coin flips, one PPOAgent.update
against the reference's, and a batched rollout + update on the GPU env.
Tolerances: logits/logprob/entropy 1e-5 relative (fp32),
det actions and env integer state exact."""
import os

import numpy as np
import pytest
import torch

from tests.torch_ref import torch_head, unpack_bits

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CFG10 = dict(arrival_rate=0.182, service_length=100, pms=10, vms=30, training_steps=10000,
             eval_steps=200, seed=1, reward_function="wr", allow_null_action=True)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")


CFG100 = dict(pms=100, vms=300, service_length=1000, arrival_rate=1.8182, training_steps=10000,
              eval_steps=100000, seed=0, reward_function="wr", sequence="uniform",
              cap_target_util=True, beta=0.5, allow_null_action=True)


def _g(name):
    return np.load(os.path.join(GOLDEN, name))


def _net512():
    from vmp.ppo import Network
    w = _g("ppo10_wr_weights.npz")
    net = Network(110, np.full(30, 12), 512).to(DEV)
    net.load_state_dict({k: torch.tensor(w[k]) for k in w.files})
    return net


def test_network_outputs_match_reference():
    from vmp.head import pack_mask
    f = _g("ppo10_fwd.npz")
    net = _net512()
    obs = torch.tensor(f["obs"], device=DEV)
    with torch.no_grad():
        logits = net.actor(obs)
        torch.testing.assert_close(logits.cpu(), torch.tensor(f["logits"]), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(net.get_value(obs).cpu(), torch.tensor(f["value"]),
                                   rtol=1e-5, atol=1e-5)
        act = torch.tensor(f["action"], device=DEV)
        mask = torch.tensor(f["mask"], device=DEV)
        a, lp, ent = net.get_action(obs, action=act, invalid_mask=mask)
        assert torch.equal(a.cpu(), act.cpu())
        np.testing.assert_allclose(lp.cpu().numpy(), f["logprob"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ent.cpu().numpy(), f["entropy"], rtol=1e-5, atol=1e-5)
        # bit-packed mask input gives the same result as the bool layout
        _, lp2, ent2 = net.get_action(obs, action=act, invalid_mask=pack_mask(mask, 30, 12))
        assert torch.equal(lp, lp2) and torch.equal(ent, ent2)
        _, lp, ent = net.get_action(obs, action=act)
        np.testing.assert_allclose(lp.cpu().numpy(), f["logprob_nomask"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ent.cpu().numpy(), f["entropy_nomask"], rtol=1e-5, atol=1e-5)
        det = torch.stack([net.get_det_action(o[None]) for o in obs])
        assert np.array_equal(det.cpu().numpy(), f["det"])
        assert np.array_equal(net.get_det_action(obs).cpu().numpy(), f["det"])


def _rand_case(B, V, A, seed, p_mask=0.5, all_masked_rows=0):
    g = torch.Generator().manual_seed(seed)
    logits = (torch.randn((B, V * A), generator=g) * 3).to(DEV)
    mask = torch.rand((B, V, A), generator=g) < p_mask
    mask[..., A - 2] = False
    if all_masked_rows:
        mask[0, :all_masked_rows] = True
    act = torch.zeros((B, V), dtype=torch.int64)
    for b in range(B):
        for v in range(V):
            ok = torch.nonzero(~mask[b, v]).flatten()
            if len(ok) == 0:
                ok = torch.arange(A)
            act[b, v] = ok[torch.randint(len(ok), (1,), generator=g)]
    return logits, mask.to(DEV), act.to(DEV)


@pytest.mark.parametrize("V,A", [(30, 12), (300, 102), (7, 33), (3, 1002), (5, 64), (2, 65)])
def test_head_forward_backward_vs_torch(V, A):
    """logprob/entropy and d/dlogits of (w1*logprob + w2*entropy) against torch
    autograd through the reference's masked Categorical math."""
    from vmp.head import HeadRng, pack_mask, policy_head
    B = 6
    logits, mask, act = _rand_case(B, V, A, seed=V * 1000 + A, all_masked_rows=2)
    bits = pack_mask(mask, V, A)
    w1 = torch.randn(B, device=DEV)
    w2 = torch.randn(B, device=DEV)
    x1 = logits.clone().requires_grad_(True)
    _, lp, ent = policy_head(x1, V, A, bits=bits, action=act, rng=HeadRng(0))
    (w1 * lp + w2 * ent).sum().backward()
    x2 = logits.clone().requires_grad_(True)
    _, lp_r, ent_r = torch_head(x2, V, A, bits=bits, action=act)
    (w1 * lp_r + w2 * ent_r).sum().backward()
    torch.testing.assert_close(lp, lp_r, rtol=1e-5, atol=1e-4 * V)
    torch.testing.assert_close(ent, ent_r, rtol=1e-5, atol=1e-5 * V)
    torch.testing.assert_close(x1.grad, x2.grad, rtol=1e-4, atol=1e-5)
    assert torch.all(x1.grad.reshape(B, V, A)[mask] == 0)


def test_head_sampling_law_and_validity():
    """Sampled actions are never masked (unless a row is all masked) and follow
    softmax(masked logits): per-category frequencies within 5 sigma."""
    from vmp.head import HeadRng, pack_mask, policy_head
    V, A, B = 4, 12, 40000
    g = torch.Generator().manual_seed(7)
    row = torch.randn((V, A), generator=g)
    mask = torch.rand((V, A), generator=g) < 0.4
    mask[:, 10] = False
    logits = row.reshape(1, -1).repeat(B, 1).to(DEV)
    bits = pack_mask(mask.to(DEV).expand(B, V, A), V, A)
    rng = HeadRng(123)
    with torch.no_grad():
        act, lp, _ = policy_head(logits, V, A, bits=bits, rng=rng)
        act2, _, _ = policy_head(logits, V, A, bits=bits, rng=rng)
    act = act.cpu().long()
    assert not torch.equal(act, act2.cpu().long())  # the stream advances
    assert not mask.gather(1, act.T).any()
    p = torch.softmax(row.masked_fill(mask, -1e7), -1)
    for v in range(V):
        cnt = torch.bincount(act[:, v], minlength=A).double()
        sd = torch.sqrt(B * p[v] * (1 - p[v])).double() + 1e-9
        assert torch.all((cnt - B * p[v].double()).abs() <= 5 * sd + 1), v
    ref_lp = torch.log_softmax(row.masked_fill(mask, -1e7), -1).gather(1, act.T).sum(0)
    torch.testing.assert_close(lp.cpu(), ref_lp, rtol=1e-5, atol=1e-5)


def test_wait_coin_flips():
    """PPOAgent.act (ppo.py:154-156): rows with > 1 invalid entries and WAIT
    valid get WAIT forbidden with probability 1 - migration_ratio."""
    from vmp.head import HeadRng, pack_mask, policy_head
    V, A, B, P = 8, 12, 20000, 10
    mask = torch.ones((V, A), dtype=torch.bool)
    mask[:, P] = False
    mask[:4, 3] = False       # rows 0-3: {3, WAIT} valid -> qualify
    mask[4:6, :] = False      # rows 4-5: nothing invalid -> never flipped
    mask[6, P] = True
    mask[6, 5] = False        # row 6: WAIT already invalid
    mask[7, :] = True
    mask[7, P] = False        # row 7: only WAIT valid (count > 1) -> flip makes it all-masked
    logits = torch.zeros((B, V * A), device=DEV)
    logits.view(B, V, A)[:, :, P] = 5.0  # WAIT strongly preferred when allowed
    bits = pack_mask(mask.to(DEV).expand(B, V, A), V, A)
    with torch.no_grad():
        act, _, _ = policy_head(logits, V, A, bits=bits, rng=HeadRng(9), wait_ratio=0.3,
                                wait_index=P)
    act = act.cpu()
    for v in range(4):
        frac = (act[:, v] != P).double().mean().item()
        # P(WAIT forbidden) = 0.7 -> action 3; else WAIT wins with prob e^5/(e^5+1)
        expect = 0.7 + 0.3 * (1 / (1 + np.exp(5)))
        assert abs(frac - expect) < 0.02, (v, frac)
    assert (act[:, 6] == 5).all()
    allmasked = (act[:, 7] != P).double().mean().item()  # uniform over 12 when flipped
    assert abs(allmasked - 0.7 * 11 / 12) < 0.02
    with torch.no_grad():  # ratio 1.0: rand() > 1 never true
        act, _, _ = policy_head(logits, V, A, bits=bits, rng=HeadRng(9), wait_ratio=1.0,
                                wait_index=P)
    assert ((act.cpu()[:, :4] == P).double().mean() > 0.95)


def test_update_matches_reference_on_gpu():
    """One PPOAgent.update through the HIP head and GAE: params within 2e-6 of
    the reference's after 16 AdamW steps (the update moves them ~8e-4)."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    d = _g("ppo_update.npz")
    env = BatchedVmEnv(Config(**CFG10), 1, device=DEV)
    ag = PPOAgent(env, PPOConfig(hidden_size=64, episodes=1))
    ag.model.load_state_dict({k[3:]: torch.tensor(d[k]) for k in d.files if k.startswith("p0_")})
    st = ag.update(*[torch.tensor(d[k]) for k in ("b_mask", "b_action", "b_obs", "b_next_obs",
                                                    "b_logprob", "b_reward", "b_done")])
    assert st["minibatches"] == 16
    for k, v in ag.model.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), d["p1_" + k], rtol=0, atol=2e-6, err_msg=k)
    env.close()


def test_batched_rollout_and_update():
    """PPOTrainer on 64 GPU envs: the rollout buffers hold the env's own obs /
    masks, sampled actions are valid, and an update runs with finite stats."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    cfg = Config(**dict(CFG10, training_steps=30, arrival_rate=1.0, service_length=20))
    env = BatchedVmEnv(cfg, 64, device=DEV)
    ag = PPOAgent(env, PPOConfig(hidden_size=64, batch_size=40, minibatch_size=10))
    tr = ag.trainer()
    tr.collect()
    # buffer step 0 is the reset obs; every sampled action is valid under its mask
    m = unpack_bits(tr.bits.reshape(-1, 30, 1), 12).reshape(40, 64, 30, 12)
    taken = m.gather(-1, tr.act.long()[..., None]).squeeze(-1)
    assert not taken.any()
    assert tr.done[29].eq(1).all() and tr.done[:29].eq(0).all() and len(tr.ep_returns) == 1
    # obs[t+1] is what step t returned: re-derive the placements from obs and
    # compare with the actions that were valid (placement column = action where accepted)
    assert torch.isfinite(tr.rew).all() and torch.isfinite(tr.logp).all()
    p0 = {k: v.clone() for k, v in ag.model.state_dict().items()}
    st = tr.update()
    assert st["minibatches"] + st["kl_breaks"] >= 4
    assert any(not torch.equal(p0[k], v) for k, v in ag.model.state_dict().items())
    tr.collect()  # continues from last_obs across the episode boundary
    assert torch.isfinite(tr.logp).all()
    env.close()


def test_act_step_graph_equals_eager():
    """ActStepGraph (mask + actor + head + step as one HIP graph) replays the
    same computation as the eager calls with the counter-mode sampling stream:
    identical env state, rewards and obs after 30 steps; replays draw fresh
    actions (the counter advances). A graph of 3 steps replayed 10 times
    (ActStepGraph(steps=3), bench.py's eval leg form) gives the same state."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import ActStepGraph, PPOAgent, PPOConfig
    cfg = Config(**dict(CFG10, arrival_rate=1.0, service_length=15, eval_steps=1000))
    outs = []
    for graphed in (1, 3, 0):
        torch.manual_seed(0)
        env = BatchedVmEnv(cfg, 256, device=DEV)
        env.eval(True)
        ag = PPOAgent(env, PPOConfig(hidden_size=64, masked=True, migration_ratio=0.5))
        ag.model.rng.seed = 1234
        ag.eval(True)
        if graphed:
            g = ActStepGraph(ag, warmup=0, steps=graphed)
            c0 = int(ag.model.rng.counter[0])
            for _ in range(30 // graphed):
                obs, rew, done = g.replay()
            # the one-launch actor advances the counter itself and re-arms its ticket
            assert int(ag.model.rng.counter[0]) == c0 + 30 and int(ag.model.rng.counter[1]) == 0
        else:
            ag.model.rng.graph_counter(env.device)
            obs = env.obs()
            bits = torch.empty((256, env.V, env.W), dtype=torch.int32, device=DEV)
            rew = torch.empty(256, dtype=torch.float64, device=DEV)
            done = torch.empty(256, dtype=torch.uint8, device=DEV)
            for _ in range(30):  # capture records without running: 30 replays = 30 steps
                env.mask_bits(out=bits)
                a = ag.act_batch(obs, bits)
                env.step(a, obs=obs, reward=rew, done=done, want_valid=False)
        st = env.state()
        outs.append((obs.clone(), rew.clone(), st["vm_placement"].clone(), env.counters().clone()))
        env.close()
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert torch.equal(x, y)


def test_bf16_linear_forward_backward():
    """BF16Linear (precision="bf16"): forward and all three gradients equal the
    f32 math on bf16-rounded operands (f32 accumulation), and stay within bf16
    rounding of the f32 layer."""
    from vmp.ppo import BF16Linear
    g = torch.Generator().manual_seed(0)
    x = torch.randn(300, 110, generator=g).to(DEV).requires_grad_(True)
    w = (torch.randn(512, 110, generator=g) * 0.1).to(DEV).requires_grad_(True)
    b = torch.randn(512, generator=g).to(DEV).requires_grad_(True)
    gy = torch.randn(300, 512, generator=g).to(DEV)
    y = BF16Linear.apply(x, w, b)
    y.backward(gy)
    xr, wr = x.detach().bfloat16().float(), w.detach().bfloat16().float()
    gr = gy.bfloat16().float()
    torch.testing.assert_close(y, xr @ wr.t() + b, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(x.grad, gr @ wr, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(w.grad, gr.t() @ xr, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(b.grad, gy.sum(0))
    yf = x.detach() @ w.detach().t() + b.detach()
    assert (y - yf).abs().max() < 0.05 * yf.abs().max()


def test_bf16_training_runs_and_logprobs_are_consistent():
    """precision="bf16": the update's first-epoch log-probabilities reproduce the
    rollout's (ratio ~ 1, no KL break) and training moves the parameters."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    cfg = Config(**dict(CFG10, training_steps=1000, arrival_rate=1.0, service_length=20))
    env = BatchedVmEnv(cfg, 128, device=DEV)
    ag = PPOAgent(env, PPOConfig(hidden_size=128, batch_size=40, minibatch_size=10,
                                 precision="bf16"))
    tr = ag.trainer()
    tr.collect()
    with torch.no_grad():
        T, N = tr.T, tr.N
        _, lp, _ = ag.model._head(ag.model.actor_logits(tr.obs.reshape(T * N, -1)), tr.V, tr.A,
                                  bits=tr.bits.reshape(T * N, tr.V, -1),
                                  action=tr.act.reshape(T * N, tr.V), rng=ag.model.rng)
    assert (lp.reshape(T, N) - tr.logp).abs().max() < 1e-3
    p0 = {k: v.clone() for k, v in ag.model.state_dict().items()}
    st = tr.update()
    assert st["kl_breaks"] == 0 and st["minibatches"] == 16
    assert any(not torch.equal(p0[k], v) for k, v in ag.model.state_dict().items())
    env.close()


@pytest.mark.parametrize("V,A", [(30, 12), (300, 102)])
def test_bf16_actor_head_node_equals_linear_plus_head(V, A):
    """BF16ActorHead (the bf16 leg's last Linear + head as one node, bf16 dlogits
    from vmp_policy_head_backward_bf16) against BF16Linear followed by the HIP
    head: logprob / entropy and dh, dW equal (the same bf16 rounding of the same
    f32 dlogits); the bias gradient sums bf16-rounded dlogits, so it agrees to
    bf16 rounding of the f32 sum."""
    from vmp.head import pack_mask, policy_head
    from vmp.ppo import BF16ActorHead, BF16Linear
    g = torch.Generator().manual_seed(V + A)
    B, K = 96, 64
    x = torch.randn(B, K, generator=g).to(DEV)
    w = (torch.randn(V * A, K, generator=g) * 0.1).to(DEV)
    b = (torch.randn(V * A, generator=g) * 0.1).to(DEV)
    mask = torch.rand((B, V, A), generator=g) < 0.4
    mask[..., A - 2] = False
    mask[0, 0] = True  # an all-masked row
    bits = pack_mask(mask.to(DEV), V, A)
    act = torch.randint(0, A - 2, (B, V), generator=g).to(DEV)
    glp, gen = torch.randn(B, generator=g).to(DEV), torch.randn(B, generator=g).to(DEV)
    outs = []
    for fused in (True, False):
        xi, wi, bi = (t.clone().requires_grad_(True) for t in (x, w, b))
        if fused:
            lp, ent = BF16ActorHead.apply(xi, wi, bi, bits, act, V, A)
        else:
            _, lp, ent = policy_head(BF16Linear.apply(xi, wi, bi), V, A, bits=bits, action=act)
        (lp * glp + ent * gen).sum().backward()
        outs.append((lp.detach(), ent.detach(), xi.grad, wi.grad, bi.grad))
    (lp1, e1, gx1, gw1, gb1), (lp2, e2, gx2, gw2, gb2) = outs
    torch.testing.assert_close(lp1, lp2, rtol=1e-5, atol=1e-5 * V)
    torch.testing.assert_close(e1, e2, rtol=1e-5, atol=1e-5 * V)
    torch.testing.assert_close(gx1, gx2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gw1, gw2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gb1, gb2, rtol=1e-2, atol=1e-2 * gb2.abs().max().item())


def test_bf16_graph_reads_the_live_parameters():
    """a captured ActStepGraph in bf16 precision must act with the
    parameters of the moment it is replayed. The bf16 weight copies live in one
    buffer per parameter (fixed address) and the capture records the cast, so
    after an optimizer-style in-place update and an eager forward (which
    refreshes the copies eagerly), a replay's actions equal an uncaptured
    act_batch with the new weights; so does a replay after a `p.data` write
    (the data-parallel broadcast path, which bypasses `_version`)."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import ActStepGraph, PPOAgent, PPOConfig, _bf16_invalidate
    cfg = Config(**dict(CFG10, arrival_rate=1.0, service_length=15, eval_steps=1000))
    torch.manual_seed(0)
    env = BatchedVmEnv(cfg, 128, device=DEV)
    env.eval(True)
    ag = PPOAgent(env, PPOConfig(hidden_size=64, masked=True, det=True, precision="bf16"))
    ag.eval(True)
    g = ActStepGraph(ag, warmup=1)
    g.replay()
    last = ag.model.actor[-1]
    for how in ("step", "data"):
        expect_old = ag.act_batch(g.obs.clone())
        with torch.no_grad():
            noise = torch.randn_like(last.weight) * 0.5
            if how == "step":  # in place, as AdamW: bumps _version
                last.weight.add_(noise)
                ag.model.actor_logits(g.obs.clone())  # eager forward: refreshes the copy
            else:  # a p.data write (dist.broadcast) + the trainer's invalidation
                last.weight.data.add_(noise)
                _bf16_invalidate(ag.model.parameters())
        obs = g.obs.clone()
        expect = ag.act_batch(obs)
        assert not torch.equal(expect, expect_old), "the update should change some actions"
        g.replay()
        assert torch.equal(g.actions, expect), how
    env.close()


def _change_rel_cos(sd, d, pre):
    """(relative L2 of sd - reference over the reference's change, cosine of
    the two parameter changes) over every parameter."""
    keys = sorted(sd)
    ours = np.concatenate([(sd[k] - d["p0_" + k]).ravel() for k in keys]).astype(np.float64)
    ref = np.concatenate([(d[pre + k] - d["p0_" + k]).ravel() for k in keys]).astype(np.float64)
    rel = float(np.linalg.norm(ours - ref) / np.linalg.norm(ref))
    return rel, float(ours @ ref / np.linalg.norm(ours) / np.linalg.norm(ref))


def test_bf16_update_vs_reference_update_10yml():
    """the bf16 training leg (precision="bf16": bf16 GEMM
    inputs, f32 accumulate, the fused matrix-core actor head at hidden 64)
    against the reference's f32 update() on its recorded batch
    (tests/golden/ppo_update.npz, src/agents/ppo.py:229-295): the same 16
    minibatch steps and no KL break, the parameter change within 3e-2 relative
    L2 of the reference's and pointing the same way (cosine >= 0.999). Bound:
    bf16 keeps 8 significand bits, and AdamW's first steps move every element
    by ~lr whatever its gradient's size, so rounding that flips a near-zero
    gradient element moves that element the other way; a CPU emulation of the
    same bf16 GEMM rounding with the torch head gives 1.2e-2 / 0.99993."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    d = _g("ppo_update.npz")
    env = BatchedVmEnv(Config(**CFG10), 1, device=DEV)
    ag = PPOAgent(env, PPOConfig(hidden_size=64, episodes=1, precision="bf16"))
    assert ag.model.bf16_fused()  # the fused head kernels run this update
    ag.model.load_state_dict({k[3:]: torch.tensor(d[k]) for k in d.files if k.startswith("p0_")})
    st = ag.update(*[torch.tensor(d[k]) for k in ("b_mask", "b_action", "b_obs", "b_next_obs",
                                                    "b_logprob", "b_reward", "b_done")])
    assert st["minibatches"] == 16 and st["kl_breaks"] == 0
    sd = {k: v.detach().cpu().numpy() for k, v in ag.model.state_dict().items()}
    rel, cos = _change_rel_cos(sd, d, "p1_")
    print(f"bf16 update vs reference (10.yml, hidden 64): rel L2 {rel:.3e}, cos {cos:.6f}")
    assert rel <= 3e-2 and cos >= 0.999, (rel, cos)
    env.close()


@pytest.mark.parametrize("k_epochs", [2, 4])
def test_bf16_update_vs_reference_update_100yml(k_epochs):
    """The bf16 leg at the 100.yml shape (V 300, A 102, D 1100) against the
    reference's update on its own sampled batch (tests/golden/ppo100_update.npz,
    hidden 8: the bf16 logits path, BF16ActorHead): the reference's minibatch /
    KL-break sequence (2 epochs: 8 steps; 4 epochs: 14 steps and the epoch-4
    break) and the parameter change within 0.15 relative L2 (cosine >= 0.99).
    Bound: the 1 100-wide first layer sees bf16-rounded observations; CPU
    emulation of the rounding measures 0.103 / 0.093 (cosine 0.995 / 0.996)."""
    from tests.test_ppo_cpu import _ppo100_update
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    env = BatchedVmEnv(Config(**CFG100), 1, device=DEV)
    ag = PPOAgent(env, PPOConfig(hidden_size=8, episodes=1, batch_size=100, minibatch_size=25,
                                 migration_ratio=0.002, k_epochs=k_epochs, precision="bf16"))
    d, ag, st = _ppo100_update(k_epochs, agent=ag)
    calls = d[("e2_" if k_epochs == 2 else "") + "ref_calls"]
    assert st["minibatches"] == calls[1] and st["minibatches"] + st["kl_breaks"] == calls[0]
    sd = {k: v.detach().cpu().numpy() for k, v in ag.model.state_dict().items()}
    rel, cos = _change_rel_cos(sd, d, "p1_e2_" if k_epochs == 2 else "p1_")
    print(f"bf16 update vs reference (100.yml, {k_epochs} epochs): rel L2 {rel:.3e}, cos {cos:.6f}")
    assert rel <= 0.15 and cos >= 0.99, (rel, cos)
    env.close()
