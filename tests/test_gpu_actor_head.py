"""vmp_actor_head: the actor's last Linear fused with the
masked multi-categorical head (ppo.py:115-131) against the unfused path
(torch addmm = nn.Linear, then vmp_policy_head / det_action) and the torch fp32
reference of the head. Tolerances as SURVEY App. C: logits / logprob /
entropy 1e-5 relative (fp32; the fused GEMM sums K in another order),
get_det_action identical where the top two logits are apart, sampling law
within 5 sigma, sampled actions never masked."""
import numpy as np
import pytest
import torch

from tests.torch_ref import torch_head

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")


def _case(B, K, V, A, seed, p_mask=0.4):
    g = torch.Generator().manual_seed(seed)
    h = torch.tanh(torch.randn((B, K), generator=g)).to(DEV)
    w = (torch.randn((V * A, K), generator=g) * (2.0 / K ** 0.5)).to(DEV)
    b = (torch.randn((V * A,), generator=g) * 0.1).to(DEV)
    mask = torch.rand((B, V, A), generator=g) < p_mask
    mask[..., A - 2] = False
    mask[0, : min(2, V)] = True  # all-masked rows (logprob -2 quirk, uniform sample)
    act = torch.zeros((B, V), dtype=torch.int64)
    for bb in range(B):
        for v in range(V):
            ok = torch.nonzero(~mask[bb, v]).flatten()
            ok = ok if len(ok) else torch.arange(A)
            act[bb, v] = ok[torch.randint(len(ok), (1,), generator=g)]
    return h, w, b, mask.to(DEV), act.to(DEV)


@pytest.mark.parametrize("B,K,V,A", [(64, 512, 30, 12), (200, 512, 300, 102), (37, 64, 7, 33),
                                     (130, 96, 3, 128), (5, 32, 40, 120), (9, 64, 5, 65)])
def test_given_mode_and_logits_match_unfused(B, K, V, A):
    from vmp.head import HEAD_GIVEN, actor_head, pack_mask, policy_head
    h, w, b, mask, act = _case(B, K, V, A, seed=B + K + V + A)
    bits = pack_mask(mask, V, A)
    logits_ref = torch.addmm(b, h, w.t())
    out = torch.empty_like(logits_ref)
    a, lp, ent = actor_head(h, w, b, V, A, bits=bits, action=act, mode=HEAD_GIVEN,
                            logits_out=out)
    torch.testing.assert_close(out, logits_ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(a.long(), act)
    _, lp_u, ent_u = policy_head(logits_ref, V, A, bits=bits, action=act)
    _, lp_r, ent_r = torch_head(logits_ref, V, A, bits=bits, action=act)
    torch.testing.assert_close(lp, lp_u, rtol=1e-5, atol=1e-4 * V)
    torch.testing.assert_close(ent, ent_u, rtol=1e-5, atol=1e-5 * V)
    torch.testing.assert_close(lp, lp_r, rtol=1e-5, atol=1e-4 * V)
    torch.testing.assert_close(ent, ent_r, rtol=1e-5, atol=1e-5 * V)
    # without logits_out nothing changes
    _, lp2, ent2 = actor_head(h, w, b, V, A, bits=bits, action=act, mode=HEAD_GIVEN)
    assert torch.equal(lp, lp2) and torch.equal(ent, ent2)


def test_argmax_matches_det_action():
    from vmp.head import HEAD_ARGMAX, actor_head, det_action
    B, K, V, A = 256, 512, 300, 102
    h, w, b, _, _ = _case(B, K, V, A, seed=3)
    logits = torch.addmm(b, h, w.t())
    a, lp, _ = actor_head(h, w, b, V, A, mode=HEAD_ARGMAX)
    assert lp is None
    ref = det_action(logits, V, A)
    top2 = logits.reshape(B, V, A).topk(2, -1).values
    clear = (top2[..., 0] - top2[..., 1]) > 1e-4
    assert clear.float().mean() > 0.99
    assert torch.equal(a[clear], ref[clear])


def test_sample_law_validity_and_stream():
    """Inverse-CDF draws follow softmax(masked logits) (5 sigma per category),
    never pick a masked action, and the stream advances between calls."""
    from vmp.head import HeadRng, actor_head, pack_mask
    V, A, K, B = 4, 12, 64, 40000
    g = torch.Generator().manual_seed(7)
    h = torch.tanh(torch.randn((1, K), generator=g)).repeat(B, 1).to(DEV)
    w = (torch.randn((V * A, K), generator=g) * 0.3).to(DEV)
    b = torch.zeros(V * A, device=DEV)
    mask = torch.rand((V, A), generator=g) < 0.4
    mask[:, 10] = False
    bits = pack_mask(mask.to(DEV).expand(B, V, A), V, A)
    rng = HeadRng(123)
    with torch.no_grad():
        act, lp, _ = actor_head(h, w, b, V, A, bits=bits, rng=rng)
        act2, _, _ = actor_head(h, w, b, V, A, bits=bits, rng=rng)
    act = act.cpu().long()
    assert not torch.equal(act, act2.cpu().long())
    assert not mask.gather(1, act.T).any()
    row = (h[:1] @ w.t() + b).reshape(V, A).cpu()
    p = torch.softmax(row.masked_fill(mask, -1e7), -1)
    for v in range(V):
        cnt = torch.bincount(act[:, v], minlength=A).double()
        sd = torch.sqrt(B * p[v] * (1 - p[v])).double() + 1e-9
        assert torch.all((cnt - B * p[v].double()).abs() <= 5 * sd + 1), v
    ref_lp = torch.log_softmax(row.masked_fill(mask, -1e7), -1).gather(1, act.T).sum(0)
    torch.testing.assert_close(lp.cpu(), ref_lp, rtol=1e-5, atol=1e-4)


def test_wait_coin_flips_fused():
    """PPOAgent.act's WAIT flips (ppo.py:154-156) inside the fused kernel: the
    same rows qualify and WAIT is forbidden with probability 1 - ratio."""
    from vmp.head import HeadRng, actor_head, pack_mask
    V, A, K, B, P = 8, 12, 32, 20000, 10
    mask = torch.ones((V, A), dtype=torch.bool)
    mask[:, P] = False
    mask[:4, 3] = False
    mask[4:6, :] = False
    mask[6, P] = True
    mask[6, 5] = False
    mask[7, :] = True
    mask[7, P] = False
    h = torch.zeros((B, K), device=DEV)
    w = torch.zeros((V * A, K), device=DEV)
    b = torch.zeros((V, A), device=DEV)
    b[:, P] = 5.0
    bits = pack_mask(mask.to(DEV).expand(B, V, A), V, A)
    with torch.no_grad():
        act, _, _ = actor_head(h, w, b.reshape(-1), V, A, bits=bits, rng=HeadRng(9),
                               wait_ratio=0.3, wait_index=P)
    act = act.cpu()
    expect = 0.7 + 0.3 * (1 / (1 + np.exp(5)))
    for v in range(4):
        assert abs((act[:, v] != P).double().mean().item() - expect) < 0.02, v
    assert (act[:, 6] == 5).all()
    assert abs((act[:, 7] != P).double().mean().item() - 0.7 * 11 / 12) < 0.02


def test_sample_equals_unfused_draws():
    """Fused and unfused heads take the same per-row uniform: on the same
    weights they draw the same actions except where the f32 rounding of the
    GEMM moves a CDF boundary across the uniform (rare)."""
    from vmp.head import HeadRng, actor_head, pack_mask, policy_head
    B, K, V, A = 2048, 512, 300, 102
    h, w, b, mask, _ = _case(B, K, V, A, seed=11)
    bits = pack_mask(mask, V, A)
    with torch.no_grad():
        a_f, lp_f, _ = actor_head(h, w, b, V, A, bits=bits, rng=HeadRng(5))
        a_u, lp_u, _ = policy_head(torch.addmm(b, h, w.t()), V, A, bits=bits, rng=HeadRng(5))
    same = (a_f == a_u).double().mean().item()
    assert same > 0.999, same
    rows = (a_f == a_u).all(1)
    torch.testing.assert_close(lp_f[rows], lp_u[rows], rtol=1e-5, atol=1e-4 * V)


def test_network_sample_fused_path_matches_logits_path():
    """Network.sample / Network.det (the rollout paths of PPOTrainer.collect,
    act_batch and ActStepGraph) on the fused kernel against the same network
    through the logits path, at the config/100.yml action space."""
    from vmp.head import HeadRng, actor_head_preferred, pack_mask
    from vmp.ppo import Network
    B, D, V, A = 512, 1100, 300, 102
    assert actor_head_preferred(V, A)
    torch.manual_seed(3)
    net = Network(D, np.full(V, A), 64).to(DEV)
    obs = torch.rand((B, D), device=DEV)
    g = torch.Generator().manual_seed(4)
    mask = torch.rand((B, V, A), generator=g) < 0.5
    mask[..., A - 2] = False
    bits = pack_mask(mask.to(DEV), V, A)
    with torch.no_grad():
        assert net._fused(obs)
        net.rng = HeadRng(9)
        a_f, lp_f = net.sample(obs, bits, wait_ratio=0.5, wait_index=A - 2)
        d_f = net.det(obs)
        net._fused = lambda o: False
        net.rng = HeadRng(9)
        a_u, lp_u = net.sample(obs, bits, wait_ratio=0.5, wait_index=A - 2)
        d_u = net.det(obs)
    assert (a_f == a_u).double().mean().item() > 0.999
    assert not mask.to(DEV).gather(-1, a_f.long()[..., None]).any()
    rows = (a_f == a_u).all(1)
    torch.testing.assert_close(lp_f[rows], lp_u[rows], rtol=1e-5, atol=1e-4 * V)
    assert (d_f == d_u).double().mean().item() > 0.999
