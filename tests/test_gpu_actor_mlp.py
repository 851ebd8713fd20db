"""vmp_actor_mlp_f32 (csrc/vmp_mlp.hip): the PPO actor's forward, ppo.py:98-109
(Linear D->H, Tanh, Linear H->H, Tanh, Linear H->N), in one launch on the f32
matrix cores, against a plain-PyTorch reference of the same op in float64
(the exact value the f32 arithmetic approximates) and torch's own f32 layers
on the device. Tolerance: 1e-5 relative to the output scale, the bar of
test_network_outputs_match_reference (f32 rounding of K = 512 sums in a
different order than hipBLASLt's)."""
import os

import numpy as np
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")


def _mlp(D, H, N, seed):
    g = torch.Generator().manual_seed(seed)
    seq = nn.Sequential(nn.Linear(D, H), nn.Tanh(), nn.Linear(H, H), nn.Tanh(), nn.Linear(H, N))
    with torch.no_grad():
        for m in seq:
            if isinstance(m, nn.Linear):
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (1.5 / m.in_features ** 0.5))
                m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)
    return seq


def _ref64(seq, x, layers):
    """float64 restatement: layers 3 = the whole stack, 2 = self.actor[:-1]."""
    h = x.double().cpu()
    for m in list(seq)[:5 if layers == 3 else 4]:
        if isinstance(m, nn.Linear):
            h = h @ m.weight.detach().double().cpu().t() + m.bias.detach().double().cpu()
        else:
            h = torch.tanh(h)
    return h


@pytest.mark.parametrize("B,D,H,N,layers", [
    (4096, 110, 512, 360, 3),   # config/10.yml eval (weights-10 shape)
    (1000, 110, 512, 360, 3),   # ragged last row block
    (333, 37, 64, 30, 3),       # small hidden, D % 4 != 0, N < 16 * 8
    (257, 1100, 512, 512, 2),   # config/100.yml rollout: self.actor[:-1] (D % 16 != 0)
    (64, 64, 512, 512, 3),      # every layer float4, N = 512 (4 tiles per wave)
    (17, 1536, 256, 5, 3),      # D at the limit, N < 16
])
def test_actor_mlp_matches_float64_and_torch(B, D, H, N, layers):
    from vmp import head as Hd
    seq = _mlp(D, H, N, seed=B + D + H + N).to(DEV)
    g = torch.Generator().manual_seed(7)
    x = torch.rand((B, D), generator=g).to(DEV)
    out = Hd.actor_mlp(x, seq[0], seq[2], seq[4] if layers == 3 else None)
    torch.cuda.synchronize()
    assert out.shape == (B, N if layers == 3 else H)
    ref = _ref64(seq, x, layers)
    scale = float(ref.abs().max())
    err = float((out.double().cpu() - ref).abs().max())
    assert err <= 1e-5 * max(1.0, scale), (err, scale)
    with torch.no_grad():
        tor = seq(x) if layers == 3 else seq[:-1](x)
    torch.testing.assert_close(out, tor, rtol=1e-5, atol=1e-5 * max(1.0, scale))


def test_actor_mlp_run_to_run_identical_and_rows_independent():
    """Fixed order: the same inputs give the same bits; a row's result does not
    depend on the other rows of its block (rows past B are zero-filled)."""
    from vmp import head as Hd
    seq = _mlp(110, 512, 360, seed=3).to(DEV)
    x = torch.rand((100, 110), generator=torch.Generator().manual_seed(1)).to(DEV)
    a = Hd.actor_mlp(x, seq[0], seq[2], seq[4])
    b = Hd.actor_mlp(x, seq[0], seq[2], seq[4])
    c = Hd.actor_mlp(x[37:38].clone(), seq[0], seq[2], seq[4])
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert torch.equal(a[37], c[0])


def test_network_uses_the_kernel_and_keeps_reference_outputs(monkeypatch):
    """Network.actor_logits under no_grad runs vmp_actor_mlp_f32 and reproduces
    the reference Network's recorded logits (weights-10/ppo-wr.pt, ppo10_fwd.npz)
    within 1e-5; with grad enabled (the update) it stays on the torch layers."""
    from vmp import head as Hd
    from vmp.ppo import Network
    w, f = np.load(os.path.join(GOLDEN, "ppo10_wr_weights.npz")), \
        np.load(os.path.join(GOLDEN, "ppo10_fwd.npz"))
    net = Network(110, np.full(30, 12), 512).to(DEV)
    net.load_state_dict({k: torch.tensor(w[k]) for k in w.files})
    obs = torch.tensor(f["obs"], device=DEV)
    calls = []
    real = Hd.actor_mlp
    monkeypatch.setattr(Hd, "actor_mlp", lambda *a, **k: calls.append(1) or real(*a, **k))
    with torch.no_grad():
        lg = net.actor_logits(obs)
    assert calls, "no-grad actor forward did not take the MLP kernel"
    torch.testing.assert_close(lg.cpu(), torch.tensor(f["logits"]), rtol=1e-5, atol=1e-5)
    calls.clear()
    lg2 = net.actor_logits(obs)
    assert not calls and lg2.requires_grad
    torch.testing.assert_close(lg2.detach(), lg, rtol=1e-5, atol=1e-5)


def test_actor_mlp_rejects_unsupported_shapes():
    from vmp import head as Hd
    seq = _mlp(16, 520, 8, seed=1).to(DEV)   # H > 512
    with pytest.raises(ValueError):
        Hd.actor_mlp(torch.zeros((4, 16), device=DEV), seq[0], seq[2], seq[4])
    seq = _mlp(16, 40, 8, seed=1).to(DEV)    # H % 16 != 0
    with pytest.raises(ValueError):
        Hd.actor_mlp(torch.zeros((4, 16), device=DEV), seq[0], seq[2], seq[4])


@pytest.mark.parametrize("B,D,H,V,A", [(4096, 110, 512, 30, 12), (1000, 110, 512, 30, 12),
                                       (333, 37, 64, 5, 100), (77, 64, 128, 16, 32)])
def test_mlp_head_equals_policy_head_on_its_logits(B, D, H, V, A):
    """vmp_actor_mlp_head_f32 against the unfused head (vmp_policy_head) run on
    the same launch's logits (logits_out): SAMPLE with the mask and the WAIT
    coin, GIVEN and ARGMAX give identical actions, logprob and entropy (the
    per-row code is shared, vmp_head_dev.h); all-masked and one-valid rows
    included, ragged B."""
    from vmp import head as Hd
    seq = _mlp(D, H, V * A, seed=B + V).to(DEV)
    g = torch.Generator().manual_seed(B)
    x = torch.rand((B, D), generator=g).to(DEV)
    mask = torch.rand((B, V, A), generator=g) < 0.5
    mask[..., A - 1] = False
    mask[0, :2] = True                 # all-masked rows
    mask[1, :2] = True
    mask[1, :2, A - 1] = False         # one valid action
    bits = Hd.pack_mask(mask.to(DEV), V, A)
    for mode in ("sample", "given", "argmax"):
        lg = torch.empty((B, V * A), dtype=torch.float32, device=DEV)
        r1, r2 = Hd.HeadRng(11), Hd.HeadRng(11)
        if mode == "sample":
            a1, lp1, en1 = Hd.actor_mlp_head(x, seq[0], seq[2], seq[4], V, A, bits=bits, rng=r1,
                                             wait_ratio=0.5, wait_index=A - 1, logits_out=lg)
            a2, lp2, en2 = Hd.policy_head(lg, V, A, bits=bits, rng=r2, wait_ratio=0.5,
                                          wait_index=A - 1)
        elif mode == "given":
            act = torch.randint(0, A, (B, V), generator=g).to(DEV)
            a1, lp1, en1 = Hd.actor_mlp_head(x, seq[0], seq[2], seq[4], V, A, bits=bits,
                                             action=act, logits_out=lg)
            a2, lp2, en2 = Hd.policy_head(lg, V, A, bits=bits, action=act)
        else:
            a1, _, _ = Hd.actor_mlp_head(x, seq[0], seq[2], seq[4], V, A, mode=Hd.HEAD_ARGMAX,
                                         logits_out=lg)
            a2 = Hd.det_action(lg, V, A)
            lp1 = lp2 = en1 = en2 = None
        torch.cuda.synchronize()
        assert torch.equal(a1.int(), a2.int()), mode
        if lp1 is not None:
            assert torch.equal(torch.nan_to_num(lp1), torch.nan_to_num(lp2)), mode
            assert torch.equal(en1, en2), mode
        # the logits copy is the plain MLP's output
        torch.testing.assert_close(lg, Hd.actor_mlp(x, seq[0], seq[2], seq[4]), rtol=0, atol=0)


def test_eval_step_graph_uses_the_one_launch_actor():
    """ActStepGraph at the config/10.yml eval shape samples through
    vmp_actor_mlp_head_f32 (one launch for MLP + head) and draws only valid
    actions."""
    from vmp import head as Hd
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import ActStepGraph, PPOAgent, PPOConfig
    cfg = Config(pms=10, vms=30, service_length=100, arrival_rate=0.182, training_steps=10000,
                 eval_steps=1000, seed=1, reward_function="wr", allow_null_action=True)
    env = BatchedVmEnv(cfg, 256, device=DEV)
    env.eval(True)
    ag = PPOAgent(env, PPOConfig(hidden_size=512, masked=True, migration_ratio=0.5))
    w = np.load(os.path.join(GOLDEN, "ppo10_wr_weights.npz"))
    ag.model.load_state_dict({k: torch.tensor(w[k]) for k in w.files})
    obs = env.obs()
    with torch.no_grad():
        assert ag.model._mlp_head_ok(obs)
    gr = ActStepGraph(ag)
    from tests.torch_ref import unpack_bits
    for t in range(20):
        bits = env.mask_bits()
        assert torch.equal(bits, gr.bits), t  # the mask the step carried over
        gr.replay()
        torch.cuda.synchronize()
        full = unpack_bits(bits, 12)
        taken = full.gather(-1, gr.actions.long()[..., None]).squeeze(-1)
        # PPOAgent.act's coin may forbid WAIT where it was the only valid
        # action: the row is then all masked and draws uniformly (ppo.py:151-156)
        forced = full[..., :10].all(-1) & ~full[..., 10]
        assert not (taken & ~forced).any(), (t, int(taken.sum()), int((taken & forced).sum()))
    env.close()


def test_packed_weights_follow_parameter_updates():
    """The kernel reads a fragment-order copy of the weights (vmp_actor_mlp_pack),
    re-packed when a weight's version moves (optimizer steps are in-place ops)
    and after mlp_invalidate (writes through `.data` keep the version)."""
    from vmp import head as Hd
    seq = _mlp(110, 512, 360, seed=5).to(DEV)
    x = torch.rand((64, 110), generator=torch.Generator().manual_seed(2)).to(DEV)
    y0 = Hd.actor_mlp(x, seq[0], seq[2], seq[4])
    with torch.no_grad():
        seq[2].weight.mul_(0.5)           # in place: version bump -> re-pack
        ref = seq(x)
    y1 = Hd.actor_mlp(x, seq[0], seq[2], seq[4])
    torch.testing.assert_close(y1, ref, rtol=1e-5, atol=1e-5)
    assert not torch.equal(y0, y1)
    seq[4].weight.data.mul_(2.0)          # bypasses the version counter
    Hd.mlp_invalidate([seq[0].weight])
    with torch.no_grad():
        ref = seq(x)
    torch.testing.assert_close(Hd.actor_mlp(x, seq[0], seq[2], seq[4]), ref, rtol=1e-5, atol=1e-5)


def test_mlp_head_lds_limit_matches_the_kernel():
    """vmp.head.actor_mlp_head_lds mirrors the LDS the C entry point asks:
    at H 512, V 32, A 16 a D of 1 408 fits one CU's 160 KB and runs, D 1 409
    (padded K 1 536) does not and is rejected, and Network then keeps the
    unfused MLP + head path (_mlp_head_ok False) instead of failing."""
    from vmp import head as Hd
    from vmp.ppo import Network
    assert Hd.actor_mlp_head_lds(1408, 512, 32, 16) <= Hd.ACTOR_MLP_LDS_LIMIT
    assert Hd.actor_mlp_head_lds(1409, 512, 32, 16) > Hd.ACTOR_MLP_LDS_LIMIT
    g = torch.Generator().manual_seed(3)
    for D, ok in ((1408, True), (1409, False)):
        seq = _mlp(D, 512, 32 * 16, seed=D).to(DEV)
        x = torch.rand((20, D), generator=g).to(DEV)
        bits = Hd.pack_mask(torch.zeros((20, 32, 16), dtype=torch.bool, device=DEV), 32, 16)
        if ok:
            a, lp, en = Hd.actor_mlp_head(x, seq[0], seq[2], seq[4], 32, 16, bits=bits,
                                          rng=Hd.HeadRng(5))
            torch.cuda.synchronize()
            assert a.shape == (20, 32) and torch.isfinite(lp).all()
        else:
            with pytest.raises(Exception):
                Hd.actor_mlp_head(x, seq[0], seq[2], seq[4], 32, 16, bits=bits, rng=Hd.HeadRng(5))
        net = Network(D, np.full(32, 16), 512).to(DEV)
        with torch.no_grad():
            assert net._mlp_head_ok(x) == ok
