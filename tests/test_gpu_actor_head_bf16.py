"""Training side of the fused actor head in bf16 (ppo.py:115-126
get_action(obs, action, mask) inside PPOAgent.update, ppo.py:258-287):
vmp_actor_head_bf16_fwd/_bwd (BF16FusedActorHead) against the logits path of
the same bf16 leg (BF16ActorHead: hipBLASLt bf16 GEMM with f32 logits + the
tiled HIP head) and a plain-PyTorch fp32 head on the same bf16-rounded
operands. Tolerances: logprob / entropy 1e-5 relative (f32 accumulation of
the same bf16 products in another order); x / W gradients 1e-3 relative L2
against the logits path (both paths round dlogits to bf16 before the dW / dh
GEMMs) and 1e-2 against torch fp32 autograd of a plain-PyTorch head on the
bf16-rounded operands (no HIP code on that side: the fused path's only extra
rounding is its bf16 dlogits); the bias gradient, summed in f32 inside the
backward kernel from unrounded dlogits, 1e-4 against fp32 autograd (and 1e-2
against the logits path, which sums bf16-rounded dlogits). Memory: a
bf16 update on the fused path stays below one minibatch's f32 [B, V*A]
logits; the logits path does not."""
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
    h = torch.tanh(torch.randn((B, K), generator=g))
    w = torch.randn((V * A, K), generator=g) * (2.0 / K ** 0.5)
    b = torch.randn((V * A,), generator=g) * 0.1
    mask = torch.rand((B, V, A), generator=g) < p_mask
    mask[..., A - 2] = False
    mask[0, : min(2, V)] = True  # all-masked rows (uniform over the row)
    mask[1, : min(3, V), :] = True
    mask[1, : min(3, V), A - 2] = False  # rows with one valid action
    # random valid actions, with some masked / out-of-row ones on row 0
    u = torch.rand((B, V, A), generator=g) + (~mask).float()
    act = u.argmax(-1)
    act[0, 0] = A          # out of the row: NaN logprob on both paths
    act[0, min(1, V - 1)] = A - 1 if V > 1 else A  # a masked pick on an all-masked row
    return h.to(DEV), w.to(DEV), b.to(DEV), mask.to(DEV), act.to(DEV).to(torch.int32)


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


def _torch_fp32_grads(h, w, b, bits, act, V, A, glp, gen):
    """d/d(h, W, b) of sum(glp * logprob + gen * entropy) by torch autograd in
    fp32: logits = b + bf16(h) bf16(W)^T as fp32 addmm, the masked head in plain
    PyTorch (tests/torch_ref.torch_head: masked_fill, logsumexp, softmax). The
    out-of-row action of row 0 is clamped into the row; callers give row 0 a
    zero logprob weight."""
    hr = h.bfloat16().float().requires_grad_(True)
    wr = w.bfloat16().float().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    logits = torch.addmm(br, hr, wr.t())
    _, lp, ent = torch_head(logits, V, A, bits=bits, action=act.long().clamp(0, A - 1))
    ((lp * glp).sum() + (ent * gen).sum()).backward()
    return hr.grad, wr.grad, br.grad


def _run(fused, h, w, b, bits, act, V, A, glp, gen, chunk_rows=1 << 20):
    from vmp.ppo import BF16ActorHead, BF16FusedActorHead
    x = h.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    bb = b.clone().requires_grad_(True)
    if fused:
        lp, ent = BF16FusedActorHead.apply(x, ww, bb, bits, act, V, A, chunk_rows)
    else:
        lp, ent = BF16ActorHead.apply(x, ww, bb, bits, act, V, A)
    ((lp * glp).sum() + (ent * gen).sum()).backward()
    return lp.detach(), ent.detach(), x.grad, ww.grad, bb.grad


@pytest.mark.parametrize("B,K,V,A", [(4096, 512, 30, 12), (1500, 512, 300, 102),
                                     (700, 256, 13, 39), (300, 128, 5, 128), (333, 64, 7, 22)])
def test_fused_matches_logits_path_and_torch(B, K, V, A):
    from vmp.head import pack_mask
    h, w, b, mask, act = _case(B, K, V, A, seed=B + V + A)
    bits = pack_mask(mask, V, A)
    g = torch.Generator().manual_seed(7)
    glp = torch.randn(B, generator=g).to(DEV)
    gen = torch.randn(B, generator=g).to(DEV)
    lp_f, ent_f, gx_f, gw_f, gb_f = _run(True, h, w, b, bits, act, V, A, glp, gen,
                                         chunk_rows=512)  # several backward chunks
    lp_u, ent_u, gx_u, gw_u, gb_u = _run(False, h, w, b, bits, act, V, A, glp, gen)
    valid = torch.isfinite(lp_u)
    assert torch.equal(valid, torch.isfinite(lp_f))
    assert not bool(valid[0]) and bool(valid[1:].all())  # row 0 picks out of the row
    torch.testing.assert_close(lp_f[valid], lp_u[valid], rtol=1e-5, atol=2e-5 * V)
    torch.testing.assert_close(ent_f, ent_u, rtol=1e-5, atol=1e-5 * V)
    # plain-PyTorch fp32 head on the bf16-rounded operands
    logits = torch.addmm(b, h.bfloat16().float(), w.bfloat16().float().t())
    _, lp_r, ent_r = torch_head(logits, V, A, bits=bits, action=act.long().clamp(0, A - 1))
    torch.testing.assert_close(lp_f[valid], lp_r[valid], rtol=1e-5, atol=1e-4 * V)
    torch.testing.assert_close(ent_f, ent_r, rtol=1e-5, atol=1e-5 * V)
    # gradients (row 0's NaN logprob would poison them: zero its weight)
    glp0 = glp.clone()
    glp0[0] = 0.0
    lp_f, _, gx_f, gw_f, gb_f = _run(True, h, w, b, bits, act, V, A, glp0, gen, chunk_rows=512)
    _, _, gx_u, gw_u, gb_u = _run(False, h, w, b, bits, act, V, A, glp0, gen)
    # the logits path sums bf16-rounded dlogits for db; the fused kernel sums
    # them in f32 before the rounding (closer to fp32, checked below)
    for name, f, u, tol in (("x", gx_f, gx_u, 1e-3), ("w", gw_f, gw_u, 1e-3),
                            ("b", gb_f, gb_u, 1e-2)):
        assert torch.isfinite(f).all(), name
        assert _rel(f, u) < tol, (name, _rel(f, u))
    # independent of every HIP path: torch fp32 autograd through a plain-PyTorch
    # head on the bf16-rounded operands. x / W: the fused path rounds dlogits to
    # bf16 before its dW / dh GEMMs (1e-2 relative L2 allowed, ~2e-3 expected);
    # b: f32 column sums of unrounded dlogits inside the kernel (1e-4)
    gx_r, gw_r, gb_r = _torch_fp32_grads(h, w, b, bits, act, V, A, glp0, gen)
    for name, f, r, tol in (("x", gx_f, gx_r, 1e-2), ("w", gw_f, gw_r, 1e-2),
                            ("b", gb_f, gb_r, 1e-4)):
        assert _rel(f, r) < tol, (name, "vs fp32 autograd", _rel(f, r))
    # chunking does not change the result: one chunk == many chunks (same sums per chunk row)
    _, _, gx_1, gw_1, gb_1 = _run(True, h, w, b, bits, act, V, A, glp0, gen, chunk_rows=1 << 20)
    assert _rel(gx_1, gx_f) < 1e-6 and _rel(gw_1, gw_f) < 1e-6 and _rel(gb_1, gb_f) < 1e-6


@pytest.mark.parametrize("B,K,V,A", [(25, 512, 31, 30), (25, 256, 31, 60), (25, 128, 33, 96),
                                     (27, 64, 7, 22)])
def test_mask_bits_row_views_any_alignment(B, K, V, A):
    """the update hands the fused head row views of the mask bits
    (bits[t0:t1] of a [T, N, V, W32] buffer), whose offset is a multiple of
    W32 words only. With odd N*V and W32 = 1, 2, 3 the view is 4 / 8 / 12 B
    past a 16-B boundary; the kernels need only the alignment of the vector
    load they use, so forward, backward and SAMPLE mode run on such views
    and equal the same bits copied to a fresh (aligned) buffer."""
    from vmp import head as H
    h, w, b, mask, act = _case(B + 1, K, V, A, seed=17 * A + V)
    full = H.pack_mask(mask, V, A)
    view = full[1:]                       # one row of V * W32 words in
    assert view.data_ptr() % 16 != 0
    aligned = view.clone()
    hb, wb = h[1:].bfloat16().contiguous(), w.bfloat16()
    act = act[1:]
    g = torch.Generator().manual_seed(5)
    glp = torch.randn(B, generator=g).to(DEV)
    gen = torch.randn(B, generator=g).to(DEV)
    outs = []
    for bits in (view, aligned):
        _, lp, ent = H.actor_head_bf16_fwd(hb, wb, b, V, A, bits, act)
        dl = torch.zeros((B, V * A), dtype=torch.bfloat16, device=DEV)
        db = torch.zeros((V * A,), dtype=torch.float32, device=DEV)
        H.actor_head_bf16_bwd(hb, wb, b, V, A, bits, act, glp, gen, dl, dbias=db)
        sa, slp, _ = H.actor_head_bf16_sample(hb, wb, b, V, A, bits, H.HeadRng(9), 0.5, A - 1)
        torch.cuda.synchronize()
        outs.append((lp, ent, dl, db, sa, slp))
    for name, x, y in zip(("logprob", "entropy", "dlogits", "dbias", "sample", "sample_lp"),
                          *outs):
        assert torch.equal(torch.nan_to_num(x.float()), torch.nan_to_num(y.float())), name
    # a misaligned base for the row's vector load is still refused loudly
    if (A + 31) // 32 in (2, 4):
        raw = torch.zeros(full.numel() + 1, dtype=torch.int32, device=DEV)
        bad = raw[1:].view(full.shape)[1:]
        with pytest.raises(ValueError, match="misaligned"):
            H.actor_head_bf16_fwd(hb, wb, b, V, A, bad, act)


@pytest.mark.parametrize("B,K,V,A", [(1500, 512, 300, 102), (700, 256, 13, 39),
                                     (333, 64, 7, 22), (300, 128, 5, 128)])
def test_bf16_sample_matches_given_mode(B, K, V, A):
    """SAMPLE mode (vmp_actor_head_bf16_sample): every drawn action is a valid
    one (an all-masked row draws from all A), and the returned logprob /
    entropy are bit-identical to the GIVEN-mode forward of those actions (the
    same logits tiles, the same lse / entropy arithmetic)."""
    from vmp import head as H
    h, w, b, mask, _ = _case(B, K, V, A, seed=7 * B + A)
    bits = H.pack_mask(mask, V, A)
    hb, wb = h.bfloat16(), w.bfloat16()
    act, lp, ent = H.actor_head_bf16_sample(hb, wb, b, V, A, bits, H.HeadRng(5))
    torch.cuda.synchronize()
    assert act.dtype == torch.int32 and tuple(act.shape) == (B, V)
    a64 = act.long()
    assert bool(((a64 >= 0) & (a64 < A)).all())
    picked_masked = mask.gather(2, a64[..., None])[..., 0]
    all_masked = mask.all(-1)
    assert not bool((picked_masked & ~all_masked).any())
    _, lp_g, ent_g = H.actor_head_bf16_fwd(hb, wb, b, V, A, bits, act)
    assert torch.equal(lp, lp_g) and torch.equal(ent, ent_g)


def test_bf16_sample_law_and_wait_coin():
    """The draw's law: 8 192 samples with the same hidden state give each VM
    row 8 192 draws; their frequencies match the masked softmax of the
    fp32 logits on the bf16-rounded operands (plain PyTorch) within 5 sigma.
    WAIT coin (PPOAgent.act, ppo.py:151-156): wait_ratio 1 never forbids WAIT
    (the draws equal the coin-less ones), wait_ratio 0 always does where more
    than one action is invalid."""
    from vmp import head as H
    B, K, V, A = 8192, 128, 6, 20
    g = torch.Generator().manual_seed(3)
    h1 = torch.tanh(torch.randn((1, K), generator=g))
    w = torch.randn((V * A, K), generator=g) * (1.0 / K ** 0.5)
    b = torch.randn((V * A,), generator=g) * 0.3
    m1 = torch.rand((1, V, A), generator=g) < 0.3
    m1[0, 0] = True          # all masked: uniform over A
    m1[0, 1, :] = False      # nothing masked
    m1[0, 2, :] = True
    m1[0, 2, A - 2] = False  # one valid action
    h = h1.expand(B, K).contiguous().to(DEV)
    mask = m1.expand(B, V, A).contiguous().to(DEV)
    bits = H.pack_mask(mask, V, A)
    hb, wb, bd = h.bfloat16(), w.to(DEV).bfloat16(), b.to(DEV)
    act, _, _ = H.actor_head_bf16_sample(hb, wb, bd, V, A, bits, H.HeadRng(11))
    logits = torch.addmm(bd, hb[:1].float(), wb.float().t()).reshape(V, A)
    logits = logits.masked_fill(mask[0], -1e7)
    prob = torch.softmax(logits.double(), -1)
    freq = torch.stack([torch.bincount(act[:, v].long(), minlength=A) for v in range(V)]).double() / B
    sigma = (prob * (1 - prob) / B).sqrt()
    assert bool(((freq - prob).abs() <= 5 * sigma + 1e-12).all()), (freq - prob).abs().max()
    P = A - 2  # the WAIT column of this case
    a_none, lp_none, _ = H.actor_head_bf16_sample(hb, wb, bd, V, A, bits, H.HeadRng(12))
    a_one, lp_one, _ = H.actor_head_bf16_sample(hb, wb, bd, V, A, bits, H.HeadRng(12),
                                                wait_ratio=1.0, wait_index=P)
    assert torch.equal(a_none, a_one) and torch.equal(lp_none, lp_one)
    a_zero, _, _ = H.actor_head_bf16_sample(hb, wb, bd, V, A, bits, H.HeadRng(12),
                                            wait_ratio=0.0, wait_index=P)
    inval = mask[0].sum(-1)  # per VM row: invalid actions
    for v in range(V):
        # (WAIT the only valid action: forbidding it masks the whole row,
        # which then draws uniformly over A, as the reference's Categorical)
        if int(inval[v]) > 1 and not bool(mask[0, v, P]) and A - int(inval[v]) > 1:
            assert not bool((a_zero[:, v] == P).any()), v
    # a device counter (captured graphs) moves the stream on every call
    rng = H.HeadRng(13).graph_counter(DEV)
    a1, _, _ = H.actor_head_bf16_sample(hb, wb, bd, V, A, bits, rng)
    a2, _, _ = H.actor_head_bf16_sample(hb, wb, bd, V, A, bits, rng)
    assert int(rng.counter[0].item()) == 2 and not torch.equal(a1, a2)


def test_no_mask_and_deterministic():
    """bits = None (masked=False in PPOConfig) and run-to-run identical outputs."""
    B, K, V, A = 777, 512, 300, 102
    h, w, b, _, act = _case(B, K, V, A, seed=5, p_mask=0.0)
    glp = torch.ones(B, device=DEV)
    gen = torch.full((B,), 0.01, device=DEV)
    r1 = _run(True, h, w, b, None, act, V, A, glp, gen, chunk_rows=256)
    r2 = _run(True, h, w, b, None, act, V, A, glp, gen, chunk_rows=256)
    for x, y in zip(r1, r2):  # (row 0's out-of-row pick is NaN on both)
        assert torch.equal(torch.nan_to_num(x), torch.nan_to_num(y))
    ru = _run(False, h, w, b, None, act, V, A, glp, gen)
    torch.testing.assert_close(r1[0], ru[0], rtol=1e-5, atol=2e-5 * V, equal_nan=True)
    assert _rel(r1[3], ru[3]) < 1e-3


def _trainer(n_envs, precision="bf16"):
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    torch.manual_seed(0)
    cfg = Config(pms=100, vms=300, service_length=1000, arrival_rate=1.8182,
                 training_steps=10000, eval_steps=100000, seed=0, reward_function="wr",
                 sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True)
    env = BatchedVmEnv(cfg, n_envs, seeds=4 * np.arange(n_envs, dtype=np.int64), device=DEV)
    ag = PPOAgent(env, PPOConfig(hidden_size=512, batch_size=100, minibatch_size=25,
                                 migration_ratio=0.002, masked=True, precision=precision))
    return env, ag, ag.trainer()


def test_bf16_update_peak_memory_below_one_minibatch_of_logits(monkeypatch):
    """config/100.yml (V 300, A 102), hidden 512, 1024 envs: a minibatch is
    25 x 1024 samples, whose f32 logits are 3.1 GB. The fused update's peak
    allocation above the rollout buffers stays below that; the logits path's
    does not (it allocates them)."""
    env, ag, tr = _trainer(1024)
    tr.collect()
    mb_logits = 25 * 1024 * 300 * 102 * 4
    peaks = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("VMP_BF16_FUSED", fused)
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        tr.update()
        torch.cuda.synchronize()
        peaks[fused] = torch.cuda.max_memory_allocated() - base
    env.close()
    assert peaks["1"] < mb_logits, (peaks, mb_logits)
    assert peaks["0"] > mb_logits, (peaks, mb_logits)


def test_bf16_update_fused_equals_logits_path_first_step(monkeypatch):
    """One collect, then the first minibatch's gradient of the whole network
    (actor, critic) on both bf16 paths: 1e-3 relative L2."""
    env, ag, tr = _trainer(256)
    tr.collect()
    state = {k: v.clone() for k, v in ag.model.state_dict().items()}
    opt_state = ag.optimizer.state_dict()
    grads = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("VMP_BF16_FUSED", fused)
        ag.model.load_state_dict(state)
        ag.optimizer.load_state_dict(opt_state)
        cfg = tr.cfg
        k, mbs = cfg.k_epochs, cfg.minibatch_size
        cfg.k_epochs, cfg.minibatch_size = 1, cfg.batch_size  # one minibatch, one step
        seen = []
        step = ag.optimizer.step

        def capture(*a, **kw):
            seen.append(torch.cat([p.grad.flatten() for p in ag.model.parameters()]).clone())
            return step(*a, **kw)
        ag.optimizer.step = capture
        try:
            tr.update()
        finally:
            ag.optimizer.step = step
            cfg.k_epochs, cfg.minibatch_size = k, mbs
        grads[fused] = seen[0]
    env.close()
    assert _rel(grads["1"], grads["0"]) < 1e-3, _rel(grads["1"], grads["0"])
