"""Actor head and advantage scan of the PPO path on libvmp.so (HIP, gfx950).

Reference (src/agents/ppo.py):
  Network.get_action      ppo.py:115-126  masked multi-Categorical: mask to -1e7,
                                          split into V Categoricals of A, sample /
                                          log_prob / entropy summed over V
  Network.get_det_action  ppo.py:128-131  argmax of the unmasked [V, A] logits
  PPOAgent.act            ppo.py:154-156  WAIT coin flips with migration_ratio
  PPOAgent.update (GAE)   ppo.py:232-243  reverse scan

`MaskedHead` is the autograd op: forward = vmp_policy_head, backward =
vmp_policy_head_backward, so the [B, V*A] logits are read once per pass and no
[V] list of Categorical objects or per-VM multinomial launches exist. Masks
travel bit-packed (u32 [B, V, ceil(A/32)], what vmp_mask writes); the
reference's bool [B, V, A] layout is packed on the device by `pack_mask`.
"""
import ctypes

import torch

from ._lib import check, lib, ptr

HEAD_SAMPLE, HEAD_GIVEN, HEAD_ARGMAX = 0, 1, 2
HEAD_MAX_A = 1024


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _need_device(t, what):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the policy head runs on the MI355X (libvmp.so); got a "
                           f"{t.device} tensor and there is no CPU fallback")


def pack_mask(invalid_mask, V, A):
    """bool invalid mask [..., V, A] or [..., V*A] -> int32 bits [B, V, W]
    (bit a of word a//32 set = invalid). int32 [B, V, W] passes through."""
    W = (A + 31) // 32
    m = invalid_mask
    if m.dtype == torch.int32 and m.shape[-1] == W:
        return m.reshape(-1, V, W).contiguous()
    m = m.reshape(-1, V, A).to(torch.bool)
    pad = W * 32 - A
    if pad:
        m = torch.nn.functional.pad(m, (0, pad))
    w = m.reshape(m.shape[0], V, W, 32).to(torch.int64)
    shifts = torch.arange(32, device=m.device, dtype=torch.int64)
    bits = (w << shifts).sum(-1)
    return torch.where(bits >= 2**31, bits - 2**32, bits).to(torch.int32).contiguous()


class HeadRng:
    """Counter-based sampling stream: (seed, offset) advanced by B*V per call,
    so every (sample, VM) draw of a run is distinct and reproducible.
    `graph_counter(device)` switches to a device-side counter (one int64
    tensor, advanced on the stream after each use) for captured graphs, whose
    replays repeat the launch arguments."""

    def __init__(self, seed: int):
        self.seed = int(seed) & (2**64 - 1)
        self.offset = 0
        self.counter = None

    def fold(self, k):
        """Give stream k (e.g. a data-parallel rank) its own seed: splitmix64 of
        seed ^ k * golden ratio. Stream 0 keeps the seed, so rank 0 of a job draws
        what a single process would."""
        if k:
            z = (self.seed ^ (int(k) * 0x9E3779B97F4A7C15)) & (2**64 - 1)
            z = (z + 0x9E3779B97F4A7C15) & (2**64 - 1)
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
            self.seed = z ^ (z >> 31)
        return self

    def graph_counter(self, device):
        """[0]: the counter the kernels mix into the seed; [1]: the arrival
        ticket of a kernel that advances [0] itself (vmp_actor_mlp_head_f32)."""
        if self.counter is None:
            self.counter = torch.zeros(2, dtype=torch.int64, device=device)
        return self

    def take(self, n):
        if self.counter is not None:
            return self.seed, 0
        o = self.offset
        self.offset += int(n)
        return self.seed, o

    def advance(self):
        if self.counter is not None:
            self.counter[:1].add_(1)  # [1] is a kernel's arrival ticket


class MaskedHead(torch.autograd.Function):
    """(logits [B, V*A], bits|None, action|None) -> (action i32 [B,V], logprob [B], entropy [B])."""

    @staticmethod
    def forward(ctx, logits, bits, action, V, A, rng_seed, rng_offset, wait_ratio, wait_index,
                rng_counter=None):
        _need_device(logits, "MaskedHead")
        B = logits.shape[0]
        if logits.dtype != torch.float32:
            logits = logits.float()
        logits = logits.contiguous()
        if logits.numel() != B * V * A:
            raise ValueError(f"logits {tuple(logits.shape)} do not hold {V} x {A} per sample")
        if bits is not None and tuple(bits.shape) != (B, V, (A + 31) // 32):
            raise ValueError(f"mask bits {tuple(bits.shape)} != {(B, V, (A + 31) // 32)}")
        if action is None:
            mode = HEAD_SAMPLE
            act = torch.empty((B, V), dtype=torch.int32, device=logits.device)
        else:
            mode = HEAD_GIVEN
            act = action.to(device=logits.device, dtype=torch.int32).reshape(B, V).contiguous()
        lp = torch.empty((B,), dtype=torch.float32, device=logits.device)
        ent = torch.empty((B,), dtype=torch.float32, device=logits.device)
        ws = torch.empty((2 * B * V,), dtype=torch.float32, device=logits.device)
        check(lib().vmp_policy_head(B, V, A, mode, ptr(logits), ptr(bits), float(wait_ratio),
                                    int(wait_index), rng_seed, rng_offset, ptr(rng_counter),
                                    ptr(act), ptr(lp), ptr(ent), ptr(ws), _stream(logits)))
        ctx.save_for_backward(logits, bits, act)
        ctx.V, ctx.A = V, A
        ctx.mark_non_differentiable(act)
        return act, lp, ent

    @staticmethod
    def backward(ctx, g_act, g_lp, g_ent):
        logits, bits, act = ctx.saved_tensors
        B = logits.shape[0]
        d = torch.empty_like(logits)
        glp = None if g_lp is None else g_lp.float().contiguous()
        gen = None if g_ent is None else g_ent.float().contiguous()
        check(lib().vmp_policy_head_backward(B, ctx.V, ctx.A, ptr(logits), ptr(bits), ptr(act),
                                             ptr(glp), ptr(gen), ptr(d), _stream(logits)))
        return d, None, None, None, None, None, None, None, None, None


HEAD_TILE_MAX_A = 128  # kTileMaxA: the tiled kernels (and the bf16 backward)


def head_given(logits, V, A, bits, action):
    """vmp_policy_head in GIVEN mode outside autograd -> (logprob [B], entropy [B])."""
    _need_device(logits, "head_given")
    B = logits.shape[0]
    act = action.to(device=logits.device, dtype=torch.int32).reshape(B, V).contiguous()
    lp = torch.empty((B,), dtype=torch.float32, device=logits.device)
    ent = torch.empty((B,), dtype=torch.float32, device=logits.device)
    ws = torch.empty((2 * B * V,), dtype=torch.float32, device=logits.device)
    check(lib().vmp_policy_head(B, V, A, HEAD_GIVEN, ptr(logits), ptr(bits), -1.0, -1, 0, 0, None,
                                ptr(act), ptr(lp), ptr(ent), ptr(ws), _stream(logits)))
    return act, lp, ent


def head_backward_bf16(logits, V, A, bits, act, g_lp, g_ent):
    """vmp_policy_head_backward_bf16: the head's dlogits rounded to bf16 in its
    store -> bf16 [B, V*A] (the bf16 training leg's GEMM input)."""
    B = logits.shape[0]
    d = torch.empty((B, V * A), dtype=torch.bfloat16, device=logits.device)
    glp = None if g_lp is None else g_lp.float().contiguous()
    gen = None if g_ent is None else g_ent.float().contiguous()
    check(lib().vmp_policy_head_backward_bf16(B, V, A, ptr(logits), ptr(bits), ptr(act), ptr(glp),
                                              ptr(gen), ptr(d), _stream(logits)))
    return d


def policy_head(logits, V, A, bits=None, action=None, rng: HeadRng = None, wait_ratio=-1.0,
                wait_index=-1):
    """Functional form of MaskedHead (differentiable in logits)."""
    if A > HEAD_MAX_A:
        raise ValueError(f"action_dim {A} > {HEAD_MAX_A}")
    if action is None and rng is None:
        raise ValueError("sampling needs a HeadRng")
    if wait_ratio >= 0 and torch.is_grad_enabled() and logits.requires_grad:
        raise ValueError("WAIT coin flips (PPOAgent.act) are inference-only")
    seed, off = rng.take(logits.shape[0] * V) if rng is not None else (0, 0)
    ctr = rng.counter if rng is not None else None
    out = MaskedHead.apply(logits, bits, action, V, A, seed, off, wait_ratio, wait_index, ctr)
    if rng is not None and action is None:
        rng.advance()
    return out


ACTOR_HEAD_MAX_A = 128


def actor_head_supported(h, weight, A):
    """vmp_actor_head's shape contract (include/vmp.h)."""
    return (h.is_cuda and h.dtype == torch.float32 and weight.dtype == torch.float32
            and h.shape[-1] % 32 == 0 and A <= ACTOR_HEAD_MAX_A)


def actor_head_preferred(V, A):
    """Where the fused kernel beats logits GEMM + head (tools/bench_actor_head.py
    on MI355X): wide action spaces. At config/100.yml (V*A = 30 600) the fused
    rollout call is faster than hipBLASLt + the tiled head; at config/10.yml
    (V*A = 360) the 360-column GEMM is too narrow to fill the chip and the
    unfused path wins."""
    return V * A >= 4096 and A <= ACTOR_HEAD_MAX_A


def actor_head(h, weight, bias, V, A, bits=None, action=None, rng: HeadRng = None, mode=None,
               wait_ratio=-1.0, wait_index=-1, logits_out=None):
    """The actor's last Linear + the masked head in one launch (vmp_actor_head,
    ppo.py:115-131): h f32 [B, K] -> (action i32 [B, V], logprob [B], entropy
    [B]); the [B, V*A] logits are written only into `logits_out` if given.
    mode: HEAD_SAMPLE (default without action), HEAD_GIVEN (default with
    action) or HEAD_ARGMAX (get_det_action: action only). Not differentiable."""
    _need_device(h, "actor_head")
    h = h.contiguous()
    B, K = h.shape
    if mode is None:
        mode = HEAD_SAMPLE if action is None else HEAD_GIVEN
    if mode == HEAD_SAMPLE and rng is None:
        raise ValueError("sampling needs a HeadRng")
    if bits is not None and tuple(bits.shape) != (B, V, (A + 31) // 32):
        raise ValueError(f"mask bits {tuple(bits.shape)} != {(B, V, (A + 31) // 32)}")
    if mode == HEAD_GIVEN:
        act = action.to(device=h.device, dtype=torch.int32).reshape(B, V).contiguous()
    else:
        act = torch.empty((B, V), dtype=torch.int32, device=h.device)
    lp = ent = None
    ws = None
    if mode != HEAD_ARGMAX:
        lp = torch.empty((B,), dtype=torch.float32, device=h.device)
        ent = torch.empty((B,), dtype=torch.float32, device=h.device)
        ws = torch.empty((2 * B * V,), dtype=torch.float32, device=h.device)
    seed, off = rng.take(B * V) if (rng is not None and mode == HEAD_SAMPLE) else (0, 0)
    ctr = rng.counter if rng is not None else None
    check(lib().vmp_actor_head(B, K, V, A, mode, ptr(h), ptr(weight.contiguous()),
                               ptr(bias.contiguous()), ptr(bits), float(wait_ratio),
                               int(wait_index), seed, off, ptr(ctr), ptr(act), ptr(lp), ptr(ent),
                               ptr(logits_out), ptr(ws), _stream(h)))
    if rng is not None and mode == HEAD_SAMPLE:
        rng.advance()
    return act, lp, ent


ACTOR_MLP_MAX_D = 1536  # VMP_ACTOR_MLP_MAX_D


ACTOR_MLP_LDS_LIMIT = 160 * 1024  # one CU's LDS


def actor_mlp_head_lds(D, H, V, A, with_bits=True):
    """Bytes of LDS vmp_actor_mlp_head_f32 asks per workgroup (vmp_mlp.hip
    mlp_lds + the logits, per-row results and staged mask words of its 16
    rows); the C entry point rejects a shape above ACTOR_MLP_LDS_LIMIT."""
    kp = lambda k: (k + 127) // 128 * 128  # noqa: E731  (kpad: 32 * kPf)
    ldx, ldh = kp(D) + 4, kp(H) + 4
    W = (A + 31) // 32
    return 4 * 16 * (max(ldx, ldh) + ldh + V * A + 2 * V) + (4 * 16 * V * W if with_bits else 0)


def actor_mlp_supported(D, H, N, layers):
    """vmp_actor_mlp_f32's shape contract (include/vmp.h)."""
    return (H % 32 == 0 and 32 <= H <= 512 and 1 <= D <= ACTOR_MLP_MAX_D
            and (layers == 2 or 1 <= N <= 512))


def mlp_packed(l1, l2, l3=None):
    """The actor weights in vmp_actor_mlp_f32's fragment order (vmp_actor_mlp_pack):
    one device buffer per Linear stack, kept on l1.weight and re-packed when
    any weight's `_version` moves (AdamW steps in place) or the cache is
    invalidated (ppo._bf16_invalidate, after `p.data` writes). Under HIP-graph
    capture a stale pack is recorded, so replays re-pack the live
    parameters (~2 MB, one launch per layer) unless it is fresh (see below)."""
    layers = 3 if l3 is not None else 2
    lin = (l1, l2, l3) if l3 is not None else (l1, l2)
    D, Hh = int(l1.in_features), int(l1.out_features)
    N = int(l3.out_features) if l3 is not None else Hh
    key = (layers, D, Hh, N, tuple(int(m.weight.data_ptr()) for m in lin))
    ver = tuple(int(m.weight._version) for m in lin)
    cache = getattr(l1.weight, "_vmp_mlp_pack", None)
    if cache is None:
        cache = {}
        l1.weight._vmp_mlp_pack = cache
    ent = cache.get(layers)
    dev = l1.weight.device
    if ent is None or ent[0] != key:
        n = int(lib().vmp_actor_mlp_packed_floats(D, Hh, N, layers))
        ent = [key, None, torch.empty((n,), dtype=torch.float32, device=dev)]
        cache[layers] = ent
    # under capture a fresh pack is NOT recorded: the graph's owner re-packs
    # eagerly before each replay when a weight moved (ActStepGraph.replay), so
    # replays do not pay ~15 us of packing; a stale one is recorded
    capturing = torch.cuda.is_current_stream_capturing()
    if ent[1] != ver:
        ws = [m.weight.detach().contiguous() for m in lin] + ([None] if l3 is None else [])
        check(lib().vmp_actor_mlp_pack(D, Hh, N, layers, *[ptr(w) for w in ws], ptr(ent[2]),
                                       _stream(ent[2])))
        if not capturing:  # a captured pack does not run now: keep the stamp
            ent[1] = ver
    return ent[2]


def mlp_invalidate(params):
    """Forget the packed copies kept on these parameters (after writes that
    bypass the version counter, e.g. `p.data` broadcasts)."""
    for p in params:
        c = getattr(p, "_vmp_mlp_pack", None)
        if c is not None:
            for ent in c.values():
                ent[1] = None


def actor_mlp(x, l1, l2, l3=None):
    """The actor MLP forward (ppo.py:98-109) in one launch (vmp_actor_mlp_f32):
    x f32 [B, D] through Linear l1, Tanh, Linear l2, Tanh and, with l3, Linear
    l3 -> the logits f32 [B, N]; without l3 -> self.actor[:-1](x), f32 [B, H].
    f32 matrix cores, activations in LDS between layers; no autograd."""
    _need_device(x, "actor_mlp")
    x = x.contiguous()
    B, D = x.shape
    H = int(l1.out_features)
    layers = 3 if l3 is not None else 2
    N = int(l3.out_features) if l3 is not None else H
    if not actor_mlp_supported(D, H, N, layers):
        raise ValueError(f"actor_mlp: unsupported shape D={D} H={H} N={N}")
    pk = mlp_packed(l1, l2, l3)
    bs = [l1.bias, l2.bias] + ([l3.bias] if l3 is not None else [None])
    bs = [None if b is None else b.detach().contiguous() for b in bs]
    out = torch.empty((B, N), dtype=torch.float32, device=x.device)
    check(lib().vmp_actor_mlp_f32(B, D, H, N, layers, ptr(x), ptr(pk), *[ptr(b) for b in bs],
                                  ptr(out), _stream(x)))
    return out


def actor_mlp_head(x, l1, l2, l3, V, A, bits=None, action=None, rng: HeadRng = None,
                   mode=None, wait_ratio=-1.0, wait_index=-1, logits_out=None):
    """The actor MLP and the masked head in one launch (vmp_actor_mlp_head_f32,
    ppo.py:98-131): x f32 [B, D] -> (action i32 [B, V], logprob [B], entropy
    [B]) as policy_head would give on the MLP's logits (same per-row code,
    same uniforms: bit for bit); the logits stay on chip unless `logits_out`
    (f32 [B, V*A]) asks for a copy. mode: HEAD_SAMPLE (default without
    action), HEAD_GIVEN (with action) or HEAD_ARGMAX. No autograd."""
    _need_device(x, "actor_mlp_head")
    x = x.contiguous()
    B, D = x.shape
    Hh = int(l1.out_features)
    if not actor_mlp_supported(D, Hh, V * A, 3) or A > ACTOR_HEAD_MAX_A:
        raise ValueError(f"actor_mlp_head: unsupported shape D={D} H={Hh} V={V} A={A}")
    if mode is None:
        mode = HEAD_SAMPLE if action is None else HEAD_GIVEN
    if mode == HEAD_SAMPLE and rng is None:
        raise ValueError("sampling needs a HeadRng")
    if bits is not None and tuple(bits.shape) != (B, V, (A + 31) // 32):
        raise ValueError(f"mask bits {tuple(bits.shape)} != {(B, V, (A + 31) // 32)}")
    if mode == HEAD_GIVEN:
        act = action.to(device=x.device, dtype=torch.int32).reshape(B, V).contiguous()
    else:
        act = torch.empty((B, V), dtype=torch.int32, device=x.device)
    lp = ent = None
    if mode != HEAD_ARGMAX:
        lp = torch.empty((B,), dtype=torch.float32, device=x.device)
        ent = torch.empty((B,), dtype=torch.float32, device=x.device)
    seed, off = rng.take(B * V) if (rng is not None and mode == HEAD_SAMPLE) else (0, 0)
    ctr = rng.counter if rng is not None else None
    pk = mlp_packed(l1, l2, l3)
    bs = [b.detach().contiguous() for b in (l1.bias, l2.bias, l3.bias)]
    # a device counter is advanced by the launch itself (no add_ launch)
    bump = int(ctr is not None and mode == HEAD_SAMPLE and ctr.numel() >= 2)
    check(lib().vmp_actor_mlp_head_f32(B, D, Hh, V, A, mode, ptr(x), ptr(pk), *[ptr(b) for b in bs],
                                       ptr(bits), float(wait_ratio), int(wait_index), seed, off,
                                       ptr(ctr), bump, ptr(act), ptr(lp), ptr(ent),
                                       ptr(logits_out), _stream(x)))
    if rng is not None and mode == HEAD_SAMPLE and not bump:
        rng.advance()
    return act, lp, ent


def actor_head_bf16_supported(K, A):
    """vmp_actor_head_bf16_fwd/_bwd's shape contract (include/vmp.h)."""
    return K % 64 == 0 and A <= ACTOR_HEAD_MAX_A


def bf16_bits_align_mask(A):
    """Address bits that must be 0 in the mask-bits base pointer of the bf16 head
    kernels: a row of W32 = ceil(A/32) words is read as one u32x4 (W32 = 4,
    16 B) or u32x2 (W32 = 2, 8 B), else word by word (4 B)."""
    w32 = (A + 31) // 32
    return 15 if w32 == 4 else (7 if w32 == 2 else 3)


def _bf16_operands(hb, wb, bias, V, A, bits, action, who):
    """Shape / dtype / layout contract of vmp_actor_head_bf16_fwd/_bwd
    (include/vmp.h): contiguous bf16 h [B, K] and weight [V*A, K], 16-byte
    aligned; f32 bias [V*A]; mask bits contiguous int32 [B, V, ceil(A/32)]
    aligned to the row's vector load (bf16_bits_align_mask); actions as contiguous
    int32 [B, V] (cast here, as the forward always did)."""
    _need_device(hb, who)
    if hb.dim() != 2 or hb.dtype != torch.bfloat16 or not hb.is_contiguous():
        raise ValueError(f"{who}: h must be contiguous bf16 [B, K]")
    B, K = hb.shape
    if (tuple(wb.shape) != (V * A, K) or wb.dtype != torch.bfloat16 or not wb.is_contiguous()):
        raise ValueError(f"{who}: weight must be contiguous bf16 [{V * A}, {K}]")
    if (hb.data_ptr() | wb.data_ptr()) & 15:
        raise ValueError(f"{who}: h and weight must be 16-byte aligned")
    if bias.numel() != V * A or bias.dtype != torch.float32:
        raise ValueError(f"{who}: bias must be f32 [{V * A}]")
    if bits is not None:
        if (tuple(bits.shape) != (B, V, (A + 31) // 32) or bits.dtype != torch.int32
                or not bits.is_contiguous()):
            raise ValueError(f"{who}: mask bits must be contiguous int32 {(B, V, (A + 31) // 32)}")
        if bits.data_ptr() & bf16_bits_align_mask(A):
            raise ValueError(f"{who}: mask bits misaligned for the row's "
                             f"{(A + 31) // 32}-word vector load")
    act = action.to(device=hb.device, dtype=torch.int32).reshape(B, V).contiguous()
    return B, K, act


def actor_head_bf16_fwd(hb, wb, bias, V, A, bits, action):
    """The bf16 training forward (vmp_actor_head_bf16_fwd): hb bf16 [B, K], wb bf16
    [V*A, K], bias f32 [V*A], GIVEN actions -> (logprob [B], entropy [B]); the
    logits are consumed in registers, never written."""
    B, K, act = _bf16_operands(hb, wb, bias, V, A, bits, action, "actor_head_bf16_fwd")
    lp = torch.empty((B,), dtype=torch.float32, device=hb.device)
    ent = torch.empty((B,), dtype=torch.float32, device=hb.device)
    ws = torch.empty((2 * B * V,), dtype=torch.float32, device=hb.device)
    check(lib().vmp_actor_head_bf16_fwd(B, K, V, A, ptr(hb), ptr(wb), ptr(bias.contiguous()),
                                        ptr(bits), ptr(act), ptr(lp), ptr(ent), ptr(ws),
                                        _stream(hb)))
    return act, lp, ent


def actor_head_bf16_sample(hb, wb, bias, V, A, bits, rng: HeadRng, wait_ratio=-1.0,
                           wait_index=-1):
    """The bf16 rollout's draw (vmp_actor_head_bf16_sample): the actor's last
    Linear on the bf16 matrix cores + the masked head in SAMPLE mode, with the
    PPOAgent.act WAIT coin when wait_ratio >= 0 -> (action i32 [B, V], logprob
    [B], entropy [B]); the logits never reach memory. The uniforms come from
    `rng`'s counter-based stream as in policy_head."""
    B = hb.shape[0] if hb.dim() == 2 else 0
    dummy = torch.empty((B, V), dtype=torch.int32, device=hb.device)
    B, K, _ = _bf16_operands(hb, wb, bias, V, A, bits, dummy, "actor_head_bf16_sample")
    if wait_ratio >= 0 and (bits is None or not 0 <= wait_index < A):
        raise ValueError("the WAIT coin needs mask bits and 0 <= wait_index < A")
    seed, off = rng.take(B * V)
    act = dummy
    lp = torch.empty((B,), dtype=torch.float32, device=hb.device)
    ent = torch.empty((B,), dtype=torch.float32, device=hb.device)
    ws = torch.empty((2 * B * V,), dtype=torch.float32, device=hb.device)
    check(lib().vmp_actor_head_bf16_sample(B, K, V, A, ptr(hb), ptr(wb), ptr(bias.contiguous()),
                                           ptr(bits), float(wait_ratio), int(wait_index), seed,
                                           off, ptr(rng.counter), ptr(act), ptr(lp), ptr(ent),
                                           ptr(ws), _stream(hb)))
    rng.advance()
    return act, lp, ent


def actor_head_bf16_bwd(hb, wb, bias, V, A, bits, action, g_lp, g_ent, out, dbias=None,
                        workspace=None):
    """The bf16 training backward (vmp_actor_head_bf16_bwd) over the rows of hb
    (a chunk): recomputes the logits tiles and writes bf16 dlogits into `out`
    ([rows, >= V*A], row stride out.stride(0)); with `dbias` (f32 [V*A]) the
    chunk's bias gradient is ADDED to it from inside the kernel (workspace:
    f32 of bf16_bwd_workspace(rows, V, A) elements, optional)."""
    B, K, act = _bf16_operands(hb, wb, bias, V, A, bits, action, "actor_head_bf16_bwd")
    if (out.dtype != torch.bfloat16 or out.dim() != 2 or out.shape[0] < B
            or out.shape[1] < V * A or out.stride(1) != 1):
        raise ValueError("dlogits out must be bf16 [rows, >= V*A] with unit column stride")
    if out.data_ptr() & 3:
        raise ValueError("dlogits out must be 4-byte aligned")
    glp = None if g_lp is None else g_lp.float().contiguous()
    gen = None if g_ent is None else g_ent.float().contiguous()
    if dbias is not None and (dbias.dtype != torch.float32 or dbias.numel() != V * A
                              or not dbias.is_contiguous()):
        raise ValueError("dbias must be contiguous f32 [V*A]")
    if workspace is not None and (workspace.dtype != torch.float32
                                  or workspace.numel() < bf16_bwd_workspace(B, V, A)):
        raise ValueError("workspace must be f32 with bf16_bwd_workspace(B, V, A) elements")
    check(lib().vmp_actor_head_bf16_bwd(B, K, V, A, ptr(hb), ptr(wb), ptr(bias.contiguous()),
                                        ptr(bits), ptr(act), ptr(glp), ptr(gen), ptr(out),
                                        int(out.stride(0)), ptr(dbias), ptr(workspace),
                                        _stream(hb)))
    return out


def bf16_bwd_workspace(B, V, A):
    """f32 elements of vmp_actor_head_bf16_bwd's bias-gradient partials."""
    return int(lib().vmp_actor_head_bf16_bwd_workspace(int(B), int(V), int(A)))


def det_action(logits, V, A):
    """get_det_action (ppo.py:128-131): unmasked argmax per VM row -> int32 [B, V]."""
    _need_device(logits, "det_action")
    logits = logits.float().contiguous()
    B = logits.shape[0]
    act = torch.empty((B, V), dtype=torch.int32, device=logits.device)
    check(lib().vmp_policy_head(B, V, A, HEAD_ARGMAX, ptr(logits), None, -1.0, -1, 0, 0, None,
                                ptr(act), None, None, None, _stream(logits)))
    return act


def gae(reward, done, value, next_value, gamma, lam):
    """GAE over [T, N] f32 tensors (ppo.py:232-243) -> (advantages, returns)."""
    _need_device(reward, "gae")
    T, N = reward.shape
    r, d = reward.float().contiguous(), done.float().contiguous()
    v, nv = value.float().contiguous(), next_value.float().contiguous()
    adv, ret = torch.empty_like(r), torch.empty_like(r)
    check(lib().vmp_gae(T, N, ptr(r), ptr(d), ptr(v), ptr(nv), float(gamma), float(lam),
                        ptr(adv), ptr(ret), _stream(r)))
    return adv, ret
