"""PPO on the MI355X env path: the reference's Network / PPOAgent surface
(src/agents/ppo.py:13-295) over a batched, device-resident rollout.

  PPOConfig          ppo.py:13-34   same fields and defaults (+ build options)
  ortho_init         ppo.py:86-89
  Network            ppo.py:91-131  same module tree and state_dict keys; the
                                    masked multi-Categorical head is the HIP op
                                    of vmp.head (one pass over the logits)
  PPOAgent.act       ppo.py:151-161 (mask from vmp_mask, WAIT coin flips drawn
                                    from numpy's global stream as the reference)
  PPOAgent.learn     ppo.py:172-226 -> PPOTrainer over all envs of a BatchedVmEnv
  PPOAgent.update    ppo.py:229-295 (same signature, N = 1)
  save/load_model    ppo.py:163-170 (`_orig_mod.` keys of the compiled model)

PPOTrainer is the data-parallel batched form of learn/update: each of N envs
contributes a column of the [T = batch_size, N] rollout, minibatch j is time
slice [j*mb, (j+1)*mb) of every env (the reference's sequential sampler,
ppo.py:250-252), advantage normalisation and the KL early stop use the whole
minibatch, and the update is chunked over envs so the [samples, V*A] logits
never exceed `chunk_bytes`. With torch.distributed initialised (one process per
GPU, RCCL), envs are sharded over ranks and each optimizer step all-reduces the
flat gradient once; AdamW then runs redundantly on every rank.

Reference quirks kept: the value loss broadcasts [mb, 1]
against [mb] (ppo.py:266-270, a per-env [mb, mb] mean here;
`value_loss_broadcast=False` gives the elementwise loss), the KL break
leaves only the current epoch, AdamW's default weight decay 0.01, and learn()
runs `episodes` episodes (the reference loops training_steps and raises
IndexError past `episodes`).
"""
import math
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn as nn

from . import head as H
from .agents import Base, batched_env


@dataclass
class PPOConfig:
    episodes: int = 2000
    hidden_size: int = 256
    migration_ratio: float = 0.5
    masked: bool = True
    lr: float = 5e-5
    gamma: float = 0.99
    lamda: float = 0.98
    ent_coef: float = 0.01
    vf_coef: float = 0.5
    vf_loss_clip: bool = True
    k_epochs: int = 4
    kl_max: float = 0.02
    eps_clip: float = 0.1
    max_grad_norm: float = 0.5
    batch_size: int = 100
    minibatch_size: int = 25
    det: bool = False
    network_arch: str = "separate"
    reward_scaling: bool = False
    training_progress_bar: bool = True
    device: str = "cpu"  # the reference's default; the build always uses the env's GPU
    # ---- build options (not in the reference) ----
    value_loss_broadcast: bool = True  # ppo.py:266-270 [mb,1]-[mb] broadcast
    precision: str = "f32"             # "bf16": bf16 GEMM inputs, f32 accumulate/output
    chunk_bytes: int = 0               # logits budget per update chunk (0: from free HBM, fixed at the first update)
    # bf16 fused head: dlogits bytes per backward chunk (0: from free HBM,
    # fixed at the first update: min(16 GiB, free / 2 / ranks sharing the
    # device)). 16 GiB holds a whole 204 800-row minibatch at V*A = 30 600
    # (12.5 GB): one dW / dh GEMM pair per minibatch instead of three, update
    # 0.743 -> 0.718 s (profiles/r05_dlogits_chunk_ab.log)
    dlogits_chunk_bytes: int = 0
    kl_lookahead: bool = True          # step before the KL early-stop flag reaches the host,
                                       # roll back on a break (same accepted steps)
    seed_stride: int = 4               # env/episode reset seed spacing


def ortho_init(layer, scale=np.sqrt(2)):
    nn.init.orthogonal_(layer.weight, gain=scale)
    nn.init.constant_(layer.bias, 0)
    return layer


def _bf16_weight(w):
    """bf16 copy of a parameter in ONE buffer per parameter (fixed address),
    refreshed in place once per parameter version: AdamW's in-place step bumps
    `_version`, so the cast runs once per optimizer step instead of at every
    forward of every update chunk. Under HIP-graph capture the cast is always
    recorded (the graph re-casts the live parameter on every replay), and the
    buffer is never reallocated while a graph may read it. Writes that bypass
    the version counter (`p.data` broadcasts) must call _bf16_invalidate."""
    c = getattr(w, "_vmp_bf16", None)
    if c is None or c[1].shape != w.shape or c[1].device != w.device:
        c = [None, torch.empty(w.shape, dtype=torch.bfloat16, device=w.device)]
        w._vmp_bf16 = c
    capturing = w.is_cuda and torch.cuda.is_current_stream_capturing()
    if capturing or c[0] != w._version:
        c[1].copy_(w.detach())
        if not capturing:  # a captured copy does not run now: keep the stamp
            c[0] = w._version
    return c[1]


def _bf16_invalidate(params):
    """Forget the derived weight copies (bf16 casts, the MLP kernel's packed
    weights) of these parameters after writes that bypass `_version`."""
    params = list(params)
    for p in params:
        c = getattr(p, "_vmp_bf16", None)
        if c is not None:
            c[0] = None
    H.mlp_invalidate(params)


_ADDMM_OUT_DTYPE = None


def _addmm_f32(b, xb, wb):
    """b + xb wb^T with bf16 inputs and f32 accumulate / output, the bias added
    in the GEMM's epilogue (torch.addmm(..., out_dtype=float32)) where this
    torch build has it, else as a separate add."""
    global _ADDMM_OUT_DTYPE
    if _ADDMM_OUT_DTYPE is not False:
        try:
            y = torch.addmm(b, xb, wb.t(), out_dtype=torch.float32)
            _ADDMM_OUT_DTYPE = True
            return y
        except (TypeError, RuntimeError, NotImplementedError):
            _ADDMM_OUT_DTYPE = False
    return torch.mm(xb, wb.t(), out_dtype=torch.float32) + b


class BF16Linear(torch.autograd.Function):
    """y = x W^T + b with bf16 GEMM inputs and f32 accumulation / output
    (hipBLASLt through torch.mm(..., out_dtype=float32)); the backward GEMMs
    likewise. Parameters and everything outside the GEMMs stay f32, and the
    rounding of x and W is deterministic, so the rollout's and the update's
    log-probabilities of the same sample agree to f32 accumulation noise."""

    @staticmethod
    def forward(ctx, x, w, b):
        xb, wb = x.to(torch.bfloat16), _bf16_weight(w)
        if b is not None:
            y = _addmm_f32(b, xb, wb)
        else:
            y = torch.mm(xb, wb.t(), out_dtype=torch.float32)
        ctx.save_for_backward(xb, wb)
        ctx.has_bias = b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        xb, wb = ctx.saved_tensors
        g = gy.to(torch.bfloat16)
        gx = torch.mm(g, wb, out_dtype=torch.float32) if ctx.needs_input_grad[0] else None
        gw = torch.mm(g.t(), xb, out_dtype=torch.float32) if ctx.needs_input_grad[1] else None
        gb = gy.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw, gb


class BF16ActorHead(torch.autograd.Function):
    """The bf16 leg's last actor Linear and the masked head (GIVEN actions) as one
    autograd node -> (logprob [B], entropy [B]). Forward: bias in the GEMM
    epilogue, f32 logits to the HIP head. Backward: the head writes dlogits in
    bf16 (vmp_policy_head_backward_bf16), which feed the dW / dh GEMMs as they
    are; the bias gradient sums them with f32 accumulation. Saves the passes an
    nn.Linear + head graph makes over the [B, V*A] logits: the bias add, the
    f32 -> bf16 cast of dlogits and the f32 bias-gradient read."""

    @staticmethod
    def forward(ctx, x, w, b, bits, action, V, A):
        xb, wb = x.to(torch.bfloat16), _bf16_weight(w)
        logits = _addmm_f32(b, xb, wb)
        act, lp, ent = H.head_given(logits, V, A, bits, action)
        ctx.save_for_backward(logits, bits, act, xb, wb)
        ctx.V, ctx.A = V, A
        return lp, ent

    @staticmethod
    def backward(ctx, g_lp, g_ent):
        logits, bits, act, xb, wb = ctx.saved_tensors
        g = H.head_backward_bf16(logits, ctx.V, ctx.A, bits, act, g_lp, g_ent)
        del logits
        gx = torch.mm(g, wb, out_dtype=torch.float32) if ctx.needs_input_grad[0] else None
        gw = torch.mm(g.t(), xb, out_dtype=torch.float32) if ctx.needs_input_grad[1] else None
        gb = g.sum(0, dtype=torch.float32) if ctx.needs_input_grad[2] else None
        return gx, gw, gb, None, None, None, None


class BF16FusedActorHead(torch.autograd.Function):
    """The bf16 leg's last actor Linear + masked head (GIVEN actions) on the HIP
    bf16 matrix-core kernels (vmp_actor_head_bf16_fwd/_bwd):
    the forward consumes each logits tile in registers; the backward recomputes
    the tiles chunk by chunk (`chunk_rows` samples at a time) and writes only
    that chunk's bf16 dlogits, which two GEMMs turn into dh and dW (and a
    column sum into db). No [B, V*A] tensor is allocated in either direction."""

    @staticmethod
    def forward(ctx, x, w, b, bits, action, V, A, chunk_rows):
        xb, wb = x.to(torch.bfloat16).contiguous(), _bf16_weight(w)
        act, lp, ent = H.actor_head_bf16_fwd(xb, wb, b, V, A, bits, action)
        ctx.save_for_backward(xb, wb, b, bits, act)
        ctx.V, ctx.A, ctx.chunk_rows = V, A, int(chunk_rows)
        return lp, ent

    @staticmethod
    def backward(ctx, g_lp, g_ent):
        xb, wb, b, bits, act = ctx.saved_tensors
        V, A = ctx.V, ctx.A
        B, K = xb.shape
        N = V * A
        R = max(1, min(B, ctx.chunk_rows))
        dev = xb.device
        glp = torch.zeros(B, device=dev) if g_lp is None else g_lp.float().contiguous()
        gen = torch.zeros(B, device=dev) if g_ent is None else g_ent.float().contiguous()
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        dl = torch.empty((R, N), dtype=torch.bfloat16, device=dev)
        gx = torch.empty((B, K), dtype=torch.float32, device=dev) if need_x else None
        # dW = dlogits^T h per chunk (hipBLASLt); db = 1^T dlogits is summed by
        # the backward kernel itself (f32 column sums before the bf16
        # rounding, reduced per M group in a fixed order), so no pass over the
        # dlogits and no second stream computes it (round 4 ran a 1^T d GEMV,
        # 0.87 ms per 70 144-row chunk; d^T [h | 1 | 0...] at K + 64 columns
        # costs as much, profiles/r05_dw_aug.log)
        gw = None
        gb = torch.zeros((N,), dtype=torch.float32, device=dev) if need_b else None
        ws = (torch.empty((H.bf16_bwd_workspace(R, V, A),), dtype=torch.float32, device=dev)
              if need_b else None)
        for r0 in range(0, B, R):
            r1 = min(B, r0 + R)
            n = r1 - r0
            d = dl[:n]
            H.actor_head_bf16_bwd(xb[r0:r1], wb, b, V, A, None if bits is None else bits[r0:r1],
                                  act[r0:r1], glp[r0:r1], gen[r0:r1], d, dbias=gb, workspace=ws)
            if need_x:
                gx[r0:r1] = torch.mm(d, wb, out_dtype=torch.float32)
            if need_w:
                part = torch.mm(d.t(), xb[r0:r1], out_dtype=torch.float32)
                gw = part if gw is None else gw.add_(part)
        return gx, gw, gb, None, None, None, None, None


def _host_scalar(t):
    """Start copying a one-element device tensor to the host now and return a
    callable that waits for that copy alone (an event, not a device sync) and
    gives the value as a Python float."""
    if not t.is_cuda:
        v = float(t.reshape(-1)[0])
        return lambda: v
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))

    def read():
        ev.synchronize()
        return float(h.reshape(-1)[0])
    return read


DLOGITS_CHUNK_MAX = 1 << 34  # the dlogits budget's cap (16 GiB)


def _keep_f32(layer):
    """Mark a Linear that stays f32 in the bf16 leg (the critic's value head)."""
    layer._vmp_keep_f32 = True
    return layer


def _run_mlp(seq, x, precision):
    """seq(x); in bf16 precision every Linear runs as BF16Linear except the one
    marked by _keep_f32, the critic's 512 -> 1 value head, which stays an f32
    Linear (a width threshold would also move every layer of a small-hidden
    model to f32). Its
    GEMV is a bandwidth-bound 2 KB-per-row read, and hipBLASLt's bf16 -> f32
    addmm at N = 1 costs ~17 ms of host time per call on ROCm 7 / torch 2.10
    (tools/host_prof_values.py), which serialised the update's value pass."""
    if precision != "bf16":
        return seq(x)
    for m in seq:
        if isinstance(m, nn.Linear) and not getattr(m, "_vmp_keep_f32", False):
            x = BF16Linear.apply(x, m.weight, m.bias)
        else:
            x = m(x)
    return x


def _nvec(action_space):
    nvec = np.asarray(getattr(action_space, "nvec", action_space), dtype=np.int64)
    if nvec.ndim != 1 or not np.all(nvec == nvec[0]):
        raise ValueError("the VmEnv action space is MultiDiscrete([A] * V)")
    return nvec


class Network(nn.Module):
    """ppo.py:91-131. `head` defaults to the HIP op (vmp.head.policy_head); a
    callable with the same signature can be injected (tests use a torch
    reference of the op to exercise the update logic on CPU)."""

    def __init__(self, input_size: int, action_space, hidden_size: int,
                 dtype: torch.dtype = torch.float32, head=None, seed=None):
        super().__init__()
        self.action_nvec = _nvec(action_space)
        self.V, self.A = int(self.action_nvec.size), int(self.action_nvec[0])
        self.critic = nn.Sequential(
            ortho_init(nn.Linear(input_size, hidden_size, dtype=dtype)), nn.Tanh(),
            ortho_init(nn.Linear(hidden_size, hidden_size, dtype=dtype)), nn.Tanh(),
            _keep_f32(ortho_init(nn.Linear(hidden_size, 1, dtype=dtype), scale=1)))
        self.actor = nn.Sequential(
            ortho_init(nn.Linear(input_size, hidden_size, dtype=dtype)), nn.Tanh(),
            ortho_init(nn.Linear(hidden_size, hidden_size, dtype=dtype)), nn.Tanh(),
            ortho_init(nn.Linear(hidden_size, int(self.action_nvec.sum()), dtype=dtype),
                       scale=0.01))
        self._head = head if head is not None else H.policy_head
        self.rng = H.HeadRng(torch.initial_seed() if seed is None else seed)
        self.precision = "f32"

    def actor_logits(self, obs):
        """self.actor(obs), in the configured GEMM precision (no-grad f32 on the
        device: the one-launch MLP kernel, vmp_actor_mlp_f32)."""
        if self._mlp_ok(obs, 3):
            return H.actor_mlp(obs, self.actor[0], self.actor[2], self.actor[4])
        return _run_mlp(self.actor, obs, self.precision)

    def actor_hidden(self, obs):
        """self.actor[:-1](obs): the last hidden layer after its Tanh. Stays on
        torch's layers: at the config/100.yml rollout (B 8 192, D 1 100) one
        16-row workgroup per CU re-streams the 2.3 MB of trunk weights per
        block and takes 180 us against hipBLASLt's 122 us
        (profiles/r06_mlp_bench.log); vmp_actor_mlp_f32(layers = 2) is there
        for callers that want it."""
        return _run_mlp(self.actor[:-1], obs, self.precision)

    def _mlp_ok(self, obs, layers):
        """The actor forward runs as one HIP launch (vmp_actor_mlp_f32) for
        rollouts and eval: f32, on the device, no autograd graph wanted, the
        reference's Linear/Tanh/Linear/Tanh/Linear stack within the kernel's
        shape contract (VMP_ACTOR_MLP=0: the torch layers, for A/B)."""
        a = self.actor
        return (self.precision == "f32" and obs.is_cuda and obs.dtype == torch.float32
                and obs.dim() == 2 and not torch.is_grad_enabled()
                and os.environ.get("VMP_ACTOR_MLP", "1") != "0"
                and len(a) == 5 and isinstance(a[1], nn.Tanh) and isinstance(a[3], nn.Tanh)
                and all(isinstance(a[i], nn.Linear) and a[i].weight.dtype == torch.float32
                        and a[i].bias is not None for i in (0, 2, 4))
                and H.actor_mlp_supported(a[0].in_features, a[0].out_features,
                                          a[4].out_features, layers))

    def get_value(self, obs):
        return _run_mlp(self.critic, obs, self.precision)

    def head(self, logits, invalid_mask=None, action=None, wait_ratio=-1.0, wait_index=-1):
        """Masked head on precomputed logits -> (action int32 [B,V], logprob [B], entropy [B])."""
        bits = None if invalid_mask is None else H.pack_mask(invalid_mask, self.V, self.A)
        return self._head(logits, self.V, self.A, bits=bits, action=action, rng=self.rng,
                          wait_ratio=wait_ratio, wait_index=wait_index)

    def _fused(self, obs):
        """The actor's last Linear + the HIP head as one kernel (vmp_actor_head)
        where it is supported and faster; injected heads and bf16 GEMMs take the
        logits path."""
        last = self.actor[-1]
        return (self._head is H.policy_head and self.precision == "f32" and obs.is_cuda
                and obs.dtype == torch.float32 and H.actor_head_preferred(self.V, self.A)
                and last.weight.dtype == torch.float32 and last.in_features % 32 == 0
                and self.A <= H.ACTOR_HEAD_MAX_A)

    def sample(self, obs, bits=None, wait_ratio=-1.0, wait_index=-1):
        """Rollout sampling (ppo.py:115-126 with the mask as packed bits; the WAIT
        coin flips of PPOAgent.act when wait_ratio >= 0) -> (action int32 [B, V],
        logprob [B]). On the fused path the [B, V*A] logits never reach HBM."""
        if self._fused(obs):
            last = self.actor[-1]
            h = self.actor_hidden(obs)
            act, lp, _ = H.actor_head(h, last.weight, last.bias, self.V, self.A, bits=bits,
                                      rng=self.rng, wait_ratio=wait_ratio, wait_index=wait_index)
            return act, lp
        if self._bf16_sample(obs, bits):
            # the bf16 leg's rollout: last Linear + head in SAMPLE mode on the
            # matrix-core kernel the update's forward uses (no [B, V*A] logits)
            last = self.actor[-1]
            h = _run_mlp(self.actor[:-1], obs, self.precision).to(torch.bfloat16).contiguous()
            act, lp, _ = H.actor_head_bf16_sample(h, _bf16_weight(last.weight), last.bias, self.V,
                                                  self.A, bits, self.rng, wait_ratio, wait_index)
            return act, lp
        if self._mlp_head_ok(obs):
            # the whole actor + head in one launch (the config/10.yml eval shape)
            a = self.actor
            act, lp, _ = H.actor_mlp_head(obs, a[0], a[2], a[4], self.V, self.A, bits=bits,
                                          rng=self.rng, wait_ratio=wait_ratio,
                                          wait_index=wait_index)
            return act, lp
        act, lp, _ = self._head(self.actor_logits(obs), self.V, self.A, bits=bits, rng=self.rng,
                                wait_ratio=wait_ratio, wait_index=wait_index)
        return act, lp

    def refresh_packs(self):
        """Re-pack the MLP kernel's weights if a parameter moved since the last
        pack (a host-side version check; captured graphs do not re-pack)."""
        a = self.actor
        if len(a) == 5 and isinstance(a[4], nn.Linear) and getattr(a[0].weight, "_vmp_mlp_pack",
                                                                    None):
            with torch.no_grad():
                for layers in tuple(a[0].weight._vmp_mlp_pack):
                    H.mlp_packed(a[0], a[2], a[4] if layers == 3 else None)

    def _mlp_head_ok(self, obs):
        """The actor MLP + the HIP head as one launch (vmp_actor_mlp_head_f32):
        its logits fit one workgroup (V*A <= 512) and the head is the HIP op."""
        return (self._head is H.policy_head and self.V * self.A <= 512
                and self.A <= H.ACTOR_HEAD_MAX_A
                and H.actor_mlp_head_lds(int(obs.shape[-1]), self.actor[0].out_features,
                                         self.V, self.A) <= H.ACTOR_MLP_LDS_LIMIT
                and self._mlp_ok(obs, 3))

    def _bf16_sample(self, obs, bits):
        """Rollouts of the bf16 leg draw on the fused bf16 kernel where it
        applies (VMP_BF16_SAMPLE=0: the logits path, for A/B measurement)."""
        return (obs.is_cuda and self.bf16_fused()
                and os.environ.get("VMP_BF16_SAMPLE", "1") != "0"
                and (bits is None or (bits.is_contiguous()
                                      and (bits.data_ptr() & H.bf16_bits_align_mask(self.A)) == 0)))

    def det(self, obs):
        """get_det_action's argmax (ppo.py:128-131) -> int32 [B, V]."""
        if self._fused(obs):
            last = self.actor[-1]
            act, _, _ = H.actor_head(self.actor_hidden(obs), last.weight, last.bias, self.V,
                                     self.A, mode=H.HEAD_ARGMAX)
            return act
        if self._mlp_head_ok(obs):
            a = self.actor
            act, _, _ = H.actor_mlp_head(obs, a[0], a[2], a[4], self.V, self.A,
                                         mode=H.HEAD_ARGMAX)
            return act
        return H.det_action(self.actor_logits(obs), self.V, self.A)

    def bf16_fused(self):
        """The bf16 update runs the fused matrix-core head (BF16FusedActorHead)
        where its kernels apply; VMP_BF16_FUSED=0 selects the logits path
        (BF16ActorHead) for A/B measurement."""
        last = self.actor[-1]
        return (self.precision == "bf16" and self._head is H.policy_head
                and os.environ.get("VMP_BF16_FUSED", "1") != "0"
                and H.actor_head_bf16_supported(last.in_features, self.A))

    def logits_bytes_per_sample(self):
        """HBM the update holds per sample of a chunk: the activations the MLPs
        keep for backward (per hidden layer of actor and critic the f32
        pre-activation and tanh output and, in bf16, the GEMM input copy:
        <= 10 H bytes, 4 layers) plus the head's own: the f32 logits of the
        logits paths, or the fused head's 2 V f32 row workspace (its dlogits
        are bounded separately by dlogits_chunk_bytes)."""
        H = int(self.actor[0].out_features)
        head = 8 * self.V if self.bf16_fused() else 4 * self.V * self.A
        return head + 40 * H

    def logprob_entropy(self, obs, bits, action, dlogits_chunk_bytes=DLOGITS_CHUNK_MAX):
        """get_action(obs, action, mask)'s logprob and entropy (ppo.py:115-126) for
        the update, differentiable. The bf16 leg with the HIP head runs the last
        Linear and the head as one node: fused on the bf16 matrix cores
        (BF16FusedActorHead, the backward's dlogits chunked to
        `dlogits_chunk_bytes`), else over f32 logits (BF16ActorHead)."""
        if (self.precision == "bf16" and self._head is H.policy_head and obs.is_cuda
                and self.A <= H.HEAD_TILE_MAX_A):
            last = self.actor[-1]
            h = _run_mlp(self.actor[:-1], obs, "bf16")
            if self.bf16_fused():
                rows = max(256, int(dlogits_chunk_bytes) // (2 * self.V * self.A) // 256 * 256)
                return BF16FusedActorHead.apply(h, last.weight, last.bias, bits, action, self.V,
                                                self.A, rows)
            return BF16ActorHead.apply(h, last.weight, last.bias, bits, action, self.V, self.A)
        _, lp, ent = self._head(self.actor_logits(obs), self.V, self.A, bits=bits, action=action,
                                rng=self.rng)
        return lp, ent

    def get_action(self, obs, action=None, invalid_mask=None):
        """ppo.py:115-126 -> (action int64 [B,V], logprob [B], entropy [B])."""
        logits = self.actor_logits(obs)
        act, lp, ent = self.head(logits, invalid_mask, action)
        return act.long(), lp, ent

    def get_det_action(self, obs, action=None):
        """ppo.py:128-131: argmax of the unmasked logits; [V] for one observation."""
        a = self.det(obs if obs.dim() > 1 else obs[None]).long()
        return a[0] if obs.dim() == 1 or obs.shape[0] == 1 else a


class ActStepGraph:
    """One batched `PPOAgent.act` + `env.step` for every env (the Base.test loop
    body, base.py:71-86, with the PPO agent) captured as a HIP graph: actor MLP
    and masked head with the WAIT coin flips (one launch at the config/10.yml
    shape, vmp_actor_mlp_head_f32, which also advances the sampling counter),
    then vmp_step_mask, which writes the next step's mask bits with the step.
    A replay advances all envs one step with no host work; the head's sampling
    stream moves through a device counter (HeadRng.graph_counter), so replays
    draw fresh actions. obs / reward / done / bits are static buffers updated
    in place. The mask bits are computed once here and then carried by the
    steps: after changing the envs outside the graph (a reset), call
    refresh_mask(). steps > 1 captures that many consecutive steps in the
    one graph (a replay then advances every env `steps` steps and the
    buffers hold the last one's results): the graph boundary's launch gap is
    paid once per replay, not once per step."""

    def __init__(self, agent, warmup=2, steps=1):
        env = agent.benv
        dev = env.device
        self.agent, self.env = agent, env
        agent.model.rng.graph_counter(dev)
        self.obs = env.obs()
        self.bits = torch.empty((env.n_envs, env.V, env.W), dtype=torch.int32, device=dev)
        self.reward = torch.empty((env.n_envs,), dtype=torch.float64, device=dev)
        self.done = torch.empty((env.n_envs,), dtype=torch.uint8, device=dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side), torch.no_grad():
            # hipBLASLt sets up a GEMM shape on its first call, which is not
            # allowed under capture: run the actor once even when warmup == 0
            # (no env step, so the envs' state is untouched); it also packs
            # the MLP kernel's weights
            agent.model.actor_logits(self.obs.to(agent.float_dtype))
            env.mask_bits(out=self.bits)
            for _ in range(warmup):
                self._step()
        torch.cuda.current_stream(dev).wait_stream(side)
        if steps < 1:
            raise ValueError(f"steps must be >= 1, not {steps}")
        self.steps = steps
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            for _ in range(steps):
                self._step()

    def _step(self):
        a = self.agent.act_batch(self.obs, self.bits)
        self.env.step(a, obs=self.obs, reward=self.reward, done=self.done, want_valid=False,
                      bool_done=False, mask_out=self.bits)
        self.actions = a  # the captured step's action buffer: the last replay's actions

    def refresh_mask(self):
        """Recompute the mask bits from the envs' current state (after a reset
        or any other change made outside the graph)."""
        self.env.mask_bits(out=self.bits)

    def replay(self):
        self.agent.model.refresh_packs()  # host check; re-packs only if a weight moved
        self.graph.replay()
        return self.obs, self.reward, self.done


def strip_compiled_prefix(sd):
    return {k.replace("_orig_mod.", "", 1) if k.startswith("_orig_mod.") else k: v
            for k, v in sd.items()}


class PPOAgent(Base):
    def __init__(self, env, config: PPOConfig, head=None, gae=None):
        super().__init__(type(self).__name__, env, config)
        self.benv = batched_env(env)
        self.device = self.benv.device
        self._head_impl = head  # default: the HIP head (vmp.head.policy_head)
        self._gae_impl = gae    # default: the HIP scan (vmp.head.gae)
        self.init_model()

    def init_model(self):
        self.float_dtype = torch.float32
        self.obs_dim = self.benv.D
        nvec = np.full(self.benv.V, self.benv.A, dtype=np.int64)
        self.model = Network(self.obs_dim, nvec, self.config.hidden_size, self.float_dtype,
                             head=self._head_impl).to(self.device)
        if self.config.precision not in ("f32", "bf16"):
            raise ValueError(f"precision must be 'f32' or 'bf16', not {self.config.precision!r}")
        self.model.precision = self.config.precision
        self.optimizer = torch.optim.AdamW(self.model.parameters(), lr=self.config.lr)

    def eval(self, mode=True):
        self.model.train(not mode)

    # ---------------------------------------------------------------- act
    def _coin_flip_bits(self, bits):
        """ppo.py:153-156 on one env's mask bits (host copy, V x W words): numpy's
        global stream is consumed exactly as the reference does (one rand()
        per qualifying row, in row order)."""
        P, A = self.benv.P, self.benv.A
        words = bits.cpu().numpy().astype(np.uint32).reshape(self.benv.V, -1)
        full = np.unpackbits(words.view(np.uint8), axis=1, bitorder="little")[:, :A]
        out = words.copy()
        for row in range(self.benv.V):
            if (np.count_nonzero(full[row]) > 1 and not full[row, P]
                    and np.random.rand() > self.config.migration_ratio):
                out[row, P >> 5] |= np.uint32(1 << (P & 31))
        return torch.from_numpy(out.view(np.int32)).to(self.device).reshape(bits.shape)

    def act(self, obs):
        """Action for one env (numpy int64 [V]); for a BatchedVmEnv use act_batch."""
        with torch.no_grad():
            o = torch.as_tensor(np.asarray(obs), dtype=self.float_dtype,
                                device=self.device).reshape(1, -1)
            if self.config.det:
                return self.model.get_det_action(o).flatten().cpu().numpy()
            bits = None
            if self.config.masked:
                bits = self._coin_flip_bits(self.benv.mask_bits()[:1])
            act, _, _ = self.model.head(self.model.actor_logits(o), bits)
            return act.flatten().long().cpu().numpy()

    def act_batch(self, obs, bits=None):
        """PPOAgent.act for every env of the batch on the device: int32 [N, V].
        The WAIT coin flips use the head's counter-based stream."""
        with torch.no_grad():
            if self.config.det:
                return self.model.det(obs)
            if self.config.masked and bits is None:
                bits = self.benv.mask_bits()
            ratio = float(self.config.migration_ratio) if self.config.masked else -1.0
            act, _ = self.model.sample(obs, bits, wait_ratio=ratio, wait_index=self.benv.P)
            return act

    # ------------------------------------------------------------ weights
    def save_model(self, modelpath):
        """ppo.py:163-166: keys carry the torch.compile `_orig_mod.` prefix, so the
        reference's load_model reads the file."""
        if modelpath:
            parent = os.path.dirname(modelpath)
            if parent:
                os.makedirs(parent, exist_ok=True)
            sd = {"_orig_mod." + k: v.detach().cpu() for k, v in self.model.state_dict().items()}
            torch.save(sd, modelpath)

    def load_model(self, modelpath):
        """ppo.py:168-170; accepts compiled (`_orig_mod.`) and plain state dicts."""
        sd = torch.load(modelpath, map_location="cpu", weights_only=True)
        self.model.load_state_dict(strip_compiled_prefix(sd))
        self.model.eval()

    # ------------------------------------------------------------ training
    def trainer(self, group=None):
        if getattr(self, "_trainer", None) is None:
            self._trainer = PPOTrainer(self, group=group)
        return self._trainer

    def learn(self):
        """ppo.py:172-226 over every env of the (batched) env; see PPOTrainer."""
        return self.trainer().learn()

    def update(self, invalid_mask_batch, action_batch, obs_batch, next_obs_batch, logprob_batch,
               rewards_batch, done_batch):
        """ppo.py:229-295 on one env's batch (leading dim = batch_size)."""
        tr = PPOTrainer(self, group=None, allocate=False, distributed=False)
        dev = self.device
        T = obs_batch.shape[0]
        obs = obs_batch.to(dev, torch.float32).reshape(T, 1, -1)
        nobs = next_obs_batch.to(dev, torch.float32).reshape(T, 1, -1)
        bits = H.pack_mask(invalid_mask_batch.to(dev), self.benv.V, self.benv.A).reshape(
            T, 1, self.benv.V, -1)
        act = action_batch.to(dev).to(torch.int32).reshape(T, 1, -1)
        lp = logprob_batch.to(dev, torch.float32).reshape(T, 1)
        rew = rewards_batch.to(dev, torch.float32).reshape(T, 1)
        done = done_batch.to(dev).to(torch.float32).reshape(T, 1)
        with torch.no_grad():
            values = self.model.get_value(obs.reshape(T, -1)).reshape(T, 1)
            next_values = self.model.get_value(nobs.reshape(T, -1)).reshape(T, 1)
        return tr.update_from(obs, bits, act, lp, rew, done, values, next_values)


class PPOTrainer:
    """Batched PPO (rollout + update) over all envs of the agent's BatchedVmEnv."""

    def __init__(self, agent: PPOAgent, group=None, allocate=True, distributed=True):
        import torch.distributed as dist
        self.agent, self.cfg = agent, agent.config
        self.env, self.model = agent.benv, agent.model
        self.gae = agent._gae_impl if agent._gae_impl is not None else H.gae
        use = distributed and dist.is_available() and dist.is_initialized()
        self.dist = dist if use else None
        self.group = group
        self.world = self.dist.get_world_size(group) if self.dist else 1
        self.rank = self.dist.get_rank(group) if self.dist else 0
        e = self.env
        self.N, self.V, self.A, self.D, self.W = e.n_envs, e.V, e.A, e.D, e.W
        self.T = int(self.cfg.batch_size)
        self.dev = e.device
        self.episode = 0
        self.ep_t = 0
        self.ep_returns = []
        self.stats = {}
        if self.dist and not getattr(self.model.rng, "rank_folded", False):
            # every rank seeds torch alike (same initial parameters): its sampling
            # stream must still differ, or env b of every rank draws the same
            # uniforms and the global batch is correlated across ranks
            self.model.rng.fold(self.rank)
            self.model.rng.rank_folded = True
        if self.dist and allocate:
            self._sync_params()
        if allocate:
            T, N = self.T, self.N
            f = dict(device=self.dev)
            self.obs = torch.empty((T, N, self.D), dtype=torch.float32, **f)
            self.last_obs = torch.empty((N, self.D), dtype=torch.float32, **f)
            self.bits = (torch.empty((T, N, self.V, self.W), dtype=torch.int32, **f)
                         if self.cfg.masked else None)
            self.act = torch.empty((T, N, self.V), dtype=torch.int32, **f)
            self.logp = torch.empty((T, N), dtype=torch.float32, **f)
            self.rew = torch.empty((T, N), dtype=torch.float32, **f)
            self.done = torch.zeros((T, N), dtype=torch.float32, **f)
            self.r64 = torch.empty((N,), dtype=torch.float64, **f)
            self.d8 = torch.empty((N,), dtype=torch.uint8, **f)
            self.ep_ret = torch.zeros((N,), dtype=torch.float64, **f)
            if self.cfg.reward_scaling:
                self.rs_R = torch.zeros((N,), dtype=torch.float64, **f)
                self.rs_n = 0
                self.rs_mean = torch.zeros((N,), dtype=torch.float64, **f)
                self.rs_S = torch.zeros((N,), dtype=torch.float64, **f)
                self.rs_std = torch.zeros((N,), dtype=torch.float64, **f)
            self._started = False

    # ------------------------------------------------------------ plumbing
    def _sync_params(self):
        for p in self.model.parameters():
            self.dist.broadcast(p.data, src=0, group=self.group)
        _bf16_invalidate(self.model.parameters())  # p.data writes keep `_version`

    def _allreduce(self, t):
        if self.dist:
            self.dist.all_reduce(t, group=self.group)
        return t

    def _episode_seeds(self, episode):
        """reset seed of env i in `episode`: seed + stride*(episode*N_global + global i)
        (disjoint PCG64 streams for every env and episode; the reference uses
        seed + i_episode for its single env, ppo.py:192)."""
        n_glob = self.N * self.world
        gi = self.rank * self.N + torch.arange(self.N, device=self.dev, dtype=torch.int64)
        return int(self.env.config.seed) + int(self.cfg.seed_stride) * (episode * n_glob + gi)

    def _start_episode(self, out_obs):
        self.env.eval(False)
        out_obs.copy_(self.env.reset(self._episode_seeds(self.episode)))
        self.ep_t = 0
        self.ep_ret.zero_()

    def _scale_reward(self, r):
        """RewardScaler (ppo.py:55-68) per env: R = gamma R + r, running std of R
        (the reference's RunningMeanStd, incl. std = x at n = 1)."""
        self.rs_R.mul_(self.cfg.gamma).add_(r)
        self.rs_n += 1
        x = self.rs_R
        if self.rs_n == 1:
            self.rs_mean.copy_(x)
            self.rs_std.copy_(x)
        else:
            old = self.rs_mean.clone()
            self.rs_mean.add_((x - old) / self.rs_n)
            self.rs_S.add_((x - old) * (x - self.rs_mean))
            self.rs_std.copy_(torch.sqrt(self.rs_S / self.rs_n))
        return r / (self.rs_std + 1e-8)

    # ------------------------------------------------------------ rollout
    @torch.no_grad()
    def collect(self):
        """batch_size steps of every env (ppo.py:194-217): mask, sample, step."""
        T, cfg, env, m = self.T, self.cfg, self.env, self.model
        ep_len = int(env.config.training_steps)
        if not self._started:
            self._start_episode(self.obs[0])
            self._started = True
        else:
            self.obs[0].copy_(self.last_obs)
        for t in range(T):
            o = self.obs[t]
            bits = None
            if self.bits is not None:
                bits = env.mask_bits(out=self.bits[t])
            act, lp = m.sample(o, bits)
            self.act[t].copy_(act)
            self.logp[t].copy_(lp)
            nxt = self.obs[t + 1] if t + 1 < T else self.last_obs
            env.step(act, obs=nxt, reward=self.r64, done=self.d8, want_valid=False,
                     bool_done=False)
            self.ep_ret.add_(self.r64)
            r = self._scale_reward(self.r64) if cfg.reward_scaling else self.r64
            self.rew[t].copy_(r)
            self.ep_t += 1
            if self.ep_t >= ep_len:
                # every env terminates together (timestep >= training_steps, env.py:160-163)
                self.done[t].fill_(1.0)
                self._end_episode()
                self.episode += 1
                self._start_episode(nxt)
            else:
                self.done[t].zero_()
        self.agent.total_steps += T * self.N

    def _end_episode(self):
        rets = self.ep_ret.clone()
        if self.dist:
            parts = [torch.empty_like(rets) for _ in range(self.world)]
            self.dist.all_gather(parts, rets, group=self.group)
            rets = torch.cat(parts)
        self.ep_returns.append(rets.cpu().numpy())

    # ------------------------------------------------------------- update
    @torch.no_grad()
    def _values(self, obs):
        T, N = obs.shape[:2]
        flat = obs.reshape(T * N, -1)
        out = torch.empty((T * N,), dtype=torch.float32, device=obs.device)
        step = 1 << 16
        for i in range(0, T * N, step):
            out[i:i + step] = self.model.get_value(flat[i:i + step]).flatten()
        return out.reshape(T, N)

    def update(self):
        """ppo.py:229-295 on the collected [T, N] rollout."""
        with torch.no_grad():
            values = self._values(self.obs)
            next_values = torch.empty_like(values)
            next_values[:-1] = values[1:]
            next_values[-1] = self._values(self.last_obs[None])[0]
        return self.update_from(self.obs, self.bits, self.act, self.logp, self.rew, self.done,
                                values, next_values)

    def update_from(self, obs, bits, act, old_lp, rew, done, values, next_values):
        cfg, m = self.cfg, self.model
        T, N = rew.shape
        with torch.no_grad():
            adv, ret = self.gae(rew, done, values, next_values, cfg.gamma, cfg.lamda)
        mbs = int(cfg.minibatch_size)
        n_mb = math.ceil(T / mbs)
        params = [p for p in m.parameters()]
        stats = dict(minibatches=0, kl_breaks=0, clipfracs=[], rollbacks=0)
        clipfracs = []  # device scalars, read once after the update (no per-minibatch sync)
        batch = (obs, bits, act, old_lp, values, adv, ret, N)

        def after(pos):  # the reference's loop order: minibatches of an epoch, epochs
            e, j = pos
            return (e, j + 1) if j + 1 < n_mb else ((e + 1, 0) if e + 1 < cfg.k_epochs else None)

        if not cfg.kl_lookahead:
            pos = (0, 0) if cfg.k_epochs > 0 and n_mb > 0 else None
            while pos is not None:
                kl_sum, clip_n, m_glob = self._minibatch_backward(batch, pos[1] * mbs,
                                                                  min(T, (pos[1] + 1) * mbs))
                # the one host sync per minibatch: the reference's loop control
                # (ppo.py:263-264) decides on the host whether this minibatch steps
                kl = float(-kl_sum / m_glob)
                if kl > cfg.kl_max:  # ppo.py:263-264: leaves this epoch's minibatch loop
                    self._zero_grads(params)
                    stats["kl_breaks"] += 1
                    pos = (pos[0] + 1, 0) if pos[0] + 1 < cfg.k_epochs else None
                    continue
                clipfracs.append(self._optimizer_step(params, clip_n, m_glob))
                stats["minibatches"] += 1
                stats["kl"] = kl
                pos = after(pos)
        else:
            # KL look-ahead: minibatch i's optimizer step is taken before its KL is
            # known on the host, and minibatch i + 1 is enqueued behind it; the
            # host reads KL_i while the device runs i + 1. If KL_i breaks the
            # epoch (ppo.py:263-264), the parameters and AdamW state go back to
            # the copy taken before step i and minibatch i + 1 is discarded: the
            # accepted steps are the reference's sequence, bit for bit, without a
            # drained queue at every minibatch.
            inflight = None
            pos = (0, 0) if cfg.k_epochs > 0 and n_mb > 0 else None
            while pos is not None or inflight is not None:
                cur = None
                if pos is not None:
                    snap = self._opt_snapshot(params)
                    kl_sum, clip_n, m_glob = self._minibatch_backward(
                        batch, pos[1] * mbs, min(T, (pos[1] + 1) * mbs))
                    kl_host = _host_scalar(kl_sum)
                    cf = self._optimizer_step(params, clip_n, m_glob)
                    cur = dict(pos=pos, kl=kl_host, m_glob=m_glob, snap=snap, cf=cf)
                    pos = after(pos)
                if inflight is not None:
                    kl = -inflight["kl"]() / inflight["m_glob"]
                    if kl > cfg.kl_max:
                        self._opt_restore(params, inflight["snap"])
                        stats["kl_breaks"] += 1
                        stats["rollbacks"] += 1 + (cur is not None)
                        e = inflight["pos"][0]
                        pos = (e + 1, 0) if e + 1 < cfg.k_epochs else None
                        cur = None
                    else:
                        clipfracs.append(inflight["cf"])
                        stats["minibatches"] += 1
                        stats["kl"] = kl
                inflight = cur
        if clipfracs:
            stats["clipfracs"] = torch.cat(clipfracs).double().cpu().tolist()
        self.stats = stats
        return stats

    def _minibatch_backward(self, batch, t0, t1):
        """Loss of time slice [t0, t1) of every env (ppo.py:250-287), backward into
        the parameters' grads -> (kl_sum, clip count) device f64 [1] (KL sum
        all-reduced), and the global sample count."""
        obs, bits, act, old_lp, values, adv, ret, N = batch
        cfg, m = self.cfg, self.model
        eps = cfg.eps_clip
        params = [p for p in m.parameters()]
        mt = t1 - t0
        m_glob = mt * N * self.world
        dev = adv.device
        with torch.no_grad():
            a_mb = adv[t0:t1]
            s = self._allreduce(a_mb.sum().reshape(1).double())
            mean = (s / m_glob).float()
            ss = self._allreduce(((a_mb - mean) ** 2).sum().reshape(1).double())
            std = torch.sqrt(ss / max(m_glob - 1, 1)).float()
            adv_n = (a_mb - mean) / (std + 1e-10)
        per_env = mt * m.logits_bytes_per_sample()
        ce = max(1, min(N, self._chunk_budget(dev) // per_env))
        self._zero_grads(params)
        kl_sum = torch.zeros(1, dtype=torch.float64, device=dev)
        clip_n = torch.zeros(1, dtype=torch.float64, device=dev)
        for n0 in range(0, N, ce):
            n1 = min(N, n0 + ce)
            nc = n1 - n0
            o = obs[t0:t1, n0:n1].reshape(mt * nc, -1)
            b = None if bits is None else bits[t0:t1, n0:n1].reshape(mt * nc, self.V, -1)
            a = act[t0:t1, n0:n1].reshape(mt * nc, self.V)
            newlp, ent = m.logprob_entropy(o, b, a, self._dlogits_budget(dev))
            newlp = newlp.reshape(mt, nc)
            logratio = newlp - old_lp[t0:t1, n0:n1]
            ratio = torch.exp(logratio)
            kl_sum += logratio.detach().double().sum()
            clip_n += ((ratio.detach() - 1.0).abs() > eps).double().sum()
            an = adv_n[:, n0:n1]
            surr = -ratio * an
            surr_c = -torch.clamp(ratio, 1 - eps, 1 + eps) * an
            loss_clip = torch.max(surr, surr_c).sum() / m_glob
            newv = m.get_value(o).reshape(mt, nc)
            R, Vb = ret[t0:t1, n0:n1], values[t0:t1, n0:n1]
            if cfg.value_loss_broadcast:
                # newvalues [mb,1] - returns [mb] -> [mb, mb] (ppo.py:266-270), per env
                du = newv[:, None, :] - R[None, :, :]
                vcl = Vb[None, :, :] + torch.clamp(newv[:, None, :] - Vb[None, :, :], -eps, eps)
                dc = vcl - R[None, :, :]
                denom = mt * mt * N * self.world
            else:
                du = newv - R
                dc = Vb + torch.clamp(newv - Vb, -eps, eps) - R
                denom = m_glob
            if cfg.vf_loss_clip:
                lvf = torch.max(du * du, dc * dc).sum() / denom
            else:
                lvf = (du * du).sum() / denom
            loss = loss_clip - cfg.ent_coef * ent.sum() / m_glob + cfg.vf_coef * 0.5 * lvf
            loss.backward()
        self._allreduce(kl_sum)
        return kl_sum, clip_n, m_glob

    def _optimizer_step(self, params, clip_n, m_glob):
        """Clip fraction all-reduce, gradient all-reduce (data parallel), grad-norm
        clipping and the AdamW step (ppo.py:283-287) -> the clip fraction
        (device scalar)."""
        self._allreduce(clip_n)
        if self.dist:  # the grads are views of one flat buffer: one all-reduce
            self.dist.all_reduce(self._gflat, group=self.group)
        nn.utils.clip_grad_norm_(params, self.cfg.max_grad_norm)
        self.agent.optimizer.step()
        return clip_n / m_glob

    def _opt_snapshot(self, params):
        """Device copies of the parameters and of AdamW's per-parameter state
        (its host `step` counters too) before a look-ahead step."""
        opt = self.agent.optimizer
        with torch.no_grad():
            ps = [p.detach().clone() for p in params]
            st = [{k: v.clone() for k, v in opt.state[p].items()} if p in opt.state else None
                  for p in params]
        return ps, st

    def _opt_restore(self, params, snap):
        opt = self.agent.optimizer
        ps, st = snap
        with torch.no_grad():
            for p, c, s in zip(params, ps, st):
                p.copy_(c)  # bumps p._version: the bf16 weight copies re-cast
                if s is None:
                    opt.state.pop(p, None)
                else:
                    for k, v in s.items():
                        opt.state[p][k].copy_(v)

    def _min_over_ranks(self, b, dev):
        if self.dist:
            t = torch.tensor([b], dtype=torch.int64, device=dev)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
            b = int(t.item())
        return b

    def _chunk_budget(self, dev):
        """The update's chunk budget, fixed once per trainer (the chunk count sets
        the f32 gradient summation order, so it must not move with the free
        memory between minibatches or runs); data parallel: the minimum over
        ranks, so every rank chunks alike."""
        if getattr(self, "_budget", None) is None:
            self._dlogits_budget(dev)  # sized first: the activations get what it leaves
            self._budget = self._min_over_ranks(self._chunk_bytes(dev), dev)
        return self._budget

    def _device_sharers(self, dev):
        """Ranks of the group on this process's device (gloo rehearsals put
        several on one GPU): one all-reduce of each rank's device key."""
        if not self.dist or dev.type != "cuda":
            return 1
        if getattr(self, "_sharers", None) is None:
            import socket
            import zlib
            props = torch.cuda.get_device_properties(dev)
            ident = getattr(props, "uuid", None)
            ident = str(ident) if ident is not None else "%s:%s" % (
                getattr(props, "pci_bus_id", ""), dev.index)
            key = zlib.crc32(("%s/%s" % (socket.gethostname(), ident)).encode()) + 1
            keys = torch.zeros(self.world, dtype=torch.int64, device=dev)
            keys[self.rank] = key
            self.dist.all_reduce(keys, group=self.group)
            self._sharers = max(1, int((keys == key).sum().item()))
        return self._sharers

    def _dlogits_budget(self, dev):
        """Bytes of bf16 dlogits per fused-head backward chunk: PPOConfig.
        dlogits_chunk_bytes, or min(16 GiB, half the memory free on the device
        / the ranks sharing it), fixed at the first update and min-reduced over
        ranks (the chunking sets dW's summation order)."""
        if getattr(self, "_dl_budget", None) is None:
            if int(self.cfg.dlogits_chunk_bytes) > 0:
                b = int(self.cfg.dlogits_chunk_bytes)
            elif dev.type != "cuda":
                b = DLOGITS_CHUNK_MAX
            else:
                b = min(DLOGITS_CHUNK_MAX, self._free_bytes(dev) // 2 // self._device_sharers(dev))
            self._dl_budget = self._min_over_ranks(max(1 << 26, b), dev)
        return self._dl_budget

    @staticmethod
    def _free_bytes(dev):
        """Memory free on the device, incl. blocks torch has cached but not handed out."""
        free, _ = torch.cuda.mem_get_info(dev)
        return int(free + torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev))

    def _chunk_bytes(self, dev):
        """Logits budget per update chunk: PPOConfig.chunk_bytes, or what the
        device can hold now: a chunk's peak is its f32 logits, the dlogits of
        the backward and the saved activations (<= 3x the logits), so the
        budget is a third of the memory free on the device (incl. blocks torch
        has cached but not handed out), capped at 1/8 of the device. On an idle
        288 GB MI355X that is 36 GB: a whole config/100.yml minibatch of 8192
        envs (25 GB of f32 logits) is one chunk, so backward writes each
        gradient once instead of accumulating chunk by chunk; on a smaller or
        shared GPU the chunks shrink instead of running out of memory (ranks
        sharing the device split it; the bf16 fused head's dlogits budget is
        taken off first)."""
        if int(self.cfg.chunk_bytes) > 0:
            return int(self.cfg.chunk_bytes)
        if dev.type != "cuda":
            return 4 << 30
        _, total = torch.cuda.mem_get_info(dev)
        free = self._free_bytes(dev)
        if self.model.bf16_fused():  # the fused head's dlogits chunk comes out of it
            free -= self._dlogits_budget(dev)
        n = self._device_sharers(dev)
        return max(1 << 28, min(int(total) // 8 // n, free // 3 // n))

    def _zero_grads(self, params):
        """Single process: grads re-created by backward. Data parallel: every
        grad is a view of one flat f32 buffer, zeroed here, which backward
        accumulates into and one RCCL all-reduce averages — no
        per-step concatenation of the 69 MB of gradients."""
        if not self.dist:
            for p in params:
                p.grad = None
            return
        n = sum(p.numel() for p in params)
        if getattr(self, "_gflat", None) is None or self._gflat.numel() != n:
            self._gflat = torch.zeros(n, dtype=params[0].dtype, device=params[0].device)
            self._gviews = []
            o = 0
            for p in params:
                self._gviews.append(self._gflat[o:o + p.numel()].view_as(p))
                o += p.numel()
        self._gflat.zero_()
        for p, g in zip(params, self._gviews):
            p.grad = g

    # ------------------------------------------------------------- driver
    def train_updates(self, n_updates):
        for _ in range(int(n_updates)):
            self.collect()
            self.update()

    def learn(self):
        """ppo.py:186-224: `episodes` episodes of training_steps steps per env,
        one update every batch_size steps (batches straddle episodes)."""
        total = int(self.cfg.episodes) * int(self.env.config.training_steps)
        n_updates = total // self.T
        show = bool(self.cfg.training_progress_bar) and self.rank == 0
        for u in range(n_updates):
            self.collect()
            self.update()
            if show and self.ep_returns:
                print("update %d/%d  episodes %d  median return %.3f" %
                      (u + 1, n_updates, len(self.ep_returns),
                       float(np.median(self.ep_returns[-1]))), flush=True)
        return self.ep_returns

