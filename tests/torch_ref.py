"""Plain-PyTorch fp32 references of the PPO ops (test infrastructure only).

`torch_head` restates Network.get_action's masked multi-Categorical
(src/agents/ppo.py:115-126) with torch.distributions-equivalent math; `torch_gae`
the reverse GAE loop (ppo.py:236-241). They are what the HIP ops are checked
against, and let the update / data-parallel logic run on CPU (gloo) tests."""
import torch


def unpack_bits(bits, A):
    B, V, W = bits.shape
    w = bits.to(torch.int64) & 0xFFFFFFFF
    shifts = torch.arange(32, dtype=torch.int64, device=bits.device)
    full = ((w[..., None] >> shifts) & 1).reshape(B, V, W * 32)[..., :A]
    return full.bool()


def torch_head(logits, V, A, bits=None, action=None, rng=None, wait_ratio=-1.0, wait_index=-1):
    B = logits.shape[0]
    lg = logits.reshape(B, V, A)
    if bits is not None:
        lg = lg.masked_fill(unpack_bits(bits, A), -1e7)  # ppo.py:119; no grad at masked
    # Categorical(logits=...): logits - logsumexp (ppo.py:121), rounded in f32 as torch does
    logp = lg - torch.logsumexp(lg, dim=-1, keepdim=True)
    if action is None:
        seed, off = rng.take(B * V) if rng else (0, 0)
        g = torch.Generator(device=logits.device).manual_seed((seed ^ off) & (2**63 - 1))
        action = torch.multinomial(logp.exp().reshape(B * V, A).detach(), 1, generator=g).reshape(B, V)
    a = action.reshape(B, V).long()
    lp = logp.gather(-1, a[..., None]).squeeze(-1).sum(-1)
    probs = torch.softmax(logp, dim=-1)
    ent = -(logp.clamp(min=torch.finfo(logp.dtype).min) * probs).sum(-1).sum(-1)
    return a.to(torch.int32), lp, ent


def torch_gae(rew, done, values, next_values, gamma, lam):
    adv = torch.zeros_like(rew)
    g = torch.zeros_like(rew[0])
    for t in reversed(range(rew.shape[0])):
        nd = 1 - done[t]
        delta = rew[t] + nd * gamma * next_values[t] - values[t]
        g = delta + nd * gamma * lam * g
        adv[t] = g
    return adv, adv + values


class StubEnv:
    """The attributes PPOAgent/PPOTrainer read from a BatchedVmEnv, on CPU."""

    def __init__(self, config, n_envs=1, device="cpu"):
        self.config = config
        self.n_envs = n_envs
        self.P, self.V = int(config.pms), int(config.vms)
        self.A = self.P + 2 if config.allow_null_action else self.P + 1
        self.D = 3 * self.V + 2 * self.P
        self.W = (self.A + 31) // 32
        self.device = torch.device(device)
