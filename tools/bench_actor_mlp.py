"""Time vmp_actor_mlp_f32 against torch's layers (hipBLASLt GEMMs + tanh) at
the PPO eval shape (config/10.yml: B 4096, D 110, H 512, N 360) and the
rollout trunk of config/100.yml (B 8192, D 1100, H 512, self.actor[:-1]),
then bench.py's ppo_eval leg with the kernel on and off (VMP_ACTOR_MLP).
HIP events on the current stream, 200 back-to-back calls each."""
import json
import os
import sys
import types

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3  # us


def main():
    from vmp import head as H
    dev = torch.device("cuda", 0)
    out = {}
    for name, B, D, Hd, N, layers in (("eval_10yml", 4096, 110, 512, 360, 3),
                                      ("rollout_100yml_trunk", 8192, 1100, 512, 30600, 2)):
        torch.manual_seed(0)
        seq = nn.Sequential(nn.Linear(D, Hd), nn.Tanh(), nn.Linear(Hd, Hd), nn.Tanh(),
                            nn.Linear(Hd, min(N, 512))).to(dev)
        x = torch.rand((B, D), device=dev)
        l3 = seq[4] if layers == 3 else None
        with torch.no_grad():
            t_k = timeit(lambda: H.actor_mlp(x, seq[0], seq[2], l3))
            t_t = timeit(lambda: (seq if layers == 3 else seq[:-1])(x))
        flops = 2.0 * B * (D * Hd + Hd * Hd + (Hd * N if layers == 3 else 0))
        out[name] = {"kernel_us": t_k, "torch_us": t_t, "kernel_TFLOPs": flops / t_k / 1e6,
                     "frac_f32_peak": flops / t_k / 1e6 / 157.3}
        print(name, json.dumps(out[name]), flush=True)
    import bench
    args = types.SimpleNamespace(ppo_eval_envs=4096)
    for flag in ("1", "0", "1"):
        os.environ["VMP_ACTOR_MLP"] = flag
        r = bench.bench_ppo_eval(args, dev, 0, 1, None)
        out[f"ppo_eval_mlp{flag}"] = {"ms_per_step": r["ms_per_step"], "frac": r["roofline"]["frac"]}
        print(f"ppo_eval VMP_ACTOR_MLP={flag}", json.dumps(out[f"ppo_eval_mlp{flag}"]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
