"""Host-side cost of the PPO critic forward in the bf16 update (diagnostic):
wall time of get_value on 65 536 and 8 192 rows, synchronised, then a cProfile
of a few calls (top functions by cumulative time).
Usage: python tools/host_prof_values.py"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import torch  # noqa: E402


def main():
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    torch.manual_seed(0)
    cfg = Config(pms=100, vms=300, service_length=1000, arrival_rate=1.8182, training_steps=10000,
                 eval_steps=100000, seed=0, reward_function="wr", cap_target_util=True,
                 sequence="uniform", beta=0.5, allow_null_action=True)
    env = BatchedVmEnv(cfg, 256, device="cuda:0")
    ag = PPOAgent(env, PPOConfig(hidden_size=512, precision=os.environ.get("PREC", "bf16")))
    m = ag.model
    for rows in (65536, 8192, 256):
        x = torch.rand((rows, env.D), device="cuda")
        with torch.no_grad():
            for _ in range(3):
                m.get_value(x)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(5):
                m.get_value(x)
            h = time.perf_counter() - t
            torch.cuda.synchronize()
            w = time.perf_counter() - t
        print(f"get_value rows {rows}: host {h / 5 * 1e3:.2f} ms/call, wall {w / 5 * 1e3:.2f} ms/call",
              flush=True)
    x = torch.rand((65536, env.D), device="cuda")
    pr = cProfile.Profile()
    with torch.no_grad():
        pr.enable()
        for _ in range(5):
            m.get_value(x)
        torch.cuda.synchronize()
        pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(15)
    env.close()


if __name__ == "__main__":
    main()
