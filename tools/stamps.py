"""Phase breakdown of the env kernel from a -DVMP_STAMPS build (diagnostic).
Usage: VMP_LIB_PATH=.../libvmp_stamps.so python tools/stamps.py [envs] [vms] [ff] [K]
(ff fast-forward steps of phase-aligned envs, then K stamped steps: ff 2000
times the refill burst, ff 2500 the quiet phase after it)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vmp import _lib  # noqa: E402
from vmp.batched import BatchedVmEnv  # noqa: E402
from vmp.config import Config  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
V = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
cfg = Config(pms=100, vms=V, arrival_rate=1.8182, service_length=1000, training_steps=10000,
             eval_steps=100000, seed=0, reward_function="wr", allow_null_action=True)
env = BatchedVmEnv(cfg, N)
env.eval(os.environ.get("STAMP_TRAIN") is None)
FF = int(sys.argv[3]) if len(sys.argv) > 3 else 2500
G = int(os.environ.get("STAMP_GROUPS", "1"))  # > 1: phases staggered as bench.py's headline
if G > 1:
    import bench  # noqa: E402
    bench.fast_forward(env, "firstfit", 4 * np.arange(N, dtype=np.int64), FF - (G - 1) * 100, G, 100, 100)
else:
    for _ in range(FF // 100):
        env.rollout("firstfit", 100)
NS = 24
buf = torch.zeros((N, NS), dtype=torch.int64, device="cuda")
_lib.check(_lib.lib().vmp_debug_stamps(env._bind(), _lib.ptr(buf)))
K = int(sys.argv[4]) if len(sys.argv) > 4 else 50
c0 = env.counters().cpu().numpy()
for _ in range(K):
    env.heuristic_step("firstfit")
torch.cuda.synchronize()
_lib.check(_lib.lib().vmp_debug_stamps(env._bind(), _lib.ptr(buf)))
torch.cuda.synchronize()
st = buf.cpu().numpy().astype(np.float64) / K
names = ["loop-end", "act+apply(rest)", "run_vms", "accept", "stats(rest)+reward", "obs", "store",
         "-", "-", "-", "-", "stats:compress", "stats:pw-sums",
         "pro:start->hdr/pm loaded", "pro:predraw", "pro:VM words loaded",
         "heur:prep", "heur:fitmax+hits", "heur:earliest", "apply:requery", "apply:scan+place",
         "apply:f32 update", "-", "apply:fitmax"]
tot = st.sum(1) - st[:, 7] - st[:, 9]
c1 = env.counters().cpu().numpy()
d = (c1 - c0).sum(0) / (N * K)
print(f"N={N} V={V} steps {FF + 1}-{FF + K}: mean cycles per env-step (per wave) = "
      f"{tot.mean():.0f}; per env-step: accepted {d[0] - d[4]:.3f}, finished {d[1]:.3f}, "
      f"placed {d[3]:.3f}, suspended {d[2]:.3f}")
for i in range(NS):
    if names[i] != "-":
        print(f"  {names[i]:20s} {st[:, i].mean():10.0f}  ({100 * st[:, i].mean() / tot.mean():5.1f}%)")
ctr = env.counters().cpu().numpy()
pl = env.state()["vm_placement"].cpu().numpy()
wall_us = st[:, 7] / 1000 / 100.0  # 100 MHz realtime ticks
cyc = st[:, 9]
print(f"wave lifetime: {wall_us.mean():.1f} us wall (mean), {cyc.mean():.0f} shader cycles -> "
      f"{cyc.mean() / wall_us.mean() / 1e3:.2f} GHz")
print("mean waiting", (pl == 100).sum(1).mean(), "running", (pl < 100).sum(1).mean())
q = np.percentile(wall_us, [10, 50, 90, 99])
print(f"wave lifetime percentiles (us): p10 {q[0]:.1f} p50 {q[1]:.1f} p90 {q[2]:.1f} p99 {q[3]:.1f} "
      f"max {wall_us.max():.1f}")
if G > 1:  # env i is in phase group i mod G (reset (i mod G) * 100 steps late)
    for g in range(G):
        print(f"  group {g} (age {FF - 100 * g}): lifetime {wall_us[g::G].mean():.1f} us")
