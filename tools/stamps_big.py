"""Phase breakdown of k_env_big (C5: P1000 / V10000, BestFit kl) from a
-DVMP_STAMPS build (diagnostic). Per-workgroup shader clocks, thread 0's view.
Usage: VMP_LIB_PATH=.../libvmp_stamps.so python tools/stamps_big.py [envs] [ff_steps] [policy]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vmp import _lib  # noqa: E402
from vmp.batched import BatchedVmEnv  # noqa: E402
from vmp.config import Config  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
FF = int(sys.argv[2]) if len(sys.argv) > 2 else 100
POL = sys.argv[3] if len(sys.argv) > 3 else "bestfit"
P, V = 1000, 10000
cfg = Config(pms=P, vms=V, arrival_rate=round(1000 / 0.55 / 1000, 3), service_length=1000,
             training_steps=10000, eval_steps=100000, seed=0, reward_function="kl",
             sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True)
env = BatchedVmEnv(cfg, N, seeds=4 * np.arange(N, dtype=np.int64), device="cuda:0")
left = FF
while left > 0:
    env.rollout(POL, min(250, left))
    left -= 250
NS = 24
buf = torch.zeros((N, NS), dtype=torch.int64, device="cuda")
_lib.check(_lib.lib().vmp_debug_stamps(env._bind(), _lib.ptr(buf)))
K = 10
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(K):
    env.heuristic_step(POL)
ev1.record()
torch.cuda.synchronize()
_lib.check(_lib.lib().vmp_debug_stamps(env._bind(), _lib.ptr(buf)))
torch.cuda.synchronize()
st = buf.cpu().numpy().astype(np.float64) / K
names = {13: "pro:load+predraw", 22: "heur:bitmaps", 17: "heur:query", 18: "heur:min+pick",
         19: "heur:choose+place(w0)", 16: "heur:rest", 2: "run_vms", 3: "accept",
         11: "stats:rank+compact", 20: "stats:phase A (+obs)", 21: "stats:phase B",
         12: "stats:final", 4: "tail-rest", 6: "obs+store"}
tot = st.sum(1)
pl = env.state()["vm_placement"].cpu().numpy()
print(f"N={N} ff={FF} policy={POL}: {ev0.elapsed_time(ev1) / K:.3f} ms/step, mean cycles per "
      f"env-step (thread 0) = {tot.mean():.0f}")
for i, nm in names.items():
    print(f"  {nm:24s} {st[:, i].mean():10.0f}  ({100 * st[:, i].mean() / tot.mean():5.1f}%)")
print("mean waiting", (pl == P).sum(1).mean(), "running", (pl < P).sum(1).mean(),
      "placements/step", float(env.counters().cpu().numpy()[:, 0].mean()) / (FF + K))
