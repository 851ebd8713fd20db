"""Time vmp_actor_mlp_head_f32 (SAMPLE, mask bits, WAIT coin, device counter)
against vmp_actor_mlp_f32 at the eval shape (B 4096, D 110, H 512, V 30, A 12)
for the library VMP_LIB_PATH names (default: the in-tree libvmp.so)."""
import os
import sys

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
from tools.bench_actor_mlp import timeit  # noqa: E402


def main():
    from vmp import head as H
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    seq = nn.Sequential(nn.Linear(110, 512), nn.Tanh(), nn.Linear(512, 512), nn.Tanh(),
                        nn.Linear(512, 360)).to(dev)
    x = torch.rand((4096, 110), device=dev)
    mask = torch.rand((4096, 30, 12), device=dev) < 0.4
    mask[..., 11] = False
    bits = H.pack_mask(mask, 30, 12)
    rng = H.HeadRng(3).graph_counter(dev)
    with torch.no_grad():
        t_mlp = timeit(lambda: H.actor_mlp(x, seq[0], seq[2], seq[4]))
        t_head = timeit(lambda: H.actor_mlp_head(x, seq[0], seq[2], seq[4], 30, 12, bits=bits,
                                                 rng=rng, wait_ratio=0.5, wait_index=11))
    print(f"{os.environ.get('VMP_LIB_PATH', 'libvmp.so')}: mlp {t_mlp:.2f} us, mlp+head {t_head:.2f} us",
          flush=True)


if __name__ == "__main__":
    main()
