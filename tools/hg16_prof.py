"""Profile driver for the bf16 training head: N forward calls
(vmp_actor_head_bf16_fwd) at B samples of the config/100.yml shape (K 512,
V 300, A 102), for rocprofv3 --pmc passes.
Usage: python tools/hg16_prof.py [B] [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import torch  # noqa: E402

from vmp import head as H  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    K, V, A = 512, 300, 102
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    hb = torch.tanh(torch.randn((B, K), device=dev, generator=g)).bfloat16()
    wb = (torch.randn((V * A, K), device=dev, generator=g) * 0.05).bfloat16()
    b = torch.randn((V * A,), device=dev, generator=g) * 0.1
    bits = torch.zeros((B, V, 4), dtype=torch.int32, device=dev)
    for i in range(0, B, 16384):
        m = torch.rand((min(B, i + 16384) - i, V, A), device=dev, generator=g) < 0.5
        m[..., A - 2] = False
        bits[i:i + m.shape[0]] = H.pack_mask(m, V, A)
    act = torch.randint(0, A - 2, (B, V), device=dev, dtype=torch.int32)
    for _ in range(n):
        H.actor_head_bf16_fwd(hb, wb, b, V, A, bits, act)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
