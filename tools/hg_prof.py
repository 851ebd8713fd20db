"""Profile driver for the fused actor head: runs one shape of
tools/bench_actor_head.py (fused only) N times, for rocprofv3 --pmc passes.
Usage: python tools/hg_prof.py [collect|update|eval] [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import torch  # noqa: E402

from vmp import head as H  # noqa: E402

SHAPES = {"collect": (8192, 512, 300, 102, "sample"), "update": (34816, 512, 300, 102, "given"),
          "eval": (4096, 512, 30, 12, "sample")}


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "collect"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    B, K, V, A, mode = SHAPES[name]
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.tanh(torch.randn((B, K), device=dev, generator=g))
    w = torch.randn((V * A, K), device=dev, generator=g) * 0.05
    b = torch.randn((V * A,), device=dev, generator=g) * 0.1
    mask = torch.rand((B, V, A), device=dev, generator=g) < 0.5
    mask[..., A - 2] = False
    bits = H.pack_mask(mask, V, A)
    del mask
    act = torch.randint(0, A - 2, (B, V), device=dev, dtype=torch.int32)
    logits = torch.empty((B, V * A), device=dev) if mode == "given" else None
    rng = H.HeadRng(1)
    with torch.no_grad():
        for _ in range(n):
            if mode == "sample":
                H.actor_head(h, w, b, V, A, bits=bits, rng=rng)
            else:
                H.actor_head(h, w, b, V, A, bits=bits, action=act, logits_out=logits)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
