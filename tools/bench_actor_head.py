"""Fused actor head (vmp_actor_head) vs the unfused path (torch addmm =
nn.Linear on hipBLASLt, then vmp_policy_head) at the PPO shapes:
  collect  config/100.yml rollout: B 8192, K 512, V 300, A 102, SAMPLE
  update   config/100.yml training forward chunk: B 34816, GIVEN (+ logits kept)
  eval     config/10.yml PPO eval: B 4096, K 512, V 30, A 12, SAMPLE + WAIT flips
Prints one JSON line per shape: ms per call (HIP events) and TFLOP/s of the GEMM."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import torch  # noqa: E402

from vmp import head as H  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    dev = "cuda:0"
    for name, B, K, V, A, mode, flips in (("collect", 8192, 512, 300, 102, "sample", False),
                                          ("update", 34816, 512, 300, 102, "given", False),
                                          ("eval", 4096, 512, 30, 12, "sample", True)):
        g = torch.Generator(device=dev).manual_seed(0)
        h = torch.tanh(torch.randn((B, K), device=dev, generator=g))
        w = torch.randn((V * A, K), device=dev, generator=g) * 0.05
        b = torch.randn((V * A,), device=dev, generator=g) * 0.1
        mask = torch.rand((B, V, A), device=dev, generator=g) < 0.5
        mask[..., A - 2] = False
        bits = H.pack_mask(mask, V, A)
        del mask
        act = torch.randint(0, A - 2, (B, V), device=dev, dtype=torch.int32)
        rng = H.HeadRng(1)
        kw = dict(wait_ratio=0.5, wait_index=A - 2) if flips else {}
        logits = torch.empty((B, V * A), device=dev)

        def unfused():
            torch.addmm(b, h, w.t(), out=logits)
            if mode == "sample":
                H.policy_head(logits, V, A, bits=bits, rng=rng, **kw)
            else:
                H.policy_head(logits, V, A, bits=bits, action=act)

        def fused():
            if mode == "sample":
                H.actor_head(h, w, b, V, A, bits=bits, rng=rng, **kw)
            else:
                H.actor_head(h, w, b, V, A, bits=bits, action=act, logits_out=logits)

        def gemm_only():
            torch.addmm(b, h, w.t(), out=logits)
        with torch.no_grad():
            tu, tf, tg = timeit(unfused), timeit(fused), timeit(gemm_only)
        fl = 2.0 * B * K * V * A
        print(json.dumps({"shape": name, "B": B, "K": K, "V": V, "A": A, "mode": mode,
                          "unfused_ms": tu, "fused_ms": tf, "hipblaslt_gemm_ms": tg,
                          "fused_tflops": fl / tf / 1e9, "hipblaslt_tflops": fl / tg / 1e9,
                          "speedup": tu / tf}), flush=True)
        del logits, h, w, bits


if __name__ == "__main__":
    main()
