"""A/B of the bf16 backward's bias-gradient options at the 100.yml update
shape (one 70 144-row dlogits chunk, V*A = 30 600, K = 512), HIP events:
  dW = d^T h (hipBLASLt) + db = 1^T d (GEMV)           (round-4 HEAD)
  d^T [h | 1 | 0 ...] with K + 8 / K + 64 / K + 128 columns (db from the GEMM)
Usage: python tools/bench_dw_aug.py"""
import json

import torch


def timed(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    R, N, K = 70144, 30600, 512
    g = torch.Generator(device="cuda").manual_seed(0)
    d = (torch.randn((R, N), generator=g, device="cuda") * 1e-3).bfloat16()
    h = torch.randn((R, K), generator=g, device="cuda").bfloat16()
    ones = torch.ones((1, R), dtype=torch.bfloat16, device="cuda")
    out = {}
    out["dW_K512"] = timed(lambda: torch.mm(d.t(), h, out_dtype=torch.float32))
    out["db_gemv"] = timed(lambda: torch.mm(ones, d, out_dtype=torch.float32))
    for extra in (8, 64, 128):
        ha = torch.zeros((R, K + extra), dtype=torch.bfloat16, device="cuda")
        ha[:, :K] = h
        ha[:, K] = 1
        out[f"dW_aug_K{K + extra}"] = timed(lambda: torch.mm(d.t(), ha, out_dtype=torch.float32))
    out["dh"] = timed(lambda: torch.mm(d, torch.randn((N, K), device="cuda").bfloat16(),
                                       out_dtype=torch.float32))
    print(json.dumps({k: round(v, 4) for k, v in out.items()}))


if __name__ == "__main__":
    main()
