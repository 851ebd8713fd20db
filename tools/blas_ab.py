"""f32 GEMM time of the ppo_eval actor (4 096 x {110, 512, 512} -> {512, 512, 360}
as addmm with bias) under torch's two BLAS back ends on ROCm: hipBLASLt
(default) and rocBLAS ("cublas"). Usage: python tools/blas_ab.py"""
import json
import torch


def t_ms(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us


def main():
    dev = "cuda:0"
    B = 4096
    shapes = [(110, 512), (512, 512), (512, 360)]
    xs = [torch.randn(B, k, device=dev) for k, _ in shapes]
    ws = [torch.randn(n, k, device=dev) * 0.05 for k, n in shapes]
    bs = [torch.randn(n, device=dev) for _, n in shapes]
    out = {}
    for lib in ("cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        r = {}
        for (k, n), x, w, b in zip(shapes, xs, ws, bs):
            r[f"{k}->{n}"] = round(t_ms(lambda: torch.addmm(b, x, w.t())), 2)
            r[f"{k}->{n} linear"] = round(t_ms(lambda: torch.nn.functional.linear(x, w, b)), 2)
        out[lib] = r
    print(json.dumps(out))


if __name__ == "__main__":
    main()
