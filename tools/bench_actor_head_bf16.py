"""The bf16 training head at the config/100.yml update shape (one minibatch of
8192 envs x 25 steps = 204 800 samples, K 512, V 300, A 102):
  fused   vmp_actor_head_bf16_fwd, then per backward chunk vmp_actor_head_bf16_bwd
          + dh / [dW | db] GEMMs (BF16FusedActorHead)
  logits  hipBLASLt bf16 GEMM -> f32 logits + tiled head, head backward -> bf16
          dlogits + GEMMs + bias column sum (BF16ActorHead)
HIP events per stage; TFLOP/s of the head GEMM work (2 B K N per product).
Usage: python tools/bench_actor_head_bf16.py [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import torch  # noqa: E402

from vmp import head as H  # noqa: E402
from vmp.ppo import BF16ActorHead, BF16FusedActorHead  # noqa: E402


def timeit(fn, n=5, warm=2):
    for _ in range(warm):
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 204800
    K, V, A = 512, 300, 102
    N = V * A
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.tanh(torch.randn((B, K), device=dev, generator=g))
    w = torch.randn((N, K), device=dev, generator=g) * 0.05
    b = torch.randn((N,), device=dev, generator=g) * 0.1
    bits = torch.zeros((B, V, 4), dtype=torch.int32, device=dev)
    for i in range(0, B, 16384):  # random masks, chunked (the bool mask is large)
        m = torch.rand((min(B, i + 16384) - i, V, A), device=dev, generator=g) < 0.5
        m[..., A - 2] = False
        bits[i:i + m.shape[0]] = H.pack_mask(m, V, A)
    act = torch.randint(0, A - 2, (B, V), device=dev, dtype=torch.int32)
    hb = h.bfloat16()
    wb = w.bfloat16()
    glp = torch.randn(B, device=dev, generator=g)
    gen = torch.randn(B, device=dev, generator=g) * 0.01
    flop = 2.0 * B * K * N
    out = {"B": B, "K": K, "V": V, "A": A}

    if os.environ.get("GEMM_AB") == "1":  # the backward's dh / dW GEMM layouts (hipBLASLt)
        r = min(B, 70144)
        d = (torch.randn((r, N), device=dev, generator=g) * 1e-3).bfloat16()
        wbT = wb.t().contiguous()                       # [K, N]
        haug = torch.zeros((r, K + 8), dtype=torch.bfloat16, device=dev)
        haug[:, :K] = hb[:r]
        haug[:, K] = 1
        f = 2.0 * r * N * K
        res = {}
        for ka in (576, 640):  # [h | 1 | 0...] padded to a multiple of 64 / 128
            hk = torch.zeros((r, ka), dtype=torch.bfloat16, device=dev)
            hk[:, :K] = hb[:r]
            hk[:, K] = 1
            t = timeit(lambda: torch.mm(d.t(), hk, out_dtype=torch.float32), n=10)
            res[f"dW d^T@[h|1] KA {ka}"] = {"ms": round(t, 3), "tflops": round(f / t / 1e9, 1)}
            del hk
        t = timeit(lambda: d.sum(0, dtype=torch.float32), n=10)
        res["db d.sum(0, f32)"] = {"ms": round(t, 3), "GB/s": round(2.0 * r * N / t / 1e6, 1)}
        ones = torch.ones((1, r), dtype=torch.bfloat16, device=dev)
        t = timeit(lambda: torch.mm(ones, d, out_dtype=torch.float32), n=10)
        res["db 1^T d"] = {"ms": round(t, 3), "GB/s": round(2.0 * r * N / t / 1e6, 1)}
        for name, fn in (("dh d@W [N,K] row-major", lambda: torch.mm(d, wb, out_dtype=torch.float32)),
                         ("dh d@(W^T)^T", lambda: torch.mm(d, wbT.t(), out_dtype=torch.float32)),
                         ("dh (W^T @ d^T)^T", lambda: torch.mm(wbT, d.t(), out_dtype=torch.float32)),
                         ("dW d^T@[h|1]", lambda: torch.mm(d.t(), haug, out_dtype=torch.float32)),
                         ("dW d^T@h", lambda: torch.mm(d.t(), hb[:r], out_dtype=torch.float32)),
                         ("dW ([h|1]^T@d)^T", lambda: torch.mm(haug.t(), d, out_dtype=torch.float32))):
            t = timeit(fn, n=10)
            res[name] = {"ms": round(t, 3), "tflops": round(f / t / 1e9, 1)}
        print(json.dumps(res), flush=True)
        return
    if os.environ.get("FWD_ONLY") == "1":  # variant A/B: the fused kernels alone
        t = timeit(lambda: H.actor_head_bf16_fwd(hb, wb, b, V, A, bits, act), n=10)
        r = min(B, 70144)
        dl = torch.empty((r, N), dtype=torch.bfloat16, device=dev)
        tb = timeit(lambda: H.actor_head_bf16_bwd(hb[:r], wb, b, V, A, bits[:r], act[:r], glp[:r],
                                                  gen[:r], dl), n=10)
        db = torch.zeros((N,), dtype=torch.float32, device=dev)
        ws = torch.empty((H.bf16_bwd_workspace(r, V, A),), dtype=torch.float32, device=dev)
        tbd = timeit(lambda: H.actor_head_bf16_bwd(hb[:r], wb, b, V, A, bits[:r], act[:r],
                                                   glp[:r], gen[:r], dl, dbias=db, workspace=ws),
                     n=10)
        ones = torch.ones((1, r), dtype=torch.bfloat16, device=dev)
        tg = timeit(lambda: torch.mm(ones, dl, out_dtype=torch.float32), n=10)
        print(json.dumps({"lib": os.environ.get("VMP_LIB_PATH", "default").split("/")[-1],
                          "fused_fwd_ms": t, "fused_fwd_tflops": flop / t / 1e9,
                          "bwd_ms_per_204800": tb * B / r,
                          "bwd_with_dbias_ms_per_204800": tbd * B / r,
                          "db_gemv_ms_per_204800": tg * B / r,
                          "bwd_tflops": 2.0 * r * K * N / tb / 1e9}), flush=True)
        return
    # hipBLASLt on the same GEMM: f32 logits out (what the logits path writes), bf16 out
    lg = torch.empty((B, N), dtype=torch.float32, device=dev)
    t = timeit(lambda: torch.mm(hb, wb.t(), out_dtype=torch.float32, out=lg))
    out["hipblaslt_f32out_ms"] = t
    out["hipblaslt_f32out_tflops"] = flop / t / 1e9
    del lg
    lg = torch.empty((B, N), dtype=torch.bfloat16, device=dev)
    t = timeit(lambda: torch.mm(hb, wb.t(), out=lg))
    out["hipblaslt_bf16out_ms"] = t
    out["hipblaslt_bf16out_tflops"] = flop / t / 1e9
    del lg
    torch.cuda.empty_cache()
    t = timeit(lambda: H.actor_head_bf16_fwd(hb, wb, b, V, A, bits, act))
    out["fused_fwd_ms"] = t
    out["fused_fwd_tflops"] = flop / t / 1e9
    rows = (1 << 32) // (2 * N) // 256 * 256
    dl = torch.empty((rows, N), dtype=torch.bfloat16, device=dev)
    r = min(rows, B)
    t = timeit(lambda: H.actor_head_bf16_bwd(hb[:r], wb, b, V, A, bits[:r], act[:r], glp[:r],
                                             gen[:r], dl))
    out["fused_bwd_kernel_ms_per_chunk"] = t
    out["fused_bwd_kernel_tflops"] = 2.0 * r * K * N / t / 1e9
    out["chunk_rows"] = r

    def fused_full():
        x = h.detach().requires_grad_(True)
        ww = w.detach().requires_grad_(True)
        bb = b.detach().requires_grad_(True)
        lp, ent = BF16FusedActorHead.apply(x, ww, bb, bits, act, V, A, rows)
        torch.autograd.backward([lp, ent], [glp, gen])

    def logits_full():
        x = h.detach().requires_grad_(True)
        ww = w.detach().requires_grad_(True)
        bb = b.detach().requires_grad_(True)
        lp, ent = BF16ActorHead.apply(x, ww, bb, bits, act, V, A)
        torch.autograd.backward([lp, ent], [glp, gen])

    torch.cuda.reset_peak_memory_stats()
    t = timeit(fused_full, n=3, warm=1)
    out["fused_fwd_bwd_ms"] = t
    out["fused_fwd_bwd_tflops_useful"] = 3 * flop / t / 1e9
    out["fused_peak_gb"] = torch.cuda.max_memory_allocated() / 1e9
    del dl
    torch.cuda.empty_cache()
    if os.environ.get("SKIP_LOGITS") != "1":
        torch.cuda.reset_peak_memory_stats()
        t = timeit(logits_full, n=3, warm=1)
        out["logits_fwd_bwd_ms"] = t
        out["logits_fwd_bwd_tflops_useful"] = 3 * flop / t / 1e9
        out["logits_peak_gb"] = torch.cuda.max_memory_allocated() / 1e9
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
