"""PPO legs: FLOP-based matrix utilisation vs the PMC MFMA-busy of the same
profiled run, on one time base (the run's summed kernel time).
  FLOP side: bench.py's GEMM-shape FLOPs of the profiled work / kernel time / peak
  PMC side:  sum SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel time x clock)
Usage: python tools/ppo_pmc_reconcile.py [profiles/r04_final_ppo_{f32,bf16,eval}_summary.json dir prefix]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

CLOCK = 2.4e9  # MI355X_MICROARCH.md: the peaks are quoted at this clock


def main():
    pre = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r04_final_ppo_")
    # the profiled runs: one collect + one update at 8 192 envs (tools/bench_ppo.py
    # --updates 1 --warmup 0); the eval run's batched steps (tools/prof_ppo_eval.py)
    D, H, VA, T, E = 3 * 300 + 2 * 100, 512, 300 * 102, 100, 8192
    col, upd = bench.ppo_update_flops(D, H, VA, T, E, 16, 25)
    # the fused bf16 head's logits recompute: one more forward of the last
    # layer per evaluated sample (16 minibatches x 25 x 8 192)
    rec = 16 * 25 * E * 2.0 * H * VA
    f32p, bf16p = bench.F32_MFMA_PEAK_TFLOPS * 1e12, bench.BF16_MFMA_PEAK_TFLOPS * 1e12
    cases = {"f32": (col + upd, f32p), "bf16": (col + upd + rec, bf16p)}
    out = {}
    for p in ("f32", "bf16", "eval"):
        d = json.load(open(pre + p + "_summary.json"))
        kt = d["kernel_ms_total"] * 1e-3
        busy = sum(v["SQ_VALU_MFMA_BUSY_CYCLES"] for v in d["pmc"].values())
        if p == "eval":
            steps = int(os.environ.get("EVAL_STEPS", "213"))  # k_env dispatches of the run
            # config/10.yml actor forward per env-step, 4 096 envs per step
            flops, peak = steps * 4096 * bench.mlp_flops([110, 512, 512, 360]), f32p
        else:
            flops, peak = cases[p]
        f = flops / kt / peak
        m = busy / (1024 * kt * CLOCK)
        out[p] = {"kernel_s": kt, "flops": flops, "flop_util": f, "pmc_util": m,
                  "rel_diff": abs(f - m) / m}
        print(f"{p:5s} kernel {kt * 1e3:8.1f} ms  FLOP util {f:.3f}  PMC MFMA busy {m:.3f}  "
              f"rel diff {abs(f - m) / m:.1%}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
