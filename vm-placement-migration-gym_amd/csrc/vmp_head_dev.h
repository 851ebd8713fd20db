// vmp_head_dev.h — per-row device code of the masked multi-categorical head
// (src/agents/ppo.py:115-131 Network.get_action / get_det_action and the
// PPOAgent.act WAIT coin, ppo.py:151-156), shared by the tiled head kernel
// (vmp_policy.hip k_head_fwd_tile) and the one-launch actor MLP + head
// (vmp_mlp.hip), so equal logits give equal actions, log-probabilities and
// entropies bit for bit on both paths.
//
// Quad layout: the 4 lanes of a quad (c = lane % 4) share one (sample, VM)
// row and take elements j = c + 4k; row reductions are two quad shuffles.
// Row pointers are generic (the callers' rows live in LDS).
#ifndef VMP_HEAD_DEV_H
#define VMP_HEAD_DEV_H

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/vmp.h"

namespace vmp {
namespace hd {

constexpr float kMaskedLogit = -1e7f;  // ppo.py:119 `logits[invalid_mask] = -1e7`

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// Counter-based uniform in [0, 1) with 24 random bits: stream (seed, ctr).
__device__ __forceinline__ float uniform_at(uint64_t seed, uint64_t ctr) {
  uint64_t h = mix64(seed ^ mix64(ctr));
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}
// Seed of a launch: with a device counter (captured graphs replay the same
// arguments) the counter's current value is mixed in.
__device__ __forceinline__ uint64_t eff_seed(uint64_t seed, const uint64_t *ctr) {
  return ctr ? seed ^ mix64(*ctr + 0x5851F42D4C957F2Dull) : seed;
}

__device__ __forceinline__ float qmax(float x) {
  x = fmaxf(x, __shfl_xor(x, 1));
  return fmaxf(x, __shfl_xor(x, 2));
}
__device__ __forceinline__ float qsum(float x) {
  x += __shfl_xor(x, 1);
  return x + __shfl_xor(x, 2);
}

// The row's invalid-action bits (bits u32[rows][W], W = ceil(A/32) <= 4), bits
// past A cleared; no mask: all valid.
__device__ __forceinline__ void mask_words(const uint32_t *bits, int W, int A, int64_t row,
                                           uint32_t (&mw)[4]) {
#pragma unroll
  for (int w = 0; w < 4; w++) mw[w] = 0u;
  if (!bits) return;
  const uint32_t *mb = bits + row * W;
#pragma unroll
  for (int w = 0; w < 4; w++)
    if (w < W) mw[w] = mb[w];
  const int tail = A - 32 * (W - 1);  // bits past A are ignored
#pragma unroll
  for (int w = 0; w < 4; w++)
    if (w == W - 1 && tail < 32) mw[w] &= (1u << tail) - 1u;
}

__device__ __forceinline__ bool bit_of(const uint32_t (&mw)[4], int j) {
  const uint32_t w = j < 32 ? mw[0] : (j < 64 ? mw[1] : (j < 96 ? mw[2] : mw[3]));
  return (w >> (j & 31)) & 1u;
}

// WAIT coin flip of PPOAgent.act (ppo.py:154-156): more than one invalid
// action, WAIT (column wait_index) valid and rand() > ratio -> the column to
// forbid, else -1. seed: the launch's effective seed.
__device__ __forceinline__ int coin_flip(float wait_ratio, int wait_index, bool has_bits,
                                         uint64_t seed, uint64_t offset, int64_t row,
                                         const uint32_t (&mw)[4]) {
  if (!(wait_ratio >= 0.f) || !has_bits) return -1;
  int cnt = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) cnt += __popc(mw[w]);
  const bool wait_bad = bit_of(mw, wait_index);
  if (cnt > 1 && !wait_bad && uniform_at(seed ^ 0xC0FFEE5EEDull, offset + (uint64_t)row) > wait_ratio)
    return wait_index;
  return -1;
}

struct RowStats {
  float m, S, lse, H;
};
// Pass 1 writes the masked row back (-1e7 at invalid entries, ppo.py:119) and
// finds the max; pass 2 sums p = exp(x - m) and p*x.
__device__ __forceinline__ RowStats quad_row_stats(float *row, const uint32_t (&mw)[4], int A,
                                                   int c, int fw) {
  float m = -INFINITY;
  for (int j = c; j < A; j += 4) {
    float x = row[j];
    if (bit_of(mw, j) || j == fw) {
      x = kMaskedLogit;
      row[j] = x;
    }
    m = fmaxf(m, x);
  }
  m = qmax(m);
  float S = 0.f, T = 0.f;
  for (int j = c; j < A; j += 4) {
    const float x = row[j];
    const float p = __expf(x - m);
    S += p;
    T += p * x;
  }
  S = qsum(S);
  T = qsum(T);
  RowStats r;
  r.m = m;
  r.S = S;
  r.lse = m + logf(S);
  r.H = r.lse - T / S;
  return r;
}

// get_det_action: unmasked, first max (NaN never wins)
__device__ __forceinline__ int quad_argmax(const float *row, int A, int c) {
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int j = c; j < A; j += 4) {
    const float x = row[j];
    if (x == x && (x > best || bi == 0x7fffffff)) {
      best = x;
      bi = j;
    }
  }
#pragma unroll
  for (int o = 1; o < 4; o <<= 1) {
    const float ob = __shfl_xor(best, o);
    const int oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  return bi == 0x7fffffff ? 0 : bi;
}

// SAMPLE: inverse CDF over the masked row (after quad_row_stats) in lane-major
// order with the row's uniform u (the same value on the 4 lanes).
__device__ __forceinline__ int quad_sample(const float *row, const RowStats &st, int A, int c,
                                           float u) {
  float t = 0.f;
  for (int j = c; j < A; j += 4) t += __expf(row[j] - st.m);
  float incl = t + __shfl_up(t, 1, 4) * (c >= 1);
  incl += __shfl_up(incl, 2, 4) * (c >= 2);
  const float excl = incl - t;  // per-lane range [excl, incl) of the quad total
  const float total = __shfl(incl, 3, 4);
  const float target = u * total;
  int pick = -1, last = -1;
  float cum = excl;
  for (int j = c; j < A; j += 4) {
    const float p = __expf(row[j] - st.m);
    if (p > 0.f) {
      cum += p;
      last = j;
      if (pick < 0 && target >= excl && target < cum) pick = j;
    }
  }
  if (pick < 0 && last >= 0 && target >= excl && target < incl) pick = last;
  // lane-major order: the last lane of the quad whose range starts <= target
  int any = pick;
#pragma unroll
  for (int o = 1; o < 4; o <<= 1) any = max(any, __shfl_xor(any, o));
  if (any < 0) {  // target past the rounded total: last positive entry
    int lk = last >= 0 ? c * 1024 + last : -1;
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) lk = max(lk, __shfl_xor(lk, o));
    any = lk & 1023;
  } else {  // more than one lane can claim only through rounding: lowest lane wins
    int mine = pick >= 0 ? c : 4;
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) mine = min(mine, __shfl_xor(mine, o));
    any = __shfl(pick, mine, 4);
  }
  return any;
}

// ---- the same row code for ONE lane (no shuffles) -------------------------
// A single-lane restatement of quad_row_stats + quad_sample / quad_argmax:
// lane c's partial sums over its elements j = c, c + 4, ... are formed in the
// same order, and the quad shuffles' combinations are evaluated explicitly
// ((S0 + S1) + (S2 + S3), the shfl_up prefix incl_c, excl_c = incl_c - t_c,
// the lowest claiming lane), so the results are the quad code's bit for bit
// (vmp_mlp.hip's fused head runs one row per lane: ~4x fewer dependent
// shuffle round trips per workgroup than 4 rows per quad).
struct LaneRow {
  int act;
  float lp, H;
};
// mode: VMP_HEAD_SAMPLE (u: the row's uniform), VMP_HEAD_GIVEN (given: the
// action), VMP_HEAD_ARGMAX (stats not formed). fw: coin_flip's column or -1.
// AMAX > 0 (A <= AMAX): the masked row and its exp(x - m) are held in
// registers and every loop is unrolled to AMAX with a j < A guard (no LDS
// re-reads, exp once per element); AMAX = 0: any A, every pass re-reads the
// row. Both evaluate the same expressions in the same order.
// for (j = j0; j < A; j += 4) f(j): unrolled to AMAX (with the j < A guard)
// when AMAX > 0, a plain loop otherwise.
template <int AMAX, int STEP, class F>
__device__ __forceinline__ void each_j(int j0, int A, F &&f) {
  if constexpr (AMAX > 0) {
#pragma unroll
    for (int j = j0; j < AMAX; j += STEP)
      if (j < A) f(j);
  } else {
    for (int j = j0; j < A; j += STEP) f(j);
  }
}

template <int AMAX = 0>
__device__ __forceinline__ LaneRow lane_row(const float *row, const uint32_t (&mw)[4], int A,
                                            int fw, int mode, float u, int given) {
  constexpr bool R = AMAX > 0;
  constexpr int NR = R ? AMAX : 1;
  float xr[NR], pr[NR];
  auto xm_mem = [&](int j) { return (bit_of(mw, j) || j == fw) ? kMaskedLogit : row[j]; };
  if (R) {
#pragma unroll
    for (int j = 0; j < NR; j++) xr[j] = j < A ? xm_mem(j) : 0.f;
  }
  LaneRow o;
  o.lp = 0.f;
  o.H = 0.f;
  if (mode == VMP_HEAD_ARGMAX) {  // unmasked
    float best = -INFINITY;
    int bi = 0x7fffffff;
    each_j<AMAX, 1>(0, A, [&](int j) {
      const float x = row[j];
      if (x == x && (x > best || bi == 0x7fffffff)) {
        best = x;
        bi = j;
      }
    });
    o.act = bi == 0x7fffffff ? 0 : bi;
    return o;
  }
  float m = -INFINITY;  // max: exact in any order
  each_j<AMAX, 1>(0, A, [&](int j) { m = fmaxf(m, R ? xr[j] : xm_mem(j)); });
  float Sc[4], Tc[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    float S = 0.f, T = 0.f;
    each_j<AMAX, 4>(c, A, [&](int j) {
      const float x = R ? xr[j] : xm_mem(j);
      const float p = __expf(x - m);
      if (R) pr[j] = p;
      S += p;
      T += p * x;
    });
    Sc[c] = S;
    Tc[c] = T;
  }
  const float S = (Sc[0] + Sc[1]) + (Sc[2] + Sc[3]);  // qsum
  const float T = (Tc[0] + Tc[1]) + (Tc[2] + Tc[3]);
  const float lse = m + logf(S);
  o.H = lse - T / S;
  int act = given;
  if (mode == VMP_HEAD_SAMPLE) {
    float t[4], incl[4], excl[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      t[c] = 0.f;
      each_j<AMAX, 4>(c, A, [&](int j) { t[c] += R ? pr[j] : __expf(xm_mem(j) - m); });
    }
    // incl = t + shfl_up(t, 1) * (c >= 1); incl += shfl_up(incl, 2) * (c >= 2)
    float i1[4];
#pragma unroll
    for (int c = 0; c < 4; c++) i1[c] = t[c] + (c >= 1 ? t[c - 1] : t[c]) * (float)(c >= 1);
#pragma unroll
    for (int c = 0; c < 4; c++) incl[c] = i1[c] + (c >= 2 ? i1[c - 2] : i1[c]) * (float)(c >= 2);
#pragma unroll
    for (int c = 0; c < 4; c++) excl[c] = incl[c] - t[c];
    const float target = u * incl[3];
    int pick[4], last[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      pick[c] = -1;
      last[c] = -1;
      float cum = excl[c];
      each_j<AMAX, 4>(c, A, [&](int j) {
        const float p = R ? pr[j] : __expf(xm_mem(j) - m);
        if (p > 0.f) {
          cum += p;
          last[c] = j;
          if (pick[c] < 0 && target >= excl[c] && target < cum) pick[c] = j;
        }
      });
      if (pick[c] < 0 && last[c] >= 0 && target >= excl[c] && target < incl[c]) pick[c] = last[c];
    }
    const int any = max(max(pick[0], pick[1]), max(pick[2], pick[3]));
    if (any < 0) {  // target past the rounded total: last positive entry
      int lk = -1;
#pragma unroll
      for (int c = 0; c < 4; c++) lk = max(lk, last[c] >= 0 ? c * 1024 + last[c] : -1);
      act = lk & 1023;
    } else {  // the lowest claiming lane
      act = pick[0] >= 0 ? pick[0] : pick[1] >= 0 ? pick[1] : pick[2] >= 0 ? pick[2] : pick[3];
    }
  }
  o.act = act;
  if (act >= 0 && act < A) {
    float xa = 0.f;
    if (R) {
#pragma unroll
      for (int j = 0; j < NR; j++) xa = j == act ? xr[j] : xa;
    } else {
      xa = xm_mem(act);
    }
    o.lp = xa - lse;
  } else {
    o.lp = NAN;
  }
  return o;
}

}  // namespace hd
}  // namespace vmp

#endif  // VMP_HEAD_DEV_H
