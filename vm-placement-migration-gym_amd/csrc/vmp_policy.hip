// vmp_policy.hip — gfx950 kernels for the PPO side of the path
// (src/agents/ppo.py): the masked multi-categorical actor head of
// Network.get_action / get_det_action (ppo.py:115-131) forward and backward,
// the PPOAgent.act WAIT coin flips (ppo.py:154-156), and the GAE reverse scan
// of PPOAgent.update (ppo.py:232-243).
//
// Head layout: logits f32 [B][V][A] (the actor's last Linear output, row-major
// [B, V*A] exactly as ppo.py:116 produces it), invalid-action bits u32
// [B][V][W] (W = ceil(A/32), bit set = invalid, the layout vmp_mask writes).
// One workgroup per sample b; its lanes form groups of G lanes, one group per
// (b, v) row at a time; lane g of a group holds elements j = g + G*e (e < E) of
// the row in registers, so each wave load reads G consecutive floats per row
// and 64/G adjacent rows (coalesced, every byte read once). Row reductions are
// xor shuffles inside the group; the per-sample sums over V (ppo.py:124-125)
// are a fixed-order block reduction (deterministic, no atomics).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/vmp.h"
#include "vmp_head_dev.h"

namespace vmp {

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

template <int G>
__device__ __forceinline__ float gsum(float x) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}
template <int G>
__device__ __forceinline__ float gmax(float x) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
  return x;
}
template <int G>
__device__ __forceinline__ int gmaxi(int x) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o));
  return x;
}

struct HeadArgs {
  int B, V, A, W, mode, wait_index;
  float wait_ratio;
  uint64_t seed, offset;
  const uint64_t *ctr;   // nullable device counter mixed into the seed (graph replays)
  const float *logits;
  const uint32_t *bits;
  int32_t *action;       // in (GIVEN) or out (SAMPLE / ARGMAX), [B][V]
  float *logprob;        // [B] (nullable)
  float *entropy;        // [B] (nullable)
  const float *g_logprob, *g_entropy;  // backward: dL/dlogprob[B], dL/dentropy[B]
  float *dlogits;        // backward output [B][V][A] (may alias logits)
  uint16_t *dlogits_bf16;  // or: bf16 backward output [B][V][A] (tiles only)
  float *row_lp, *row_ent;  // tiled kernels: per-row results [B*V]
};

// Seed of this launch: with a device counter (captured graphs replay the same
// arguments) the counter's current value is mixed in.
__device__ __forceinline__ uint64_t eff_seed(const HeadArgs &a) {
  return a.ctr ? a.seed ^ mix64(*a.ctr + 0x5851F42D4C957F2Dull) : a.seed;
}

// Loads one row into registers with the mask applied and, for SAMPLE/GIVEN,
// the WAIT coin flip of PPOAgent.act (ppo.py:154-156):
//   count_nonzero(invalid[row]) > 1 and not invalid[row, P] and rand() > ratio
//   -> invalid[row, P] = True.
template <int G, int E>
__device__ __forceinline__ void load_row(const HeadArgs &a, int64_t row, int g, float (&x)[E],
                                         float (&raw)[E], bool flip_wait) {
  const float *lg = a.logits + row * a.A;
  const uint32_t *mb = a.bits ? a.bits + row * a.W : nullptr;
  bool forbid_wait = false;
  if (mb && flip_wait) {
    int cnt = 0;
    for (int w = 0; w < a.W; w++) {
      uint32_t word = mb[w];
      int lo = w * 32;
      if (a.A - lo < 32) word &= (1u << (a.A - lo)) - 1u;
      cnt += __popc(word);
    }
    int P = a.wait_index;
    bool wait_bad = (mb[P >> 5] >> (P & 31)) & 1u;
    if (cnt > 1 && !wait_bad)
      forbid_wait = uniform_at(eff_seed(a) ^ 0xC0FFEE5EEDull, a.offset + (uint64_t)row) > a.wait_ratio;
  }
#pragma unroll
  for (int e = 0; e < E; e++) {
    int j = g + G * e;
    float v = -INFINITY, r = -INFINITY;
    if (j < a.A) {
      r = v = lg[j];
      if (mb && (((mb[j >> 5] >> (j & 31)) & 1u) || (forbid_wait && j == a.wait_index)))
        v = kMaskedLogit;
    }
    x[e] = v;
    raw[e] = r;
  }
}

// Softmax statistics of a register-resident row: p[e] = exp(x - max),
// S = sum p, lse = max + log S, H = -sum (p/S)(x - lse) (Categorical.entropy).
template <int G, int E>
__device__ __forceinline__ void row_stats(const float (&x)[E], int g, int A, float (&p)[E],
                                          float &S, float &lse, float &H) {
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < E; e++)
    if (g + G * e < A) mx = fmaxf(mx, x[e]);
  mx = gmax<G>(mx);
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < E; e++) {
    p[e] = (g + G * e < A) ? expf(x[e] - mx) : 0.f;
    s += p[e];
  }
  S = gsum<G>(s);
  lse = mx + logf(S);
  float inv = 1.0f / S, h = 0.f;
#pragma unroll
  for (int e = 0; e < E; e++)
    if (p[e] > 0.f) h += (p[e] * inv) * (x[e] - lse);
  H = -gsum<G>(h);
}

// Inverse-CDF draw over the row in lane-major order (lane g's E elements, then
// lane g+1's ...): any fixed order of the categories samples the same law.
template <int G, int E>
__device__ __forceinline__ int sample_row(const float (&p)[E], int g, int A, float u) {
  float t = 0.f;
#pragma unroll
  for (int e = 0; e < E; e++) t += p[e];
  float incl = t;
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    float y = __shfl_up(incl, o, G);
    if (g >= o) incl += y;
  }
  float excl = __shfl_up(incl, 1, G);
  if (g == 0) excl = 0.f;
  float total = __shfl(incl, G - 1, G);
  float target = u * total;
  int pick = -1, last = -1;
  float c = excl;
#pragma unroll
  for (int e = 0; e < E; e++) {
    if (p[e] > 0.f) {
      c += p[e];
      last = g * E + e;
      if (pick < 0 && target >= excl && target < incl && target < c) pick = g + G * e;
    }
  }
  if (pick < 0 && t > 0.f && target >= excl && target < incl) pick = g + G * ((last - g * E));
  int any = gmaxi<G>(pick);
  if (any >= 0) return any;
  // target fell past the rounded total: take the last positive category
  int lk = gmaxi<G>(last);
  int lg = lk / E, le = lk - lg * E;
  return lg + G * le;
}

// Block-wide fixed-order sum of one value per group leader; result in thread 0.
template <int G>
__device__ __forceinline__ float block_sum_groups(float v, float *lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o >= G; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) s += lds[w];
  return s;
}

// Forward: mode VMP_HEAD_SAMPLE draws action[b][v]; VMP_HEAD_GIVEN reads it;
// both write logprob[b] = sum_v log_softmax(masked)[a] and entropy[b] =
// sum_v H_v (ppo.py:117-126). VMP_HEAD_ARGMAX is get_det_action (ppo.py:128-131):
// argmax of the UNMASKED row, first index on ties (torch.argmax).
template <int G, int E>
__global__ __launch_bounds__(256) void k_head_fwd(HeadArgs a) {
  __shared__ float lds[2][4];
  const int b = blockIdx.x;
  const int g = threadIdx.x & (G - 1);
  const int grp = threadIdx.x / G, ngrp = blockDim.x / G;
  const bool sample = a.mode == VMP_HEAD_SAMPLE, argmax = a.mode == VMP_HEAD_ARGMAX;
  const bool flip = a.wait_ratio >= 0.f && !argmax;
  float lp_acc = 0.f, ent_acc = 0.f;
  for (int v = grp; v < a.V; v += ngrp) {
    const int64_t row = (int64_t)b * a.V + v;
    float x[E], raw[E], p[E];
    load_row<G, E>(a, row, g, x, raw, flip);
    if (argmax) {
      float best = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int e = 0; e < E; e++) {  // strict > keeps the first index of a tie
        int j = g + G * e;
        if (j < a.A && raw[e] == raw[e] && (raw[e] > best || bi == 0x7fffffff)) {
          best = raw[e];
          bi = j;
        }
      }
#pragma unroll
      for (int o = G / 2; o > 0; o >>= 1) {
        float ob = __shfl_xor(best, o);
        int oi = __shfl_xor(bi, o);
        if (ob > best || (ob == best && oi < bi)) {
          best = ob;
          bi = oi;
        }
      }
      if (g == 0) a.action[row] = bi == 0x7fffffff ? 0 : bi;
      continue;
    }
    float S, lse, H;
    row_stats<G, E>(x, g, a.A, p, S, lse, H);
    int act;
    if (sample) {
      act = sample_row<G, E>(p, g, a.A, uniform_at(eff_seed(a), a.offset + (uint64_t)row));
      if (g == 0) a.action[row] = act;
    } else {
      act = a.action[row];
    }
    float xa = 0.f;
#pragma unroll
    for (int e = 0; e < E; e++)
      if (g + G * e == act) xa = x[e];
    xa = gsum<G>(xa);
    float lp = (act >= 0 && act < a.A) ? xa - lse : NAN;
    lp_acc += lp;
    ent_acc += H;
  }
  if (argmax) return;
  // one value per group (all lanes of a group agree); count each group once
  float lp_v = (g == 0) ? lp_acc : 0.f, en_v = (g == 0) ? ent_acc : 0.f;
  float lp_s = block_sum_groups<G>(lp_v, lds[0]);
  float en_s = block_sum_groups<G>(en_v, lds[1]);
  if (threadIdx.x == 0) {
    if (a.logprob) a.logprob[b] = lp_s;
    if (a.entropy) a.entropy[b] = en_s;
  }
}

// Backward of (logprob, entropy) w.r.t. the pre-mask logits:
//   d/dz_j = g_lp (1[j=a] - q_j) - g_ent q_j (log q_j + H),  q = softmax(masked z),
// and 0 at masked entries (the in-place `logits[mask] = -1e7` of ppo.py:119
// passes no gradient there). Recomputes the row statistics from the logits.
template <int G, int E>
__global__ __launch_bounds__(256) void k_head_bwd(HeadArgs a) {
  const int b = blockIdx.x;
  const int g = threadIdx.x & (G - 1);
  const int grp = threadIdx.x / G, ngrp = blockDim.x / G;
  const float glp = a.g_logprob ? a.g_logprob[b] : 0.f;
  const float gen = a.g_entropy ? a.g_entropy[b] : 0.f;
  for (int v = grp; v < a.V; v += ngrp) {
    const int64_t row = (int64_t)b * a.V + v;
    float x[E], raw[E], p[E];
    load_row<G, E>(a, row, g, x, raw, false);
    float S, lse, H;
    row_stats<G, E>(x, g, a.A, p, S, lse, H);
    const int act = a.action[row];
    const uint32_t *mb = a.bits ? a.bits + row * a.W : nullptr;
    float *d = a.dlogits + row * a.A;
    const float inv = 1.0f / S;
#pragma unroll
    for (int e = 0; e < E; e++) {
      int j = g + G * e;
      if (j < a.A) {
        bool masked = mb && ((mb[j >> 5] >> (j & 31)) & 1u);
        float q = p[e] * inv;
        float l = x[e] - lse;
        float gj = glp * ((j == act ? 1.f : 0.f) - q);
        if (q > 0.f) gj -= gen * q * (l + H);
        d[j] = masked ? 0.f : gj;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Tiled row kernels (A <= kTileMaxA, the 10.yml / 100.yml shapes): one
// 256-thread block per tile of 64 consecutive (b, v) rows, a quad of lanes per
// row. The tile (64*A floats, contiguous in HBM) is copied into LDS by the
// block with 16-B loads (fully coalesced, every byte read once), then each
// quad runs its row out of LDS. Row statistics follow
// Categorical(logits=masked) exactly as the group kernels: lse = m + log S
// rounded in f32, l_j = x_j - lse, logprob = l_a, entropy = -sum q_j l_j
// = lse - (sum p_j x_j)/S. Per-row results go to a row buffer; k_rowsum adds
// them per sample in a fixed order (deterministic).
constexpr int kTileMaxA = 128;

// The whole block copies the tile once (thread t takes float4 t, t + 256, ...).
__device__ __forceinline__ void tile_load(const float *src, float *lds, int n) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int n4 = n >> 2;
  const float4 *s4 = reinterpret_cast<const float4 *>(src);
  float4 *d4 = reinterpret_cast<float4 *>(lds);
  for (int i = t; i < n4; i += nt) d4[i] = s4[i];
  for (int i = (n4 << 2) + t; i < n; i += nt) lds[i] = src[i];
}
__device__ __forceinline__ void tile_store(float *dst, const float *lds, int n) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int n4 = n >> 2;
  const float4 *s4 = reinterpret_cast<const float4 *>(lds);
  float4 *d4 = reinterpret_cast<float4 *>(dst);
  for (int i = t; i < n4; i += nt) d4[i] = s4[i];
  for (int i = (n4 << 2) + t; i < n; i += nt) dst[i] = lds[i];
}

// f32 tile -> bf16 rows (round to nearest even, v_cvt_pk_bf16_f32), 8-B stores
__device__ __forceinline__ void tile_store_bf16(uint16_t *dst, const float *lds, int n) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int n4 = n >> 2;
  const float4 *s4 = reinterpret_cast<const float4 *>(lds);
  for (int i = t; i < n4; i += nt) {
    const float4 v = s4[i];
    const __bf16 h[4] = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    uint2 u;
    __builtin_memcpy(&u, h, 8);
    reinterpret_cast<uint2 *>(dst)[i] = u;
  }
  for (int i = (n4 << 2) + t; i < n; i += nt) {
    const __bf16 h = (__bf16)lds[i];
    __builtin_memcpy(dst + i, &h, 2);
  }
}

// Quad layout inside a tile: wave w owns rows 16w..16w+15, lane l works on
// row 16w + l/4 with the 4 lanes of its quad taking elements j = c + 4k
// (c = l%4): row reductions are 2 quad shuffles (DPP), per-lane work is A/4.
// The per-row code (mask, WAIT coin, stats, draw) is vmp_head_dev.h's, shared
// with the one-launch actor MLP + head (vmp_mlp.hip).

template <int ROWS>
__device__ __forceinline__ void tile_rows(int64_t &r0, int &nr) {
  const int64_t rows = r0;  // caller passes total rows in r0
  r0 = (int64_t)blockIdx.x * ROWS;
  nr = (int)min((int64_t)ROWS, rows - r0);
}

// Forward over a tile of 64 rows (256 threads): per-row logprob / entropy to
// a.row_lp / a.row_ent; SAMPLE draws by inverse CDF in lane-major order.
__global__ __launch_bounds__(256) void k_head_fwd_tile(HeadArgs a) {
  extern __shared__ __align__(16) float tl[];
  int64_t r0 = (int64_t)a.B * a.V;
  int nr;
  tile_rows<64>(r0, nr);
  tile_load(a.logits + r0 * a.A, tl, nr * a.A);
  __syncthreads();
  const int lr = threadIdx.x >> 2, c = threadIdx.x & 3;
  if (lr >= nr) return;  // whole quads leave together
  const int64_t row = r0 + lr;
  float *rp = tl + lr * a.A;
  if (a.mode == VMP_HEAD_ARGMAX) {  // get_det_action: unmasked, first max
    const int bi = hd::quad_argmax(rp, a.A, c);
    if (c == 0) a.action[row] = bi;
    return;
  }
  uint32_t mw[4];
  hd::mask_words(a.bits, a.W, a.A, row, mw);
  const uint64_t seed = eff_seed(a);
  const int fw = hd::coin_flip(a.wait_ratio, a.wait_index, a.bits != nullptr, seed, a.offset, row,
                               mw);
  const hd::RowStats st = hd::quad_row_stats(rp, mw, a.A, c, fw);
  int act;
  if (a.mode == VMP_HEAD_SAMPLE) {
    act = hd::quad_sample(rp, st, a.A, c, hd::uniform_at(seed, a.offset + (uint64_t)row));
    if (c == 0) a.action[row] = act;
  } else {
    act = a.action[row];
  }
  if (c == 0) {
    const float lp = (act >= 0 && act < a.A) ? rp[act] - st.lse : NAN;
    a.row_lp[row] = lp;
    a.row_ent[row] = st.H;
  }
}

// Backward over a tile: d/dz_j of (g_lp * logprob + g_ent * entropy)
//   = -q_j (g_lp + g_ent (x_j - lse + H)) + g_lp [j = a],  0 at masked j,
// written into the tile in place and streamed out with 16-B stores.
__global__ __launch_bounds__(256) void k_head_bwd_tile(HeadArgs a) {
  extern __shared__ __align__(16) float tl[];
  int64_t r0 = (int64_t)a.B * a.V;
  int nr;
  tile_rows<64>(r0, nr);
  tile_load(a.logits + r0 * a.A, tl, nr * a.A);
  __syncthreads();
  const int lr = threadIdx.x >> 2, c = threadIdx.x & 3;
  if (lr < nr) {
    const int64_t row = r0 + lr;
    float *rp = tl + lr * a.A;
    uint32_t mw[4];
    hd::mask_words(a.bits, a.W, a.A, row, mw);
    const hd::RowStats st = hd::quad_row_stats(rp, mw, a.A, c, -1);
    const int b = (int)(row / a.V);
    const float glp = a.g_logprob ? a.g_logprob[b] : 0.f;
    const float gen = a.g_entropy ? a.g_entropy[b] : 0.f;
    const int act = a.action[row];
    const float inv = 1.0f / st.S;
    const float c1 = glp + gen * (st.H - st.lse);
    for (int j = c; j < a.A; j += 4) {
      const float x = rp[j];
      const float q = __expf(x - st.m) * inv;
      float g = -q * fmaf(gen, x, c1);
      if (j == act) g += glp;
      rp[j] = hd::bit_of(mw, j) ? 0.f : g;
    }
  }
  __syncthreads();
  if (a.dlogits_bf16) tile_store_bf16(a.dlogits_bf16 + r0 * a.A, tl, nr * a.A);
  else tile_store(a.dlogits + r0 * a.A, tl, nr * a.A);
}

// Per-sample sums of the row results (ppo.py:124-125), fixed order: one wave per sample.
__global__ __launch_bounds__(256) void k_rowsum(int B, int V, const float *row_lp,
                                                const float *row_ent, float *lp, float *ent) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float s0 = 0.f, s1 = 0.f;
  for (int v = lane; v < V; v += 64) {
    s0 += row_lp[(int64_t)b * V + v];
    s1 += row_ent[(int64_t)b * V + v];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o);
    s1 += __shfl_xor(s1, o);
  }
  if (lane == 0) {
    if (lp) lp[b] = s0;
    if (ent) ent[b] = s1;
  }
}

// PPOAgent.update GAE (ppo.py:232-243): one lane per env column, reverse scan
// over T; f32 as the reference's rewards_batch / values.
__global__ void k_gae(int T, int N, const float *r, const float *d, const float *v,
                      const float *nv, float gamma, float lam, float *adv, float *ret) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float g = 0.f;
  for (int t = T - 1; t >= 0; t--) {
    int64_t i = (int64_t)t * N + n;
    float nd = 1.f - d[i];
    float delta = r[i] + nd * gamma * nv[i] - v[i];
    g = delta + nd * gamma * lam * g;
    adv[i] = g;
    ret[i] = g + v[i];
  }
}

}  // namespace vmp

// ------------------------------------------------------------ host dispatch
namespace {
using namespace vmp;

// groups of G lanes, E elements per lane: smallest G with A <= 16 G, then the
// smallest E in {4, 8, 16} covering ceil(A / G).
int pick_g(int A) { return A <= 64 ? 4 : (A <= 256 ? 16 : 64); }
int pick_e(int A, int G) {
  int need = (A + G - 1) / G;
  return need <= 4 ? 4 : (need <= 8 ? 8 : 16);
}
int block_threads(int V, int G) {
  int t = V * G;
  if (t <= 64) return 64;
  if (t <= 128) return 128;
  return 256;
}

#define VMP_HEAD_CASE(KERN, GG, EE)                                                      \
  if (G == GG && E == EE) {                                                              \
    hipLaunchKernelGGL((KERN<GG, EE>), dim3(a.B), dim3(block_threads(a.V, GG)), 0, st, a); \
    return hipGetLastError();                                                            \
  }
#define VMP_HEAD_ALL(KERN)                                                               \
  VMP_HEAD_CASE(KERN, 4, 4) VMP_HEAD_CASE(KERN, 4, 8) VMP_HEAD_CASE(KERN, 4, 16)         \
  VMP_HEAD_CASE(KERN, 16, 4) VMP_HEAD_CASE(KERN, 16, 8) VMP_HEAD_CASE(KERN, 16, 16)      \
  VMP_HEAD_CASE(KERN, 64, 4) VMP_HEAD_CASE(KERN, 64, 8) VMP_HEAD_CASE(KERN, 64, 16)

bool use_tiles(const HeadArgs &a) {
  return a.A <= kTileMaxA && ((uintptr_t)a.logits & 15) == 0 &&
         (!a.dlogits || ((uintptr_t)a.dlogits & 15) == 0);
}

hipError_t launch_fwd(const HeadArgs &a0, hipStream_t st) {
  if (use_tiles(a0)) {
    HeadArgs a = a0;
    const int64_t rows = (int64_t)a.B * a.V;
    const unsigned grid = (unsigned)((rows + 63) / 64);
    const size_t lds = (size_t)64 * a.A * sizeof(float);
    const bool need_sums = a.mode != VMP_HEAD_ARGMAX;
    float *scratch = nullptr;
    if (need_sums) {
      float *ws = a.row_lp;  // caller's workspace (2*B*V floats) if given
      if (!ws) {
        hipError_t e = hipMallocAsync((void **)&scratch, 2 * rows * sizeof(float), st);
        if (e != hipSuccess) return e;
        ws = scratch;
      }
      a.row_lp = ws;
      a.row_ent = ws + rows;
    }
    hipLaunchKernelGGL(k_head_fwd_tile, dim3(grid), dim3(256), lds, st, a);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && need_sums) {
      hipLaunchKernelGGL(k_rowsum, dim3((a.B + 3) / 4), dim3(256), 0, st, a.B, a.V, a.row_lp,
                         a.row_ent, a.logprob, a.entropy);
      e = hipGetLastError();
    }
    if (scratch) {
      hipError_t f = hipFreeAsync(scratch, st);
      if (e == hipSuccess) e = f;
    }
    return e;
  }
  const HeadArgs &a = a0;
  const int G = pick_g(a.A), E = pick_e(a.A, G);
  VMP_HEAD_ALL(k_head_fwd)
  return hipErrorInvalidValue;
}
hipError_t launch_bwd(const HeadArgs &a, hipStream_t st) {
  if (use_tiles(a)) {
    const int64_t rows = (int64_t)a.B * a.V;
    const unsigned grid = (unsigned)((rows + 63) / 64);
    const size_t lds = (size_t)64 * a.A * sizeof(float);
    hipLaunchKernelGGL(k_head_bwd_tile, dim3(grid), dim3(256), lds, st, a);
    return hipGetLastError();
  }
  const int G = pick_g(a.A), E = pick_e(a.A, G);
  VMP_HEAD_ALL(k_head_bwd)
  return hipErrorInvalidValue;
}
}  // namespace

namespace vmp {
// shared with vmp_capi.cpp's vmp_last_error()
int policy_fail(int code, const char *msg);
}

extern "C" {

int vmp_policy_head(int32_t B, int32_t V, int32_t A, int32_t mode, const float *logits,
                    const uint32_t *mask_bits, float wait_ratio, int32_t wait_index,
                    uint64_t seed, uint64_t offset, const uint64_t *rng_counter, int32_t *action,
                    float *logprob, float *entropy, float *workspace, void *stream) {
  if (B < 0 || V < 1 || A < 1 || A > VMP_HEAD_MAX_A || !logits || !action)
    return vmp::policy_fail(VMP_EINVAL, "vmp_policy_head: bad shape or null pointer");
  if (mode != VMP_HEAD_SAMPLE && mode != VMP_HEAD_GIVEN && mode != VMP_HEAD_ARGMAX)
    return vmp::policy_fail(VMP_EINVAL, "vmp_policy_head: unknown mode");
  if (wait_ratio >= 0.f && (!mask_bits || wait_index < 0 || wait_index >= A))
    return vmp::policy_fail(VMP_EINVAL, "vmp_policy_head: WAIT coin flips need the mask and 0 <= wait_index < A");
  if (B == 0) return VMP_OK;
  HeadArgs a{};
  a.B = B, a.V = V, a.A = A, a.W = (A + 31) / 32, a.mode = mode, a.wait_index = wait_index;
  a.wait_ratio = wait_ratio, a.seed = seed, a.offset = offset, a.ctr = rng_counter;
  a.row_lp = workspace;
  a.logits = logits, a.bits = mask_bits, a.action = action, a.logprob = logprob,
  a.entropy = entropy;
  hipError_t e = launch_fwd(a, (hipStream_t)stream);
  if (e != hipSuccess) return vmp::policy_fail(VMP_EDEVICE, hipGetErrorString(e));
  return VMP_OK;
}

int vmp_policy_head_backward(int32_t B, int32_t V, int32_t A, const float *logits,
                             const uint32_t *mask_bits, const int32_t *action,
                             const float *g_logprob, const float *g_entropy, float *dlogits,
                             void *stream) {
  if (B < 0 || V < 1 || A < 1 || A > VMP_HEAD_MAX_A || !logits || !action || !dlogits)
    return vmp::policy_fail(VMP_EINVAL, "vmp_policy_head_backward: bad shape or null pointer");
  if (B == 0) return VMP_OK;
  HeadArgs a{};
  a.B = B, a.V = V, a.A = A, a.W = (A + 31) / 32, a.mode = VMP_HEAD_GIVEN, a.wait_index = -1;
  a.wait_ratio = -1.f;
  a.logits = logits, a.bits = mask_bits, a.action = const_cast<int32_t *>(action);
  a.g_logprob = g_logprob, a.g_entropy = g_entropy, a.dlogits = dlogits;
  hipError_t e = launch_bwd(a, (hipStream_t)stream);
  if (e != hipSuccess) return vmp::policy_fail(VMP_EDEVICE, hipGetErrorString(e));
  return VMP_OK;
}

int vmp_policy_head_backward_bf16(int32_t B, int32_t V, int32_t A, const float *logits,
                                  const uint32_t *mask_bits, const int32_t *action,
                                  const float *g_logprob, const float *g_entropy,
                                  uint16_t *dlogits_bf16, void *stream) {
  if (B < 0 || V < 1 || A < 1 || A > VMP_HEAD_MAX_A || !logits || !action || !dlogits_bf16)
    return vmp::policy_fail(VMP_EINVAL, "vmp_policy_head_backward_bf16: bad shape or null pointer");
  if (B == 0) return VMP_OK;
  HeadArgs a{};
  a.B = B, a.V = V, a.A = A, a.W = (A + 31) / 32, a.mode = VMP_HEAD_GIVEN, a.wait_index = -1;
  a.wait_ratio = -1.f;
  a.logits = logits, a.bits = mask_bits, a.action = const_cast<int32_t *>(action);
  a.g_logprob = g_logprob, a.g_entropy = g_entropy, a.dlogits_bf16 = dlogits_bf16;
  if (!use_tiles(a) || ((uintptr_t)dlogits_bf16 & 7))
    return vmp::policy_fail(VMP_EINVAL, "vmp_policy_head_backward_bf16: needs A <= 128, 16-B aligned "
                                        "logits and 8-B aligned dlogits");
  hipError_t e = launch_bwd(a, (hipStream_t)stream);
  if (e != hipSuccess) return vmp::policy_fail(VMP_EDEVICE, hipGetErrorString(e));
  return VMP_OK;
}

int vmp_gae(int32_t T, int32_t N, const float *reward, const float *done, const float *value,
            const float *next_value, float gamma, float lam, float *adv, float *ret,
            void *stream) {
  if (T < 0 || N < 0 || !reward || !done || !value || !next_value || !adv || !ret)
    return vmp::policy_fail(VMP_EINVAL, "bad gae arguments");
  if (T == 0 || N == 0) return VMP_OK;
  hipLaunchKernelGGL(k_gae, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, T, N,
                     reward, done, value, next_value, gamma, lam, adv, ret);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return vmp::policy_fail(VMP_EDEVICE, hipGetErrorString(e));
  return VMP_OK;
}

}  // extern "C"
