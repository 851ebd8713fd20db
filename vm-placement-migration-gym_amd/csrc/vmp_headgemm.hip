// vmp_headgemm.hip — the actor's last Linear fused with the masked
// multi-categorical head of Network.get_action / get_det_action
// (src/agents/ppo.py:115-131): logits = h W^T + b are formed
// tile by tile on the f32 matrix cores and consumed in the same workgroup, so
// the [B, V*A] logits never reach HBM (unless the caller asks for them, as the
// training forward does for its backward).
//
// GEMM: C[B, N = V*A] = H[B, K] * W[N, K]^T, f32 in / f32 accumulate on
// v_mfma_f32_16x16x4_f32 (exact f32 products, one rounding per step). A
// workgroup of 8 waves owns a BM = 128 x BN tile whose columns are S whole
// action segments (BN = S*A rounded up to a multiple of 16, at most 208), so
// every (sample, VM) row of A logits is complete inside one workgroup. Wave w
// owns rows 16w..16w+15 and all BN columns (NT = BN/16 accumulator tiles of
// 4 VGPRs), computed transposed (W as the MFMA's A operand): each lane ends
// with 4 consecutive logits of one row, one 16-B LDS store in the epilogue.
// The W tile (BN x 32 per K step) is staged through LDS (double buffered, one
// barrier per K step); each lane reads its H fragments straight from global
// memory as float4 (K-permuted: lane l holds k = 4*(l>>4) + j of the 16-deep
// half, element j feeding MFMA j, the W fragment read the same way from LDS;
// the K order only changes f32 rounding, inside the 1e-5 contract).
//
// Epilogue: the C tile (+ bias) is staged in LDS, 64 rows at a time, and one
// quad of lanes per (row, segment) applies the mask (`logits[mask] = -1e7`,
// ppo.py:119) and the PPOAgent.act WAIT coin flip (ppo.py:154-156), then
// lse = m + log S (f32, torch's Categorical order), logprob of the sampled /
// given action, entropy -sum q (x - lse). SAMPLE draws by inverse CDF with
// one counter-based uniform per row (the unfused head's stream: equal logits
// draw equal actions), the law of Categorical.sample. ARGMAX is
// get_det_action: first max of the UNMASKED row. Per-row results go to
// row_lp / row_ent; k_rowsum (vmp_policy.hip) adds them per sample in a fixed
// order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/vmp.h"

namespace vmp {

__global__ void k_rowsum(int B, int V, const float *row_lp, const float *row_ent, float *lp,
                         float *ent);

namespace {

constexpr int kBK = 32;
constexpr int kLdsStride = kBK + 4;  // W tile row stride (floats)
constexpr float kMasked = -1e7f;     // ppo.py:119

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// the same counter-based uniforms as vmp_policy.hip (coin flips agree with the
// unfused head draw for draw)
__device__ __forceinline__ float uniform_at(uint64_t seed, uint64_t ctr) {
  const uint64_t h = mix64(seed ^ mix64(ctr));
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}

struct HGArgs {
  int B, K, V, A, W32, S, BN, n_tiles, mode, wait_index, stage_waves;
  float wait_ratio;
  uint64_t seed, offset;
  const uint64_t *ctr;
  const float *h, *w, *bias;
  const uint32_t *bits;
  int32_t *action;
  float *row_lp, *row_ent;
  float *logits;  // nullable: raw logits [B][V*A] out
};

__device__ __forceinline__ uint64_t eff_seed(const HGArgs &a) {
  return a.ctr ? a.seed ^ mix64(*a.ctr + 0x5851F42D4C957F2Dull) : a.seed;
}

// get_det_action: first max of the unmasked row (quad lanes c, c+4k)
__device__ __forceinline__ void row_argmax(const HGArgs &a, const float *x, int64_t row, int c) {
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int j = c; j < a.A; j += 4) {
    const float xj = x[j];
    if (xj == xj && (xj > best || bi == 0x7fffffff)) {
      best = xj;
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
  if (c == 0) a.action[row] = bi == 0x7fffffff ? 0 : bi;
}

// One (row, segment) of A <= 4 KQ logits on a quad: lane c takes x[c + 4k]
// into registers with one LDS read each (no branches: the tile's LDS carries
// 4 KQ floats of slack past the last row) and keeps exp(x - m), so the
// passes cost ~13 VALU per element: entries past A are folded into the mask
// (x = -1e7, p = 0), the entropy is (1/S) sum p (x - lse), and the inverse
// CDF counts the running sums <= target instead of tracking a pick.
template <int KQ>
__device__ __forceinline__ void row_task(const HGArgs &a, const float *x, int64_t row, int c,
                                         uint64_t seed, bool sample, bool flip, uint32_t w0,
                                         int32_t given) {
  constexpr int kWords = (4 * KQ + 31) / 32;
  static_assert(kWords <= 4, "A <= 128: lane c of the quad holds mask word c");
  uint32_t mw[kWords], me[kWords], ob[kWords];  // the row's mask; mask | (j >= A); j >= A
  int cnt = 0;
#pragma unroll
  for (int q = 0; q < kWords; q++) {
    mw[q] = __shfl(w0, q, 4);
    const int tail = a.A - 32 * q;  // bits past A are not actions
    const uint32_t in = tail >= 32 ? ~0u : (tail > 0 ? (1u << tail) - 1u : 0u);
    mw[q] &= in;
    cnt += __popc(mw[q]);
    me[q] = ~in;
    ob[q] = ~in >> c;
  }
  if (flip) {  // PPOAgent.act's WAIT coin (ppo.py:154-156): forbid WAIT for this row
    const int P = a.wait_index;
    bool wait_bad = false;
#pragma unroll
    for (int q = 0; q < kWords; q++)
      if (q == (P >> 5)) wait_bad = (mw[q] >> (P & 31)) & 1u;
    if (cnt > 1 && !wait_bad &&
        uniform_at(seed ^ 0xC0FFEE5EEDull, a.offset + (uint64_t)row) > a.wait_ratio) {
#pragma unroll
      for (int q = 0; q < kWords; q++)
        if (q == (P >> 5)) mw[q] |= 1u << (P & 31);
    }
  }
  bool all_masked = true;
#pragma unroll
  for (int q = 0; q < kWords; q++) {
    all_masked = all_masked && (mw[q] | me[q]) == ~0u;
    me[q] = (me[q] | mw[q]) >> c;  // lane c's bits: element k at bit 4 (k % 8)
  }
  // pairs of elements in packed f32 registers (v_pk_add / v_pk_mul / v_pk_fma)
  static_assert(KQ % 2 == 0, "KQ buckets are even");
  f32x2 xv[KQ / 2], pv[KQ / 2];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < KQ; k++) {
    // bit 4 (k % 8) of the lane's word -> 0 / all ones; select -1e7 bit-wise
    const int sel = (int)(me[k >> 3] << (31 - 4 * (k & 7))) >> 31;
    const int xb = __float_as_int(x[c + 4 * k]);
    const float v = __int_as_float((sel & __float_as_int(kMasked)) | (~sel & xb));
    xv[k >> 1][k & 1] = v;
    m = fmaxf(m, v);
  }
  m = fmaxf(m, __shfl_xor(m, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  // __expf(x - m) = exp2((x - m) * log2 e), the same roundings as the unfused head
  const f32x2 m2 = {m, m}, l2e = {1.44269504088896341f, 1.44269504088896341f};
#pragma unroll
  for (int k = 0; k < KQ / 2; k++) {
    const f32x2 d = (xv[k] - m2) * l2e;
    pv[k] = f32x2{__builtin_amdgcn_exp2f(d[0]), __builtin_amdgcn_exp2f(d[1])};  // 0 at masked
  }
  if (all_masked) {  // ... unless the row is all masked: then only entries past A drop out
#pragma unroll
    for (int k = 0; k < KQ; k++)
      if ((ob[k >> 3] >> (4 * (k & 7))) & 1u) pv[k >> 1][k & 1] = 0.f;
  }
  float sl = 0.f;  // this lane's share of S, in element order
#pragma unroll
  for (int k = 0; k < KQ; k++) sl += pv[k >> 1][k & 1];
  float S = sl + __shfl_xor(sl, 1);
  S += __shfl_xor(S, 2);
  const float lse = m + logf(S);
  // Categorical.entropy -sum q (x - lse), as (1/S) sum p (x - lse)
  const f32x2 lse2 = {lse, lse};
  f32x2 h2 = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < KQ / 2; k++) h2 = __builtin_elementwise_fma(pv[k], xv[k] - lse2, h2);
  float hs = h2[0] + h2[1];
  hs += __shfl_xor(hs, 1);
  hs += __shfl_xor(hs, 2);
  hs *= 1.0f / S;
  int act;
  if (sample) {
    // inverse CDF in lane-major order over the quad (vmp_policy.hip's tiled
    // head: the same uniform per row, so equal logits draw equal actions)
    float incl = sl + __shfl_up(sl, 1, 4) * (c >= 1);
    incl += __shfl_up(incl, 2, 4) * (c >= 2);
    const float excl = incl - sl;
    const float target = uniform_at(seed, a.offset + (uint64_t)row) * __shfl(incl, 3, 4);
    // the first k whose running sum passes target has p_k > 0: the running
    // sums are non-decreasing, so it is the count of sums <= target
    int below = 0;
    float cum = excl;
#pragma unroll
    for (int k = 0; k < KQ; k++) {
      cum += pv[k >> 1][k & 1];
      below += cum <= target;
    }
    const bool mine = target >= excl && target < incl;
    int pick = -1;
    if (mine) {
      if (below < KQ) {
        pick = c + 4 * below;
      } else {  // rounding: incl passed target, the lane's own sum did not
#pragma unroll
        for (int k = 0; k < KQ; k++)
          if (pv[k >> 1][k & 1] > 0.f) pick = c + 4 * k;
      }
    }
    int any = pick;
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) any = max(any, __shfl_xor(any, o));
    if (any < 0) {  // target past the rounded total: last positive entry
      int last = -1;
#pragma unroll
      for (int k = 0; k < KQ; k++)
        if (pv[k >> 1][k & 1] > 0.f) last = c + 4 * k;
      int lk = last >= 0 ? c * 1024 + last : -1;
#pragma unroll
      for (int o = 1; o < 4; o <<= 1) lk = max(lk, __shfl_xor(lk, o));
      any = lk & 1023;
    } else {  // more than one lane can claim only through rounding: lowest lane wins
      int mn = pick >= 0 ? c : 4;
#pragma unroll
      for (int o = 1; o < 4; o <<= 1) mn = min(mn, __shfl_xor(mn, o));
      any = __shfl(pick, mn, 4);
    }
    act = any;
    if (c == 0) a.action[row] = act;
  } else {
    act = given;
  }
  if (c == 0) {
    float lp = NAN;
    if (act >= 0 && act < a.A) {
      bool msk = false;
#pragma unroll
      for (int q = 0; q < kWords; q++)
        if (q == (act >> 5)) msk = (mw[q] >> (act & 31)) & 1u;
      lp = (msk ? kMasked : x[act]) - lse;
    }
    a.row_lp[row] = lp;
    a.row_ent[row] = -hs;
  }
}

// NW waves (BM = 16 NW rows) per workgroup, NT accumulator tiles per wave; 4
// waves per SIMD (<= 128 VGPRs). Blocks are numbered M-fastest, so the
// workgroups resident at a time share few W column slabs (L2 / MALL reuse).
template <int NT, int NW>
__global__ __launch_bounds__(64 * NW, 4) void k_head_gemm(HGArgs a) {
  extern __shared__ __align__(16) float lds[];
  constexpr int kThreads = 64 * NW, kBM = 16 * NW;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int m_blocks = (a.B + kBM - 1) / kBM;
  const int m_blk = blockIdx.x % m_blocks, n_tile = blockIdx.x / m_blocks;
  const int m0 = m_blk * kBM;
  const int v0 = n_tile * a.S;                        // first VM row of the tile
  const int nseg = min(a.S, a.V - v0);                 // segments in this tile
  const int N = a.V * a.A, n0 = v0 * a.A;
  const int K = a.K;
  float *wl0 = lds, *wl1 = lds + NT * 16 * kLdsStride;

  // ---- W tile staging: BN rows x 32 floats = NT*128 float4, 512 threads ----
  constexpr int kStage = (NT * 128 + kThreads - 1) / kThreads;
  f32x4 st[kStage];
  auto stage_load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < kStage; r++) {
      const int i = t + r * kThreads;             // float4 index in the tile
      const int row = i >> 3, c4 = i & 7;          // 8 float4 per 32-wide row
      const int n = min(n0 + row, N - 1);          // pad rows read a valid row (ignored)
      st[r] = (i < NT * 128) ? *reinterpret_cast<const f32x4 *>(a.w + (int64_t)n * K + k0 + 4 * c4)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto stage_store = [&](float *wl) {
#pragma unroll
    for (int r = 0; r < kStage; r++) {
      const int i = t + r * kThreads;
      if (i < NT * 128) {
        const int row = i >> 3, c4 = i & 7;
        *reinterpret_cast<f32x4 *>(wl + row * kLdsStride + 4 * c4) = st[r];
      }
    }
  };
  // ---- H fragments: lane l -> row 16*wid + (l & 15), k = 16*kk + 4*(l >> 4) + j ----
  const int arow = min(m0 + 16 * wid + (lane & 15), a.B - 1);
  const float *hrow = a.h + (int64_t)arow * K + 4 * (lane >> 4);
  f32x4 acc[NT];
#pragma unroll
  for (int c = 0; c < NT; c++) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 a0 = *reinterpret_cast<const f32x4 *>(hrow);
  f32x4 a1 = *reinterpret_cast<const f32x4 *>(hrow + 16);
  stage_load(0);
  stage_store(wl0);
  __syncthreads();
  const float *wrd = nullptr;
#pragma unroll 1
  for (int k0 = 0, it = 0; k0 < K; k0 += kBK, it++) {
    float *cur = (it & 1) ? wl1 : wl0, *nxt = (it & 1) ? wl0 : wl1;
    const bool more = k0 + kBK < K;
    f32x4 na0 = a0, na1 = a1;
    if (more) {  // next step's W tile and H fragments, in flight during the MFMAs
      stage_load(k0 + kBK);
      na0 = *reinterpret_cast<const f32x4 *>(hrow + k0 + kBK);
      na1 = *reinterpret_cast<const f32x4 *>(hrow + k0 + kBK + 16);
    }
    wrd = cur + (lane & 15) * kLdsStride + 4 * (lane >> 4);
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      const f32x4 av = kk ? a1 : a0;
#pragma unroll
      for (int c0 = 0; c0 < NT; c0 += 4) {  // 4 accumulators in flight per fragment
        f32x4 bv[4];
#pragma unroll
        for (int c = 0; c < 4; c++)
          if (c0 + c < NT)
            bv[c] = *reinterpret_cast<const f32x4 *>(wrd + (c0 + c) * 16 * kLdsStride + 16 * kk);
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
          for (int c = 0; c < 4; c++)
            if (c0 + c < NT)
              acc[c0 + c] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv[c][j], av[j], acc[c0 + c], 0, 0, 0);
      }
    }
    if (more) stage_store(nxt);
    a0 = na0;
    a1 = na1;
    __syncthreads();
  }

#ifdef VMP_HG_GEMM_ONLY  // timing-only build: the main loop alone (outputs wrong)
  {
    float z = 0.f;
#pragma unroll
    for (int c = 0; c < NT; c++) z += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    if (z == 12345.f) a.row_lp[0] = z;  // keeps every MFMA live
  }
  return;
#endif
  // ---- epilogue: 16 gw rows (one group of gw waves) at a time through LDS ----
  // gw = NW when the whole C tile fits the LDS budget, else 4. Group g waits
  // out stages 0..g-1, stages its accumulators for stage g, and from then on
  // helps process stages g..G-1: stage h is processed by groups 0..h, whose
  // accumulators are dead, so the row passes get the registers (a loop over
  // stages would keep every wave's accumulators live throughout). Every group
  // executes 2 G barriers.
  const int gw = a.stage_waves, G = NW / gw, SR = 16 * gw;
  const int BNp = a.BN + 4;  // 16-B aligned rows (b128 staging and logits reads)
  float *ct = lds;
  const int g = __builtin_amdgcn_readfirstlane(wid / gw);
#pragma unroll 1
  for (int h = 0; h < g; h++) {
    __syncthreads();  // half h staged
    __syncthreads();  // half h processed
  }
  {  // lane l holds columns 16c + 4 (l >> 4) + 0..3 of tile row 16 (wid % 4) + (l & 15)
    float *dst = ct + (16 * (wid - g * gw) + (lane & 15)) * BNp;
    const int w = nseg * a.A;
#pragma unroll
    for (int c = 0; c < NT; c++) {
      const int col = c * 16 + 4 * (lane >> 4);
      if (col < a.BN) {  // the template's NT may exceed this launch's BN / 16
        f32x4 v = acc[c];
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] += (col + i < w) ? a.bias[n0 + col + i] : 0.f;
        *reinterpret_cast<f32x4 *>(dst + col) = v;
      }
    }
  }
  const uint64_t seed = eff_seed(a);
  const bool sample = a.mode == VMP_HEAD_SAMPLE, argmax = a.mode == VMP_HEAD_ARGMAX;
  const bool flip = a.wait_ratio >= 0.f && a.bits && !argmax;
  const int c = t & 3;
  // per-task inputs (lane c: mask word c; lane 0: the given action) are
  // fetched one task ahead, the first before the staging barrier
  auto fetch = [&](int task, int h, int ntask, uint32_t &w, int32_t &given) {
    w = 0u;
    given = 0;
    if (task < ntask) {
      const int r = task / nseg, s = task - r * nseg;
      const int64_t row = (int64_t)(m0 + SR * h + r) * a.V + v0 + s;
      if (a.bits && c < a.W32) w = a.bits[row * a.W32 + c];
      if (!sample && !argmax && c == 0) given = a.action[row];
    }
  };
#pragma unroll 1
  for (int h = g; h < G; h++) {
    const int rows = min(SR, a.B - (m0 + SR * h));
    const int nwave = gw * (h + 1);  // groups 0..h take part
    const int ntask = rows * nseg, step = 16 * nwave;
    int task = t >> 2;
    uint32_t wn;
    int32_t gn;
    fetch(task, h, ntask, wn, gn);
    __syncthreads();  // half h staged (by group h)
    if (a.logits) {  // raw logits of the half's rows: streaming (non-temporal) stores
      const int w = nseg * a.A;
      float *gl = a.logits + (int64_t)(m0 + SR * h) * N + n0;
      if (((N | n0 | w) & 3) == 0 && ((uintptr_t)a.logits & 15) == 0) {
        const int w4 = w >> 2;
        for (int i = t; i < rows * w4; i += 64 * nwave) {
          const int r = i / w4, c4 = i - r * w4;
          const f32x4 v = *reinterpret_cast<const f32x4 *>(ct + r * BNp + 4 * c4);
          __builtin_nontemporal_store(v, reinterpret_cast<f32x4 *>(gl + (int64_t)r * N + 4 * c4));
        }
      } else {
        for (int r = wid; r < rows; r += nwave)
          for (int cc = lane; cc < w; cc += 64)
            __builtin_nontemporal_store(ct[r * BNp + cc], gl + (int64_t)r * N + cc);
      }
    }
    // one quad of lanes per (row, segment): lane c takes elements j = c + 4k
#pragma unroll 1
    for (; task < ntask; task += step) {
      const uint32_t w = wn;
      const int32_t given = gn;
      fetch(task + step, h, ntask, wn, gn);
      const int r = task / nseg, s = task - r * nseg;
      const int64_t row = (int64_t)(m0 + SR * h + r) * a.V + v0 + s;
      const float *x = ct + r * BNp + s * a.A;
      if (argmax) row_argmax(a, x, row, c);
      else switch ((a.A + 15) >> 4) {  // KQ = 4 ceil(A / 16) elements per lane
        case 1: row_task<4>(a, x, row, c, seed, sample, flip, w, given); break;
        case 2: row_task<8>(a, x, row, c, seed, sample, flip, w, given); break;
        case 3: row_task<12>(a, x, row, c, seed, sample, flip, w, given); break;
        case 4: row_task<16>(a, x, row, c, seed, sample, flip, w, given); break;
        case 5: row_task<20>(a, x, row, c, seed, sample, flip, w, given); break;
        case 6: row_task<24>(a, x, row, c, seed, sample, flip, w, given); break;
        case 7: row_task<28>(a, x, row, c, seed, sample, flip, w, given); break;
        default: row_task<32>(a, x, row, c, seed, sample, flip, w, given); break;
      }
    }
    __syncthreads();  // half h processed: LDS free for half h + 1
  }
}

template <int NT, int NW>
hipError_t launch_nw(const HGArgs &a, hipStream_t st) {
  HGArgs b = a;
  const size_t lds_w = (size_t)2 * NT * 16 * kLdsStride * sizeof(float);
  // + 128 floats: the row passes read 4 KQ <= 128 floats from each segment start
  auto lds_c = [&](int gw) { return ((size_t)16 * gw * (a.BN + 4) + 128) * sizeof(float); };
  // the whole tile in one stage when two workgroups still fit a CU (80 KB each)
  b.stage_waves = lds_c(NW) <= 80 * 1024 ? NW : 4;
  const size_t lds = lds_w > lds_c(b.stage_waves) ? lds_w : lds_c(b.stage_waves);
  const int64_t m_blocks = (a.B + 16 * NW - 1) / (16 * NW);
  hipLaunchKernelGGL((k_head_gemm<NT, NW>), dim3((unsigned)(m_blocks * a.n_tiles)), dim3(64 * NW),
                     lds, st, b);
  return hipGetLastError();
}

// 8 waves (128 rows per W slab) unless that leaves CUs idle; measured: 16
// waves per workgroup (one per CU) ran 20 % slower, 4 waves 50 % slower at the
// 100.yml shapes.
template <int NT>
hipError_t launch_nt(const HGArgs &a, hipStream_t st) {
  const int64_t tiles = a.n_tiles;
  if (const char *f = getenv("VMP_HG_NW")) {  // measurement override
    if (f[0] == '4') return launch_nw<NT, 4>(a, st);
    if (f[0] == '8') return launch_nw<NT, 8>(a, st);
    if (f[0] == '1') return launch_nw<NT, 16>(a, st);
  }
  if (((a.B + 127) / 128) * tiles >= 256) return launch_nw<NT, 8>(a, st);
  return launch_nw<NT, 4>(a, st);
}

}  // namespace

int policy_fail(int code, const char *msg);

}  // namespace vmp

using namespace vmp;

extern "C" int vmp_actor_head(int32_t B, int32_t K, int32_t V, int32_t A, int32_t mode,
                              const float *h, const float *weight, const float *bias,
                              const uint32_t *mask_bits, float wait_ratio, int32_t wait_index,
                              uint64_t seed, uint64_t offset, const uint64_t *rng_counter,
                              int32_t *action, float *logprob, float *entropy, float *logits_out,
                              float *workspace, void *stream) {
  if (B < 0 || K < 1 || V < 1 || A < 1 || !h || !weight || !bias || !action)
    return policy_fail(VMP_EINVAL, "vmp_actor_head: bad shape or null pointer");
  if (K % 32 != 0 || A > VMP_ACTOR_HEAD_MAX_A)
    return policy_fail(VMP_EINVAL, "vmp_actor_head: needs K % 32 == 0 and A <= 128");
  if ((((uintptr_t)h) | ((uintptr_t)weight)) & 15)
    return policy_fail(VMP_EINVAL, "vmp_actor_head: h and weight must be 16-byte aligned");
  if (mode != VMP_HEAD_SAMPLE && mode != VMP_HEAD_GIVEN && mode != VMP_HEAD_ARGMAX)
    return policy_fail(VMP_EINVAL, "vmp_actor_head: unknown mode");
  if (wait_ratio >= 0.f && (!mask_bits || wait_index < 0 || wait_index >= A))
    return policy_fail(VMP_EINVAL, "vmp_actor_head: WAIT coin flips need the mask and 0 <= wait_index < A");
  if (B == 0) return VMP_OK;
  HGArgs a{};
  a.B = B, a.K = K, a.V = V, a.A = A, a.W32 = (A + 31) / 32, a.mode = mode;
  // whole segments per tile, at most 13 accumulator tiles (208 columns: no
  // spills at 4 waves / SIMD)
  a.S = 208 / A;
  if (const char *f = getenv("VMP_HG_SMAX")) a.S = std::max(1, std::min(a.S, atoi(f)));  // measurement
  if (a.S > V) a.S = V;
  // small batches: narrower tiles until >= 512 four-wave workgroups fill the
  // chip (config/10.yml eval, B 4096 x 360 columns, would run 64 workgroups)
  while (a.S > 1 && (int64_t)((B + 63) / 64) * ((V + a.S - 1) / a.S) < 512) a.S = (a.S + 1) / 2;
  a.BN = (a.S * A + 15) / 16 * 16;
  a.n_tiles = (V + a.S - 1) / a.S;
  a.wait_index = wait_index, a.wait_ratio = wait_ratio;
  a.seed = seed, a.offset = offset, a.ctr = rng_counter;
  a.h = h, a.w = weight, a.bias = bias, a.bits = mask_bits, a.action = action;
  a.logits = logits_out;
  hipStream_t st = (hipStream_t)stream;
  const bool sums = mode != VMP_HEAD_ARGMAX;
  const int64_t rows = (int64_t)B * V;
  float *scratch = nullptr;
  if (sums) {
    float *ws = workspace;
    if (!ws) {
      hipError_t e = hipMallocAsync((void **)&scratch, 2 * rows * sizeof(float), st);
      if (e != hipSuccess) return policy_fail(VMP_EOOM, hipGetErrorString(e));
      ws = scratch;
    }
    a.row_lp = ws;
    a.row_ent = ws + rows;
  }
  const int nt = a.BN / 16;
  hipError_t e;
  if (nt <= 4) e = launch_nt<4>(a, st);
  else if (nt <= 8) e = launch_nt<8>(a, st);
  else e = launch_nt<13>(a, st);
  if (e == hipSuccess && sums) {
    hipLaunchKernelGGL(k_rowsum, dim3((B + 3) / 4), dim3(256), 0, st, B, V, a.row_lp, a.row_ent,
                       logprob, entropy);
    e = hipGetLastError();
  }
  if (scratch) {
    hipError_t f = hipFreeAsync(scratch, st);
    if (e == hipSuccess) e = f;
  }
  if (e != hipSuccess) return policy_fail(VMP_EDEVICE, hipGetErrorString(e));
  return VMP_OK;
}
