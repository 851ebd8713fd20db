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
// action segments (BN = S*A rounded up to a multiple of 16, at most 256), so
// every (sample, VM) row of A logits is complete inside one workgroup. Wave w
// owns rows 16w..16w+15 and all BN columns (NT = BN/16 accumulator tiles of
// 4 VGPRs). The W tile (BN x 32 per K step) is staged through LDS (double
// buffered, one barrier per K step); each lane reads its H fragments straight
// from global memory as float4 (K-permuted: lane l holds k = 4*(l>>4) + j of
// the 16-deep half, element j feeding MFMA j, the W fragment read the same way
// from LDS; the K order only changes f32 rounding, inside the 1e-5 contract).
//
// Epilogue: the C tile (+ bias) is staged in LDS, 64 rows at a time, and one
// quad of lanes per (row, segment) applies the mask (`logits[mask] = -1e7`,
// ppo.py:119) and the PPOAgent.act WAIT coin flip (ppo.py:154-156), then
// lse = m + log S (f32, torch's Categorical order), logprob of the sampled /
// given action, entropy -sum q (x - lse). SAMPLE draws by inverse CDF with
// one counter-based uniform per row (the unfused head's stream: equal logits
// draw equal actions), the law of Categorical.sample. ARGMAX is
// get_det_action: first max of the UNMASKED row. Per-row results go to row_lp / row_ent; k_rowsum (vmp_policy.hip) adds
// them per sample in a fixed order.
#include <hip/hip_runtime.h>
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
  int B, K, V, A, W32, S, BN, n_tiles, mode, wait_index;
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
              acc[c0 + c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[c][j], acc[c0 + c], 0, 0, 0);
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
  // ---- epilogue: 64 rows at a time through LDS (reuses the W buffers) ----
  const int BNp = a.BN + 1;  // odd row stride: the per-row scans hit distinct banks
  float *ct = lds;
  const uint64_t seed = eff_seed(a);
  const bool sample = a.mode == VMP_HEAD_SAMPLE, argmax = a.mode == VMP_HEAD_ARGMAX;
  const bool flip = a.wait_ratio >= 0.f && a.bits && !argmax;
#pragma unroll 1
  for (int half = 0; half < NW / 4; half++) {
    // waves 4*half .. 4*half+3 hold rows 64*half .. 64*half+63 of the tile
    if ((wid >> 2) == half) {
      const int rw = 16 * (wid & 3) + 4 * (lane >> 4);
#pragma unroll
      for (int c = 0; c < NT; c++) {
        const int col = c * 16 + (lane & 15);
        if (col < a.BN) {  // the template's NT may exceed this launch's BN / 16
          const float bcol = (col < nseg * a.A) ? a.bias[n0 + col] : 0.f;
#pragma unroll
          for (int i = 0; i < 4; i++) ct[(rw + i) * BNp + col] = acc[c][i] + bcol;
        }
      }
    }
    __syncthreads();
    const int rows = min(64, a.B - (m0 + 64 * half));
    if (a.logits) {  // raw logits of the tile's rows, row-contiguous stores
      const int w = nseg * a.A;
      for (int i = t; i < rows * w; i += kThreads) {
        const int r = i / w, c = i - r * w;
        a.logits[(int64_t)(m0 + 64 * half + r) * N + n0 + c] = ct[r * BNp + c];
      }
    }
    // one quad of lanes per (row, segment): lane c takes elements j = c + 4k
    const int c = t & 3;
#pragma unroll 1
    for (int task = t >> 2; task < rows * nseg; task += kThreads >> 2) {
      const int r = task / nseg, s = task - r * nseg;
      const int b = m0 + 64 * half + r, v = v0 + s;
      const int64_t row = (int64_t)b * a.V + v;
      const float *x = ct + r * BNp + s * a.A;
      if (argmax) {  // get_det_action: first max of the unmasked row
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
        continue;
      }
      uint32_t mw[8];
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        mw[q] = (a.bits && q < a.W32) ? a.bits[row * a.W32 + q] : 0u;
        if (q == a.W32 - 1 && a.A - 32 * q < 32) mw[q] &= (1u << (a.A - 32 * q)) - 1u;
        cnt += __popc(mw[q]);
      }
      int forbid = -1;
      if (flip) {
        const int P = a.wait_index;
        const bool wait_bad = (mw[P >> 5] >> (P & 31)) & 1u;
        if (cnt > 1 && !wait_bad &&
            uniform_at(seed ^ 0xC0FFEE5EEDull, a.offset + (uint64_t)row) > a.wait_ratio)
          forbid = P;
      }
      auto xm = [&](int j) {
        return (((mw[j >> 5] >> (j & 31)) & 1u) || j == forbid) ? kMasked : x[j];
      };
      float m = -INFINITY;
      for (int j = c; j < a.A; j += 4) m = fmaxf(m, xm(j));
      m = fmaxf(m, __shfl_xor(m, 1));
      m = fmaxf(m, __shfl_xor(m, 2));
      float sl = 0.f;  // this lane's share of S
      for (int j = c; j < a.A; j += 4) sl += __expf(xm(j) - m);
      float S = sl + __shfl_xor(sl, 1);
      S += __shfl_xor(S, 2);
      const float lse = m + logf(S);
      // Categorical.entropy: -sum q_j (x_j - lse), the normalised logits rounded
      // in f32 as torch forms them (an all-masked row then gives lse's rounding)
      const float inv = 1.0f / S;
      float hs = 0.f;
      for (int j = c; j < a.A; j += 4) {
        const float xj = xm(j);
        const float p = __expf(xj - m);
        if (p > 0.f) hs += (p * inv) * (xj - lse);
      }
      hs += __shfl_xor(hs, 1);
      hs += __shfl_xor(hs, 2);
      int act;
      if (sample) {
        // inverse CDF in lane-major order over the quad (vmp_policy.hip's tiled
        // head: the same uniform per row, so equal logits draw equal actions)
        float incl = sl + __shfl_up(sl, 1, 4) * (c >= 1);
        incl += __shfl_up(incl, 2, 4) * (c >= 2);
        const float excl = incl - sl;
        const float total = __shfl(incl, 3, 4);
        const float target = uniform_at(seed, a.offset + (uint64_t)row) * total;
        int pick = -1, last = -1;
        float cum = excl;
        for (int j = c; j < a.A; j += 4) {
          const float pj = __expf(xm(j) - m);
          if (pj > 0.f) {
            cum += pj;
            last = j;
            if (pick < 0 && target >= excl && target < cum) pick = j;
          }
        }
        if (pick < 0 && last >= 0 && target >= excl && target < incl) pick = last;
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
        act = any;
        if (c == 0) a.action[row] = act;
      } else {
        act = a.action[row];
      }
      if (c == 0) {
        a.row_lp[row] = (act >= 0 && act < a.A) ? xm(act) - lse : NAN;
        a.row_ent[row] = -hs;
      }
    }
    __syncthreads();
  }
}

template <int NT, int NW>
hipError_t launch_nw(const HGArgs &a, hipStream_t st) {
  const size_t lds_w = (size_t)2 * NT * 16 * kLdsStride * sizeof(float);
  const size_t lds_c = (size_t)64 * (a.BN + 1) * sizeof(float);
  const size_t lds = lds_w > lds_c ? lds_w : lds_c;
  const int64_t m_blocks = (a.B + 16 * NW - 1) / (16 * NW);
  hipLaunchKernelGGL((k_head_gemm<NT, NW>), dim3((unsigned)(m_blocks * a.n_tiles)), dim3(64 * NW),
                     lds, st, a);
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
    return policy_fail(VMP_EINVAL, "vmp_actor_head: needs K % 32 == 0 and A <= 256");
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
  // spills at 4 waves / SIMD); 208 < A <= 256 takes one segment of 16 tiles
  a.S = A <= 208 ? 208 / A : 1;
  if (a.S > V) a.S = V;
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
  else if (nt <= 13) e = launch_nt<13>(a, st);
  else e = launch_nt<16>(a, st);
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
