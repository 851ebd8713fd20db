// vmp_headgemm_bf16.hip — the training side of the fused actor head
// (src/agents/ppo.py:115-126 get_action(obs, action, mask) and
// the PPOAgent.update backward through it, ppo.py:258-287), on the bf16
// matrix cores.
//
// Forward (GIVEN actions): logits = h W^T + b are formed tile by tile with
// v_mfma_f32_16x16x32_bf16 (bf16 h and W, f32 accumulate) and consumed in
// registers: masked max / sum / lse, entropy lse - (sum p x)/S and the given
// action's logprob per (sample, VM row) -> row buffers -> k_rowsum. The
// [B, V*A] logits never reach HBM.
// Backward: the same tiles are recomputed, and dlogits
//   d_j = -q_j (g_lp + g_ent (x_j - lse + H)) + g_lp [j = a],  0 at masked j
// is formed in registers and rounded to bf16 for the dW / dh GEMMs, written
// for the caller's row chunk only (the host runs the backward chunk by chunk,
// so at most one chunk of dlogits exists; the bias gradient comes out of the
// dW GEMM as the product with a column of ones appended to h).
//
// Tile: a workgroup of 8 waves owns BM = 256 samples x NT 16-column tiles.
// The columns are S whole action segments, each padded to SA = 16 TS columns
// (TS tiles), so a tile column's segment is known at compile time: tile
// column n = 16 TS s + j holds logit j of VM row v0 + s. Wave w owns samples
// 32w..32w+31; the accumulators are computed transposed (W as the A operand):
// lane (q = l >> 4, c = l & 15) holds columns 16 nt + 4q + 0..3 of sample
// 16 mc + c, so a segment's row reductions are in-lane sums plus two xor
// shuffles over q. Operands are staged through LDS with global_load_lds
// (16 B per lane, two stages of BK = 64; 128-B rows, 16-B chunk index XOR
// (row >> 1) & 7 on the source address and on the read: conflict-free
// ds_read_b128 fragments). The bias is the accumulators' initial value.
//
// Each workgroup keeps one column tile and loops over the M blocks of its M
// group; workgroups of one XCD run the same M block at about the same time,
// so the h tile is an L2 hit for all but the first.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/vmp.h"

#define LDSP __attribute__((address_space(3)))
#define GLBP __attribute__((address_space(1)))

namespace vmp {

__global__ void k_rowsum(int B, int V, const float *row_lp, const float *row_ent, float *lp,
                         float *ent);
int policy_fail(int code, const char *msg);

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int kBM = 256;       // samples per M block (NW waves x MC 16-sample columns)
constexpr int kBK = 64;        // K per LDS stage
constexpr int kRow = 2 * kBK;  // bytes per staged row
constexpr int kMaxNT = 14;     // 16-column accumulator tiles per workgroup
constexpr float kMasked = -1e7f;   // ppo.py:119
constexpr float kPad = -1e30f;     // tile columns past A: p = 0, never the max
constexpr float kLog2e = 1.44269504088896341f;
constexpr int kPipe = 4;       // W fragments in flight ahead of their MFMAs
constexpr int kTeam = 8;       // XCD team size (hg16_tile)

struct H16Args {
  int B, K, V, A, W32, n_tiles, m_blocks, m_groups, ld;
  int team, teams;  // XCD teams (launch_hg16); team 0: one column tile per block index
  const uint16_t *h, *w;
  const float *bias;
  const uint32_t *bits;
  const int32_t *action;
  const float *g_lp, *g_ent;
  float *row_lp, *row_ent;  // forward: per (sample, VM row)
  uint16_t *dl;             // backward: bf16 dlogits [B][ld]
  float *dpart;             // backward, nullable: bias-gradient partials [M group][V*A]
  // sampling (vmp_actor_head_bf16_sample): action is the output [B][V]; the
  // launch seed is seed, mixed with *ctr when ctr is set (vmp_policy.hip's
  // stream); wait_ratio >= 0: PPOAgent.act's WAIT coin per row
  uint64_t seed, offset;
  const uint64_t *ctr;
  float wait_ratio;
  int wait_index;
  int32_t *act_out;  // sampling: the drawn actions [B][V]
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// the counter-based uniforms of vmp_policy.hip / vmp_headgemm.hip (stream
// (seed, ctr), 24 random bits)
__device__ __forceinline__ float uniform_at(uint64_t seed, uint64_t ctr) {
  const uint64_t h = mix64(seed ^ mix64(ctr));
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ uint64_t eff_seed(const H16Args &a) {
  return a.ctr ? a.seed ^ mix64(*a.ctr + 0x5851F42D4C957F2Dull) : a.seed;
}

__device__ __forceinline__ int lds_chunk(int row, int cl) { return cl ^ ((row >> 1) & 7); }

__device__ __forceinline__ bf16x8 frag(const char LDSP *base, int row, int cl) {
  return *reinterpret_cast<const bf16x8 LDSP *>(base + row * kRow + (lds_chunk(row, cl) << 4));
}

// global -> LDS staging of one K stage: W rows (tile columns, segment-padded)
// then h rows, 8 rows of 128 B per wave instruction; lane L writes LDS
// position L % 8 of row L / 8 with the logical chunk that position holds.
// NW issuing waves (wid < NW), BM h rows.
template <int TS, int NT, int NW, int BM = kBM>
__device__ __forceinline__ void stage_issue(const H16Args &a, char LDSP *buf, int v0, int m0,
                                            int k0, int wid, int lane) {
  constexpr int SA = 16 * TS, BNp = 16 * NT, PW = BNp / 8, PIECES = (BNp + BM) / 8;
  const int rl = lane >> 3, p = lane & 7;
#pragma unroll
  for (int i0 = 0; i0 < PIECES; i0 += NW) {
    const int i = i0 + wid;
    if (i < PIECES) {  // wave-uniform
      const uint16_t *src;
      int r;
      if (i < PW) {
        r = 8 * i + rl;
        const int s = r / SA, j = r - s * SA;
        const int v = v0 + s;
        const int wr = (v < a.V && j < a.A) ? v * a.A + j : v0 * a.A;  // pad rows: any row
        src = a.w + (int64_t)wr * a.K;
      } else {
        r = 8 * (i - PW) + rl;
        src = a.h + (int64_t)min(m0 + r, a.B - 1) * a.K;
      }
      src += k0 + 8 * lds_chunk(r, p);
      char LDSP *dst = buf + (i < PW ? 0 : BNp * kRow) + (r - rl) * kRow;
      __builtin_amdgcn_global_load_lds((const GLBP void *)src, (LDSP void *)dst, 16, 0, 0);
    }
  }
}

__device__ __forceinline__ float xsum(float v) {
  v += __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}
__device__ __forceinline__ float xmax(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}

// The row's raw mask words, branch-free (no mask: any readable 16 B, the
// weight matrix, cleared by mask_fix): loads behind a null test join at a
// phi, and the compiler waits for them right there instead of at their use.
template <int W32>
__device__ __forceinline__ void load_mask_raw(const H16Args &a, int64_t row, uint32_t (&mw)[4]) {
  const uint32_t *src = a.bits ? a.bits + row * W32 : reinterpret_cast<const uint32_t *>(a.w);
  mw[0] = mw[1] = mw[2] = mw[3] = 0u;
  if (W32 == 4) {
    const u32x4 v = *reinterpret_cast<const u32x4 *>(src);
    mw[0] = v[0], mw[1] = v[1], mw[2] = v[2], mw[3] = v[3];
  } else if (W32 == 2) {
    const u32x2 v = *reinterpret_cast<const u32x2 *>(src);
    mw[0] = v[0], mw[1] = v[1];
  } else {
#pragma unroll
    for (int i = 0; i < W32; i++) mw[i] = src[i];
  }
}
// ... at its use: nothing when there is no mask, bits past A cleared
template <int W32>
__device__ __forceinline__ void mask_fix(const H16Args &a, uint32_t (&mw)[4]) {
  const uint32_t on = a.bits ? ~0u : 0u;
#pragma unroll
  for (int i = 0; i < 4; i++) mw[i] = i < W32 ? (mw[i] & on) : 0u;
  const int tail = a.A - 32 * (W32 - 1);  // 1..32 bits in the last word
  mw[W32 - 1] &= tail >= 32 ? ~0u : (1u << tail) - 1u;
}

// the row's mask words (bit j of word j >> 5 = action j invalid), bits past A
// cleared; W32 = ceil(A / 32) words per (sample, VM) row
template <int W32>
__device__ __forceinline__ void load_mask(const H16Args &a, int64_t row, uint32_t (&mw)[4]) {
  mw[0] = mw[1] = mw[2] = mw[3] = 0u;
  if (!a.bits) return;
  const uint32_t *src = a.bits + row * W32;
  if (W32 == 4) {
    const u32x4 v = *reinterpret_cast<const u32x4 *>(src);
    mw[0] = v[0], mw[1] = v[1], mw[2] = v[2], mw[3] = v[3];
  } else if (W32 == 2) {
    const u32x2 v = *reinterpret_cast<const u32x2 *>(src);
    mw[0] = v[0], mw[1] = v[1];
  } else {
#pragma unroll
    for (int i = 0; i < W32; i++) mw[i] = src[i];
  }
  const int tail = a.A - 32 * (W32 - 1);  // 1..32 bits in the last word
  mw[W32 - 1] &= tail >= 32 ? ~0u : (1u << tail) - 1u;
}

// The workgroup's column tile and M group. XCD teams (a.team > 0): blocks b
// and b + 8 share an XCD (dealt round-robin), so the team members i = b / 8 ..
// of one XCD take the same column tile (its W tile stays in that XCD's L2
// while they walk M blocks j, j + G, ...) and the 32 / team teams resident on
// an XCD walk the same M blocks (h tiles shared): at team 8, an L2 working set
// of 4 W tiles + 8 h tiles instead of 32 W tiles (kTeam; 0 / 2 / 4 / 8
// measured, profiles/r04_hg16_team.log). False: a padding block.
__device__ __forceinline__ bool hg16_tile(const H16Args &a, int &n_tile, int &g) {
  if (a.team > 0) {
    const int b = blockIdx.x, i = b >> 3;
    const int T = (i / a.team) * 8 + (b & 7);
    if (T >= a.teams) return false;  // padding to whole teams on every XCD
    n_tile = T % a.n_tiles;
    g = (T / a.n_tiles) * a.team + i % a.team;
  } else {
    n_tile = blockIdx.x % a.n_tiles;
    g = blockIdx.x / a.n_tiles;
  }
  return g < a.m_blocks;
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
// Column sums of four values d[0..3] (columns 4 q + r of one tile, sample c =
// lane & 15) over the 16 samples of a DPP row, reduce-scatter style: two
// quad exchanges leave each lane one column summed over its quad, two
// row_shr prefix adds sum the four quads; lane c = 12..15 returns the total
// of column r = 2 (c & 1) + ((c >> 1) & 1). A fixed order: run-to-run
// identical. 11 VALU per four columns.
__device__ __forceinline__ float row16_colsum4(const float (&d)[4], int c) {
  const bool odd = c & 1, b2 = (c >> 1) & 1;
  float k0 = odd ? d[2] : d[0], k1 = odd ? d[3] : d[1];
  const float s0 = odd ? d[0] : d[2], s1 = odd ? d[1] : d[3];
  k0 += dpp_f<0xB1>(s0);  // quad_perm [1, 0, 3, 2]: the partner c ^ 1
  k1 += dpp_f<0xB1>(s1);
  float k = b2 ? k1 : k0;
  k += dpp_f<0x4E>(b2 ? k0 : k1);  // quad_perm [2, 3, 0, 1]: the partner c ^ 2
  k += dpp_f<0x114>(k);            // row_shr:4
  k += dpp_f<0x118>(k);            // row_shr:8
  return k;
}

// The epilogue of one wave's samples (MC columns of 16) of an M block, one
// (column mc, segment s) row at a time: begin() loads the per-sample
// gradients and row 0's mask / action, row(pi) consumes row pi and prefetches
// row pi + 1 (the ping-pong kernel spreads the rows over the other group's
// K steps, so the state between rows is these few registers and acc).
// colL (backward with a.dpart, else null): the wave's f32 column sums of
// dlogits over every sample it has processed, one float per tile column.
typedef uint32_t u32x2u __attribute__((ext_vector_type(2), aligned(4)));

// One tile's bf16 dlogits of one lane, pk0 = columns j0, j0 + 1 and pk1 =
// j0 + 2, j0 + 3 (j0 = 16 u + 4 q) of sample m, VM row v. Even A and ld:
// the lane's 8 bytes go out as one dwordx2 (4-byte aligned: the unaligned
// access mode of the HSA targets; two dword stores per tile were a third of
// the backward's store instructions' issue time).
template <int TS>
__device__ __forceinline__ void store_dl_tile(const H16Args &a, int m, int v, int u, int q,
                                              uint32_t pk0, uint32_t pk1) {
  const bool live = m < a.B;
  const int j0 = 16 * u + 4 * q;
  uint16_t *dst = a.dl + (int64_t)m * a.ld + (int64_t)v * a.A + j0;
  if (((a.A | a.ld) & 1) == 0) {
    // inner tiles hold only real columns (TS = ceil(A / 16)); in the last
    // one j0 is a multiple of 4, so a lane's valid columns are 0, 2 or 4
    if (live && (u < TS - 1 || j0 + 2 < a.A)) {
      *reinterpret_cast<u32x2u *>(dst) = u32x2u{pk0, pk1};
    } else if (live && j0 < a.A) {
      *reinterpret_cast<uint32_t *>(dst) = pk0;
    }
  } else if (live && j0 < a.A) {
    dst[0] = (uint16_t)pk0;
    if (j0 + 1 < a.A) dst[1] = (uint16_t)(pk0 >> 16);
    if (j0 + 2 < a.A) dst[2] = (uint16_t)pk1;
    if (j0 + 3 < a.A) dst[3] = (uint16_t)(pk1 >> 16);
  }
}

// SMP (forward only): draw the action instead of reading it (SAMPLE mode).
template <int TS, bool BWD, int MC, int SEG = kMaxNT / TS, bool SMP = false>
struct Hg16Epi {
  static_assert(!(SMP && BWD), "sampling is a forward mode");
  static constexpr int S = SEG, NP = MC * S;  // S segments of TS tiles per column tile
  uint64_t seed = 0;  // SMP: the launch seed (eff_seed), set by the kernel
  static constexpr int W32 = (16 * TS + 31) / 32;  // = ceil(A / 32) for every A with ceil(A / 16) = TS
  // The (mc, s) rows' mask words and actions are loaded one row ahead (and
  // the backward's per-sample gradients up front), so a row's compute runs
  // under the next row's loads: loaded where used, every row waited on two
  // dependent global round trips, and each wait also drained the previous
  // row's dlogits stores.
  float glp_[MC], gen_[MC];
  uint32_t mwn[4];
  int actn;

  __device__ __forceinline__ static int64_t row_of(const H16Args &a, int pi, int m0, int v0, int wid,
                                                   int c) {
    const int m = m0 + 16 * (MC * wid + pi / S) + c;
    return (int64_t)(m < a.B ? m : a.B - 1) * a.V + min(v0 + pi % S, a.V - 1);
  }

  __device__ __forceinline__ void keep_live() {
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("" : "+v"(mwn[i]));
    asm volatile("" : "+v"(actn));
    if (BWD)
#pragma unroll
      for (int mc = 0; mc < MC; mc++) asm volatile("" : "+v"(glp_[mc]), "+v"(gen_[mc]));
  }

  __device__ __forceinline__ void begin(const H16Args &a, int m0, int v0, int wid, int lane) {
    const int c = lane & 15;
#pragma unroll
    for (int mc = 0; mc < MC; mc++) {
      const int m = m0 + 16 * (MC * wid + mc) + c;
      const int mm = m < a.B ? m : a.B - 1;
      glp_[mc] = (BWD && a.g_lp) ? a.g_lp[mm] : 0.f;
      gen_[mc] = (BWD && a.g_ent) ? a.g_ent[mm] : 0.f;
    }
    load_mask_raw<W32>(a, row_of(a, 0, m0, v0, wid, c), mwn);
    actn = SMP ? -1 : a.action[row_of(a, 0, m0, v0, wid, c)];
  }

  __device__ __forceinline__ void row(const H16Args &a, f32x4 (&acc)[S * TS][MC], const int pi,
                                      int m0, int v0, int wid, int lane, float LDSP *colL) {
    const int q = lane >> 4, c = lane & 15;
    const int mc = pi / S, s = pi % S;
    const int m = m0 + 16 * (MC * wid + mc) + c;
    const bool live = m < a.B;
    const int mm = live ? m : a.B - 1;
    const float glp = glp_[mc], gen = gen_[mc];
    uint32_t mw[4] = {mwn[0], mwn[1], mwn[2], mwn[3]};
    const int act = actn;
    if (pi + 1 < NP) {
      load_mask_raw<W32>(a, row_of(a, pi + 1, m0, v0, wid, c), mwn);
      actn = SMP ? -1 : a.action[row_of(a, pi + 1, m0, v0, wid, c)];
    }
    mask_fix<W32>(a, mw);
    const int v = v0 + s;
    if (v >= a.V) return;  // workgroup-uniform: the last tile's missing segments
    const int64_t row = (int64_t)mm * a.V + v;
    if (SMP && a.wait_ratio >= 0.f && a.bits) {
      // PPOAgent.act's WAIT coin (ppo.py:151-156, vmp_policy.hip coin_flip):
      // more than one invalid action and WAIT valid -> WAIT forbidden with
      // probability 1 - wait_ratio, by the unfused head's per-row uniform
      const int cnt = __popc(mw[0]) + __popc(mw[1]) + __popc(mw[2]) + __popc(mw[3]);
      const int P = a.wait_index, pw = P >> 5;
      const uint32_t pb = 1u << (P & 31);
      const uint32_t wword = pw == 0 ? mw[0] : pw == 1 ? mw[1] : pw == 2 ? mw[2] : mw[3];
      if (cnt > 1 && !(wword & pb) &&
          uniform_at(seed ^ 0xC0FFEE5EEDull, a.offset + (uint64_t)row) > a.wait_ratio) {
#pragma unroll
        for (int i = 0; i < 4; i++) mw[i] |= i == pw ? pb : 0u;
      }
    }
    const int tgt = (act >= 0 && act < a.A) ? act : -1;
    // pass 1: masked logits (-1e7 at invalid actions, kPad past A) and the row max
    float xm[TS][4];
    uint32_t nib[TS];
    float mx = kPad;
#pragma unroll
    for (int u = 0; u < TS; u++) {
      nib[u] = mw[u >> 1] >> (16 * (u & 1) + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int j = 16 * u + 4 * q + r;
        const float x = ((nib[u] >> r) & 1u) ? kMasked : acc[s * TS + u][mc][r];
        // TS = ceil(A / 16): only the segment's last tile reaches past A
        xm[u][r] = (u < TS - 1 || j < a.A) ? x : kPad;
        mx = fmaxf(mx, xm[u][r]);
      }
    }
    mx = xmax(mx);
    // pass 2: p = exp(x - m) (x - m first: exact at x = m, so an all-masked
    // row gets p = 1 everywhere, as the unfused head), S, T = sum p x
    float p[TS][4];
    float Ss = 0.f, Ts = 0.f;
#pragma unroll
    for (int u = 0; u < TS; u++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        p[u][r] = __builtin_amdgcn_exp2f((xm[u][r] - mx) * kLog2e);
        Ss += p[u][r];
        Ts = __builtin_fmaf(p[u][r], xm[u][r], Ts);
      }
    float xa = 0.f;
    if (!BWD && !SMP) {  // the given action's logit: tile u_t, register r_t of lane q_t
      const int ut = tgt >> 4, rt = tgt & 3, qt = (tgt >> 2) & 3;
      float sel[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < TS; u++)
#pragma unroll
        for (int r = 0; r < 4; r++) sel[r] = u == ut ? xm[u][r] : sel[r];
      xa = rt == 0 ? sel[0] : rt == 1 ? sel[1] : rt == 2 ? sel[2] : sel[3];
      xa = (tgt >= 0 && q == qt) ? xa : 0.f;
    }
    Ss = xsum(Ss);
    Ts = xsum(Ts);
    const float lse = mx + logf(Ss);
    const float inv = 1.0f / Ss;
    const float H = lse - Ts * inv;  // Categorical.entropy, the tiled head's order
    if (!BWD && SMP) {
      // inverse CDF over the row in action order j = 16 u + 4 q + r: the tile
      // totals T[u] (same value on every lane), the tile u* holding target,
      // then the first element of u* whose running sum passes target (the
      // running sums of the lanes q are built in q order by every lane)
      float tl[TS], T[TS];
#pragma unroll
      for (int u = 0; u < TS; u++) {
        tl[u] = ((p[u][0] + p[u][1]) + p[u][2]) + p[u][3];
        T[u] = xsum(tl[u]);
      }
      float tot = 0.f;
#pragma unroll
      for (int u = 0; u < TS; u++) tot += T[u];
      const float target = uniform_at(seed, a.offset + (uint64_t)row) * tot;
      int us = -1;
      float base = 0.f, cum = 0.f;
#pragma unroll
      for (int u = 0; u < TS; u++) {
        const float nx = cum + T[u];
        if (us < 0 && nx > target) {
          us = u;
          base = cum;
        }
        cum = nx;
      }
      int ulast = 0;  // rounding: target past every sum -> the last tile with mass
#pragma unroll
      for (int u = 0; u < TS; u++) ulast = T[u] > 0.f ? u : ulast;
      if (us < 0) {
        us = ulast;
        base = 0.f;
#pragma unroll
        for (int u = 0; u < TS; u++) base += u < ulast ? T[u] : 0.f;
      }
      float pu[4], xu[4], tu = 0.f;
#pragma unroll
      for (int r = 0; r < 4; r++) pu[r] = xu[r] = 0.f;
#pragma unroll
      for (int u = 0; u < TS; u++)
        if (u == us) {
          tu = tl[u];
#pragma unroll
          for (int r = 0; r < 4; r++) pu[r] = p[u][r], xu[r] = xm[u][r];
        }
      // the tile's lane sums in q order: lane q's running sum starts at
      // base + t_0 + ... + t_{q-1}
      const float t0 = __shfl(tu, c), t1 = __shfl(tu, 16 + c), t2 = __shfl(tu, 32 + c);
      float pre = base;
      pre = q > 0 ? pre + t0 : pre;
      pre = q > 1 ? pre + t1 : pre;
      pre = q > 2 ? pre + t2 : pre;
      int pick = 0x7fffffff, lastpos = -1;
      float cr = pre, xpick = 0.f, xlast = 0.f;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        cr += pu[r];
        const int j = 16 * us + 4 * q + r;
        if (pick == 0x7fffffff && cr > target && pu[r] > 0.f) {
          pick = j;
          xpick = xu[r];
        }
        if (pu[r] > 0.f) {
          lastpos = j;
          xlast = xu[r];
        }
      }
      // the smallest passing j over the 4 lanes of the sample (its logit
      // travels with it); none (rounding inside the tile): the tile's last
      // element with mass
      int jb = pick;
      float xb = xpick;
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        const int jo = __shfl_xor(jb, o);
        const float xo = __shfl_xor(xb, o);
        if (jo < jb) jb = jo, xb = xo;
      }
      if (jb == 0x7fffffff) {
        int jl = lastpos;
        float xl = xlast;
#pragma unroll
        for (int o = 16; o < 64; o <<= 1) {
          const int jo = __shfl_xor(jl, o);
          const float xo = __shfl_xor(xl, o);
          if (jo > jl) jl = jo, xl = xo;
        }
        jb = jl < 0 ? 0 : jl;
        xb = xl;
      }
      if (live && q == 0) {
        a.act_out[row] = jb;
        a.row_lp[row] = xb - lse;
        a.row_ent[row] = H;
      }
    } else if (!BWD) {
      xa = xsum(xa);  // one lane-element holds it, the others 0
      if (live && q == 0) {
        a.row_lp[row] = tgt >= 0 ? xa - lse : NAN;
        a.row_ent[row] = H;
      }
    } else {
      const float c1 = glp + gen * (H - lse);
      // pass 1's per-element mask compares are recomputed from the nibbles
      // here (kept live across pass 2 they are 64-bit SGPR pairs each, and
      // spilled)
#pragma unroll
      for (int u = 0; u < TS; u++) asm volatile("" : "+v"(nib[u]));
      int tq = tgt - 4 * q;
      asm volatile("" : "+v"(tq));
#pragma unroll
      for (int u = 0; u < TS; u++) {
        float d[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int j = 16 * u + 4 * q + r;
          float dd = -(p[u][r] * inv) * __builtin_fmaf(gen, xm[u][r], c1);
          dd += (16 * u + r == tq) ? glp : 0.f;
          d[r] = ((u < TS - 1 || j < a.A) && !((nib[u] >> r) & 1u)) ? dd : 0.f;  // inner tiles: j < A
        }
        if (colL) {
          // the bias gradient db = 1^T dlogits (ppo.py:258-287 through the
          // last Linear's bias): this row group's f32 column sums before the
          // bf16 rounding, added to the wave's LDS sums by lane c = 15
          float dl4[4];
#pragma unroll
          for (int r = 0; r < 4; r++) dl4[r] = live ? d[r] : 0.f;
          const float cs = row16_colsum4(dl4, c);
          if (c >= 12) colL[16 * (s * TS + u) + 4 * q + 2 * (c & 1) + ((c >> 1) & 1)] += cs;
        }
        // bf16 dlogits (round to nearest even), columns v A + j of row m
        const __bf16 b0 = (__bf16)d[0], b1 = (__bf16)d[1], b2 = (__bf16)d[2], b3 = (__bf16)d[3];
        const uint32_t pk0 = (uint32_t)__builtin_bit_cast(uint16_t, b0) |
                             ((uint32_t)__builtin_bit_cast(uint16_t, b1) << 16);
        const uint32_t pk1 = (uint32_t)__builtin_bit_cast(uint16_t, b2) |
                             ((uint32_t)__builtin_bit_cast(uint16_t, b3) << 16);
        store_dl_tile<TS>(a, m, v, u, q, pk0, pk1);
      }
    }
  }
};

// The workgroup's bias-gradient partial: its waves' LDS column sums added in
// wave order and stored to a.dpart[g][v A + j] (one workgroup per (column
// tile, M group) pair, so every partial is written exactly once; k_dsum
// reduces the M groups in order).
template <int TS, int NW>
__device__ __forceinline__ void hg16_dsum_flush(const H16Args &a, const float LDSP *cols, int v0,
                                                int g) {
  constexpr int S = kMaxNT / TS, NT = S * TS, SA = 16 * TS, BNp = 16 * NT;
  __syncthreads();
  for (int n = threadIdx.x; n < BNp; n += 64 * NW) {
    const int s = n / SA, j = n - s * SA, v = v0 + s;
    float x = 0.f;
#pragma unroll
    for (int w = 0; w < NW; w++) x += cols[w * BNp + n];
    if (v < a.V && j < a.A) a.dpart[(int64_t)g * a.V * a.A + v * a.A + j] = x;
  }
}

// db[n] += sum over the M groups g < G of part[g][n], in g order
__global__ void k_dsum(int64_t N, int G, const float *part, float *db) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float x = 0.f;
  for (int g = 0; g < G; g++) x += part[(int64_t)g * N + n];
  db[n] += x;
}

// NW waves per workgroup, each owning MC = 16 / NW columns of 16 samples
// (built: 8 waves x 2 columns, two waves per SIMD). Two LDS stages of BK = 64.
template <int TS, bool BWD, int NW, bool SMP = false>
__global__ __launch_bounds__(64 * NW, NW / 4) void k_hg16(H16Args a) {
  constexpr int S = kMaxNT / TS, NT = S * TS, SA = 16 * TS, BNp = 16 * NT;
  constexpr int MC = 16 / NW, kThreads = 64 * NW;
  constexpr int kStageW = BNp * kRow, kStage = kStageW + kBM * kRow;
  extern __shared__ __align__(16) char lds_raw[];
  char LDSP *lds = (char LDSP *)lds_raw;
  float LDSP *biasL = reinterpret_cast<float LDSP *>(lds + 2 * kStage);
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int q = lane >> 4, c = lane & 15;
  int n_tile, g;
  if (!hg16_tile(a, n_tile, g)) return;
  const int v0 = n_tile * S;
  const bool dsum = BWD && a.dpart;  // backward: the bias gradient's column sums too
  float LDSP *colL = dsum ? biasL + BNp + wid * BNp : nullptr;

  // the tile's bias in tile-column order (0 past A / past V)
  for (int n = t; n < BNp; n += kThreads) {
    const int s = n / SA, j = n - s * SA, v = v0 + s;
    biasL[n] = (v < a.V && j < a.A) ? a.bias[v * a.A + j] : 0.f;
  }
  if (dsum)
    for (int n = t; n < NW * BNp; n += kThreads) biasL[BNp + n] = 0.f;
  __syncthreads();

  const int nk = a.K / kBK;
  int sb = 0;  // LDS stage of K step 0 of this M block
  // K step 0 of the first M block; later blocks' step 0 is issued during the
  // previous block's last K step, into the stage that step does not read
  stage_issue<TS, NT, NW>(a, lds, v0, g * kBM, 0, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll 1
  for (int mb = g; mb < a.m_blocks; mb += a.m_groups) {
    const int m0 = mb * kBM;
    const int mn = mb + a.m_groups;  // next M block of this workgroup
    f32x4 acc[NT][MC];
#pragma unroll
    for (int nt = 0; nt < NT; nt++) {
      const f32x4 b4 = *reinterpret_cast<const f32x4 LDSP *>(biasL + 16 * nt + 4 * q);
#pragma unroll
      for (int mc = 0; mc < MC; mc++) acc[nt][mc] = b4;
    }
    // ---- GEMM: two LDS stages, the next stage's DMA under this stage's MFMAs ----
#pragma unroll 1
    for (int s = 0; s < nk; s++) {
      const char LDSP *cur = lds + ((sb + s) & 1) * kStage;
      char LDSP *nxt = lds + ((sb + s + 1) & 1) * kStage;
      if (s + 1 < nk)
        stage_issue<TS, NT, NW>(a, nxt, v0, m0, (s + 1) * kBK, wid, lane);
      else if (mn < a.m_blocks)
        stage_issue<TS, NT, NW>(a, nxt, v0, mn * kBM, 0, wid, lane);
      const char LDSP *Hs = cur + kStageW;
      // the stage's 2 x NT W fragments are read kPipe ahead of their two MFMAs
      // (an LDS read's latency is several 16-cycle MFMA pairs: read right
      // before its use, every pair waited on it); both K halves' h fragments
      // up front. The sched_group_barriers pin the pattern
      // {MFMA, MFMA, ds_read} so the compiler does not sink the reads again.
      constexpr int NF = 2 * NT;
      bf16x8 hf[2][MC];
#pragma unroll
      for (int kk = 0; kk < 2; kk++)
#pragma unroll
        for (int mc = 0; mc < MC; mc++) hf[kk][mc] = frag(Hs, 16 * (MC * wid + mc) + c, 4 * kk + q);
      bf16x8 wf[kPipe];
#pragma unroll
      for (int i = 0; i < kPipe; i++) wf[i] = frag(cur, 16 * (i % NT) + c, 4 * (i / NT) + q);
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * MC + kPipe, 0);
#pragma unroll
      for (int i = 0; i < NF; i++) {
        const int kk = i / NT, nt = i % NT;
#pragma unroll
        for (int mc = 0; mc < MC; mc++)
          acc[nt][mc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i % kPipe], hf[kk][mc], acc[nt][mc], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, MC, 0);
        if (i + kPipe < NF) {
          const int j = i + kPipe;
          wf[i % kPipe] = frag(cur, 16 * (j % NT) + c, 4 * (j / NT) + q);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    sb = (sb + nk) & 1;
    {
      Hg16Epi<TS, BWD, MC, S, SMP> ep;
      if (SMP) ep.seed = eff_seed(a);
      ep.begin(a, m0, v0, wid, lane);
#pragma unroll
      for (int pi = 0; pi < Hg16Epi<TS, BWD, MC, S, SMP>::NP; pi++)
        ep.row(a, acc, pi, m0, v0, wid, lane, colL);
    }
  }
  if (dsum) hg16_dsum_flush<TS, NW>(a, biasL + BNp, v0, g);
}

// stages, the tile's bias, the 8 waves' bias-gradient column sums (backward)
template <int TS>
constexpr size_t lds_bytes() {
  return 2 * (size_t)(16 * (kMaxNT / TS * TS) + kBM) * kRow + 9 * 16 * (kMaxNT / TS * TS) * sizeof(float);
}
static_assert(lds_bytes<1>() <= 160 * 1024, "stages exceed LDS");

int pick_ts(int A) { return (A + 15) / 16; }  // segment width: 16 TS columns, TS = ceil(A / 16)

// M groups: the grid is n_tiles x m_groups workgroups at one per CU; pick the
// group count whose last dispatch round is fullest (ties: fewer workgroups)
int pick_groups(int n_tiles, int m_blocks) {
  int best = 1;
  double best_eff = -1.0;
  for (int g = 1; g <= m_blocks && g <= 64; g++) {
    const int64_t wg = (int64_t)n_tiles * g;
    const double rounds = (double)((wg + 255) / 256);
    const double eff = (double)wg / (rounds * 256.0);
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = g;
    }
    if (eff > 0.97) break;
  }
  return best;
}

template <bool BWD, int NW, bool SMP = false>
hipError_t launch_ts(const H16Args &a, int TS, hipStream_t st) {
  const int64_t n_wg = a.team > 0 ? (int64_t)(a.teams + 7) / 8 * 8 * a.team
                                  : (int64_t)a.n_tiles * a.m_groups;
  const dim3 grid((unsigned)n_wg), block(64 * NW);
  switch (TS) {
#define VMP_HG16_CASE(T) \
  case T: hipLaunchKernelGGL((k_hg16<T, BWD, NW, SMP>), grid, block, lds_bytes<T>(), st, a); break;
    VMP_HG16_CASE(1) VMP_HG16_CASE(2) VMP_HG16_CASE(3) VMP_HG16_CASE(4)
    VMP_HG16_CASE(5) VMP_HG16_CASE(6) VMP_HG16_CASE(7)
    default: hipLaunchKernelGGL((k_hg16<8, BWD, NW, SMP>), grid, block, lds_bytes<8>(), st, a); break;
#undef VMP_HG16_CASE
  }
  return hipGetLastError();
}

template <bool BWD, bool SMP = false>
hipError_t launch_hg16(H16Args &a, hipStream_t st) {
  const int TS = pick_ts(a.A);
  const int S = kMaxNT / TS;
  a.n_tiles = (a.V + S - 1) / S;
  a.m_blocks = (a.B + kBM - 1) / kBM;
  const int team = kTeam;
  a.team = 0;
  if (team > 0 && a.m_blocks >= team) {
    // r walks per team member: the grid n_tiles x team x r (rounded to whole
    // teams per XCD) whose last round of 256 one-per-CU workgroups is fullest
    int best = 1;
    double best_eff = -1.0;
    for (int r = 1; r * team <= a.m_blocks && r <= 64; r++) {
      const int64_t teams = (int64_t)a.n_tiles * r;
      const int64_t wg = (teams + 7) / 8 * 8 * team;
      const double eff = (double)(teams * team) / ((double)((wg + 255) / 256) * 256.0);
      if (eff > best_eff + 1e-9) {
        best_eff = eff;
        best = r;
      }
      if (eff > 0.97) break;
    }
    a.team = team;
    a.teams = a.n_tiles * best;
    a.m_groups = team * best;
  } else {
    a.m_groups = pick_groups(a.n_tiles, a.m_blocks);
  }
  return launch_ts<BWD, 8, SMP>(a, TS, st);
}

int check_common(int32_t B, int32_t K, int32_t V, int32_t A, const void *h, const void *w,
                 const float *bias, const uint32_t *bits, const int32_t *action,
                 const char *who) {
  if (B < 0 || K < 1 || V < 1 || A < 1 || !h || !w || !bias || !action)
    return policy_fail(VMP_EINVAL, who);
  if (K % kBK != 0 || A > VMP_ACTOR_HEAD_MAX_A)
    return policy_fail(VMP_EINVAL, "bf16 actor head: needs K % 64 == 0 and A <= 128");
  if ((((uintptr_t)h) | ((uintptr_t)w)) & 15)
    return policy_fail(VMP_EINVAL, "bf16 actor head: h and weight must be 16-byte aligned");
  // the epilogue reads a row's W32 = ceil(A / 32) mask words as one u32x4
  // (W32 = 4) or u32x2 (W32 = 2), else word by word; rows are W32 words apart,
  // so the base alignment of that vector width is all it needs
  const int W32 = (A + 31) / 32;
  const uintptr_t need = W32 == 4 ? 15 : (W32 == 2 ? 7 : 3);
  if (((uintptr_t)bits) & need)
    return policy_fail(VMP_EINVAL, "bf16 actor head: mask_bits misaligned for its row width");
  return VMP_OK;
}

}  // namespace
}  // namespace vmp

using namespace vmp;

extern "C" int vmp_actor_head_bf16_fwd(int32_t B, int32_t K, int32_t V, int32_t A,
                                       const uint16_t *h, const uint16_t *weight,
                                       const float *bias, const uint32_t *mask_bits,
                                       const int32_t *action, float *logprob, float *entropy,
                                       float *workspace, void *stream) {
  int rc = check_common(B, K, V, A, h, weight, bias, mask_bits, action,
                        "vmp_actor_head_bf16_fwd: bad shape or null pointer");
  if (rc) return rc;
  if (!logprob || !entropy) return policy_fail(VMP_EINVAL, "vmp_actor_head_bf16_fwd: null output");
  if (B == 0) return VMP_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rows = (int64_t)B * V;
  float *scratch = nullptr, *ws = workspace;
  if (!ws) {
    hipError_t e = hipMallocAsync((void **)&scratch, 2 * rows * sizeof(float), st);
    if (e != hipSuccess) return policy_fail(VMP_EOOM, hipGetErrorString(e));
    ws = scratch;
  }
  H16Args a{};
  a.B = B, a.K = K, a.V = V, a.A = A, a.W32 = (A + 31) / 32, a.ld = V * A;
  a.h = h, a.w = weight, a.bias = bias, a.bits = mask_bits, a.action = action;
  a.row_lp = ws, a.row_ent = ws + rows;
  hipError_t e = launch_hg16<false>(a, st);
  if (e == hipSuccess) {
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

extern "C" int vmp_actor_head_bf16_sample(int32_t B, int32_t K, int32_t V, int32_t A,
                                          const uint16_t *h, const uint16_t *weight,
                                          const float *bias, const uint32_t *mask_bits,
                                          float wait_ratio, int32_t wait_index, uint64_t seed,
                                          uint64_t offset, const uint64_t *rng_counter,
                                          int32_t *action, float *logprob, float *entropy,
                                          float *workspace, void *stream) {
  int rc = check_common(B, K, V, A, h, weight, bias, mask_bits, action,
                        "vmp_actor_head_bf16_sample: bad shape or null pointer");
  if (rc) return rc;
  if (!logprob || !entropy)
    return policy_fail(VMP_EINVAL, "vmp_actor_head_bf16_sample: null output");
  if (wait_ratio >= 0.f && (!mask_bits || wait_index < 0 || wait_index >= A))
    return policy_fail(VMP_EINVAL, "vmp_actor_head_bf16_sample: the WAIT coin needs mask bits "
                                   "and 0 <= wait_index < A");
  if (B == 0) return VMP_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rows = (int64_t)B * V;
  float *scratch = nullptr, *ws = workspace;
  if (!ws) {
    hipError_t e = hipMallocAsync((void **)&scratch, 2 * rows * sizeof(float), st);
    if (e != hipSuccess) return policy_fail(VMP_EOOM, hipGetErrorString(e));
    ws = scratch;
  }
  H16Args a{};
  a.B = B, a.K = K, a.V = V, a.A = A, a.W32 = (A + 31) / 32, a.ld = V * A;
  a.h = h, a.w = weight, a.bias = bias, a.bits = mask_bits, a.act_out = action;
  a.row_lp = ws, a.row_ent = ws + rows;
  a.seed = seed, a.offset = offset, a.ctr = rng_counter;
  a.wait_ratio = wait_ratio, a.wait_index = wait_index;
  hipError_t e = launch_hg16<false, true>(a, st);
  if (e == hipSuccess) {
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

extern "C" int vmp_actor_head_bf16_bwd(int32_t B, int32_t K, int32_t V, int32_t A,
                                       const uint16_t *h, const uint16_t *weight,
                                       const float *bias, const uint32_t *mask_bits,
                                       const int32_t *action, const float *g_logprob,
                                       const float *g_entropy, uint16_t *dlogits, int32_t ld,
                                       float *dbias, float *workspace, void *stream) {
  int rc = check_common(B, K, V, A, h, weight, bias, mask_bits, action,
                        "vmp_actor_head_bf16_bwd: bad shape or null pointer");
  if (rc) return rc;
  if (!dlogits || ld < V * A)
    return policy_fail(VMP_EINVAL, "vmp_actor_head_bf16_bwd: null dlogits or ld < V*A");
  // even A and ld: the dlogits go out as 4-byte pairs
  if (((uintptr_t)dlogits) & 3)
    return policy_fail(VMP_EINVAL, "vmp_actor_head_bf16_bwd: dlogits must be 4-byte aligned");
  if (B == 0) return VMP_OK;
  H16Args a{};
  a.B = B, a.K = K, a.V = V, a.A = A, a.W32 = (A + 31) / 32, a.ld = ld;
  a.h = h, a.w = weight, a.bias = bias, a.bits = mask_bits, a.action = action;
  a.g_lp = g_logprob, a.g_ent = g_entropy, a.dl = dlogits;
  hipStream_t st = (hipStream_t)stream;
  float *scratch = nullptr;
  if (dbias) {  // partials per M group (at most bf16_bwd_workspace_floats floats)
    a.dpart = workspace;
    if (!a.dpart) {
      hipError_t e = hipMallocAsync((void **)&scratch,
                                    sizeof(float) * (size_t)vmp_actor_head_bf16_bwd_workspace(B, V, A),
                                    st);
      if (e != hipSuccess) return policy_fail(VMP_EOOM, hipGetErrorString(e));
      a.dpart = scratch;
    }
  }
  hipError_t e = launch_hg16<true>(a, st);
  if (e == hipSuccess && dbias) {
    const int64_t N = (int64_t)V * A;
    const int G = a.m_groups < a.m_blocks ? a.m_groups : a.m_blocks;
    hipLaunchKernelGGL(k_dsum, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, N, G, a.dpart,
                       dbias);
    e = hipGetLastError();
  }
  if (scratch) {
    hipError_t f = hipFreeAsync(scratch, st);
    if (e == hipSuccess) e = f;
  }
  if (e != hipSuccess) return policy_fail(VMP_EDEVICE, hipGetErrorString(e));
  return VMP_OK;
}

// floats of bias-gradient partials vmp_actor_head_bf16_bwd may use: V*A per M
// group, at most 64 groups x 8 (XCD teams) of 256-sample blocks
extern "C" int64_t vmp_actor_head_bf16_bwd_workspace(int32_t B, int32_t V, int32_t A) {
  const int64_t blocks = ((int64_t)B + kBM - 1) / kBM;
  const int64_t groups = blocks < 512 ? blocks : 512;
  return (groups < 1 ? 1 : groups) * (int64_t)V * A;
}
