// vmp_mlp.hip — the PPO actor's MLP for rollouts and eval (src/agents/ppo.py:
// 98-109: self.actor = Linear(D, H), Tanh, Linear(H, H), Tanh, Linear(H, N)),
// forward only, f32 (the reference's precision), in ONE launch.
//
// At the eval shape (config/10.yml: B 4 096, D 110, H 512, N 360) the three
// GEMMs are 0.46 / 2.1 / 1.5 GFLOP: hipBLASLt takes 18.6 / 20.5 / 21.3 us per
// call (profiles/r05_eval_blas_ab.log) and two torch tanh passes and their
// launches come on top. Here a workgroup owns 16 rows (one 16x16x4 MFMA row
// tile; B / 16 = 256 workgroups = one per CU at B = 4 096) and runs all three
// layers on them: the activations stay in LDS between layers (bias and tanh
// in the accumulator epilogue), so nothing but the logits reaches memory, and
// the weights stream from L2 (2 MB per workgroup; every workgroup of an XCD
// reads the same 2 MB, resident in its 4 MB L2).
//
// Layer Y[16][Nout] = X[16][K] W^T + b on v_mfma_f32_16x16x4_f32 (f32 in,
// f32 accumulate, exact f32 products). 8 waves, 2 per SIMD; wave w owns the
// 16-column tiles w, w + 8, ... of the layer. The weights are read in
// MFMA-fragment order from a PACKED copy (vmp_actor_mlp_pack, re-packed by
// the caller whenever a parameter changes): per (tile T, K step s of 32
// columns) 64 lanes x 8 floats, lane (c = l & 15, g = l >> 4) holding
// W[16 T + c][32 s + 8 g .. 8 g + 7], stored as two 1 KB halves, so every
// weight load of a wave is 1 KB contiguous. Read straight from the nn.Linear
// rows, a wave's float4 load touched 16 rows x 64 B: the texture path then
// paced the kernel at ~2.6x its MFMA time (81 us at the eval shape against
// 31 us of MFMA work). MFMA i takes element i of the lane's weight and
// activation float4s, so its K index g stands for column 32 s + 8 g + 4 h +
// i: every product of the 32 columns is summed once (a permuted order inside
// each MFMA, not a GEMM library's; the f32 rounding differs from
// hipBLASLt's at the last bit, both within the 1e-5 of
// test_network_outputs_match_reference). K is zero-padded in the packed
// weights and in the LDS activations to a multiple of 32 kPf; weight loads
// are issued kPf K steps ahead of their MFMAs. LDS activation rows are padded
// to a stride of 4 x odd words, so the 16 rows' float4 reads of one lane
// group g cover the 64 banks once.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "../../include/vmp.h"
#include "vmp_head_dev.h"

#define LDSP __attribute__((address_space(3)))

namespace vmp {

int policy_fail(int code, const char *msg);

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = 16;     // rows per workgroup (the MFMA's M)
constexpr int kWaves = 8;     // 2 per SIMD (16 waves, 2 tiles each: no faster)
constexpr int kPf = 4;        // K steps (of 32 columns) of weight loads in flight
constexpr int kMaxTpw = 4;    // 16-column tiles per wave: N <= 8 * 16 * 4 = 512

struct MlpArgs {
  int B, D, H, N, layers;
  int Dp, Hp, ldx, ldh;  // D, H rounded up to 32 kPf; LDS row strides (words)
  const float *x, *b1, *b2, *b3;
  const float *p1, *p2, *p3;  // the layers' packed weights (vmp_actor_mlp_pack)
  float *out;  // [B][N] (layers 3) or [B][H] (layers 2); head: the nullable logits copy
  // the masked head on the logits (vmp_actor_mlp_head_f32): N = V * A
  int V, A, W, mode, wait_index;
  float wait_ratio;
  uint64_t seed, offset;
  const uint64_t *ctr;
  uint64_t *ctr_bump;  // non-null: add 1 to ctr[0] after every workgroup read it (ctr[1]: ticket)
  const uint32_t *bits;
  int32_t *action;  // in (GIVEN) or out (SAMPLE / ARGMAX), [B][V]
  float *logprob, *entropy;  // [B], nullable
};

__device__ __forceinline__ f32x4 ld4(const float *p) { return *reinterpret_cast<const f32x4 *>(p); }

typedef f32x4 Frags[kPf][kMaxTpw][2];  // a wave's weight fragments for kPf K steps

// The first TPW tiles' fragment pointers of a wave (tiles past the last:
// the last tile) and their loads for K steps 0 .. kPf - 1.
template <int TPW>
__device__ __forceinline__ void tile_ptrs(const float *Wp, int S, int ntile, int wid, int lane,
                                          const float *(&wp)[kMaxTpw]) {
#pragma unroll
  for (int t = 0; t < TPW; t++)
    wp[t] = Wp + (int64_t)min(wid + kWaves * t, ntile - 1) * S * 512 + 4 * lane;
}
template <int TPW>
__device__ __forceinline__ void load_step(Frags &wf, int j, const float *const (&wp)[kMaxTpw],
                                          int s) {
#pragma unroll
  for (int t = 0; t < TPW; t++) {
    wf[j][t][0] = ld4(wp[t] + 512 * s);
    wf[j][t][1] = ld4(wp[t] + 512 * s + 256);
  }
}

// Y = act W^T + b for the block's 16 rows; TPW tiles per wave. `act` rows
// hold Kp columns (a multiple of 32 kPf, zeros past K); Wp: the layer's
// packed weights (Kp columns, ceil(Nout / 16) tiles). OUT: 0 = tanh into LDS
// rows (stride ldo), 1 = raw to global rows m0.. (stride ldo), 2 = tanh to
// global, 3 = raw into LDS rows (stride Nout) and, if outG is set, to global
// as 1. Tiles past Nout compute on the last tile (never stored).
// wf: the wave's fragment registers; LOADED: K steps 0 .. kPf - 1 are
// already in flight (layer 1's, issued at kernel start). Prefetching the next
// layer's first steps into the registers the last steps free measured no
// faster (49.7 / 50.1 / 49.8 us at 0 / 1 / 2 steps, eval shape) and costs
// 32 VGPRs per step: not done.
template <int TPW, int OUT, bool LOADED = false>
__device__ __forceinline__ void layer(const float LDSP *act, int lda, int Kp, const float *Wp,
                                      const float *bias, int Nout, float LDSP *outL, float *outG,
                                      int ldo, int m0, int B, int wid, int lane, Frags &wf) {
  const int c = lane & 15, g = lane >> 4;
  const int ntile = (Nout + 15) >> 4, S = Kp >> 5;  // S: a multiple of kPf
  f32x4 acc[TPW];
  const float *wp[kMaxTpw];
  tile_ptrs<TPW>(Wp, S, ntile, wid, lane, wp);
  if (!LOADED) {
#pragma unroll
    for (int j = 0; j < kPf; j++) load_step<TPW>(wf, j, wp, j);
  }
#pragma unroll
  for (int t = 0; t < TPW; t++) {
    const float b = bias[min(min(wid + kWaves * t, ntile - 1) * 16 + c, Nout - 1)];
    acc[t] = f32x4{b, b, b, b};  // the bias is the accumulators' start
  }
  const float LDSP *arow = act + c * lda + 8 * g;
  // one K step: its 8 TPW MFMAs on wf[j], then (LOAD) wf[j]'s reload for
  // step s + kPf into the same registers, issued after their last use. The
  // main loop always reloads and the last kPf steps never do, so no branch
  // merges loaded and unloaded fragments (a merge made the compiler copy the
  // fresh loads and wait for all of them: the prefetch collapsed to ~1 step)
  auto kstep = [&](int s, int j, bool load) {
    const f32x4 a0 = *reinterpret_cast<const f32x4 LDSP *>(arow + 32 * s);
    const f32x4 a1 = *reinterpret_cast<const f32x4 LDSP *>(arow + 32 * s + 4);
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int t = 0; t < TPW; t++)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[i], wf[j][t][0][i], acc[t], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int t = 0; t < TPW; t++)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i], wf[j][t][1][i], acc[t], 0, 0, 0);
    if (load) load_step<TPW>(wf, j, wp, s + kPf);
    __builtin_amdgcn_sched_barrier(0);  // keep the reloads here (the scheduler sank them all
                                        // to the loop's end, behind a vmcnt(0))
  };
#pragma unroll 1
  for (int s0 = 0; s0 + kPf < S; s0 += kPf) {
#pragma unroll
    for (int j = 0; j < kPf; j++) kstep(s0 + j, j, true);
  }
#pragma unroll
  for (int j = 0; j < kPf; j++) kstep(S - kPf + j, j, false);
  // accumulator layout: acc[t][i] = Y[row 4 g + i][column 16 tile + c]
#pragma unroll
  for (int t = 0; t < TPW; t++) {
    const int n = (wid + kWaves * t) * 16 + c;
    if (n >= Nout) continue;  // (also every tile past the last)
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int r = 4 * g + i;
      if (OUT == 0) {
        outL[r * ldo + n] = tanhf(acc[t][i]);
      } else if (OUT == 3) {
        outL[r * Nout + n] = acc[t][i];
        if (outG && m0 + r < B) outG[(int64_t)(m0 + r) * ldo + n] = acc[t][i];
      } else if (m0 + r < B) {
        outG[(int64_t)(m0 + r) * ldo + n] = OUT == 2 ? tanhf(acc[t][i]) : acc[t][i];
      }
    }
  }
}

// The masked head (ppo.py:115-131, PPOAgent.act's WAIT coin ppo.py:151-156)
// on the block's logits in LDS (16 rows x N, N = V * A): one (sample, VM) row
// per lane through hd::lane_row, the single-lane restatement of the quad code
// k_head_fwd_tile runs, then the per-sample sums over V in k_rowsum's order:
// equal logits give the unfused head's actions, log-probabilities and
// entropies bit for bit.
// ctr0: thread 0's copy of the device counter, loaded at kernel start.
__device__ __forceinline__ void block_head(const MlpArgs &a, float *lg, float *rlp, float *rent,
                                           const uint32_t *mb, int m0, int t, int lane, int wid,
                                           uint64_t ctr0) {
  // the launch's seed (hd::eff_seed on the counter thread 0 read at kernel
  // start, its latency under the layers), broadcast through LDS
  __shared__ uint64_t seed_s;
  if (t == 0) seed_s = a.ctr ? a.seed ^ hd::mix64(ctr0 + 0x5851F42D4C957F2Dull) : a.seed;
  __syncthreads();
  const uint64_t seed = seed_s;
  for (int lr = t; lr < kRows * a.V; lr += 64 * kWaves) {  // one row per lane
    const int b = lr / a.V, v = lr - b * a.V;
    if (m0 + b >= a.B) continue;
    const int64_t row = (int64_t)(m0 + b) * a.V + v;
    const float *rp = lg + b * a.N + v * a.A;
    uint32_t mw[4];
    hd::mask_words(a.bits ? mb : nullptr, a.W, a.A, b * a.V + v, mw);  // staged in LDS
    const int fw = a.mode == VMP_HEAD_ARGMAX
                       ? -1
                       : hd::coin_flip(a.wait_ratio, a.wait_index, a.bits != nullptr, seed,
                                       a.offset, row, mw);
    const float u = a.mode == VMP_HEAD_SAMPLE ? hd::uniform_at(seed, a.offset + (uint64_t)row) : 0.f;
    const int given = a.mode == VMP_HEAD_GIVEN ? a.action[row] : -1;
    const hd::LaneRow r = a.A <= 16 ? hd::lane_row<16>(rp, mw, a.A, fw, a.mode, u, given)
                                    : hd::lane_row<0>(rp, mw, a.A, fw, a.mode, u, given);
    if (a.mode != VMP_HEAD_GIVEN) a.action[row] = r.act;
    if (a.mode != VMP_HEAD_ARGMAX) {
      rlp[b * a.V + v] = r.lp;
      rent[b * a.V + v] = r.H;
    }
  }
  if (a.mode == VMP_HEAD_ARGMAX) return;
  if (a.ctr_bump && t == 0) {
    // the launch advances its own sampling counter: the last workgroup to take
    // a ticket (every other one has read ctr[0]: thread 0 used its value
    // above) adds 1 and re-arms the ticket for the next launch, which is
    // stream-ordered after this one. Taken after the rows, off their path.
    // Relaxed device-scope atomics suffice: the only order needed is "read
    // before ticket", which thread 0's use of ctr0 above gives, and the next
    // launch sees the counter through the kernel boundary (a release fence
    // here writes the L2 back: ~8 us per launch, measured).
    const uint64_t k = __hip_atomic_fetch_add(a.ctr_bump + 1, 1ull, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (k == (uint64_t)gridDim.x - 1) {
      __hip_atomic_fetch_add(a.ctr_bump, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.ctr_bump + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  // per sample: lane-strided partial sums, then the xor tree (k_rowsum)
#pragma unroll
  for (int k = 0; k < kRows / kWaves; k++) {
    const int b = (kRows / kWaves) * wid + k;
    if (m0 + b >= a.B) break;  // wave-uniform
    float s0 = 0.f, s1 = 0.f;
    for (int v = lane; v < a.V; v += 64) {
      s0 += rlp[b * a.V + v];
      s1 += rent[b * a.V + v];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o);
      s1 += __shfl_xor(s1, o);
    }
    if (lane == 0) {
      if (a.logprob) a.logprob[m0 + b] = s0;
      if (a.entropy) a.entropy[m0 + b] = s1;
    }
  }
}

template <int TPW3, bool HEAD>
__global__ __launch_bounds__(64 * kWaves, kWaves / 4) void k_actor_mlp(MlpArgs a) {
  extern __shared__ __align__(16) float lds[];
  // region X: the input rows, later the second hidden layer; region H1
  float LDSP *X = (float LDSP *)lds;
  float LDSP *H1 = X + kRows * (a.ldx > a.ldh ? a.ldx : a.ldh);
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int m0 = blockIdx.x * kRows;
  // head: the block's mask words, staged in LDS under the layers' work (a
  // global round trip per (sample, VM) row in the head cost ~10 us)
  float *lg = lds + kRows * ((a.ldx > a.ldh ? a.ldx : a.ldh) + a.ldh);
  float *rlp = lg + kRows * a.N, *rent = rlp + kRows * a.V;
  uint32_t *mb = reinterpret_cast<uint32_t *>(rent + kRows * a.V);
  // layer 1's first kPf weight steps go out first, under the row staging
  Frags wf;
  {
    const float *wp[kMaxTpw];
    tile_ptrs<kMaxTpw>(a.p1, a.Dp >> 5, (a.H + 15) >> 4, wid, lane, wp);
#pragma unroll
    for (int j = 0; j < kPf; j++) load_step<kMaxTpw>(wf, j, wp, j);
  }
  uint64_t ctr0 = 0;
  if (HEAD && a.ctr && t == 0) ctr0 = *a.ctr;
  if (HEAD && a.bits) {
    const int nw = kRows * a.V * a.W;
    const int64_t w0 = (int64_t)m0 * a.V * a.W, wend = (int64_t)a.B * a.V * a.W;
    for (int i = t; i < nw; i += 64 * kWaves) mb[i] = w0 + i < wend ? a.bits[w0 + i] : 0u;
  }
  // the 16 input rows, zero-padded to Dp columns (rows past B: zeros); the
  // hidden rows' padding columns [H, Hp) zeroed once (the layers write < H)
  for (int i = t; i < kRows * a.Dp; i += 64 * kWaves) {
    const int r = i / a.Dp, k = i - r * a.Dp;
    X[r * a.ldx + k] = (m0 + r < a.B && k < a.D) ? a.x[(int64_t)(m0 + r) * a.D + k] : 0.f;
  }
  const int hpad = a.Hp - a.H;
  for (int i = t; i < kRows * hpad; i += 64 * kWaves) {
    const int r = i / hpad, k = a.H + i - r * hpad;
    H1[r * a.ldh + k] = 0.f;
  }
  __syncthreads();
  layer<kMaxTpw, 0, true>(X, a.ldx, a.Dp, a.p1, a.b1, a.H, H1, nullptr, a.ldh, m0, a.B, wid, lane,
                          wf);
  __syncthreads();
  if (a.layers == 2) {  // self.actor[:-1]: the last hidden layer, after its Tanh
    layer<kMaxTpw, 2>(H1, a.ldh, a.Hp, a.p2, a.b2, a.H, nullptr, a.out, a.H, m0, a.B, wid, lane,
                         wf);
    return;
  }
  // the second hidden layer overwrites X (row stride ldh); its padding columns
  for (int i = t; i < kRows * hpad; i += 64 * kWaves) {
    const int r = i / hpad, k = a.H + i - r * hpad;
    X[r * a.ldh + k] = 0.f;
  }
  layer<kMaxTpw, 0>(H1, a.ldh, a.Hp, a.p2, a.b2, a.H, X, nullptr, a.ldh, m0, a.B, wid, lane, wf);
  __syncthreads();
  if (!HEAD) {
    layer<TPW3, 1>(X, a.ldh, a.Hp, a.p3, a.b3, a.N, nullptr, a.out, a.N, m0, a.B, wid, lane, wf);
    return;
  }
  // the logits stay in LDS for the head (generic pointers: the head's per-row
  // code is shared with k_head_fwd_tile)
  layer<TPW3, 3>(X, a.ldh, a.Hp, a.p3, a.b3, a.N, (float LDSP *)lg, a.out, a.N, m0, a.B, wid,
                    lane, wf);
  __syncthreads();
  block_head(a, lg, rlp, rent, mb, m0, t, lane, wid, ctr0);
}

// Padded K of a layer's packed weights: a multiple of 32 kPf.
__host__ __device__ inline int kpad(int K) { return (K + 32 * kPf - 1) / (32 * kPf) * (32 * kPf); }

// The fragment-order copy of one Linear's weight W[N][K]: element
// ((T * S + s) * 2 + h) * 256 + 4 l + j = W[16 T + (l & 15)][32 s + 8 (l >> 4)
// + 4 h + j] (0 past N or K), S = kpad(K) / 32, T < ceil(N / 16).
__global__ void k_mlp_pack(const float *W, int N, int K, float *out, int64_t n_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_out) return;
  const int S = kpad(K) >> 5;
  const int j = (int)(i & 3), l = (int)((i >> 2) & 63), h = (int)((i >> 8) & 1);
  const int64_t ts = i >> 9;
  const int s = (int)(ts % S), T = (int)(ts / S);
  const int n = 16 * T + (l & 15), k = 32 * s + 8 * (l >> 4) + 4 * h + j;
  out[i] = (n < N && k < K) ? W[(int64_t)n * K + k] : 0.f;
}

}  // namespace
}  // namespace vmp

using namespace vmp;

namespace {
// floats of each layer's packed copy (tiles x 16 x padded K)
int64_t pack_floats(int N, int K) { return (int64_t)((N + 15) / 16) * 16 * kpad(K); }

// checks shared by both entry points; fills the layer part of `a`
int mlp_setup(MlpArgs &a, int32_t B, int32_t D, int32_t H, int32_t N, int32_t layers,
              const float *x, const float *packed, const float *b1, const float *b2,
              const float *b3, const char *who) {
  if (B < 0 || D < 1 || H < 32 || (layers != 2 && layers != 3) || !x || !packed || !b1 || !b2 ||
      (layers == 3 && (N < 1 || !b3)))
    return policy_fail(VMP_EINVAL, who);
  if (H % 32 != 0 || H > 16 * kWaves * kMaxTpw || (layers == 3 && N > 16 * kWaves * kMaxTpw) ||
      D > VMP_ACTOR_MLP_MAX_D)
    return policy_fail(VMP_EINVAL, "actor MLP: needs H % 32 == 0, H <= 512, N <= 512, "
                                   "D <= VMP_ACTOR_MLP_MAX_D");
  if (((uintptr_t)packed) & 15)
    return policy_fail(VMP_EINVAL, "actor MLP: packed weights must be 16-byte aligned");
  a.B = B, a.D = D, a.H = H, a.N = N, a.layers = layers;
  a.Dp = kpad(D);
  a.Hp = kpad(H);
  a.ldx = a.Dp + 4;  // 4 x odd words: conflict-free float4 rows
  a.ldh = a.Hp + 4;
  a.x = x, a.b1 = b1, a.b2 = b2, a.b3 = b3;
  a.p1 = packed;
  a.p2 = a.p1 + pack_floats(H, D);
  a.p3 = a.p2 + pack_floats(H, H);
  return VMP_OK;
}

size_t mlp_lds(const MlpArgs &a) {
  return sizeof(float) * kRows * ((size_t)(a.ldx > a.ldh ? a.ldx : a.ldh) + a.ldh);
}

int mlp_launch(const MlpArgs &a, bool head, size_t lds, void *stream) {
  if (lds > 160 * 1024) return policy_fail(VMP_EINVAL, "actor MLP: the block's LDS exceeds 160 KB");
  const dim3 grid((unsigned)((a.B + kRows - 1) / kRows)), block(64 * kWaves);
  hipStream_t st = (hipStream_t)stream;
  const int tpw3 = a.layers == 3 ? ((a.N + 15) / 16 + kWaves - 1) / kWaves : kMaxTpw;
#define VMP_MLP_LAUNCH(T, HD) hipLaunchKernelGGL((k_actor_mlp<T, HD>), grid, block, lds, st, a)
#define VMP_MLP_TPW(HD)                       \
  if (tpw3 <= 1) VMP_MLP_LAUNCH(1, HD);       \
  else if (tpw3 == 2) VMP_MLP_LAUNCH(2, HD);  \
  else if (tpw3 == 3) VMP_MLP_LAUNCH(3, HD);  \
  else VMP_MLP_LAUNCH(4, HD);
  if (head) {
    VMP_MLP_TPW(true)
  } else {
    VMP_MLP_TPW(false)
  }
#undef VMP_MLP_TPW
#undef VMP_MLP_LAUNCH
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return policy_fail(VMP_EDEVICE, hipGetErrorString(e));
  return VMP_OK;
}
}  // namespace

extern "C" int64_t vmp_actor_mlp_packed_floats(int32_t D, int32_t H, int32_t N, int32_t layers) {
  if (D < 1 || H < 1 || (layers == 3 && N < 1)) return -1;
  return pack_floats(H, D) + pack_floats(H, H) + (layers == 3 ? pack_floats(N, H) : 0);
}

extern "C" int vmp_actor_mlp_pack(int32_t D, int32_t H, int32_t N, int32_t layers, const float *w1,
                                  const float *w2, const float *w3, float *packed, void *stream) {
  if (D < 1 || H < 1 || (layers != 2 && layers != 3) || !w1 || !w2 || !packed ||
      (layers == 3 && (N < 1 || !w3)))
    return policy_fail(VMP_EINVAL, "vmp_actor_mlp_pack: bad shape or null pointer");
  hipStream_t st = (hipStream_t)stream;
  const float *src[3] = {w1, w2, w3};
  const int n[3] = {H, H, N}, k[3] = {D, H, H};
  float *dst = packed;
  for (int i = 0; i < layers; i++) {
    const int64_t m = pack_floats(n[i], k[i]);
    hipLaunchKernelGGL(k_mlp_pack, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, src[i],
                       n[i], k[i], dst, m);
    dst += m;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return policy_fail(VMP_EDEVICE, hipGetErrorString(e));
  return VMP_OK;
}

extern "C" int vmp_actor_mlp_f32(int32_t B, int32_t D, int32_t H, int32_t N, int32_t layers,
                                 const float *x, const float *packed, const float *b1,
                                 const float *b2, const float *b3, float *out, void *stream) {
  MlpArgs a{};
  int rc = mlp_setup(a, B, D, H, N, layers, x, packed, b1, b2, b3,
                     "vmp_actor_mlp_f32: bad shape or null pointer");
  if (rc) return rc;
  if (!out) return policy_fail(VMP_EINVAL, "vmp_actor_mlp_f32: null output");
  if (B == 0) return VMP_OK;
  a.out = out;
  return mlp_launch(a, false, mlp_lds(a), stream);
}

extern "C" int vmp_actor_mlp_head_f32(int32_t B, int32_t D, int32_t H, int32_t V, int32_t A,
                                      int32_t mode, const float *x, const float *packed,
                                      const float *b1, const float *b2, const float *b3,
                                      const uint32_t *mask_bits, float wait_ratio,
                                      int32_t wait_index, uint64_t seed, uint64_t offset,
                                      const uint64_t *rng_counter, int32_t advance_counter,
                                      int32_t *action, float *logprob, float *entropy,
                                      float *logits_out, void *stream) {
  MlpArgs a{};
  if (V < 1 || A < 1 || A > VMP_ACTOR_HEAD_MAX_A || (int64_t)V * A > 512 || !action ||
      (mode != VMP_HEAD_SAMPLE && mode != VMP_HEAD_GIVEN && mode != VMP_HEAD_ARGMAX))
    return policy_fail(VMP_EINVAL, "vmp_actor_mlp_head_f32: bad head shape, mode or null action");
  if (wait_ratio >= 0.f && mask_bits && (wait_index < 0 || wait_index >= A))
    return policy_fail(VMP_EINVAL, "vmp_actor_mlp_head_f32: wait_index out of the row");
  int rc = mlp_setup(a, B, D, H, V * A, 3, x, packed, b1, b2, b3,
                     "vmp_actor_mlp_head_f32: bad shape or null pointer");
  if (rc) return rc;
  if (B == 0) return VMP_OK;
  a.out = logits_out;
  a.V = V, a.A = A, a.W = (A + 31) / 32, a.mode = mode;
  a.wait_ratio = wait_ratio, a.wait_index = wait_index;
  a.seed = seed, a.offset = offset, a.ctr = rng_counter, a.bits = mask_bits;
  a.ctr_bump = (advance_counter && rng_counter) ? const_cast<uint64_t *>(rng_counter) : nullptr;
  a.action = action, a.logprob = logprob, a.entropy = entropy;
  const size_t lds = mlp_lds(a) + sizeof(float) * kRows * ((size_t)a.N + 2 * V) +
                     (mask_bits ? sizeof(uint32_t) * kRows * (size_t)V * a.W : 0);
  return mlp_launch(a, true, lds, stream);
}
