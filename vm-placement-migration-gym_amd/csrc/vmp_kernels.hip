// vmp_kernels.hip — gfx950 kernels for the batched VmEnv hot path.
//
// One 64-lane wavefront owns one env for a whole launch (4 envs per 256-thread
// workgroup, the waves never synchronise with each other after the prologue).
// Lane l holds VM slots v = s*64 + l (s < VPT) in registers: the reference's
// per-VM Python loops (env.py:68-88, 244-293) become lane-parallel passes, and
// the only truly ordered work — resource updates on one PM, which must happen
// in VM order — runs as a wave-uniform loop over the
// ballot of the slots that carry an event. PM resources (f64) live in LDS.
//
// Exactness: all f64 arithmetic follows the reference's operation order; the
// build uses -ffp-contract=off; numpy's pairwise summation, PCG64 streams,
// Poisson samplers and np.around are restated bit-for-bit (see oracle/ for the
// CPU restatement these kernels are tested against).
#include <hip/hip_runtime.h>

#include "vmp_layout.h"

// Pointers into LDS carry address space 3 explicitly: 32-bit addresses (half
// the SGPRs of generic pointers) and ds_* instructions without relying on
// address-space inference through the helpers.
#define LDSP __attribute__((address_space(3)))

// Minimum waves per SIMD the env kernel is register-allocated for
// (__launch_bounds__ 2nd argument); measured choice, see DESIGN.md.
#ifndef VMP_WAVES_PER_EU
#define VMP_WAVES_PER_EU 2
#endif
#ifndef VMP_WAVES_PER_EU_ONE  // the per-step (k_steps == 1) instantiation
#define VMP_WAVES_PER_EU_ONE 3
#endif

namespace vmp {

// Global (address space 1) views of HBM pointers. Pointers read out of the
// EnvParams / StepOut structs are generic, and generic accesses compile to
// FLAT instructions, which count in lgkmcnt as well as vmcnt: every later
// s_waitcnt lgkmcnt for an LDS access then also waits for them to complete
// (in k_env_big the mid-step state stores stalled every following LDS wait).
#define GLBP __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T GLBP *gptr(T *p) {
  return (T GLBP *)p;
}

#ifdef VMP_CHECK_QUIET
// quiet-bit check build: quiet steps in which some pending VM fit a PM
__device__ unsigned long long g_quiet_violations;
#endif
// -> the count since the last call (reset to 0); -1 in a build without the check
int64_t quiet_violations_take() {
#ifdef VMP_CHECK_QUIET
  unsigned long long v = 0, z = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_quiet_violations), sizeof(v)) != hipSuccess) return -2;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_quiet_violations), &z, sizeof(z)) != hipSuccess) return -2;
  return (int64_t)v;
#else
  return -1;
#endif
}

// Register row s of lane ln (slot v = 64 s + ln) in the blocked VM words of
// a wave kernel: the slot word's index (= vm_slot_idx(v)), + 64 for the time
// word. vm_pitch pads the env's blocks to the kernel's rows, so a padded slot
// (v >= V) reads padding inside the env's pitch, never used.
__device__ __forceinline__ int vw_row(int s, int ln) { return (s << 7) + ln; }

// Streaming stores (obs / state written once per launch, not re-read by it).
#ifdef VMP_NT_STORE
#define ST_NT(ptr, val) __builtin_nontemporal_store((val), gptr(ptr))
#else
#define ST_NT(ptr, val) (*gptr(ptr) = (val))
#endif

// ------------------------------------------------------------ wave utils --
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// An LDS base the compiler cannot tie to earlier address arithmetic: the
// pointers make_lds derives from it at a late use are recomputed there instead
// of being kept live (and spilled) from the prologue.
__device__ __forceinline__ char LDSP *opaque_base(char LDSP *b) {
  uint32_t x = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)b);  // 32-bit
  asm volatile("" : "+s"(x));
  return (char LDSP *)(uintptr_t)x;
}
// The lane id recomputed where the compiler cannot tie it to lane_id(): slot
// indices s*64 + lane built from it in a late phase (the obs / state stores)
// are not the prologue's, which the register allocator otherwise keeps live
// (spilled to scratch) from the loads at entry to the stores at exit.
__device__ __forceinline__ int fresh_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int below(uint64_t m, int lane) {
  return __popcll(m & ((1ull << lane) - 1ull));
}
// LDS hand-off between lanes of ONE wave: order the accesses, no s_barrier.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint32_t rdlane(uint32_t x, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}

// ------------------------------------------------------------- PCG64 -----
// numpy PCG64 (pcg64.h): 128-bit LCG, XSL-RR output, next_double = (u64>>11)*2^-53.
struct U128 {
  uint64_t hi, lo;
};
constexpr uint64_t kMulHi = 0x2360ED051FC65DA4ULL, kMulLo = 0x4385DF649FCCF645ULL;

__device__ __forceinline__ U128 mul128(U128 a, U128 b) {
  U128 r;
  r.lo = a.lo * b.lo;
  r.hi = __umul64hi(a.lo, b.lo) + a.lo * b.hi + a.hi * b.lo;
  return r;
}
__device__ __forceinline__ U128 add128(U128 a, U128 b) {
  U128 r;
  r.lo = a.lo + b.lo;
  r.hi = a.hi + b.hi + (r.lo < a.lo);
  return r;
}
struct Pcg {
  U128 s, inc;
};
__device__ __forceinline__ uint64_t pcg_next(Pcg &r) {
  r.s = add128(mul128(r.s, U128{kMulHi, kMulLo}), r.inc);
  uint64_t x = r.s.hi ^ r.s.lo;
  unsigned rot = (unsigned)(r.s.hi >> 58);
  return (x >> rot) | (x << ((64 - rot) & 63));
}
__device__ __forceinline__ double next_double(Pcg &r) {
  return (double)(pcg_next(r) >> 11) * (1.0 / 9007199254740992.0);
}
// pcg_advance_lcg_128: jump by delta draws.
__device__ void pcg_advance(Pcg &r, uint64_t delta) {
  U128 cur_mult{kMulHi, kMulLo}, cur_plus = r.inc, acc_mult{0, 1}, acc_plus{0, 0};
  while (delta > 0) {
    if (delta & 1) {
      acc_mult = mul128(acc_mult, cur_mult);
      acc_plus = add128(mul128(acc_plus, cur_mult), cur_plus);
    }
    cur_plus = mul128(add128(cur_mult, U128{0, 1}), cur_plus);
    cur_mult = mul128(cur_mult, cur_mult);
    delta >>= 1;
  }
  r.s = add128(mul128(acc_mult, r.s), acc_plus);
}
// SeedSequence(seed).generate_state(4, uint64) -> pcg64_set_seed (bit_generator.pyx).
__device__ void pcg_seed(Pcg &r, uint64_t seed) {
  const uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u, INIT_B = 0x8b51f9ddu,
                 MULT_B = 0x58f38dedu, MIX_L = 0xca01f9ddu, MIX_R = 0x4973f715u;
  uint32_t ent0 = (uint32_t)seed, ent1 = (uint32_t)(seed >> 32);
  int n_ent = (seed >> 32) ? 2 : 1;
  uint32_t pool[4];
  uint32_t hc = INIT_A;
  auto hashmix = [&](uint32_t v) {
    v ^= hc;
    hc *= MULT_A;
    v *= hc;
    v ^= v >> 16;
    return v;
  };
#pragma unroll
  for (int i = 0; i < 4; i++) pool[i] = hashmix(i == 0 ? ent0 : (i == 1 && n_ent == 2 ? ent1 : 0u));
#pragma unroll
  for (int s = 0; s < 4; s++)
#pragma unroll
    for (int d = 0; d < 4; d++)
      if (s != d) {
        uint32_t h = hashmix(pool[s]);
        uint32_t x = MIX_L * pool[d] - MIX_R * h;
        pool[d] = x ^ (x >> 16);
      }
  uint32_t w[8];
  uint32_t hb = INIT_B;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t d = pool[i & 3];
    d ^= hb;
    hb *= MULT_B;
    d *= hb;
    w[i] = d ^ (d >> 16);
  }
  uint64_t v0 = w[0] | ((uint64_t)w[1] << 32), v1 = w[2] | ((uint64_t)w[3] << 32);
  uint64_t v2 = w[4] | ((uint64_t)w[5] << 32), v3 = w[6] | ((uint64_t)w[7] << 32);
  U128 s{v0, v1}, inc{v2, v3};
  r.inc = U128{(inc.hi << 1) | (inc.lo >> 63), (inc.lo << 1) | 1};
  r.s = U128{0, 0};
  r.s = add128(mul128(r.s, U128{kMulHi, kMulLo}), r.inc);
  r.s = add128(r.s, s);
  r.s = add128(mul128(r.s, U128{kMulHi, kMulLo}), r.inc);
}

// random_loggam (distributions.c) — device fallback outside the host table.
__device__ double loggam_dev(double x) {
  const double a[10] = {8.333333333333333e-02, -2.777777777777778e-03, 7.936507936507937e-04,
                        -5.952380952380952e-04, 8.417508417508418e-04, -1.917526917526918e-03,
                        6.410256410256410e-03, -2.955065359477124e-02, 1.796443723688307e-01,
                        -1.39243221690590e+00};
  if (x == 1.0 || x == 2.0) return 0.0;
  int64_t n = (x < 7.0) ? (int64_t)(7 - x) : 0;
  double x0 = x + n;
  double x2 = (1.0 / x0) * (1.0 / x0);
  double gl0 = a[9];
  for (int k = 8; k >= 0; k--) {
    gl0 *= x2;
    gl0 += a[k];
  }
  double gl = gl0 / x0 + 0.5 * 1.8378770664093453e+00 + (x0 - 0.5) * log(x0) - x0;
  if (x < 7.0)
    for (int64_t k = 1; k <= n; k++) {
      gl -= log(x0 - 1.0);
      x0 -= 1.0;
    }
  return gl;
}

// loggam beyond the host table (k > lam + 16 sqrt(lam) + 64): never reached in
// practice; out of line so it costs the env kernel no registers.
__device__ __noinline__ double loggam_far(double x) { return loggam_dev(x); }

// PTRS acceptance test of random_poisson_ptrs (distributions.c), the branch
// taken by ~14% of draws: out of line so its log()s do not hold registers in
// the env kernel. loggam(k+1) comes from the host table (glibc) when in range.
__device__ __forceinline__ bool ptrs_accept(double V, double us, int64_t k, double lam, double a,
                                         double b, double loglam, double log_invalpha,
                                         const double *tab, int tab_n) {
  const double lg = (k + 1 < tab_n) ? gptr(tab)[k + 1] : loggam_far((double)(k + 1));
  return (log(V) + log_invalpha - log(a / (us * us) + b)) <= (-lam + k * loglam - lg);
}

// random_poisson (distributions.c): mult method (lam < 10) / PTRS (lam >= 10).
__device__ __forceinline__ int64_t poisson(Pcg &r, const PoisConst &c) {
  if (c.kind == 2) {
#pragma unroll 1
    for (;;) {
      const double U = next_double(r) - 0.5;
      const double V = next_double(r);
      const double us = 0.5 - fabs(U);
      const int64_t k = (int64_t)floor((2 * c.a / us + c.b) * U + c.lam + 0.43);
      if ((us >= 0.07) && (V <= c.vr)) return k;
      if ((k < 0) || ((us < 0.013) && (V > us))) continue;
      if (ptrs_accept(V, us, k, c.lam, c.a, c.b, c.loglam, c.log_invalpha, c.loggam_tab, c.tab_n))
        return k;
    }
  } else if (c.kind == 0) {
    return 0;
  }
  double prod = 1.0;
  int64_t X = 0;
#pragma unroll 1
  for (;;) {
    prod *= next_double(r);
    if (prod > c.enlam)
      X += 1;
    else
      return X;
  }
}

// Diagnostic build only (-DVMP_STAMPS): per-phase shader-clock deltas,
// accumulated per env into p.stamps[e][kStamps]. No stamp executes otherwise.
#ifdef VMP_STAMPS
constexpr int kStamps = 24;
// The accumulators live in LDS (one row per wave in k_env, one per block in
// k_env_big, written by one lane), not in registers: a 24-entry register
// array in the 256-VGPR block kernel spilled and distorted its timing ~7x.
#define STAMP_PARAMS , uint64_t LDSP *st_acc, uint64_t &st_prev
#define STAMP_ARGS , st_acc, st_prev
#define STAMP_DECL_AT(ptr)                                          \
  uint64_t LDSP *st_acc = (ptr);                                    \
  if (st_acc && lane_id() == 0)                                     \
    for (int _i = 0; _i < kStamps; _i++) st_acc[_i] = 0;            \
  uint64_t st_prev = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                      \
  do {                                                \
    const uint64_t _t = __builtin_amdgcn_s_memtime(); \
    if (st_acc && lane_id() == 0) st_acc[i] += _t - st_prev; \
    st_prev = _t;                                     \
  } while (0)
#define STAMP_FLUSH()                                                         \
  do {                                                                        \
    if (p.stamps && st_acc && lane_id() == 0)                                 \
      for (int _i = 0; _i < kStamps; _i++) p.stamps[(int64_t)e * kStamps + _i] += st_acc[_i]; \
  } while (0)
#elif defined(VMP_WGTIME)
// Workgroup timing build (k_env_big): thread 0 records the 100 MHz real-time
// clock at every stamp point into a block LDS row; tools/wgtime.py reads it.
__shared__ uint64_t wg_marks[24];
#define STAMP_PARAMS
#define STAMP_ARGS
#define STAMP_DECL_AT(ptr)
#define STAMP(i)                                                         \
  do {                                                                   \
    if (threadIdx.x == 0) wg_marks[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define STAMP_FLUSH()
#else
#define STAMP_PARAMS
#define STAMP_ARGS
#define STAMP_DECL_AT(ptr)
#define STAMP(i)
#define STAMP_FLUSH()
#endif

// ---------------------------------------------------- pairwise summation --
// numpy DOUBLE_pairwise_sum (loops_utils.h.src, PW_BLOCKSIZE 128) of
// f(0..n-1) by one wave. Leaves (<= 128 elements: 8 interleaved accumulator
// chains, an ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) combine, a sequential tail)
// run lane-parallel (8 lanes per leaf); the split n2 = n/2 - (n/2)%8 is
// enumerated and the partial sums combined by lane 0 alone on small LDS
// stacks, so no cross-lane hand-off happens inside the recursion.
struct PwLds {
  int32_t LDSP *lo, *len;  // leaf list (DFS order), n_leaf entries
  int32_t LDSP *stk;            // lane-0 stack, 3 * 64 ints
  double LDSP *val;             // leaf sums, + value stack
};

// lane 0 only: leaves of the recursion for n, left to right.
__device__ __forceinline__ int pw_plan(int n, const PwLds &S) {
  int sp = 0, nl = 0;
  S.stk[0] = 0;
  S.stk[1] = n;
  sp = 2;
  while (sp > 0) {
    sp -= 2;
    const int o = S.stk[sp], m = S.stk[sp + 1];
    if (m <= 128) {
      S.lo[nl] = o;
      S.len[nl] = m;
      nl++;
    } else {
      int n2 = m / 2;
      n2 -= n2 % 8;
      S.stk[sp] = o + n2;  // right, popped second
      S.stk[sp + 1] = m - n2;
      S.stk[sp + 2] = o;   // left, popped first
      S.stk[sp + 3] = n2;
      sp += 4;
    }
  }
  return nl;
}

// lane 0 only: pw(n) = pw(n2) + pw(n - n2) over the leaf sums in val[].
__device__ __forceinline__ double pw_combine(int n, const PwLds &S, int nl) {
  double LDSP *vs = S.val + nl;  // value stack after the leaf sums
  int sp = 0, vsp = 0, leaf = 0;
  S.stk[0] = n;
  S.stk[1] = 0;
  sp = 2;
  while (sp > 0) {
    sp -= 2;
    const int m = S.stk[sp], ph = S.stk[sp + 1];
    if (m <= 128) {
      vs[vsp++] = S.val[leaf++];
    } else if (ph == 0) {
      int n2 = m / 2;
      n2 -= n2 % 8;
      S.stk[sp + 1] = 1;  // revisit after both children
      S.stk[sp + 2] = m - n2;
      S.stk[sp + 3] = 0;
      S.stk[sp + 4] = n2;
      S.stk[sp + 5] = 0;
      sp += 6;
    } else {
      const double b = vs[--vsp];
      const double a = vs[--vsp];
      vs[vsp++] = a + b;
    }
  }
  return vs[0];
}

__device__ __forceinline__ double readlane_f64(double x, int l) {
  const int64_t b = __double_as_longlong(x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((int64_t)(((uint64_t)hi << 32) | lo));
}

// Register-resident plan (depth <= RD): leaf cnt's (offset, size) lands in
// lane cnt; the combine reads leaf sums by readlane. pw_reg_cap(RD) is the
// largest n such that every n' <= n splits into at most RD levels and 64
// leaves (1928 for RD = 4, 7688 for RD = 6; host check: vmp_capi.cpp pw_depth).
constexpr int kPwRegDepth = 4;
constexpr int pw_reg_cap(int rd) { return rd <= 4 ? 1928 : rd == 5 ? 3848 : 7688; }
template <int D>
__device__ __forceinline__ void pw_enum_r(int o, int n, int &cnt, int lane, int &my_o,
                                          int &my_m) {
  if (D == 0 || n <= 128) {
    if (lane == cnt) {
      my_o = o;
      my_m = n;
    }
    cnt++;
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  pw_enum_r<(D > 0 ? D - 1 : 0)>(o, n2, cnt, lane, my_o, my_m);
  pw_enum_r<(D > 0 ? D - 1 : 0)>(o + n2, n - n2, cnt, lane, my_o, my_m);
}
template <int D>
__device__ __forceinline__ double pw_comb_r(int n, int &cnt, double myval) {
  if (D == 0 || n <= 128) return readlane_f64(myval, cnt++);
  int n2 = n / 2;
  n2 -= n2 % 8;
  const double a = pw_comb_r<(D > 0 ? D - 1 : 0)>(n2, cnt, myval);
  const double b = pw_comb_r<(D > 0 ? D - 1 : 0)>(n - n2, cnt, myval);
  return a + b;
}

// One leaf [o, o+m) by the 8-lane group of the calling lane; the value is
// valid in the group's lane j == 0. Chain loads are issued 8 at a time.
template <class F>
__device__ __forceinline__ double pw_leaf_group(int o, int m, F &f) {
  const int j = lane_id() & 7;
  const int full = m - (m % 8);
  const int cnt = full >> 3;  // elements per accumulator chain (<= 16)
  double r = 0.0;
  if (cnt > 0) {
    double x[8];
#pragma unroll
    for (int t = 0; t < 8; t++) x[t] = t < cnt ? f(o + j + 8 * t) : 0.0;
    r = x[0];
#pragma unroll
    for (int t = 1; t < 8; t++)
      if (t < cnt) r += x[t];
    if (cnt > 8) {
#pragma unroll
      for (int t = 0; t < 8; t++) x[t] = t + 8 < cnt ? f(o + j + 8 * (t + 8)) : 0.0;
#pragma unroll
      for (int t = 0; t < 8; t++)
        if (t + 8 < cnt) r += x[t];
    }
  }
  // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)): xor-pairs reproduce the tree exactly
  // (f64 addition is commutative)
  r = r + __shfl_xor(r, 1);
  r = r + __shfl_xor(r, 2);
  r = r + __shfl_xor(r, 4);
  double res = cnt > 0 ? r : 0.0;
  if (j == 0) {
    double tl[7];
#pragma unroll
    for (int t = 0; t < 7; t++) tl[t] = full + t < m ? f(o + full + t) : 0.0;
#pragma unroll
    for (int t = 0; t < 7; t++)
      if (full + t < m) res += tl[t];
  }
  return res;
}

template <int RD = kPwRegDepth, class F>
__device__ __forceinline__ double wave_pw_sum(int n, F f, const PwLds &S) {
  static_assert(RD >= 4 && RD <= 6, "register plan depth");
  const int lane = lane_id();
  if (n < 8) {  // pairwise_sum's direct loop, evaluated by every lane alike
    double r = 0.0;
#pragma unroll 1
    for (int i = 0; i < n; i++) r += f(i);
    return r;
  }
  if (n <= 128) return readlane_f64(pw_leaf_group(0, n, f), 0);
  if (n <= pw_reg_cap(RD)) {
    int my_o = 0, my_m = 0, nl = 0;
    pw_enum_r<RD>(0, n, nl, lane, my_o, my_m);
    double myval = 0.0;
    for (int b = 0; b < nl; b += 8) {
      const int l = b + (lane >> 3);
      // both shuffles unconditional: a ds_bpermute under a partial exec mask
      // must not read a source lane that the mask left out
      const int o = __shfl(my_o, l & 63), m_src = __shfl(my_m, l & 63);
      const int m = l < nl ? m_src : 0;
      const double v = pw_leaf_group(o, m, f);
      const double moved = __shfl(v, ((lane - b) & 7) * 8);
      if (lane >= b && lane < b + 8) myval = moved;
    }
    int cnt = 0;
    return pw_comb_r<RD>(n, cnt, myval);
  }
  // deeper recursion (n > pw_reg_cap(RD), P-sized sums of big configs): LDS plan
  int nl = 1;
  if (lane == 0) S.stk[191] = pw_plan(n, S);
  wsync();
  nl = S.stk[191];
  for (int b = 0; b < nl; b += 8) {
    const int l = b + (lane >> 3);
    const int o = l < nl ? S.lo[l] : 0, m = l < nl ? S.len[l] : 0;
    const double v = pw_leaf_group(o, m, f);
    if (l < nl && (lane & 7) == 0) S.val[l] = v;
  }
  wsync();
  if (lane == 0) S.val[nl] = pw_combine(n, S, nl);
  wsync();
  const double r = S.val[nl];
  wsync();
  return r;
}

// ------------------------------------------- numpy scalar argsort (BF) ----
// aquicksort_<float_tag> / aheapsort_ (npysort), run by ONE lane on LDS
// arrays (index form of the pointer algorithm); stack arrays live in LDS.
__device__ __forceinline__ bool fless(float a, float b) { return a < b || (b != b && a == a); }
// Sort keys: an f32 array, or BestFit's fcpu[i] + fmem[i] formed at each read
// (the same f32 sum bestfit.py:31 sorts; no key array in LDS).
struct KeyArr {
  const float LDSP *a;
  __device__ __forceinline__ float operator[](int i) const { return a[i]; }
};
struct KeySum {
  const float LDSP *a, *b;
  __device__ __forceinline__ float operator[](int i) const { return a[i] + b[i]; }
};

template <class KV>
__device__ void aheapsort_lds(KV v, uint16_t LDSP *tosort, int n) {
  uint16_t LDSP *a = tosort - 1;
  int i, j, l;
  uint16_t tmp;
  for (l = n >> 1; l > 0; --l) {
    tmp = a[l];
    for (i = l, j = l << 1; j <= n;) {
      if (j < n && fless(v[a[j]], v[a[j + 1]])) j += 1;
      if (fless(v[tmp], v[a[j]])) {
        a[i] = a[j];
        i = j;
        j += j;
      } else
        break;
    }
    a[i] = tmp;
  }
  for (; n > 1;) {
    tmp = a[n];
    a[n] = a[1];
    n -= 1;
    for (i = 1, j = 2; j <= n;) {
      if (j < n && fless(v[a[j]], v[a[j + 1]])) j++;
      if (fless(v[tmp], v[a[j]])) {
        a[i] = a[j];
        i = j;
        j += j;
      } else
        break;
    }
    a[i] = tmp;
  }
}

// Only the sorted positions lo..hi are needed (BF's tie block): numpy sorts
// every partition independently of the others, so a partition that does not
// intersect [lo, hi] is dropped instead of sorted, and positions lo..hi come
// out exactly as the full sort leaves them (a quickselect-shaped walk:
// ~2n element visits instead of ~n log n).
template <class KV>
__device__ __noinline__ void aquicksort_lds(KV v, uint16_t LDSP *t, int num,
                                            int32_t LDSP *stack, int lo, int hi) {
  int32_t LDSP *depth = stack + 128;
  int pl = 0, pr = num - 1;
  int sp = 0, dp = 0;
  int cdepth = 0;
  for (int u = num; u >>= 1;) cdepth++;
  cdepth *= 2;
  for (;;) {
    if (pr < lo || pl > hi) goto stack_pop;
    if (cdepth < 0) {
      aheapsort_lds(v, t + pl, pr - pl + 1);
      goto stack_pop;
    }
    while ((pr - pl) > 15) {
      int pm = pl + ((pr - pl) >> 1);
      uint16_t x;
      if (fless(v[t[pm]], v[t[pl]])) { x = t[pm]; t[pm] = t[pl]; t[pl] = x; }
      if (fless(v[t[pr]], v[t[pm]])) { x = t[pr]; t[pr] = t[pm]; t[pm] = x; }
      if (fless(v[t[pm]], v[t[pl]])) { x = t[pm]; t[pm] = t[pl]; t[pl] = x; }
      float vp = v[t[pm]];
      int pi = pl, pj = pr - 1;
      x = t[pm]; t[pm] = t[pj]; t[pj] = x;
      for (;;) {
        do ++pi; while (fless(v[t[pi]], vp));
        do --pj; while (fless(vp, v[t[pj]]));
        if (pi >= pj) break;
        x = t[pi]; t[pi] = t[pj]; t[pj] = x;
      }
      int pk = pr - 1;
      x = t[pi]; t[pi] = t[pk]; t[pk] = x;
      if (pi - pl < pr - pi) {
        stack[sp++] = pi + 1;
        stack[sp++] = pr;
        pr = pi - 1;
      } else {
        stack[sp++] = pl;
        stack[sp++] = pi - 1;
        pl = pi + 1;
      }
      depth[dp++] = --cdepth;
      if (pr < lo || pl > hi) goto stack_pop;
    }
    for (int pi = pl + 1; pi <= pr; ++pi) {
      uint16_t vi = t[pi];
      float vp = v[vi];
      int pj = pi, pk = pi - 1;
      while (pj > pl && fless(vp, v[t[pk]])) t[pj--] = t[pk--];
      t[pj] = vi;
    }
  stack_pop:
    if (sp == 0) break;
    pr = stack[--sp];
    pl = stack[--sp];
    cdepth = depth[--dp];
  }
}

// Wave-parallel form of the same sort (all 64 lanes, uniform control flow),
// identical result. numpy's partition loop
//   do ++pi while v[pi] < vp;  do --pj while vp < v[pj];  if (pi >= pj) break;  swap
// pairs the k-th left stop A[k] (ascending positions in (pl, pr-1] with
// v >= vp; pr-1 holds the pivot) with the k-th right stop B[k] (descending
// positions in [pl, pr-2] with v <= vp; pl holds a value <= vp) while
// A[k] < B[k]: up to that point each scan only crosses unmodified positions,
// so both lists follow from the values before the loop. With K = #{k : A[k] <
// B[k]} (a prefix, A rising and B falling), the K swaps are disjoint, and the
// final left stop is min(A[K], B[K-1]) (B[K-1] holds a swapped-in value >= vp).
// Stops are ranked with ballots; the lists live in `scr` (u16, 2 x n). Small
// partitions (<= 16) get numpy's insertion sort as a stable rank sort; the
// depth-limit heapsort stays on lane 0.
//
// One partition step of numpy's loop on [pl, pr] (pr - pl > 15): median of
// three, the stops, the swaps and the pivot's final move; returns its
// position pi ([pl, pi - 1] <= pivot <= [pi + 1, pr]).
template <class KV>
__device__ __forceinline__ int wave_partition(KV v, uint16_t LDSP *t, int pl, int pr,
                                              uint16_t LDSP *scr) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1ull;
  const int pm = pl + ((pr - pl) >> 1);
  uint16_t tl = t[pl], tm = t[pm], tr = t[pr], x;
  if (fless(v[tm], v[tl])) { x = tm; tm = tl; tl = x; }
  if (fless(v[tr], v[tm])) { x = tr; tr = tm; tm = x; }
  if (fless(v[tm], v[tl])) { x = tm; tm = tl; tl = x; }
  const float vp = v[tm];
  const uint16_t tq = t[pr - 1];
  wsync();
  if (lane == 0) {
    t[pl] = tl;
    t[pm] = tq;
    t[pr] = tr;
    t[pr - 1] = tm;
  }
  wsync();
  // A (ascending stops in [pl+1, pr-1]) and B (stops in [pl, pr-2], kept
  // ascending in bas: B[k] = bas[nb-1-k]) from ONE pass over [pl, pr-1]
  // reading each key once, two 64-position batches per round trip
  uint16_t LDSP *apos = scr;
  uint16_t LDSP *bas = scr + (pr - pl + 1);
  int na = 0, nb = 0;
  for (int c = pl; c <= pr - 1; c += 128) {
    const int q0 = c + lane, q1 = c + 64 + lane;
    const bool in0 = q0 <= pr - 1, in1 = q1 <= pr - 1;
    const int i0 = t[in0 ? q0 : pl], i1 = t[in1 ? q1 : pl];
    const float x0 = v[i0], x1 = v[i1];
    const bool fa0 = in0 && q0 >= pl + 1 && !fless(x0, vp), fb0 = in0 && q0 <= pr - 2 && !fless(vp, x0);
    const bool fa1 = in1 && q1 >= pl + 1 && !fless(x1, vp), fb1 = in1 && q1 <= pr - 2 && !fless(vp, x1);
    const uint64_t ma0 = ballot(fa0), mb0 = ballot(fb0), ma1 = ballot(fa1), mb1 = ballot(fb1);
    if (fa0) apos[na + __popcll(ma0 & lt)] = (uint16_t)q0;
    if (fb0) bas[nb + __popcll(mb0 & lt)] = (uint16_t)q0;
    na += __popcll(ma0);
    nb += __popcll(mb0);
    if (fa1) apos[na + __popcll(ma1 & lt)] = (uint16_t)q1;
    if (fb1) bas[nb + __popcll(mb1 & lt)] = (uint16_t)q1;
    na += __popcll(ma1);
    nb += __popcll(mb1);
  }
  wsync();
  int kk = 0;  // K: A[k] < B[k] holds for a prefix of k
  for (int c = 0; c < na && c < nb; c += 64) {
    const int k = c + lane;
    const bool sw = k < na && k < nb && (int)apos[k] < (int)bas[nb - 1 - k];
    kk += __popcll(ballot(sw));
  }
  for (int c = 0; c < kk; c += 64) {
    const int k = c + lane;
    uint16_t xa = 0, xb = 0;
    int qa = 0, qb = 0;
    if (k < kk) {
      qa = apos[k];
      qb = bas[nb - 1 - k];
      xa = t[qa];
      xb = t[qb];
    }
    wsync();
    if (k < kk) {
      t[qa] = xb;
      t[qb] = xa;
    }
    wsync();
  }
  int pi = apos[kk];
  if (kk > 0 && (int)bas[nb - kk] < pi) pi = bas[nb - kk];
  wsync();
  if (lane == 0) {
    x = t[pi];
    t[pi] = t[pr - 1];
    t[pr - 1] = x;
  }
  wsync();
  return pi;
}

// numpy's insertion sort of [pl, pr] (<= 16 elements) = a stable rank sort.
template <class KV>
__device__ __forceinline__ void wave_leaf_sort(KV v, uint16_t LDSP *t, int pl, int pr) {
  const int lane = threadIdx.x & 63;
  const int n = pr - pl + 1;
  uint16_t me = 0;
  float vm = 0.f;
  if (lane < n) {
    me = t[pl + lane];
    vm = v[me];
  }
  int rank = 0;
  for (int j = 0; j < n; j++) {
    const float vj = __shfl(vm, j);
    rank += (fless(vj, vm) || (j < lane && !fless(vm, vj))) ? 1 : 0;
  }
  wsync();
  if (lane < n) t[pl + rank] = me;
  wsync();
}

template <class KV>
__device__ __noinline__ void wave_aquicksort(KV v, uint16_t LDSP *t, int num,
                                             int32_t LDSP *stack, int lo, int hi,
                                             uint16_t LDSP *scr) {
  const int lane = threadIdx.x & 63;
  int32_t LDSP *depth = stack + 128;
  int pl = 0, pr = num - 1;
  int sp = 0, dp = 0;
  int cdepth = 0;
  for (int u = num; u >>= 1;) cdepth++;
  cdepth *= 2;
  for (;;) {
    if (pr < lo || pl > hi) goto stack_pop;
    if (cdepth < 0) {
      if (lane == 0) aheapsort_lds(v, t + pl, pr - pl + 1);
      wsync();
      goto stack_pop;
    }
    while ((pr - pl) > 15) {
      const int pi = wave_partition(v, t, pl, pr, scr);
      if (pi - pl < pr - pi) {
        if (lane == 0) {
          stack[sp] = pi + 1;
          stack[sp + 1] = pr;
        }
        sp += 2;
        pr = pi - 1;
      } else {
        if (lane == 0) {
          stack[sp] = pl;
          stack[sp + 1] = pi - 1;
        }
        sp += 2;
        pl = pi + 1;
      }
      --cdepth;
      if (lane == 0) depth[dp] = cdepth;
      dp++;
      wsync();
      if (pr < lo || pl > hi) goto stack_pop;
    }
    wave_leaf_sort(v, t, pl, pr);
  stack_pop:
    if (sp == 0) break;
    wsync();
    sp -= 2;
    pl = stack[sp];
    pr = stack[sp + 1];
    cdepth = depth[--dp];
  }
  wsync();
}

// BestFit's tie block needs only the HIGHEST position in [lo, hi] whose PM
// fits (the first in visiting order). The walk processes the same partitions
// as wave_aquicksort(lo, hi), each with the same depth, so every position in
// [lo, hi] settles to numpy's element; partitions of disjoint ranges do not
// interact, so the order they are processed in is free. Here the upper part
// is always processed first and the lower part waits on the stack (a reverse
// in-order walk: positions settle in descending order, a partition's pivot
// after its upper part, checked when the lower part is popped), and the walk
// stops at the first settled position that fits. A tie block of e PMs whose
// highest member fits costs one root-to-leaf path (~2n element visits)
// instead of sorting the block (~e log e more partitions). The stack holds
// the pending lower parts of one path: at most 2 log2(n) + 1 entries (the
// depth limit ends a path in heapsort). Returns the position, or -1.
template <class KV, class Fit>
__device__ __noinline__ int wave_aqselect_top(KV v, uint16_t LDSP *t, int num,
                                              int32_t LDSP *stack, int lo, int hi,
                                              uint16_t LDSP *scr, Fit fit) {
  const int lane = threadIdx.x & 63;
  int32_t LDSP *depth = stack + 128;
  int pl = 0, pr = num - 1;
  int sp = 0, dp = 0;
  int cdepth = 0;
  for (int u = num; u >>= 1;) cdepth++;
  cdepth *= 2;
  // highest fitting position of the settled range [a, b] within [lo, hi]
  auto scan = [&](int a, int b) -> int {
    const int a0 = a > lo ? a : lo;
    for (int c = b < hi ? b : hi; c >= a0; c -= 64) {
      const int pos = c - lane;
      const uint64_t f = ballot(pos >= a0 && fit((int)t[pos >= a0 ? pos : a0]));
      if (f) return c - (__ffsll((unsigned long long)f) - 1);
    }
    return -1;
  };
  int found = -1;
  for (;;) {
    if (pr < lo || pl > hi) goto stack_pop;
    if (cdepth < 0) {
      if (lane == 0) aheapsort_lds(v, t + pl, pr - pl + 1);
      wsync();
      found = scan(pl, pr);
      if (found >= 0) break;
      goto stack_pop;
    }
    while ((pr - pl) > 15) {
      const int pi = wave_partition(v, t, pl, pr, scr);
      if (lane == 0) {  // the lower part waits; the upper part goes on
        stack[sp] = pl;
        stack[sp + 1] = pi - 1;
      }
      sp += 2;
      pl = pi + 1;
      --cdepth;
      if (lane == 0) depth[dp] = cdepth;
      dp++;
      wsync();
      if (pr < lo || pl > hi) goto stack_pop;
    }
    wave_leaf_sort(v, t, pl, pr);
    found = scan(pl, pr);
    if (found >= 0) break;
  stack_pop:
    if (sp == 0) break;
    wsync();
    sp -= 2;
    pl = stack[sp];
    pr = stack[sp + 1];
    cdepth = depth[--dp];
    // the popped range is the lower part of a partition whose pivot sits at
    // pr + 1, settled, and every position above it has been checked
    if (pr + 1 >= lo && pr + 1 <= hi && fit((int)t[pr + 1])) {
      found = pr + 1;
      break;
    }
  }
  wsync();
  return found;
}

// --------------------------------------------------------- env kernel ----
// Per-wave LDS carve (offsets from EnvParams, computed by the host).
struct Lds {
  EnvHdr LDSP *hdr;                  // the env's 256-B header (scalars, RNG streams)
  double LDSP *cpu, *mem;       // f64[P] PM resources (the env state)
  float LDSP *fcpu, *fmem;      // f32[P] observation view used by the heuristics
  uint8_t LDSP *tc, *tm;        // per-PM largest fitting size (hundredths), f32 semantics
  uint16_t LDSP *ord;                // BF ascending argsort, then reversed into visiting order
  uint64_t LDSP *bc, *bm;       // action phase: the any-fit table (u32 [128] at bc)
  int32_t LDSP *sortstk;             // introsort stacks
  uint16_t LDSP *nulls;              // NULL slot indices (aliases the fit bitmaps)
  uint8_t LDSP *accc, *accm;    // accepted sizes (alias the fit bitmaps)
  double LDSP *jobres;               // reduction results of the step
  int32_t LDSP *arr;                 // per-step arrivals of the launch (prologue draws)
  uint32_t LDSP *svc;                // speculative planned runtimes
  uint64_t LDSP *svcst;              // rng4 state after each speculative draw
  uint64_t LDSP *svcfb;              // rng4 state for fallback draws
  int32_t LDSP *svcinfo;             // [0] speculative count, [1] consumed
  uint8_t LDSP *ccomp, *mcomp;  // compressed sizes of existing VMs [ccomp_cap]
  uint64_t LDSP *pdirty;             // bit i: PM double i (cpu | memory) changed
  uint32_t LDSP *evw;                // k_env_big event lists [512]: VM word,
  int32_t LDSP *evt;                 //   target / value,
  uint8_t LDSP *evok;                //   result
  PwLds pw;
  char LDSP *base;                   // the wave's LDS region
};

// The wave's LDS view, rebuilt from its base address (cheap; avoids passing
// the pointer struct by value into out-of-line helpers).
__device__ __forceinline__ Lds make_lds(const EnvParams &p, char LDSP *base) {
  Lds L;
  L.hdr = reinterpret_cast<EnvHdr LDSP *>(base + p.off_hdr);
  L.cpu = reinterpret_cast<double LDSP *>(base + p.off_pm);
  L.mem = L.cpu + p.P;
  L.fcpu = reinterpret_cast<float LDSP *>(base + p.off_fpm);
  L.fmem = L.fcpu + p.fmem_off;  // k_env_big: 16-B aligned rows (vector reads in big_choose)
  L.tc = reinterpret_cast<uint8_t LDSP *>(base + p.off_thr);
  L.tm = L.tc + p.tm_off;
  L.ord = reinterpret_cast<uint16_t LDSP *>(base + p.off_ord);
  L.bc = reinterpret_cast<uint64_t LDSP *>(base + p.off_bits);
  L.bm = L.bc + 101 * p.NW;
  L.sortstk = reinterpret_cast<int32_t LDSP *>(base + p.off_sort);
  L.nulls = reinterpret_cast<uint16_t LDSP *>(base + p.off_bits);
  L.accc = reinterpret_cast<uint8_t LDSP *>(base + p.off_acc);
  L.accm = L.accc + p.acc_cap;
  L.jobres = reinterpret_cast<double LDSP *>(base + p.off_stage);
  L.svcinfo = reinterpret_cast<int32_t LDSP *>(base + p.off_stage + 8 * 12);
  L.svcfb = reinterpret_cast<uint64_t LDSP *>(base + p.off_stage + 8 * 14);
  L.svcst = reinterpret_cast<uint64_t LDSP *>(base + p.off_pre);
  L.svc = reinterpret_cast<uint32_t LDSP *>(base + p.off_pre + 16 * p.scap);
  L.arr = reinterpret_cast<int32_t LDSP *>(base + p.off_pre + 20 * p.scap);
  L.pdirty = reinterpret_cast<uint64_t LDSP *>(base + p.off_pdirty);
  L.ccomp = reinterpret_cast<uint8_t LDSP *>(base + p.off_ccomp);
  L.mcomp = L.ccomp + p.ccomp_cap;
  L.evw = reinterpret_cast<uint32_t LDSP *>(base + p.off_ev);
  L.evt = reinterpret_cast<int32_t LDSP *>(L.evw + 512);
  L.evok = reinterpret_cast<uint8_t LDSP *>(L.evt + 512);
  L.pw.lo = reinterpret_cast<int32_t LDSP *>(base + p.off_leaf);
  L.pw.len = L.pw.lo + p.n_leaf;
  L.pw.stk = L.pw.len + p.n_leaf;
  L.pw.val = reinterpret_cast<double LDSP *>(base + p.off_leafval);
  L.base = base;
  return L;
}

// Exact k/100 for k = 0..127 (np.around(., 2) values), per block.
struct Tables {
  double cent[128];
  float fcent[128];
  PoisConst pois[2];  // block copy of p.pois, read by the prologue draws
};

__device__ __forceinline__ int w_pl(uint32_t w) { return (int)(w & 0xFFFFu); }
// Register slots past V hold placement kPad: no test for running (< P), WAIT,
// NULL or existing (<= WAIT) matches it, so the per-slot loops need no lane
// range mask (keeping 16 64-bit masks live would spill SGPRs); only stores
// test live().
constexpr int kPad = 0xFFFF;
__device__ __forceinline__ bool live(uint32_t w) { return w_pl(w) != kPad; }
__device__ __forceinline__ int w_cc(uint32_t w) { return (int)((w >> 16) & 0xFFu); }
__device__ __forceinline__ int w_cm(uint32_t w) { return (int)(w >> 24); }
__device__ __forceinline__ uint32_t w_make(int pl, int cc, int cm) {
  return (uint32_t)pl | ((uint32_t)cc << 16) | ((uint32_t)cm << 24);
}

__device__ __forceinline__ Pcg ld_pcg(const EnvHdr LDSP *h, int k) {
  Pcg r;
  r.s = U128{h->rng[k][0], h->rng[k][1]};
  r.inc = U128{h->rng[k][2], h->rng[k][3]};
  return r;
}
__device__ __forceinline__ void st_pcg(EnvHdr LDSP *h, int k, const Pcg &r) {
  if (lane_id() == 0) {
    h->rng[k][0] = r.s.hi;
    h->rng[k][1] = r.s.lo;
  }
}

// FC(k) = (float)(k / 100.0), the f32 obs value of a size of k hundredths;
// (float)(k * 0.01) equals it for every k in [0, 127] (checked exhaustively).
__device__ __forceinline__ float fcent_of(int k) { return (float)((double)k * 0.01); }

// Largest k in [0, 100] with f + FC(k) <= 1 in f32 (monotone in k), or -1.
// For every f32 f in [0, 1] (PM loads, env.py:267-268 keeps them >= 0) the
// answer is one of k0 - 1, k0, k0 + 1 with k0 = (int)((1 - f) * 100): checked
// exhaustively over all 1 065 353 217 such f.
__device__ __forceinline__ int fit_threshold(float f) {
  int k0 = (int)((1.0f - f) * 100.0f);
  k0 = k0 < 0 ? 0 : (k0 > 100 ? 100 : k0);
  const bool up = k0 < 100 && f + fcent_of(k0 + 1) <= 1.0f;
  const bool at = f + fcent_of(k0) <= 1.0f;
  return up ? k0 + 1 : (at ? k0 : k0 - 1);
}

// Inclusive prefix OR across the wave (lane i: OR of lanes 0..i) with DPP row
// shifts and the GFX9 row broadcasts: 6 VALU steps, no LDS traffic.
__device__ __forceinline__ uint32_t prefix_or32(uint32_t x) {
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}
__device__ __forceinline__ uint64_t prefix_or64(uint64_t x) {
  return ((uint64_t)prefix_or32((uint32_t)(x >> 32)) << 32) | prefix_or32((uint32_t)x);
}

// Inclusive prefix max across the wave for values >= 0 (0 is the identity).
__device__ __forceinline__ uint32_t prefix_max32(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
  return x;
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// The any-fit table: M[k] = max of the +1-encoded memory thresholds tm over
// the PMs whose cpu threshold is >= k (0: none). A VM of sizes (kc, km) fits
// some PM iff M[kc] > km (firstfit.py:33, bestfit.py:35: cpu and memory both
// fit). Built per step and after each placement (only the placed PM's
// thresholds move); the heuristics' choices are then wave scans over the
// thresholds (ff_scan, bf_choose). Levels are mapped to lanes in reverse
// (row 63-i, and 127-i for levels 64..100), so the suffix max over k is a
// DPP lane prefix max.
__device__ __forceinline__ void build_fitmax(const EnvParams &p, const Lds &L, uint32_t LDSP *M) {
  const int lane = lane_id();
  M[lane] = 0;
  M[lane + 64] = 0;
  wsync();
  for (int q = lane; q < p.P; q += 64) {
    const int tcq = (int)L.tc[q];
    if (tcq > 0) __atomic_fetch_max(&M[tcq - 1], (uint32_t)L.tm[q], __ATOMIC_RELAXED);
  }
  wsync();
  const int rlo = 63 - lane, rhi = 127 - lane;
  const bool hi_ok = rhi <= 100;
  uint32_t c1 = hi_ok ? M[rhi] : 0u, c0 = M[rlo];
  c1 = prefix_max32(c1);
  c0 = max(prefix_max32(c0), (uint32_t)__builtin_amdgcn_readlane((int)c1, 63));
  wsync();
  M[rlo] = c0;
  if (hi_ok) M[rhi] = c1;
  wsync();
}

// FirstFit's PM for sizes (kc, km) (firstfit.py:33-37): the first PM in index
// order whose f32 thresholds accept both, by a wave scan over the PMs' u8
// thresholds (P/64 ballots; no fit bitmaps to build or maintain). -1 if none.
__device__ __forceinline__ int ff_scan(const EnvParams &p, const Lds &L, int kc, int km) {
  const int lane = lane_id();
  for (int b = 0; b < p.P; b += 64) {
    const int i = b + lane;
    const bool f = i < p.P && (int)L.tc[i] - 1 >= kc && (int)L.tm[i] - 1 >= km;
    const uint64_t m = ballot(f);
    if (m) return b + __ffsll((unsigned long long)m) - 1;
  }
  return -1;
}

// BestFit's choice for sizes (kc, km) (bestfit.py:33-39): the first PM in
// visiting order flip(argsort(fcpu + fmem)) that fits, i.e. the fitting PM of
// largest key. Fast path: a wave argmax over the PMs; only when two or more
// fitting PMs share the largest key m does their order matter. The keys equal
// to m occupy the ascending positions [P - above - eq, P - above) (above =
// keys > m, none of which fits); the scalar introsort (numpy's tie order,
// SURVEY App. C) is run for that block only, and its highest fitting position
// (the first in visiting order) is taken. Returns -1 if nothing fits.
__device__ __forceinline__ int bf_tie(const EnvParams &p, const Lds &L, int kc, int km, int above,
                                   int eq);
__device__ __forceinline__ int bf_choose(const EnvParams &p, const Lds &L, int kc, int km) {
  const int lane = lane_id();
  const int P = p.P;
  float best = -INFINITY;
  int cnt = 0, bi = -1;
  for (int i = lane; i < P; i += 64) {
    if ((int)L.tc[i] - 1 >= kc && (int)L.tm[i] - 1 >= km) {
      const float key = L.fcpu[i] + L.fmem[i];
      if (key > best) {
        best = key;
        cnt = 1;
        bi = i;
      } else if (key == best) {
        cnt++;
      }
    }
  }
  float m = best;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  int tot = (best == m) ? cnt : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
  if (tot == 0) return -1;
  if (tot == 1) {
    const uint64_t who = ballot(best == m && cnt == 1);
    return __builtin_amdgcn_readlane(bi, __ffsll((unsigned long long)who) - 1);
  }
  // ties at the top: numpy's order decides
  int above = 0, eq = 0;
  for (int i = lane; i < P; i += 64) {
    const float key = L.fcpu[i] + L.fmem[i];
    above += key > m;
    eq += key == m;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    above += __shfl_xor(above, o);
    eq += __shfl_xor(eq, o);
  }
  return bf_tie(p, L, kc, km, above, eq);
}

// BestFit's choice when eq >= 2 PMs share the largest fitting key m and
// `above` keys exceed it (none of which fits): the tied keys occupy the
// ascending positions [P - above - eq, P - above) of numpy's argsort; only the
// quicksort partitions that intersect that block are sorted, and the highest
// fitting position in it (the first in visiting order) is taken.
__device__ __forceinline__ int bf_tie(const EnvParams &p, const Lds &L, int kc, int km, int above,
                                   int eq) {
  const int lane = lane_id();
  const int P = p.P;
  for (int i = lane; i < P; i += 64) L.ord[i] = (uint16_t)i;
  const int hi = P - above - 1, lo = P - above - eq;
  wsync();
  const uint8_t LDSP *tc = L.tc, *tm = L.tm;
  const int pos = wave_aqselect_top(
      KeySum{L.fcpu, L.fmem}, L.ord, P, L.sortstk, lo, hi,
      reinterpret_cast<uint16_t LDSP *>(L.sortstk + 256),
      [=](int q) { return (int)tc[q] - 1 >= kc && (int)tm[q] - 1 >= km; });
  return pos >= 0 ? (int)L.ord[pos] : -1;  // visiting order: descending positions
}

// Record that PM q's cpu and memory were written (one lane: the callers'
// writes are single-lane); the state store writes back only marked PM words.
__device__ __forceinline__ void mark_pm(const Lds &L, int P, int q) {
  L.pdirty[q >> 6] |= 1ull << (q & 63);
  L.pdirty[(P + q) >> 6] |= 1ull << ((P + q) & 63);
}

// One VM placement event of the env (env.py:74-84 for a WAIT -> PM move):
// _resource_valid in f64, then _place_vm. Returns validity (wave-uniform).
__device__ __forceinline__ bool env_place(const Lds &L, const Tables &T, int P, int q, int kc,
                                          int km) {
  double cq = L.cpu[q], mq = L.mem[q];
  double vc = T.cent[kc], vm = T.cent[km];
  bool ok = (cq + vc <= 1) && (mq + vm <= 1);
  wsync();
  if (ok && lane_id() == 0) {
    L.cpu[q] = cq + vc;
    L.mem[q] = mq + vm;
    mark_pm(L, P, q);
  }
  wsync();
  return ok;
}

// ---- random draws of a launch (prologue) ---------------------------------
// All Poisson draws a launch can need are taken BEFORE the VM state is loaded
// into registers, so the samplers never share the register budget with it:
// the K arrival counts (rng3, one per step, all consumed) and up to scap
// service lengths (rng4), speculative: only the first `used` are consumed and
// rng4 is committed to the state recorded after draw used-1 (draws past scap
// come from the out-of-line fallback below).
__device__ __noinline__ uint32_t svc_fallback(uint64_t LDSP *st, const uint64_t LDSP *inc,
                                              const PoisConst *c) {
  Pcg r;
  r.s = U128{st[0], st[1]};
  r.inc = U128{inc[0], inc[1]};
  const int64_t x = poisson(r, *c);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if ((threadIdx.x & 63) == 0) {
    st[0] = r.s.hi;
    st[1] = r.s.lo;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return (uint32_t)(x + 1);
}

// Lane-parallel PCG64: lane j of a chunk holds the state after j+1 draws from
// the chunk's base state, s_j = A_j*base + M_j*inc (jump table p.jump), and
// its uniform next_double. Draws are consumed in stream order; the committed
// state after `pos` draws of the chunk is the base (pos = 0) or lane pos-1's.
struct ParRng {
  U128 base, inc;  // wave-uniform
  U128 st;         // lane j: state after j+1 draws of the chunk
  double u;        // lane j: uniform j of the chunk
  int pos;         // draws consumed in this chunk (wave-uniform)
};
__device__ __forceinline__ U128 rl128(U128 x, int l) {
  return U128{readlane_u64(x.hi, l), readlane_u64(x.lo, l)};
}
__device__ __forceinline__ void par_fill(ParRng &g, const U128 &JA, const U128 &JM) {
  g.st = add128(mul128(JA, g.base), mul128(JM, g.inc));
  const uint64_t x = g.st.hi ^ g.st.lo;
  const unsigned rot = (unsigned)(g.st.hi >> 58);
  const uint64_t out = (x >> rot) | (x << ((64 - rot) & 63));
  g.u = (double)(out >> 11) * (1.0 / 9007199254740992.0);
  g.pos = 0;
}
__device__ __forceinline__ void par_next_chunk(ParRng &g, const U128 &JA, const U128 &JM) {
  g.base = rl128(g.st, 63);
  par_fill(g, JA, JM);
}
__device__ __forceinline__ U128 par_state(const ParRng &g) {
  return g.pos == 0 ? g.base : rl128(g.st, uni(g.pos - 1));
}

// random_poisson, mult method (lam < 10): the running product is formed in
// stream order (same rounding as the sequential loop), uniforms by readlane.
__device__ __forceinline__ int64_t par_poisson_mult(ParRng &g, double enlam, const U128 &JA,
                                                    const U128 &JM) {
  double prod = 1.0;
  int64_t X = 0;
#pragma unroll 1
  for (;;) {
    if (g.pos == 64) par_next_chunk(g, JA, JM);
    prod *= readlane_f64(g.u, uni(g.pos));
    g.pos++;
    if (prod > enlam)
      X += 1;
    else
      return X;
  }
}

// random_poisson_ptrs (lam >= 10): every loop iteration consumes one (U, V)
// pair and its outcome depends on that pair only, so lanes i < 32 evaluate
// pair i of the chunk at once; the n-th draw is the n-th accepting pair.
struct PtrsChunk {
  uint64_t acc;  // accepting pairs of the chunk
  int64_t k;     // lane i: k of pair i
  bool valid;
};
__device__ __forceinline__ void par_ptrs_eval(const ParRng &g, const PoisConst &c, PtrsChunk &pc) {
  const int lane = lane_id();
  const int i = lane & 31;
  const double U = __shfl(g.u, 2 * i) - 0.5;
  const double V = __shfl(g.u, 2 * i + 1);
  const double us = 0.5 - fabs(U);
  const int64_t k = (int64_t)floor((2 * c.a / us + c.b) * U + c.lam + 0.43);
  bool ok;
  if ((us >= 0.07) && (V <= c.vr))
    ok = true;
  else if ((k < 0) || ((us < 0.013) && (V > us)))
    ok = false;
  else
    ok = ptrs_accept(V, us, k, c.lam, c.a, c.b, c.loglam, c.log_invalpha, c.loggam_tab, c.tab_n);
  pc.acc = ballot(ok && lane < 32);
  pc.k = k;
  pc.valid = true;
}
__device__ __forceinline__ int64_t par_poisson_ptrs(ParRng &g, const PoisConst &c, PtrsChunk &pc,
                                                    const U128 &JA, const U128 &JM) {
#pragma unroll 1
  for (;;) {
    if (g.pos == 64) {
      par_next_chunk(g, JA, JM);
      pc.valid = false;
    }
    if (!pc.valid) par_ptrs_eval(g, c, pc);
    const uint64_t m = pc.acc & (~0ull << (g.pos >> 1));
    if (m == 0) {
      g.pos = 64;
      continue;
    }
    const int i = uni(__builtin_ctzll(m));
    g.pos = 2 * i + 2;
    return (int64_t)readlane_u64((uint64_t)pc.k, i);
  }
}

__device__ __forceinline__ int64_t par_poisson(ParRng &g, const PoisConst &c, PtrsChunk &pc,
                                               const U128 &JA, const U128 &JM) {
  if (c.kind == 0) return 0;  // lam == 0: no draw consumed
  if (c.kind == 1) return par_poisson_mult(g, c.enlam, JA, JM);
  return par_poisson_ptrs(g, c, pc, JA, JM);
}

__device__ __forceinline__ void predraw(const EnvParams &p, const Lds &L, const Tables &T,
                                        int K, int V, const U128 &JA, const U128 &JM) {
  const int lane = lane_id();
  EnvHdr LDSP *H = L.hdr;
  ParRng g;
  PtrsChunk pc;
  pc.valid = false;
  // K arrival counts, rng3 (env.py:272)
  Pcg r3 = ld_pcg(H, 2);
  g.base = r3.s;
  g.inc = r3.inc;
  par_fill(g, JA, JM);
  int64_t need = 0;
#pragma unroll 1
  for (int k = 0; k < K; k++) {
    const int64_t a = par_poisson(g, T.pois[0], pc, JA, JM);
    if (lane == 0) L.arr[k] = (int32_t)(a < 0x7fffffff ? a : 0x7fffffff);
    need += a < V ? a : V;
  }
  r3.s = par_state(g);
  st_pcg(H, 2, r3);
  // up to scap speculative service lengths, rng4 (env.py:289), with the state
  // after each draw for the commit
  Pcg r4 = ld_pcg(H, 3);
  // a one-step launch after a step that left no NULL slot and no running VM
  // due to finish accepts nothing (_accept_vm_requests fills NULL slots only):
  // no service length is drawn. The hint (EnvHdr::pad, written by the
  // previous per-step launch) only gates this speculation: a draw it wrongly
  // skipped would come from svc_fallback, from the same stream position.
  const uint64_t hint = H->pad;
  const bool none_free = K == 1 && (hint >> 63) && ((hint >> 32) & 1u) == 0 &&
                         (uint32_t)hint > (uint32_t)H->timestep + 1u;
  const int S = none_free ? 0 : (int)(need < p.scap ? need : p.scap);
  g.base = r4.s;
  g.inc = r4.inc;
  pc.valid = false;
  if (S > 0) par_fill(g, JA, JM);
#pragma unroll 1
  for (int j = 0; j < S; j++) {
    const int64_t x = par_poisson(g, T.pois[1], pc, JA, JM);
    const U128 sj = par_state(g);
    if (lane == 0) {
      L.svc[j] = (uint32_t)(x + 1);
      L.svcst[2 * j] = sj.hi;
      L.svcst[2 * j + 1] = sj.lo;
    }
  }
  const U128 fb = S > 0 ? par_state(g) : r4.s;
  if (lane == 0) {
    L.svcfb[0] = fb.hi;  // fallback continues after the last speculative draw
    L.svcfb[1] = fb.lo;
    L.svcinfo[0] = S;
    L.svcinfo[1] = 0;  // consumed
  }
  wsync();
}

// Next planned runtime (rng4.poisson(L) + 1, env.py:289) for an accepted VM.
__device__ __forceinline__ uint32_t svc_take(const EnvParams &p, const Lds &L) {
  const int S = L.svcinfo[0], used = L.svcinfo[1];
  uint32_t x;
  if (used < S) {
    x = L.svc[used];
  } else {
    x = svc_fallback(L.svcfb, &L.hdr->rng[3][2], p.pois + 1);
  }
  wsync();
  if (lane_id() == 0) L.svcinfo[1] = used + 1;
  wsync();
  return x;
}

// Commit rng4 to the state after the last consumed draw.
__device__ __forceinline__ void svc_commit(const Lds &L) {
  const int S = L.svcinfo[0], used = L.svcinfo[1];
  if (used == 0) return;
  uint64_t hi, lo;
  if (used <= S) {
    hi = L.svcst[2 * (used - 1)];
    lo = L.svcst[2 * (used - 1) + 1];
  } else {
    hi = L.svcfb[0];
    lo = L.svcfb[1];
  }
  wsync();
  if (lane_id() == 0) {
    L.hdr->rng[3][0] = hi;
    L.hdr->rng[3][1] = lo;
  }
  wsync();
}

// FirstFitAgent.act / BestFitAgent.act (firstfit.py:21-38, bestfit.py:21-40)
// on the pre-step f32 observation, fused with the action phase of step().
// Exact w.r.t. the reference's sequential loop because:
//  - a waiting VM's choice is "first visiting position whose PM fits", answered
//    in O(P/64) from per-size fit bitmaps; the earliest VM (index order) with a
//    fit wins; VMs before it never fit again (loads only grow);
//  - after a FirstFit win on PM q only q's cpu threshold drops, so the cached
//    "has a fit" bit of a later VM can change only if q fitted it before and
//    not after (its first fit was then q or earlier; re-querying is exact
//    either way); BestFit changes both of q's thresholds and re-queries the
//    VMs q fitted before and not after; its target is bf_choose's argmax;
//  - the heuristic's state (f32 view) and the env's state (f64) are disjoint,
//    so applying each winner's env event as soon as it is decided equals
//    deciding every action first and stepping afterwards (env.py:68-88).
template <int VPT>
__device__ __forceinline__ int64_t heuristic_apply(const EnvParams &p, const Lds &L,
                                                   const Tables &T, uint32_t (&wa)[VPT],
                                                   int policy, int32_t *act_out,
                                                   uint8_t *valid_out, bool quiet, int qkind,
                                                   bool &fit_any STAMP_PARAMS) {
  const int lane = lane_id();
  const int P = p.P, WAIT = p.P;
  const bool bf = policy == 1;
  uint32_t pend = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++)
    if (w_pl(wa[s]) == WAIT) pend |= 1u << s;
  uint32_t won = 0, bad = 0;
  int64_t n_place = 0;
  fit_any = false;
  // quiet: skip the heuristic. qkind 1 (EnvHdr::pad bit 62): the previous
  // step found no pending VM that fits any PM, and since then no VM finished
  // (no PM load fell) and none arrived (no new pending VM): nothing fits now
  // either, so the heuristic places nothing and the any-fit table need not
  // be built. qkind 2 (bit 60): the previous step's placements were all
  // invalid in f64 (the f32 observation said they fit: a PM loaded to within
  // rounding of 1) and nothing finished or arrived, so the step sees the same
  // observation, makes the same decisions and the env rejects them again -
  // env_body takes this skip only where no actions / validity flags are
  // returned. The check build (-DVMP_CHECK_QUIET) runs the heuristic anyway
  // and counts the skippable steps in which some pending VM fits (qkind 1)
  // or some placement is valid (qkind 2) (vmp_debug_quiet_violations): 0
  // unless a writer of the env state left a stale bit (see EnvHdr::pad).
#ifdef VMP_CHECK_QUIET
  if (ballot(pend != 0)) {
#else
  if (!quiet && ballot(pend != 0)) {
#endif
    for (int i = lane; i < P; i += 64) {
      const float fcv = (float)L.cpu[i], fmv = (float)L.mem[i];
      L.fcpu[i] = fcv;
      L.fmem[i] = fmv;
      L.tc[i] = (uint8_t)(fit_threshold(fcv) + 1);
      L.tm[i] = (uint8_t)(fit_threshold(fmv) + 1);
    }
    wsync();
    STAMP(16);
    uint32_t hit = 0;  // bit s: VM slot s of this lane is pending and some PM fits it
    // the any-fit table M (build_fitmax) answers "does some PM accept (c, m)";
    // it is rebuilt after each placement (only the placed PM's thresholds move)
    uint32_t LDSP *M = reinterpret_cast<uint32_t LDSP *>(L.bc);
    build_fitmax(p, L, M);
#pragma unroll
    for (int s = 0; s < VPT; s++)
      hit |= (uint32_t)(((pend >> s) & 1u) && M[w_cc(wa[s])] > (uint32_t)w_cm(wa[s])) << s;
    const bool anyfit = ballot(hit != 0) != 0;
    fit_any = anyfit;
#ifdef VMP_CHECK_QUIET
    if (quiet && qkind == 1 && anyfit && lane == 0)
      __hip_atomic_fetch_add(gptr(&g_quiet_violations), 1ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
#endif
    STAMP(17);
#pragma unroll 1
    for (; anyfit;) {
      // earliest VM (index order s * 64 + lane) with a fit: each lane's lowest
      // hit slot, then a DPP max over the wave of (2047 - index)
      const int mine = hit ? (__builtin_ctz(hit) << 6) | lane : 2047;
      const int best = 2047 - (int)__builtin_amdgcn_readlane(
                                  (int)prefix_max32((uint32_t)(2047 - mine)), 63);
      STAMP(18);
      if (best == 2047) break;
      const int ws = best >> 6, wl = best & 63;
      uint32_t own = 0;
#pragma unroll
      for (int s = 0; s < VPT; s++)
        if (s == ws) own = wa[s];
      const uint32_t ww = rdlane(own, wl);
      // everything up to and including the winner is decided
#pragma unroll
      for (int s = 0; s < VPT; s++)
        if (s < ws || (s == ws && lane <= wl)) pend &= ~(1u << s);
      hit &= pend;
      const int kc = w_cc(ww), km = w_cm(ww);
      const int q = bf ? bf_choose(p, L, kc, km) : ff_scan(p, L, kc, km);  // wave-uniform
      // the env event (env.py:55-64: _resource_valid in f64, _place_vm) and the
      // heuristic's own f32 update (FF: cpu only, firstfit.py:36) read and
      // write disjoint state: one LDS round trip, one write-back
      const double cq = L.cpu[q], mq = L.mem[q];
      const float fq = L.fcpu[q], fmq = L.fmem[q];
      const int tc_old = (int)L.tc[q] - 1, tm_old = (int)L.tm[q] - 1;
      const double vc = T.cent[kc], vm = T.cent[km];
      const bool ok = (cq + vc <= 1) && (mq + vm <= 1);
      const float nc = fq + T.fcent[kc];
      const float nm = fmq + T.fcent[km];
      const int t = fit_threshold(nc);
      const int tmq = bf ? fit_threshold(nm) : tm_old;
      wsync();
      if (lane == 0) {
        if (ok) {
          L.cpu[q] = cq + vc;
          L.mem[q] = mq + vm;
          mark_pm(L, P, q);
        }
        L.fcpu[q] = nc;
        L.tc[q] = (uint8_t)(t + 1);
        if (bf) {
          L.fmem[q] = nm;
          L.tm[q] = (uint8_t)(tmq + 1);
        }
      }
      wsync();
      n_place += ok;
      STAMP(20);
      if (lane == wl) {
#pragma unroll
        for (int s = 0; s < VPT; s++)
          if (s == ws) {
            won |= 1u << s;
            if (ok) wa[s] = (wa[s] & 0xFFFF0000u) | (uint32_t)q;
            else bad |= 1u << s;
          }
        if (act_out) gptr(act_out)[ws * 64 + wl] = q;
      }
      STAMP(21);
      if (t < tc_old || tmq < tm_old) {  // q's thresholds fell: the table changes
        build_fitmax(p, L, M);
        STAMP(23);
        // re-query the VMs still pending with a fit (M is exact: "some PM
        // accepts (c, m)"), table reads batched four slots at a time
#pragma unroll
        for (int s0 = 0; s0 < VPT; s0 += 4) {
          uint32_t mc[4];
#pragma unroll
          for (int j = 0; j < 4; j++) mc[j] = s0 + j < VPT ? M[w_cc(wa[s0 + j])] : 0u;
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (s0 + j < VPT && !(mc[j] > (uint32_t)w_cm(wa[s0 + j]))) hit &= ~(1u << (s0 + j));
        }
      }
      STAMP(19);
    }
  }
#ifdef VMP_CHECK_QUIET
  if (quiet && qkind == 2 && n_place > 0 && lane == 0)
    __hip_atomic_fetch_add(gptr(&g_quiet_violations), 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
#endif
  if (act_out || valid_out) {
    const int ln = fresh_lane();
#pragma unroll
    for (int s = 0; s < VPT; s++) {
      const int v = s * 64 + ln;
      if (live(wa[s])) {
        if (act_out && !((won >> s) & 1u)) gptr(act_out)[v] = (int32_t)w_pl(wa[s]);
        if (valid_out) gptr(valid_out)[v] = (uint8_t)!((bad >> s) & 1u);
      }
    }
  }
  return n_place;
}

// Action phase of step() for external actions (env.py:68-88): per slot of 64
// VMs, the events (WAIT -> PM place attempts, PM -> WAIT suspends) are applied
// in ascending VM order by a wave-uniform loop over the ballot.
template <int VPT>
__device__ __forceinline__ void external_apply(const EnvParams &p, const Lds &L, const Tables &T,
                                               uint32_t (&wa)[VPT], const int32_t *act_row,
                                               uint8_t *valid_out, int64_t &n_place,
                                               int64_t &n_susp) {
  const int lane = lane_id();
  const int P = p.P, WAIT = p.P;
  // all action loads issued at once, unconditionally (clamped index) and
  // through the global address space: one wait for all of them instead of a
  // conditional load + wait per slot row
  const int32_t GLBP *ar = gptr(act_row);
  int32_t tv[VPT];
  __asm__ volatile("" ::: "memory");  // not hoisted above the prologue's draws
#pragma unroll
  for (int s = 0; s < VPT; s++) tv[s] = ar[min(s * 64 + lane, p.V - 1)];
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const int v = s * 64 + lane;
    const bool in = live(wa[s]);
    const int c = w_pl(wa[s]);
    const int t = in ? tv[s] : c;
    const bool isplace = in && c == WAIT && t >= 0 && t < P;
    const bool issusp = in && c < P && t == WAIT;
    uint64_t evm = ballot(isplace || issusp);
    uint64_t okm = 0;
    const uint32_t me = wa[s];
#pragma unroll 1
    while (evm) {  // wave-uniform, ascending lane = ascending VM index
      const int l = __ffsll((unsigned long long)evm) - 1;
      evm &= evm - 1;
      const uint32_t ew = rdlane(me, l);
      const int et = __builtin_amdgcn_readlane(t, l);
      const int ec = w_pl(ew);
      const double vc = T.cent[w_cc(ew)], vm = T.cent[w_cm(ew)];
      const int q = (ec == WAIT) ? et : ec;
      double cq = L.cpu[q], mq = L.mem[q];
      bool eok = true;
      if (ec == WAIT) {
        eok = (cq + vc <= 1) && (mq + vm <= 1);
        if (eok) {
          cq = cq + vc;
          mq = mq + vm;
        }
      } else {
        cq = cq - vc;
        mq = mq - vm;
      }
      wsync();
      if (lane == 0) {
        L.cpu[q] = cq;
        L.mem[q] = mq;
        mark_pm(L, P, q);
      }
      okm |= (uint64_t)eok << l;
      wsync();
    }
    bool ok = (t == c) || issusp;
    if (isplace) ok = (okm >> lane) & 1ull;
    n_place += __popcll(okm & ballot(isplace));
    n_susp += __popcll(ballot(issusp));
    if (ok && t != c && in) wa[s] = (wa[s] & 0xFFFF0000u) | (uint32_t)t;
    if (valid_out && in) gptr(valid_out)[v] = (uint8_t)ok;
  }
}

// kl_divergence (env.py:8-17) in numpy/LAPACK/OpenBLAS evaluation order.
__device__ __forceinline__ double kl_reward(double tcm, double tmm, double tcv, double tmv,
                                            double cm, double mm, double cv, double mv) {
  double det_q = exp((0.0 + log(cv)) + log(mv));
  double det_p = exp((0.0 + log(tcv)) + log(tmv));
  double qi0 = 1.0 / cv, qi1 = 1.0 / mv;
  double tr = qi0 * tcv + qi1 * tmv;
  double d0 = tcm - cm, d1 = tmm - mm;
  double m1 = fma(d1 * qi1, d1, (d0 * qi0) * d0);
  double kl = 0.5 * ((((log(det_q / det_p) - 2) + tr) + m1) - tr);
  return -kl;
}

// Everything of step() after the action phase: _run_vms, _accept_vm_requests,
// stats + reward, termination (env.py:101, 108-163, 244-293).
// LAZY (the per-step launch): the high words are not held in registers. `fb`
// bit s says whether slot s finishes this step if it runs (running: F - t <= 1;
// waiting: remaining <= 1, i.e. placed now it finishes now), accepted words are
// stored at once through `vmo`, and the caller fixes the finish keys of placed /
// suspended VMs in memory; rem[] is then unused.
template <int VPT, bool LAZY>
__device__ __forceinline__ double env_tail(const EnvParams &p, const Lds &L, const Tables &T,
                                           uint32_t (&wa)[VPT], uint32_t (&rem)[VPT],
                                           uint32_t run0, uint32_t fb, uint32_t &dirty,
                                           uint32_t *vmo, int kstep, bool ext,
                                           bool quiet_in, bool &terminated, bool &calm,
                                           bool &has_ex STAMP_PARAMS) {
  const int lane = lane_id();
  const int P = p.P, WAIT = p.P, NUL = p.P + 1;
  EnvHdr LDSP *H = L.hdr;
  // ---- _run_vms (env.py:244-268) ----
  // A running VM's word holds its finish key F = t + remaining (t = this
  // step's timestep), so the per-step decrement of every running VM is implicit
  // and its word is not rewritten; waiting VMs hold the remaining runtime
  // itself. The action phase only moves VMs between WAIT and a PM (external
  // migrations PM -> PM' are invalid, env.py:35-44), so run0 (running before the
  // action phase) tells which words switch representation.
  const uint32_t t32 = (uint32_t)H->timestep;
  int64_t n_term = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const bool running = w_pl(wa[s]) < P;
    if (running != (bool)((run0 >> s) & 1u)) {
      if (!LAZY) rem[s] = running ? rem[s] + t32 : rem[s] - t32;  // placed : suspended
      dirty |= 1u << s;
    }
    // remaining r = F - t: decrement if r > 0, finish if it reaches 0
    const bool term = running && (LAZY ? (bool)((fb >> s) & 1u) : (int32_t)(rem[s] - t32) <= 1);
    uint64_t it = ballot(term);
    n_term += __popcll(it);
    const uint32_t me = wa[s];
#pragma unroll 1
    while (it) {  // frees in ascending VM order (env.py:260-262)
      const int l = __ffsll((unsigned long long)it) - 1;
      it &= it - 1;
      const uint32_t ew = rdlane(me, l);
      const int q = w_pl(ew);
      const double cq = L.cpu[q] - T.cent[w_cc(ew)];
      const double mq = L.mem[q] - T.cent[w_cm(ew)];
      wsync();
      if (lane == 0) {
        L.cpu[q] = cq;
        L.mem[q] = mq;
        mark_pm(L, P, q);
      }
      wsync();
    }
    if (term) {
      wa[s] = w_make(NUL, 0, 0);
      if (!LAZY) rem[s] = 0;
      dirty |= 1u << s;
    }
  }
  // precision clamp (env.py:267-268): every stored load is 0 or >= 1e-7 after
  // the previous step's clamp and placements only add, so only a free or a
  // suspension (external actions) can leave a value below 1e-7
  if (n_term > 0 || ext)
    for (int i = lane; i < P; i += 64) {
      if (L.cpu[i] < 1e-7) L.cpu[i] = 0;
      if (L.mem[i] < 1e-7) L.mem[i] = 0;
    }
  STAMP(2);
  // ---- _accept_vm_requests (env.py:271-293) ----
  // only a finish makes a NULL slot: none if the previous per-step launch left
  // none (EnvHdr::pad bit 32 clear under bit 63; the launch's first step: the
  // header's hint is the state before it) and none finished now
  const uint64_t ph = H->pad;
  const bool no_null = kstep == 0 && (ph >> 63) && !((ph >> 32) & 1u) && n_term == 0;
  int n_null = 0;
  if (!no_null) {
#pragma unroll
    for (int s = 0; s < VPT; s++) {
      const int v = s * 64 + lane;
      const bool isnull = w_pl(wa[s]) == NUL;
      const uint64_t nm = ballot(isnull);
      if (isnull) L.nulls[n_null + below(nm, lane)] = (uint16_t)v;
      n_null += __popcll(nm);
    }
  }
  const int64_t arrivals = L.arr[kstep];  // rng3.poisson(lambda), drawn in the prologue
  const int64_t k = arrivals < n_null ? arrivals : n_null;
  wsync();
  if (k > 0) {
    // to_accept = the first k NULL slots; sizes popped from the rng1/rng2
    // sequences, planned runtimes from rng4 (env.py:276-290)
    Pcg r1 = ld_pcg(H, 0), r2 = ld_pcg(H, 1);
#pragma unroll 1
    for (int j = 0; j < k; j++) {
      const int cc = (int)rint((p.seq_lo + p.seq_range * next_double(r1)) * 100.0);
      const int cm = (int)rint((p.seq_lo + p.seq_range * next_double(r2)) * 100.0);
      const uint32_t rr = svc_take(p, L);
      const int v = L.nulls[j];
      if (lane == (v & 63)) {
#pragma unroll
        for (int s = 0; s < VPT; s++)
          if (s == (v >> 6)) {
            wa[s] = w_make(WAIT, cc, cm);
            if (LAZY) {  // final for this launch: stored now, skipped at the end
              ST_NT(vmo + vm_slot_idx(v), wa[s]);
              ST_NT(vmo + vm_time_idx(v), rr);
              dirty &= ~(1u << s);
            } else {
              rem[s] = rr;
              dirty |= 1u << s;
            }
          }
      }
      if (lane == 0) {
        L.accc[j] = (uint8_t)cc;
        L.accm[j] = (uint8_t)cm;
      }
    }
    st_pcg(H, 0, r1);
    st_pcg(H, 1, r2);
  }
  wsync();
  STAMP(3);
  // ---- stats + reward (env.py:112-156) ----
  // target_cpu/memory_mean (env.py:116-121) feed only the kl reward and the
  // eval-mode info; for wr/ut they are derived on demand from the stored state
  // by k_target_means (vmp_get_stats), so the step skips the two V-long sums.
  const bool kl = p.reward == 2;
  int n_ex = 0, n_w = 0;
  // wr after a quiet step in which nothing finished, arrived or was placed:
  // the VM set is the previous step's, so is its waiting ratio (stored in the
  // header) and whether any VM exists (has_ex: carried by the caller, from
  // EnvHdr::pad bit 61 at the launch's start)
  const bool same_vms = p.reward == 0 && quiet_in && n_term == 0 && k == 0;
  if (!same_vms) {
#pragma unroll
    for (int s = 0; s < VPT; s++) {
      const int c = w_pl(wa[s]);
      const bool ex = c <= WAIT;
      const uint64_t em = ballot(ex);
      if (kl && ex) {
        const int rk = n_ex + below(em, lane);
        L.ccomp[rk] = (uint8_t)w_cc(wa[s]);
        L.mcomp[rk] = (uint8_t)w_cm(wa[s]);
      }
      n_ex += __popcll(em);
      n_w += __popcll(ballot(c == WAIT));
    }
  }
  if (!same_vms) has_ex = n_ex > 0;
  wsync();
  STAMP(11);
  // the pairwise reductions of the step, one inlined body per source type:
  //  0,1  sum of the accepted sizes (total_*_requested, env.py:280/285)
  //  2,3  sum of existing VM sizes (target means, env.py:116-121)
  //  4,5  sum of PM cpu / memory (ut reward; kl means)
  //  6,7  PM squared-deviation sums (kl, np.var(cpu/memory))
  //  8,9  VM-size squared-deviation sums (kl, np.var(vm_cpu/vm_memory[existing]))
  double LDSP *res = L.jobres;
  const double *cent = T.cent;
  {  // VM-size sources: accepted sizes, existing sizes, their deviations
#pragma unroll 1
    for (int j = (k > 0 ? 0 : 2); j < (kl ? 4 : 2); j++) {
      const uint8_t LDSP *src = (j == 0) ? L.accc : (j == 1) ? L.accm : ((j & 1) ? L.mcomp : L.ccomp);
      const int n = j < 2 ? (int)k : n_ex;
      const double r = wave_pw_sum(n, [=](int i) { return cent[src[i]]; }, L.pw);
      wsync();
      if (lane == 0) res[j] = r;
      wsync();
    }
  }
  if (p.reward >= 1) {  // PM sources (ut, kl)
    const int jend = p.reward == 2 ? 8 : 6;
#pragma unroll 1
    for (int j = 4; j < jend; j++) {
      const double LDSP *src = (j & 1) ? L.mem : L.cpu;
      const double mean = j < 6 ? 0.0 : res[j - 2] / (double)P;
      const bool sq = j >= 6;
      const double r = wave_pw_sum(P, [=](int i) {
        const double x = src[i];
        const double d = x - mean;
        return sq ? d * d : x;
      }, L.pw);
      wsync();
      if (lane == 0) res[j] = r;
      wsync();
    }
  }
  if (p.reward == 2) {  // VM-size deviations (kl)
#pragma unroll 1
    for (int j = 8; j < 10; j++) {
      const uint8_t LDSP *src = (j & 1) ? L.mcomp : L.ccomp;
      const double mean = res[j - 6] / (double)n_ex;
      const double r = wave_pw_sum(n_ex, [=](int i) {
        const double d = cent[src[i]] - mean;
        return d * d;
      }, L.pw);
      wsync();
      if (lane == 0) res[j] = r;
      wsync();
    }
  }
  STAMP(12);
  const double wr = same_vms ? H->waiting_ratio : n_ex > 0 ? (double)n_w / (double)n_ex : 0.0;
  if (!kl) res[2] = res[3] = 0.0;  // unused below
  double tcm = res[2] / (double)P;
  if (p.cap_target_util && tcm > 1) tcm = 1.0;
  double tmm = res[3] / (double)P;
  if (p.cap_target_util && tmm > 1) tmm = 1.0;
  double reward = 0.0;
  if (has_ex) {
    if (p.reward == 2) {  // kl (env.py:124-149)
      double cv = res[6] / (double)P, mv = res[7] / (double)P;
      if (cv == 0) cv = 1e-6;
      if (mv == 0) mv = 1e-6;
      double tcv = res[8] / (double)n_ex, tmv = res[9] / (double)n_ex;
      if (tcv == 0) tcv = 1e-6;
      if (tmv == 0) tmv = 1e-6;
      reward = (tcm == 0 || tmm == 0)
                   ? 0.0
                   : kl_reward(tcm, tmm, tcv, tmv, res[4] / (double)P, res[5] / (double)P, cv, mv);
    } else if (p.reward == 1) {  // ut (env.py:150-151)
      reward = p.beta * res[4] + (1 - p.beta) * res[5];
    } else {  // wr (env.py:152-153)
      reward = -wr;
    }
  }
  STAMP(4);
  // ---- counters, termination (env.py:160-163, 101) ----
  const int64_t ts = H->timestep;
  terminated = ts >= p.limit;
  calm = n_term == 0 && k == 0;  // no PM load fell, no new pending VM
  (void)n_ex;
  wsync();
  if (lane == 0) {
    H->timestep = ts + 1;
    H->total_requests += arrivals;
    H->served += n_term;
    H->dropped += arrivals - k;
    H->waiting_ratio = wr;
    if (kl) {
      H->tcm = tcm;
      H->tmm = tmm;
    }
    if (k > 0) {
      H->total_cpu_req = H->total_cpu_req + res[0];
      H->total_mem_req = H->total_mem_req + res[1];
    }
  }
  wsync();
  return reward;
}

template <int VPT>
__device__ __forceinline__ void write_obs(const EnvParams &p, const Lds &L, const Tables &T,
                                          const uint32_t (&wa)[VPT], float *obs) {
  const int lane = fresh_lane();
  const int V = p.V, P = p.P;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const int v = s * 64 + lane;
    if (live(wa[s])) {
      ST_NT(obs + v, (float)w_pl(wa[s]));
      ST_NT(obs + V + v, T.fcent[w_cc(wa[s])]);
      ST_NT(obs + 2 * V + v, T.fcent[w_cm(wa[s])]);
    }
  }
  for (int i = lane; i < P; i += 64) {
    ST_NT(obs + 3 * V + i, (float)L.cpu[i]);
    ST_NT(obs + 3 * V + P + i, (float)L.mem[i]);
  }
}

// get_invalid_action_mask(masked=True) (env.py:45-53), bit-packed, 1 = invalid.
template <int VPT>
__device__ __forceinline__ void write_mask(const EnvParams &p, const Lds &L, const Tables &T,
                                           const uint32_t (&wa)[VPT], uint32_t *bits) {
  const int lane = fresh_lane();
  const int P = p.P, A = p.A, W = p.W32, WAIT = p.P, NUL = p.P + 1;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const int v = s * 64 + lane;
    const bool in = live(wa[s]);
    const int c = in ? w_pl(wa[s]) : NUL;
    const double vc = T.cent[w_cc(wa[s])], vm = T.cent[w_cm(wa[s])];
    const bool waiting = in && c == WAIT;
    const bool anyw = ballot(waiting) != 0;
#pragma unroll 1
    for (int w = 0; w < W; w++) {
      uint32_t word = 0xFFFFFFFFu;
      const int a0 = w * 32;
      if (c >= a0 && c < a0 + 32 && c < A) word &= ~(1u << (c - a0));  // stay
      if (c < P && WAIT >= a0 && WAIT < a0 + 32) word &= ~(1u << (WAIT - a0));  // suspend
      if (anyw) {
        const int hi = min(a0 + 32, P);
#pragma unroll 1
        for (int q = a0; q < hi; q++) {  // uniform q: LDS broadcast reads
          const bool fit = (L.cpu[q] + vc <= 1) && (L.mem[q] + vm <= 1);
          if (waiting && fit) word &= ~(1u << (q - a0));
        }
      }
      if (in) bits[(int64_t)v * W + w] = word;
    }
  }
}

// ONE = true is the per-step launch (k_steps == 1, the Base.test loop body); it
// is a separate instantiation so profiles tell it apart from fused rollouts.
// EXT = true: the external-action step (vmp_step), its own kernel k_env_ext so
// the heuristic's registers do not weigh on it and vice versa.
template <int VPT, bool ONE, bool EXT>
__device__ __forceinline__ void env_body(const EnvParams &p, const StepOut &o) {
  extern __shared__ __align__(16) char lds[];
  __shared__ Tables T;
#ifdef VMP_STAMPS
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
  const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
#endif
  const int lane = lane_id();
  const int wid = threadIdx.x >> 6;
  const int e_raw = uni(blockIdx.x * kEnvWavesPerBlock + wid);
  const int e = e_raw < p.N ? e_raw : p.N - 1;  // tail waves load a valid env, then leave
  char LDSP *base = (char LDSP *)lds + wid * p.lds_wave_bytes;
  const Lds L = make_lds(p, base);
  const int V = p.V, P = p.P;
  // ---- every global load of the env's state is issued up front: header and
  // PM resources (needed first, to LDS), then the VM words (to registers),
  // whose latency the random draws below overlap ----
  // (indices are clamped instead of branched on, so no load is conditional and
  // the waits below can count: a skipped load would force vmcnt(0))
  // a starting wave's state loads issue ahead of the running waves' work: its
  // critical path starts at their latency (burst launches -1.1-1.6 %,
  // profiles/r04_prio_prologue_ab.log)
  __builtin_amdgcn_s_setprio(2);
  const uint64_t hv = gptr(reinterpret_cast<const uint64_t *>(p.hdr + e))[lane & 31];
  // Poisson constants for the block's LDS copy (issued before the state loads,
  // so waiting for them never waits on the state)
  constexpr int kPoisWords = (int)(2 * sizeof(PoisConst) / 4);
  const uint32_t pw = gptr(reinterpret_cast<const uint32_t *>(p.pois))[threadIdx.x % kPoisWords];
  // this lane's PCG64 jump entry (lane-parallel draws), right behind the header
  U128 JA{0, 0}, JM{0, 0};
  if (o.k_steps > 0) {
    const uint64_t GLBP *jt = gptr(p.jump + 4 * lane);
    JA = U128{jt[0], jt[1]};
    JM = U128{jt[2], jt[3]};
  }
  const double *pm = p.pm + (int64_t)e * 2 * P;
  const int n_pm = 2 * P;
  double pv[4];
#pragma unroll
  for (int j = 0; j < 4; j++) pv[j] = pm[min(j * 64 + lane, n_pm - 1)];
  __asm__ volatile("" ::: "memory");  // keep the issue order: header/PM first
  // ONE: only the slot words (placement, sizes) go to registers here; the
  // finish keys are read after the draws and folded into one bit per slot
  // (slot and time words sit in separate 256-B runs of each 64-slot block)
  const uint32_t GLBP *vlo = gptr(p.vmw + (int64_t)e * vm_pitch(V));
  uint32_t wa[VPT], rem[VPT];
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const int v = s * 64 + lane;
    const uint32_t x = vlo[vw_row(s, lane)];
    wa[s] = v < V ? x : (uint32_t)kPad;
    if (ONE) {
      rem[s] = 0;
    } else {
      const uint32_t y = vlo[vw_row(s, lane) + 64];
      rem[s] = v < V ? y : 0u;
    }
  }
  __asm__ volatile("" ::: "memory");  // ... and the VM words before any wait
  __builtin_amdgcn_s_setprio(0);
  // size tables (k/100 in f64 and f32) while the loads are in flight; the only
  // block-wide barrier: waves are independent below
  for (int i = threadIdx.x; i < 128; i += blockDim.x) {
    T.cent[i] = (double)i / 100.0;
    T.fcent[i] = (float)((double)i / 100.0);
  }
  if (threadIdx.x < kPoisWords) reinterpret_cast<uint32_t *>(T.pois)[threadIdx.x] = pw;
  __syncthreads();
  if (e_raw >= p.N) return;
  if (lane < 32) reinterpret_cast<uint64_t LDSP *>(L.hdr)[lane] = hv;
  wsync();
#ifdef VMP_STAMPS
  const uint64_t t_loaded = __builtin_amdgcn_s_memtime();
#endif
  // the external kernel parks the PM words in LDS before the draws (issued
  // right behind the header, they are in by then): live across the draws
  // they spilled to scratch there
  if (EXT) {
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (j * 64 + lane < n_pm) L.cpu[j * 64 + lane] = pv[j];
  }
  // the draws need only the header: they run while the PM / VM loads land
  if (o.k_steps > 0) predraw(p, L, T, o.k_steps, V, JA, JM);
#ifdef VMP_STAMPS
  const uint64_t t_drawn = __builtin_amdgcn_s_memtime();
#endif
  if (!EXT) {
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (j * 64 + lane < n_pm) L.cpu[j * 64 + lane] = pv[j];
  }
  for (int i = 256 + lane; i < n_pm; i += 64) L.cpu[i] = pm[i];  // P > 128
  for (int i = lane; i < (n_pm + 63) / 64; i += 64) L.pdirty[i] = 0;
  wsync();
#ifdef VMP_STAMPS
  __shared__ uint64_t st_lds[kEnvWavesPerBlock * kStamps];
#endif
  STAMP_DECL_AT((uint64_t LDSP *)st_lds + wid * kStamps)
#ifdef VMP_STAMPS
  if (lane == 0) {
    st_acc[13] = t_loaded - t_start;
    st_acc[14] = t_drawn - t_loaded;
    st_acc[15] = st_prev - t_drawn;
  }
#endif
  bool term = false;
  int64_t ndone = 0;
  uint32_t dirty = 0;  // bit s: this lane's VM word s changed (stored at the end)
  uint32_t fb = 0;     // ONE: bit s = slot s finishes this step if it runs
  uint32_t hiv[VPT];   // ONE: the finish keys / remaining runtimes, in flight
  uint32_t nf = 0u;  // ONE: smallest finish key running on (EnvHdr::pad hint; 0: unknown)
  bool want_nf = false;
  // ONE, heuristic: a quiet step (EnvHdr::pad bit 62, or bit 60 where no
  // actions / validity flags are returned: it places nothing) whose
  // hint records the smallest finish key nf of the running VMs (the previous
  // launch left no NULL slot) with nf > t + 1 needs no time word: no VM
  // finishes and none is placed, so every finish bit is 0 and nf carries over
  // (heuristic launches suspend nothing). Its 16 time-word loads then all read
  // one line (the loads stay unconditional, so the counted waits before their
  // use are the same on both paths): 4 KB less HBM per such env-step.
  bool skip_time = false;
  uint32_t nf_carry = 0u;
  if (ONE && !EXT) {
    // (off in the check build: its quiet steps still run the fit loop and
    // may place, which a skipped step's carried nf and zero finish bits
    // would leave stale: the audited state must evolve as the product's)
#if !defined(VMP_NO_TIME_SKIP) && !defined(VMP_CHECK_QUIET)
    const uint64_t ph = L.hdr->pad;
    nf_carry = (uint32_t)ph;
    const bool skip_h = ((ph >> 62) & 1u) || (((ph >> 60) & 1u) && !o.act_out && !o.valid);
    skip_time = skip_h && (ph >> 63) && ((ph >> 32) & 1u) == 0u && nf_carry != 0u &&
                (int32_t)(nf_carry - (uint32_t)L.hdr->timestep) > 1;
#endif
    // issued before the action phase, consumed after it (latency hidden by it)
    const uint32_t GLBP *hb = vlo + 64 + (skip_time ? 0 : lane);
    const int hs = skip_time ? 0 : 128;
#pragma unroll
    for (int s = 0; s < VPT; s++) hiv[s] = hb[s * hs];
    __asm__ volatile("" ::: "memory");
  }
  uint32_t *vmo = p.vmw + (int64_t)e * vm_pitch(V);
  const int k_steps = ONE ? 1 : o.k_steps;
  // EnvHdr::pad bits 62 / 60 (qkind 1 / 2, see heuristic_apply); the
  // external-action kernel neither uses nor keeps them
  int qkind = EXT ? 0 : (((L.hdr->pad >> 62) & 1u) ? 1 : (((L.hdr->pad >> 60) & 1u) ? 2 : 0));
  bool has_ex = (L.hdr->pad >> 61) & 1u;  // bit 61: some VM exists (read with bit 62 only)
#pragma unroll 1
  for (int k = 0; k < k_steps; k++) {
    const bool last = k == k_steps - 1;
    uint8_t *valid_row = (last && o.valid) ? o.valid + (int64_t)e * V : nullptr;
    int32_t *act_row = (last && o.act_out) ? o.act_out + (int64_t)e * V : nullptr;
    int64_t n_place = 0, n_susp = 0;
    uint32_t run0 = 0;
#pragma unroll
    for (int s = 0; s < VPT; s++) run0 |= (uint32_t)(w_pl(wa[s]) < P) << s;
    bool fit_any = false;
    // qkind 2 repeats rejected placements: skipped only where no actions or
    // validity flags leave this step
    const bool quiet = qkind == 1 || (qkind == 2 && !act_row && !valid_row);
    if (!EXT)
      n_place = heuristic_apply<VPT>(p, L, T, wa, o.policy, act_row, valid_row, quiet, qkind,
                                     fit_any STAMP_ARGS);
    else {
      // the external kernel loads the time words after its action phase: live
      // across it beside the 16 action words they spilled 10 VGPRs
      external_apply<VPT>(p, L, T, wa, o.actions + (int64_t)e * V, valid_row, n_place, n_susp);
      if (ONE) {
        const int ln = fresh_lane();
#pragma unroll
        for (int s = 0; s < VPT; s++) hiv[s] = vlo[vw_row(s, ln) + 64];
      }
    }
    STAMP(1);
    if (ONE) {  // the time words' last use: bit s = slot s finishes this step if it runs
      const uint32_t t32 = (uint32_t)L.hdr->timestep;
      // the next launch's draw hint needs the smallest finish key of the VMs
      // that run on only where the last step left no NULL slot (else nf = 0)
      const uint64_t ph = L.hdr->pad;
      want_nf = !((ph >> 63) && ((ph >> 32) & 1u));
      nf = want_nf ? 0xFFFFFFFFu : 0u;
      if (skip_time) {  // (want_nf holds: the hint's NULL bit is 0)
        nf = nf_carry;
      } else {
#pragma unroll
      for (int s = 0; s < VPT; s++) {  // by the placement before the action phase
        const bool was_run = (run0 >> s) & 1u;
        const bool f = was_run ? (int32_t)(hiv[s] - t32) <= 1 : hiv[s] <= 1u;
        fb |= (uint32_t)f << s;
      }
      }
      if (want_nf && !skip_time) {
#pragma unroll
        for (int s = 0; s < VPT; s++) {
          const bool was_run = (run0 >> s) & 1u;
          const bool f = (fb >> s) & 1u;
          if (w_pl(wa[s]) < P && !f) nf = min(nf, was_run ? hiv[s] : hiv[s] + t32);
        }
      }
    }
    wsync();
    if (lane == 0) {
      L.hdr->place_action += n_place;
      L.hdr->suspend_action += n_susp;
    }
    wsync();
    bool calm = false;
    const double r = env_tail<VPT, ONE>(p, L, T, wa, rem, run0, fb, dirty, vmo, k, EXT, quiet,
                                        term, calm, has_ex STAMP_ARGS);
    // the next step's skip: nothing fit (1), or every placement was rejected
    // (2); a skipped step passes its kind on while nothing changes
    qkind = (EXT || !calm) ? 0 : quiet ? qkind : (!fit_any ? 1 : (n_place == 0 ? 2 : 0));
    if (o.reward && lane == 0) gptr(o.reward)[(int64_t)k * p.N + e] = r;
    ndone += term;
  }
  if (o.k_steps > 0) svc_commit(make_lds(p, opaque_base(base)));
  if (!EXT && o.k_steps == 0 && o.policy >= 0 && o.act_out) {
    // act only: decide on a scratch copy of the VM words; nothing is stored
    uint32_t wt[VPT];
#pragma unroll
    for (int s = 0; s < VPT; s++) wt[s] = wa[s];
    bool fit_any;
    heuristic_apply<VPT>(p, L, T, wt, o.policy, o.act_out + (int64_t)e * V, nullptr, qkind == 1,
                         qkind, fit_any STAMP_ARGS);
  }
  STAMP(0);
  if (o.obs) write_obs<VPT>(p, L, T, wa, o.obs + (int64_t)e * p.D);
  if (o.mask_bits) write_mask<VPT>(p, L, T, wa, o.mask_bits + (int64_t)e * V * p.W32);
  STAMP(5);
  if (o.k_steps > 0) {
    if (o.done && lane == 0) gptr(o.done)[e] = (uint8_t)term;
    if (o.done_count && lane == 0) gptr(o.done_count)[e] += ndone;
    const uint32_t t32 = (uint32_t)(L.hdr->timestep - 1);  // this launch's step
    const int ln = fresh_lane();
#pragma unroll
    for (int s = 0; s < VPT; s++) {
      if (live(wa[s]) && ((dirty >> s) & 1u)) {  // unchanged words stay as they are
        const int iw = (s << 7) + ln;  // live: slot 64 s + ln < V, so its vm_slot_idx
        if (!ONE) {
          ST_NT(vmo + iw, wa[s]);
          ST_NT(vmo + iw + 64, rem[s]);
        } else if (w_pl(wa[s]) == P + 1) {  // finished: NULL, remaining 0
          ST_NT(vmo + iw, wa[s]);
          ST_NT(vmo + iw + 64, 0u);
        } else {  // placed (r -> F = t + r) or suspended (F -> r = F - t)
          uint32_t GLBP *w32 = gptr(vmo);
          w32[iw] = wa[s];
          __hip_atomic_fetch_add(w32 + iw + 64, w_pl(wa[s]) < P ? t32 : 0u - t32,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    // only the PM words written this launch (place / suspend / free: the
    // precision clamp changes no other value, as every stored value is 0 or
    // >= 1e-7 after the previous launch's clamp)
    double *pmo = p.pm + (int64_t)e * 2 * P;
    for (int i = lane, j = 0; i < 2 * P; i += 64, j++)
      if ((L.pdirty[j] >> lane) & 1ull) ST_NT(pmo + i, (double)L.cpu[i]);
    {  // the next launch's draw hint (predraw): per-step launches only
      uint64_t hint = 0;
      if (ONE) {  // (the NULL count is recorded as 0 or 1: only "none" is read)
        bool anynull = false;
#pragma unroll
        for (int s = 0; s < VPT; s++) anynull |= w_pl(wa[s]) == P + 1;
        uint32_t m = nf;
        const bool nn = ballot(anynull) != 0;
        if (!nn && want_nf) {
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o));
        }
        hint = (1ull << 63) | ((uint64_t)nn << 32) | m;
      }
      hint |= ((uint64_t)(qkind == 1) << 62) | ((uint64_t)(qkind == 2) << 60) |
              ((uint64_t)has_ex << 61);
      wsync();
      if (lane == 0) L.hdr->pad = hint;
      wsync();
    }
    if (lane < 32)
      gptr(reinterpret_cast<uint64_t *>(p.hdr + e))[lane] = reinterpret_cast<uint64_t LDSP *>(L.hdr)[lane];
  }
  STAMP(6);
#ifdef VMP_STAMPS
  if (lane == 0) {
    st_acc[7] = (__builtin_amdgcn_s_memrealtime() - rt_start) * 1000;  // x1000 (100 MHz ticks)
    st_acc[9] = __builtin_amdgcn_s_memtime() - t_start;
  }
#endif
  STAMP_FLUSH();
}

template <int VPT, bool ONE>
__global__ __launch_bounds__(64 * kEnvWavesPerBlock, ONE ? VMP_WAVES_PER_EU_ONE : VMP_WAVES_PER_EU) void k_env(EnvParams p, StepOut o) {
  env_body<VPT, ONE, false>(p, o);
}
// VPT 1 (V <= 64, the PPO eval's config/10.yml): 4 waves per SIMD, so a
// 4 096-env step is one round of waves on the 256 CUs (at 3, 131 VGPRs, a
// third of the envs ran in a second round)
template <int VPT>
__global__ __launch_bounds__(64 * kEnvWavesPerBlock, VPT == 1 ? 4 : VMP_WAVES_PER_EU_ONE) void k_env_ext(EnvParams p, StepOut o) {
  env_body<VPT, true, true>(p, o);
}

template __global__ void k_env_ext<1>(EnvParams, StepOut);
template __global__ void k_env_ext<2>(EnvParams, StepOut);
template __global__ void k_env_ext<4>(EnvParams, StepOut);
template __global__ void k_env_ext<8>(EnvParams, StepOut);
template __global__ void k_env_ext<16>(EnvParams, StepOut);
template __global__ void k_env<1, false>(EnvParams, StepOut);
template __global__ void k_env<1, true>(EnvParams, StepOut);
template __global__ void k_env<2, false>(EnvParams, StepOut);
template __global__ void k_env<2, true>(EnvParams, StepOut);
template __global__ void k_env<4, false>(EnvParams, StepOut);
template __global__ void k_env<4, true>(EnvParams, StepOut);
template __global__ void k_env<8, false>(EnvParams, StepOut);
template __global__ void k_env<8, true>(EnvParams, StepOut);
template __global__ void k_env<16, false>(EnvParams, StepOut);
template __global__ void k_env<16, true>(EnvParams, StepOut);

// ------------------------------------------------------------- reset -----
// VmEnv.reset (env.py:180-226) for masked envs, one wave per env.
__global__ __launch_bounds__(256) void k_reset(EnvParams p, const int64_t *seeds,
                                               const uint8_t *env_mask, float *obs) {
  const int lane = lane_id();
  const int e = uni(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
  if (e >= p.N) return;
  if (env_mask && !env_mask[e]) return;
  EnvHdr *h = p.hdr + e;
  const int V = p.V, P = p.P;
  if (lane < 4) {
    Pcg r;
    if (seeds) {
      pcg_seed(r, (uint64_t)(seeds[e] + lane));  // seed() env.py:172-178
    } else {
      r.s = U128{h->rng[lane][0], h->rng[lane][1]};
      r.inc = U128{h->rng[lane][2], h->rng[lane][3]};
      if (lane < 2) {  // sequences restart 2M draws after the last reset
        r.s = U128{h->seqbase[lane][0], h->seqbase[lane][1]};
        pcg_advance(r, (uint64_t)p.M2);
      }
    }
    h->rng[lane][0] = r.s.hi;
    h->rng[lane][1] = r.s.lo;
    h->rng[lane][2] = r.inc.hi;
    h->rng[lane][3] = r.inc.lo;
    if (lane < 2) {
      h->seqbase[lane][0] = r.s.hi;
      h->seqbase[lane][1] = r.s.lo;
    }
  }
  if (lane >= 20 && lane < 32) {
    reinterpret_cast<uint64_t *>(h)[lane] = (lane == 20) ? 1ull : 0ull;  // timestep = 1
  }
  uint32_t *vw = p.vmw + (int64_t)e * vm_pitch(V);
  for (int v = lane; v < V; v += 64) {
    vw[vm_slot_idx(v)] = (uint32_t)(P + 1);
    vw[vm_time_idx(v)] = 0u;
  }
  for (int i = lane; i < 2 * P; i += 64) p.pm[(int64_t)e * 2 * P + i] = 0.0;
  if (obs) {
    float *o = obs + (int64_t)e * p.D;
    for (int i = lane; i < p.D; i += 64) o[i] = i < V ? (float)(P + 1) : 0.0f;
  }
}

// ------------------------------------------------------- state export ----
__global__ void k_export(EnvParams p, int64_t *placement, double *vm_cpu, double *vm_mem,
                         double *cpu, double *mem, int64_t *remaining, int64_t *rank) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t nv = (int64_t)p.N * p.V;
  if (i < nv) {
    const uint32_t *vw = p.vmw + (i / p.V) * vm_pitch(p.V);
    const int v = (int)(i % p.V);
    const uint64_t w = (uint64_t)vw[vm_slot_idx(v)] | ((uint64_t)vw[vm_time_idx(v)] << 32);
    if (placement) placement[i] = (int64_t)(w & 0xFFFF);
    if (vm_cpu) vm_cpu[i] = (double)((w >> 16) & 0xFF) / 100.0;
    if (vm_mem) vm_mem[i] = (double)((w >> 24) & 0xFF) / 100.0;
    if (remaining) {  // running VMs hold their finish key F = timestep + remaining
      const int64_t hi = (int64_t)(w >> 32);
      remaining[i] = (int)(w & 0xFFFF) < p.P ? (int64_t)(uint32_t)((uint32_t)hi - (uint32_t)p.hdr[i / p.V].timestep) : hi;
    }
  }
  int64_t np_ = (int64_t)p.N * p.P;
  if (i < np_) {
    int64_t e = i / p.P, q = i % p.P;
    if (cpu) cpu[i] = p.pm[e * 2 * p.P + q];
    if (mem) mem[i] = p.pm[e * 2 * p.P + p.P + q];
  }
  if (rank && i < p.N) {  // _get_rank (env.py:320-325): distinct PMs hosting a VM
    int64_t r = 0;
    const uint32_t *row = p.vmw + i * vm_pitch(p.V);
    for (int q = 0; q < p.P; q++) {
      bool used = false;
      for (int v = 0; v < p.V && !used; v++) used = (int)(row[vm_slot_idx(v)] & 0xFFFF) == q;
      r += used;
    }
    rank[i] = r;
  }
}

// target_cpu_mean / target_memory_mean (env.py:116-121) from the stored state,
// one wave per env. Both are pure functions of the post-step state (existing =
// placement <= WAIT, their sizes in index order), so deriving them here gives
// the values step() would have left, through the same pairwise order; the step
// kernel itself computes them only for the kl reward. vmp_get_stats runs this
// before k_counters.
__global__ __launch_bounds__(256) void k_target_means(EnvParams p) {
  __shared__ uint8_t comp[kWavesPerBlock][2][kMaxVPT * 64];
  __shared__ double cent[128];
  for (int i = threadIdx.x; i < 128; i += blockDim.x) cent[i] = (double)i / 100.0;
  __syncthreads();
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  const int e = uni(blockIdx.x * kWavesPerBlock + wid);
  if (e >= p.N) return;
  const int V = p.V, P = p.P;
  const uint32_t *row = p.vmw + (int64_t)e * vm_pitch(V);
  uint8_t *cc = comp[wid][0], *cm = comp[wid][1];
  int n_ex = 0;
  for (int b = 0; b < V; b += 64) {
    const int v = b + lane;
    const uint32_t w = v < V ? row[vm_slot_idx(v)] : (uint32_t)(P + 1);
    const bool ex = v < V && (int)(w & 0xFFFFu) <= P;
    const uint64_t m = ballot(ex);
    if (ex) {
      const int rk = n_ex + below(m, lane);
      cc[rk] = (uint8_t)((w >> 16) & 0xFFu);
      cm[rk] = (uint8_t)((w >> 24) & 0xFFu);
    }
    n_ex += __popcll(m);
  }
  wsync();
  const PwLds none{};  // n <= 1024: the register plan, no LDS plan needed
  const double *ct = cent;
  const double sc = wave_pw_sum(n_ex, [=](int i) { return ct[cc[i]]; }, none);
  const double sm = wave_pw_sum(n_ex, [=](int i) { return ct[cm[i]]; }, none);
  if (lane == 0) {
    double tcm = sc / (double)P, tmm = sm / (double)P;
    if (p.cap_target_util && tcm > 1) tcm = 1.0;
    if (p.cap_target_util && tmm > 1) tmm = 1.0;
    p.hdr[e].tcm = tcm;
    p.hdr[e].tmm = tmm;
  }
}

__global__ void k_counters(EnvParams p, int64_t *ctr, double *st) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.N) return;
  const EnvHdr *h = p.hdr + e;
  if (ctr) {
    int64_t *c = ctr + (int64_t)e * 6;
    c[0] = h->total_requests;
    c[1] = h->served;
    c[2] = h->suspend_action;
    c[3] = h->place_action;
    c[4] = h->dropped;
    c[5] = h->timestep;
  }
  if (st) {
    double *s = st + (int64_t)e * 5;
    s[0] = h->waiting_ratio;
    s[1] = h->tcm;
    s[2] = h->tmm;
    s[3] = h->total_cpu_req;
    s[4] = h->total_mem_req;
  }
}

__global__ void k_mask_bool(int64_t rows, int A, int W, const uint32_t *bits, uint8_t *mask) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * A) return;
  int64_t r = i / A;
  int a = (int)(i % A);
  mask[i] = (bits[r * W + (a >> 5)] >> (a & 31)) & 1u;
}


// ------------------------------------------------------- large-V env kernel
// V > 1024 (e.g. the P1000 / V10000 stress config): one workgroup of NT =
// 64 * NWV threads per env. Thread t owns VM slots v = s*NT + t (s < SPT), so
// slot order (s, t) is ascending VM order. The VM words live in LDS (W[v]),
// the remaining service times in registers (rem[s], only touched by fully
// unrolled loops, so they stay statically indexed: a dynamically indexed
// register array would live in scratch, which at 512 threads x 500 B per CU
// misses L2). PM-level work (fit bitmaps, BF sort, placements, frees, RNG
// draws, pairwise sums, reward) runs on wave 0 with the wave kernel's helpers;
// per-VM events that the reference applies in VM order are ranked across the
// block (row_counts + slot_rank: one barrier pair for all SPT slot rows) and
// applied by wave 0 in that order. Same arithmetic, same
// order as k_env: the two kernels are interchangeable (VMP_BIG_KERNEL=1
// forces this one for any V, which the parity tests use).
// Slot-row loops of the block kernel (s = 0..SPT-1), unrolled by 4: 4 LDS
// reads in flight per round trip (a full unroll hoists enough per-slot
// temporaries to grow the scratch from 496 to 3296 B per lane at SPT = 20;
// one row per iteration costs one LDS round trip per row).
#define VMP_SLOOP _Pragma("unroll 4")

// k_env_big's workgroup: 6 waves (two workgroups per CU at 3 waves/SIMD); a
// compile-time thread count so slot s of a thread sits at a constant LDS
// offset s * kBigNT * 4 (immediate ds offsets, no per-slot address registers).
// Up to kBigMaxSPT slots per thread (V <= kBigNT * kBigMaxSPT).
#ifndef VMP_BIG_NT
#define VMP_BIG_NT 256
#endif
constexpr int kBigNT = VMP_BIG_NT;
// per-thread slot sets (bit s: slot s * kBigNT + t)
typedef uint64_t SMask;
#define SBIT(s) ((SMask)1 << (s))
constexpr int kBigMaxSPT = (10240 + kBigNT - 1) / kBigNT, kBigMaxWaves = kBigNT / 64;
static_assert(kBigNT % 64 == 0 && kBigNT <= 512 && kBigMaxSPT <= 64, "block shape");
// k_env_big's per-step helpers (pairwise-sum jobs, reward, draws): inlined
// (round 3: out of line, every call saved and restored the caller's live
// registers through scratch, 224 B per lane; inlined the kernel needs 193
// VGPRs instead of 250 and runs 8 % faster with the 4-row slot loops)
#define VMP_BIG_CALL __forceinline__
struct BigShared {
  int32_t wcnt[16];   // per-wave counts of a compaction
  int32_t bc[8];      // broadcast scalars
  int64_t b64[4];
  int32_t rc[kBigMaxSPT * kBigMaxWaves];  // per slot row, per wave flag counts (row_counts)
  int32_t rtot[kBigMaxWaves];             // per wave flag totals
  double half[20];    // big_sum_phase: the two halves of a split job j at 2j, 2j + 1
  uint32_t fmax[kBigMaxWaves][128];  // big_heuristic: any-fit table per PM chunk
  int32_t wmin[kBigMaxWaves];         // block_min_1b
  int32_t klflag[2];                  // big_kl_sums: means of jobs 2 / 3 published
};

// Rank of this thread's flag among the flagged threads of the block
// (ascending t) and the block total. Two barriers.
__device__ __forceinline__ int bcx_rank(bool flag, BigShared &B, int &total) {
  const int lane = lane_id(), wid = threadIdx.x >> 6, nwv = kBigNT >> 6;
  const uint64_t m = ballot(flag);
  __syncthreads();
  if (lane == 0) B.wcnt[wid] = __popcll(m);
  __syncthreads();
  int off = 0, tot = 0;
  for (int i = 0; i < nwv; i++) {
    const int c = B.wcnt[i];
    off += i < wid ? c : 0;
    tot += c;
  }
  total = tot;
  return off + below(m, lane);
}

// Flag counts of all SPT slot rows at once (bit s of fl = slot s*NT + t):
// B.rc[s][wave] and the block total. Two barriers for all rows.
// With xsum: *xsum (a per-thread int) is summed over the block on the same
// two barriers.
template <int SPT>
__device__ __forceinline__ int row_counts(SMask fl, BigShared &B, int *xsum = nullptr) {
  const int lane = lane_id(), wid = threadIdx.x >> 6, nwv = kBigNT >> 6;
  int x = 0;
  if (xsum) {
    x = *xsum;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  }
  __syncthreads();
  int wt = 0;
#pragma unroll
  for (int s = 0; s < SPT; s++) {
    const int c = __popcll(ballot((fl >> s) & 1u));
    wt += c;
    if (lane == 0) B.rc[s * kBigMaxWaves + wid] = c;
  }
  if (lane == 0) {
    B.rtot[wid] = wt;
    if (xsum) B.wcnt[wid] = x;
  }
  __syncthreads();
  int tot = 0, xt = 0;
  for (int i = 0; i < nwv; i++) {
    tot += B.rtot[i];
    if (xsum) xt += B.wcnt[i];
  }
  if (xsum) *xsum = xt;
  return tot;
}

// Rank (ascending VM order) of slot row s of this thread in the flag set
// counted by row_counts; `base` carries the flags of rows < s (start at 0 and
// call for s = 0, 1, ... in order). Valid for flagged slots only.
__device__ __forceinline__ int slot_rank(SMask fl, int s, const BigShared &B, int &base) {
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  const uint64_t m = ballot((fl >> s) & 1u);
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBigMaxWaves; w++) {  // rows of absent waves stay 0
    const int c = B.rc[s * kBigMaxWaves + w];
    pre += w < wid ? c : 0;
    tot += c;
  }
  const int r = base + pre + below(m, lane);
  base += tot;
  return r;
}

// After row_counts: the block rank (VM order) of this wave's first flagged
// slot of row s, in lane s (s < SPT), and in `rowbase` the rank of row s's
// first flagged slot. One set of LDS reads per wave and a lane scan, instead
// of eight LDS reads per row in slot_rank; then the rank of a flagged slot in
// row s is readlane(result, s) + its position among the wave's flags.
template <int SPT>
__device__ __forceinline__ int row_prefix(const BigShared &B, int &rowbase) {
  static_assert(SPT <= 64, "one lane per slot row");
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  int tot = 0, mine = 0;
  if (lane < SPT) {
#pragma unroll
    for (int w = 0; w < kBigMaxWaves; w++) {  // rows of absent waves stay 0
      const int c = B.rc[lane * kBigMaxWaves + w];
      tot += c;
      mine += w < wid ? c : 0;
    }
  }
  int incl = tot;
#pragma unroll
  for (int o = 1; o < (SPT > 32 ? 64 : 32); o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  rowbase = incl - tot;
  return rowbase + mine;
}

__device__ __forceinline__ int block_sum_int(int x, BigShared &B) {
  const int lane = lane_id(), wid = threadIdx.x >> 6, nwv = kBigNT >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  __syncthreads();
  if (lane == 0) B.wcnt[wid] = x;
  __syncthreads();
  int s = 0;
  for (int i = 0; i < nwv; i++) s += B.wcnt[i];
  return s;
}

__device__ __forceinline__ int block_min_int(int x, BigShared &B) {
  const int lane = lane_id(), wid = threadIdx.x >> 6, nwv = kBigNT >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o));
  __syncthreads();
  if (lane == 0) B.wcnt[wid] = x;
  __syncthreads();
  int s = 0x7fffffff;
  for (int i = 0; i < nwv; i++) s = min(s, B.wcnt[i]);
  return s;
}

// Block-wide min with ONE barrier. Precondition: another block barrier lies
// between two calls (the resolve loop's choose barrier), so no wave can
// overwrite B.wmin while another still reads the previous call's values.
__device__ __forceinline__ int block_min_1b(int x, BigShared &B) {
  const int lane = lane_id(), wid = threadIdx.x >> 6, nwv = kBigNT >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o));
  if (lane == 0) B.wmin[wid] = x;
  __syncthreads();
  int s = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < nwv; i++) s = min(s, B.wmin[i]);
  return s;
}

// PM chunk c of the block (one per wave): PMs [c*CP, min((c+1)*CP, P)).
__device__ __forceinline__ int big_chunk_len(int P) { return (P + kBigMaxWaves - 1) / kBigMaxWaves; }

// The any-fit table of PM chunk c (build_fitmax over that chunk's PMs), built
// by the calling wave alone: the table of the whole env is the max over the
// chunks' tables, and a placement changes one PM, so only its chunk is rebuilt.
template <class MT>  // uint32_t * into the block's static LDS (BigShared)
__device__ __forceinline__ void big_build_chunk(const Lds &L, MT *M, int lo, int hi) {
  const int lane = lane_id();
  M[lane] = 0;
  M[lane + 64] = 0;
  wsync();
  for (int q = lo + lane; q < hi; q += 64) {
    const int tcq = (int)L.tc[q];
    if (tcq > 0) __atomic_fetch_max(&M[tcq - 1], (uint32_t)L.tm[q], __ATOMIC_RELAXED);
  }
  wsync();
  const int rlo = 63 - lane, rhi = 127 - lane;
  const bool hi_ok = rhi <= 100;
  uint32_t c1 = hi_ok ? M[rhi] : 0u, c0 = M[rlo];
  c1 = prefix_max32(c1);
  c0 = max(prefix_max32(c0), (uint32_t)__builtin_amdgcn_readlane((int)c1, 63));
  wsync();
  M[rlo] = c0;
  if (hi_ok) M[rhi] = c1;
  wsync();
}

// Does some PM accept sizes (c, m): the max over the chunk tables.
__device__ __forceinline__ bool big_anyfit(const BigShared &B, int c, int m) {
  uint32_t x = B.fmax[0][c];
#pragma unroll
  for (int i = 1; i < kBigMaxWaves; i++) x = max(x, B.fmax[i][c]);
  return x > (uint32_t)m;
}

// Wave 0's choice for sizes (kc, km): FirstFit's first fitting PM in index
// order (firstfit.py:33-37) or BestFit's fitting PM of largest f32 key
// (bestfit.py:33-39, ties by numpy's introsort in bf_choose). Lane l scans the
// 16 consecutive PMs [b + 16l, b + 16l + 16) of each 1024-PM block b with
// vector LDS reads (thresholds 16 B, f32 view 4 x 16 B per row), so a scan is
// one round trip per block instead of one per 64 PMs. -1 if nothing fits.
__device__ __forceinline__ int big_choose(const EnvParams &p, const Lds &L, bool bf, int kc, int km) {
  const int lane = lane_id();
  const int P = p.P;
  float best = -INFINITY;
  int cnt = 0, bi = -1, first = 0x7fffffff;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 kfc[4], kfm[4];  // the last block's f32 view (the tie count reads it for P <= 1024)
  for (int b = 0; b < P; b += 1024) {
    const int q0 = b + 16 * lane;
    const u32x4 tcw = *reinterpret_cast<const u32x4 LDSP *>(L.tc + q0);
    const u32x4 tmw = *reinterpret_cast<const u32x4 LDSP *>(L.tm + q0);
    f32x4 fc[4], fm[4];
    if (bf) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        fc[j] = *reinterpret_cast<const f32x4 LDSP *>(L.fcpu + q0 + 4 * j);
        fm[j] = *reinterpret_cast<const f32x4 LDSP *>(L.fmem + q0 + 4 * j);
        kfc[j] = fc[j];
        kfm[j] = fm[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int q = q0 + j;
      const int tcq = (int)((tcw[j >> 2] >> (8 * (j & 3))) & 0xFFu) - 1;
      const int tmq = (int)((tmw[j >> 2] >> (8 * (j & 3))) & 0xFFu) - 1;
      if (q < P && tcq >= kc && tmq >= km) {
        first = min(first, q);
        if (bf) {
          const float key = fc[j >> 2][j & 3] + fm[j >> 2][j & 3];  // the f32 sum bestfit.py sorts
          if (key > best) {
            best = key;
            cnt = 1;
            bi = q;
          } else if (key == best) {
            cnt++;
          }
        }
      }
    }
    if (!bf) {  // FirstFit: the first block with a fit decides
      const uint64_t f = ballot(first != 0x7fffffff);
      if (f) return __builtin_amdgcn_readlane(first, __ffsll((unsigned long long)f) - 1);
    }
  }
  if (!bf) return -1;
  float m = best;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  int tot = (best == m) ? cnt : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
  if (tot == 0) return -1;
  if (tot == 1) {
    const uint64_t who = ballot(best == m && cnt == 1);
    return __builtin_amdgcn_readlane(bi, __ffsll((unsigned long long)who) - 1);
  }
#ifdef VMP_WGTIME
  if (threadIdx.x == 0) wg_marks[23] += 1;  // tie count (timing build)
#endif
  if (P > 1024) return bf_choose(p, L, kc, km);  // tied top keys: numpy's order decides
  // one block: every key is still in this lane's registers
  int above = 0, eq = 0;
  {
    const int q0 = 16 * lane;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const float key = kfc[j >> 2][j & 3] + kfm[j >> 2][j & 3];
      above += (q0 + j < P) && key > m;
      eq += (q0 + j < P) && key == m;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    above += __shfl_xor(above, o);
    eq += __shfl_xor(eq, o);
  }
  return bf_tie(p, L, kc, km, above, eq);
}

// FirstFit / BestFit act fused with the action phase (heuristic_apply, block form).
// Per step: each wave builds the f32 view, thresholds and any-fit table of its
// PM chunk (no barrier until all are built), the pending VMs' hits are read
// from the chunk tables, and each placement costs two block barriers: the
// earliest winner (block_min_1b) and wave 0's choose + place + rebuild of the
// placed PM's chunk table.
template <int SPT>
__device__ __forceinline__ int64_t big_heuristic(const EnvParams &p, const Lds &L, const Tables &T,
                                                 BigShared &B, uint32_t LDSP *W, int policy,
                                                 int32_t *act_out, uint8_t *valid_out STAMP_PARAMS) {
  const int t = threadIdx.x, NT = kBigNT, lane = lane_id(), wid = t >> 6;
  const bool w0 = t < 64;
  const int P = p.P, WAIT = p.P;
  const bool bf = policy == 1;
  SMask pend = 0;
VMP_SLOOP
  for (int s = 0; s < SPT; s++)
    if (w_pl(W[s * NT + t]) == WAIT) pend |= SBIT(s);
  SMask won = 0, bad = 0;
  int64_t n_place = 0;
  const int CP = big_chunk_len(P);
  {  // this wave's PM chunk: f32 view, thresholds, any-fit table
    const int lo = wid * CP, hi = min(P, lo + CP);
    for (int i = lo + lane; i < hi; i += 64) {
      const float fcv = (float)L.cpu[i], fmv = (float)L.mem[i];
      L.fcpu[i] = fcv;
      L.fmem[i] = fmv;
      L.tc[i] = (uint8_t)(fit_threshold(fcv) + 1);
      L.tm[i] = (uint8_t)(fit_threshold(fmv) + 1);
    }
    wsync();
    big_build_chunk(L, B.fmax[wid], lo, hi);
  }
  __syncthreads();
  STAMP(22);
  SMask hit = 0;
  for (SMask r = pend; r; r &= r - 1) {
    const int s = __builtin_ctzll(r);
    const uint32_t w = W[s * NT + t];
    if (big_anyfit(B, w_cc(w), w_cm(w))) hit |= SBIT(s);
  }
  STAMP(17);
#pragma unroll 1
  for (;;) {
    // earliest VM (index order) with a fit: this thread's lowest hit slot
    const int mine = hit ? __builtin_ctzll(hit) * NT + t : 0x7fffffff;
    const int vw = block_min_1b(mine, B);
    if (vw == 0x7fffffff) break;
    {  // VMs before the winner never fit again (PM loads only grow)
      const int sm = vw >= t ? (vw - t) / NT : -1;  // slots s <= sm have s*NT + t <= vw
      if (sm >= 0) pend &= sm >= 63 ? (SMask)0 : ~(SBIT(sm + 1) - 1);
    }
    hit &= pend;
    const int ws = vw / NT, wt = vw - ws * NT;
    const uint32_t ww = W[vw];
    const int kc = w_cc(ww), km = w_cm(ww);
    STAMP(18);
    if (w0) {
      const int q = big_choose(p, L, bf, kc, km);
      const bool ok = env_place(L, T, P, q, kc, km);
      const int tc_old = (int)L.tc[q] - 1, tm_old = (int)L.tm[q] - 1;
      const float nc = L.fcpu[q] + T.fcent[kc];
      const float nm = bf ? L.fmem[q] + T.fcent[km] : L.fmem[q];
      const int tc_new = fit_threshold(nc), tm_new = bf ? fit_threshold(nm) : tm_old;
      wsync();
      if (lane == 0) {
        L.fcpu[q] = nc;
        L.tc[q] = (uint8_t)(tc_new + 1);
        if (bf) {
          L.fmem[q] = nm;
          L.tm[q] = (uint8_t)(tm_new + 1);
        }
        B.bc[1] = q;
        B.bc[2] = ok;
        B.bc[3] = tc_old;
        B.bc[4] = tc_new;
        B.bc[5] = tm_new;
        B.bc[7] = tm_old;
      }
      wsync();
      if (tc_new != tc_old || tm_new != tm_old) {  // q's chunk table
        const int c = q / CP;
        big_build_chunk(L, B.fmax[c], c * CP, min(P, c * CP + CP));
      }
    }
    __syncthreads();
    STAMP(19);
    const int q = B.bc[1];
    const bool ok = B.bc[2] != 0;
    n_place += ok;
    if (t == wt) {
      won |= SBIT(ws);
      if (ok) W[vw] = (ww & 0xFFFF0000u) | (uint32_t)q;
      else bad |= SBIT(ws);
      if (act_out) act_out[vw] = q;
    }
    {  // re-query the VMs q fitted before and not after
      const int tq = B.bc[4], tc_old = B.bc[3], tmq = B.bc[5], tm_old = B.bc[7];
      if (tq != tc_old || tmq != tm_old)
        for (SMask r = hit; r; r &= r - 1) {
          const int s = __builtin_ctzll(r);
          const uint32_t w = W[s * NT + t];
          const int c = w_cc(w), m = w_cm(w);
          if (c <= tc_old && m <= tm_old && !(c <= tq && m <= tmq) && !big_anyfit(B, c, m))
            hit &= ~SBIT(s);
        }
    }
  }
  if (act_out || valid_out) {
VMP_SLOOP
    for (int s = 0; s < SPT; s++) {
      const int v = s * NT + t;
      const uint32_t w = W[v];
      if (live(w)) {
        if (act_out && !((won >> s) & 1u)) act_out[v] = (int32_t)w_pl(w);
        if (valid_out) valid_out[v] = (uint8_t)!((bad >> s) & 1u);
      }
    }
  }
  __syncthreads();
  return n_place;
}

// External actions (external_apply, block form): per slot row s, the events
// are compacted in ascending VM order and applied by wave 0 one by one.
template <int SPT>
__device__ __forceinline__ void big_external(const EnvParams &p, const Lds &L, const Tables &T,
                                             BigShared &B, uint32_t LDSP *W,
                                             const int32_t *act_row, uint8_t *valid_out,
                                             int64_t &n_place, int64_t &n_susp) {
  const int t = threadIdx.x, NT = kBigNT, lane = lane_id();
  const int P = p.P, WAIT = p.P;
#pragma unroll 1
  for (int s = 0; s < SPT; s++) {
    const int v = s * NT + t;
    const uint32_t wv = W[v];
    const bool in = live(wv);
    const int c = w_pl(wv);
    const int tg = in ? act_row[v] : c;
    const bool isplace = in && c == WAIT && tg >= 0 && tg < P;
    const bool issusp = in && c < P && tg == WAIT;
    int nev = 0;
    const int r = bcx_rank(isplace || issusp, B, nev);
    if (isplace || issusp) {
      L.evw[r] = wv;
      L.evt[r] = tg;
    }
    __syncthreads();
    if (t < 64) {
#pragma unroll 1
      for (int i = 0; i < nev; i++) {  // ascending VM index
        const uint32_t ew = L.evw[i];
        const int et = L.evt[i];
        const int ec = w_pl(ew);
        const double vc = T.cent[w_cc(ew)], vm = T.cent[w_cm(ew)];
        const int q = (ec == WAIT) ? et : ec;
        double cq = L.cpu[q], mq = L.mem[q];
        bool eok = true;
        if (ec == WAIT) {
          eok = (cq + vc <= 1) && (mq + vm <= 1);
          if (eok) {
            cq = cq + vc;
            mq = mq + vm;
          }
        } else {
          cq = cq - vc;
          mq = mq - vm;
        }
        wsync();
        if (lane == 0) {
          L.cpu[q] = cq;
          L.mem[q] = mq;
          mark_pm(L, P, q);
          L.evok[i] = (uint8_t)eok;
        }
        wsync();
      }
    }
    __syncthreads();
    bool ok = (tg == c) || issusp;
    if (isplace) ok = L.evok[r] != 0;
    n_place += block_sum_int(isplace && ok, B);
    n_susp += block_sum_int(issusp, B);
    if (ok && tg != c && in) W[v] = (wv & 0xFFFF0000u) | (uint32_t)tg;
    if (valid_out && in) valid_out[v] = (uint8_t)ok;
  }
}

// The step's pairwise sums in k_env_big (env_tail's stats section, block
// form): job j computes res[j] with the numbers of env_tail (0,1 accepted
// sizes; 2,3 existing VM sizes; 4,5 PM cpu / memory; 6,7 PM squared
// deviations; 8,9 VM-size squared deviations), each by one whole wave in
// numpy's pairwise order. Out of line so its temporaries do not share the
// register budget with the block's slot arrays.
#ifndef VMP_BIG_PW_DEPTH
#define VMP_BIG_PW_DEPTH 6
#endif
#ifndef VMP_BIG_SPLIT_A
#define VMP_BIG_SPLIT_A 0
#endif
constexpr int kBigPwDepth = VMP_BIG_PW_DEPTH;  // register plan up to n = 7688 (6), 1928 (4)
constexpr bool kBigSplitA = VMP_BIG_SPLIT_A;   // split phase A's long sums too
// Job j over elements [o, o + m) of its source (the whole job: o = 0, m = n),
// result to *dst.
// spill: bit 0 the accepted sizes (jobs 0, 1), bit 1 the existing-VM sizes
// (jobs 2, 3, 8, 9) are in the env's HBM spill instead of LDS.
__device__ VMP_BIG_CALL void big_sum_job(const EnvParams &p, const Tables &T, char LDSP *base,
                                         int j, int n_ex, int o, int m, double LDSP *dst,
                                         uint32_t spill) {
  const Lds L = make_lds(p, base);
  const int P = p.P;
  double LDSP *res = L.jobres;
  const double *cent = T.cent;
  // job j's u8 source in the spill: accc | accm | ccomp | mcomp, V bytes each
  const int part = j < 2 ? j : 2 + (j & 1);
  const bool g = (spill >> (j < 2 ? 0 : 1)) & 1u;
  const uint8_t GLBP *gsrc = gptr(p.bigscr) + ((int64_t)blockIdx.x * 4 + part) * p.V + o;
  double r;
  if (j < 4) {
    const uint8_t LDSP *src = ((j == 0) ? L.accc : (j == 1) ? L.accm : ((j & 1) ? L.mcomp : L.ccomp)) + o;
    if (g) r = wave_pw_sum<kBigPwDepth>(m, [=](int i) { return cent[gsrc[i]]; }, L.pw);
    else r = wave_pw_sum<kBigPwDepth>(m, [=](int i) { return cent[src[i]]; }, L.pw);
  } else if (j < 8) {
    const double LDSP *src = ((j & 1) ? L.mem : L.cpu) + o;
    const double mean = j < 6 ? 0.0 : res[j - 2] / (double)P;
    const bool sq = j >= 6;
    r = wave_pw_sum<kBigPwDepth>(m, [=](int i) {
      const double x = src[i];
      const double d = x - mean;
      return sq ? d * d : x;
    }, L.pw);
  } else {
    const uint8_t LDSP *src = ((j & 1) ? L.mcomp : L.ccomp) + o;
    const double mean = res[j - 6] / (double)n_ex;
    if (g)
      r = wave_pw_sum<kBigPwDepth>(m, [=](int i) {
        const double d = cent[gsrc[i]] - mean;
        return d * d;
      }, L.pw);
    else
      r = wave_pw_sum<kBigPwDepth>(m, [=](int i) {
        const double d = cent[src[i]] - mean;
        return d * d;
      }, L.pw);
  }
  wsync();
  if (lane_id() == 0) *dst = r;
  wsync();
}

// The jobs of bit set `jobs` spread over the block's waves (all threads call
// it; returns after a barrier). A sum past the register plan uses the LDS
// plan, of which the carve holds one copy: those run on wave 0 in turn.
// halves: a job with n > kBigSplitMin runs as numpy's top-level split, pairwise(n) =
// pairwise(n2) + pairwise(n - n2) with n2 = n/2 - (n/2) % 8, the two halves on
// two waves and their sum formed by wave 0 after the barrier (so only wave 0
// may read those results).
__device__ __forceinline__ int big_sum_n(const EnvParams &p, int j, int k, int n_ex) {
  return j < 2 ? k : (j >= 4 && j < 8) ? p.P : n_ex;
}
// Number of wave tasks big_sum_phase deals for `jobs`.
// A job is split only when its halves save a pass: one wave sums 8 leaves of
// <= 128 elements per pass (8-lane groups), so n <= 1024 takes one pass whole.
#ifndef VMP_BIG_SPLIT_MIN
#define VMP_BIG_SPLIT_MIN 1024
#endif
constexpr int kBigSplitMin = VMP_BIG_SPLIT_MIN;
__device__ __forceinline__ int big_sum_ntask(const EnvParams &p, uint32_t jobs, int k, int n_ex,
                                             bool halves) {
  int n = 0;
  for (; jobs; jobs &= jobs - 1) n += (halves && big_sum_n(p, __builtin_ctz(jobs), k, n_ex) > kBigSplitMin) ? 2 : 1;
  return n;
}
// block_combine: the split results are formed before a block barrier (every
// wave may read them), else by wave 0 alone after it.
__device__ __forceinline__ void big_sum_phase(const EnvParams &p, const Tables &T, char LDSP *base,
                                              BigShared &B, uint32_t jobs, int k, int n_ex,
                                              bool halves, bool block_combine, uint32_t spill) {
  const int wid = threadIdx.x >> 6, nwv = kBigNT >> 6;
  double LDSP *res = reinterpret_cast<double LDSP *>(base + p.off_stage);  // L.jobres
  int slot = 0;
  uint32_t split = 0;
#pragma unroll 1
  while (jobs) {
    const int j = __builtin_ctz(jobs);
    jobs &= jobs - 1;
    const int n = big_sum_n(p, j, k, n_ex);
    const bool two = halves && n > kBigSplitMin;
    const int n2 = (n / 2) - (n / 2) % 8;
#pragma unroll 1
    for (int h = 0; h < (two ? 2 : 1); h++) {
      const int o = two && h ? n2 : 0, m = two ? (h ? n - n2 : n2) : n;
      const int w = m > pw_reg_cap(kBigPwDepth) ? 0 : (slot++ % nwv);
      double LDSP *dst = two ? (double LDSP *)&B.half[2 * j + h] : res + j;
      if (w == wid) big_sum_job(p, T, base, j, n_ex, o, m, dst, spill);
    }
    if (two) split |= 1u << j;
  }
#ifdef VMP_WGTIME
  STAMP(block_combine ? 18 : 19);  // wave 0: its sum tasks of phase A / B done
#endif
  __syncthreads();
  if (split && wid == 0) {
    if (lane_id() == 0)
      for (uint32_t s = split; s; s &= s - 1) {
        const int j = __builtin_ctz(s);
        res[j] = B.half[2 * j] + B.half[2 * j + 1];
      }
    wsync();
  }
  if (split && block_combine) __syncthreads();
}

// kl's ten sums on the block's four waves with no barrier between a plain sum
// and the squared deviations that need its mean: each wave runs the chain
// whose mean it computes itself (PM sums 4 -> 6 on wave 0, 5 -> 7 on wave 1,
// existing-VM sums 2 -> 8 on wave 2, 3 -> 9 on wave 3; the accepted sizes 0 /
// 1 on waves 0 / 1), and a VM-size job past one pass (n_ex > kBigSplitMin) is
// split at numpy's top level with its second half on wave 0 / 1 once wave 2 /
// 3 has published the mean (LDS flag). Same jobs, same order of additions as
// big_sum_phase: three passes on the longest wave instead of four.
__device__ __forceinline__ void big_kl_sums(const EnvParams &p, const Tables &T, char LDSP *base,
                                            BigShared &B, int k, int n_ex, uint32_t spill,
                                            int mark) {
  const int wid = threadIdx.x >> 6, lane = lane_id();
  double LDSP *res = reinterpret_cast<double LDSP *>(base + p.off_stage);  // L.jobres
  const bool split = n_ex > kBigSplitMin;
  const int n2 = (n_ex / 2) - (n_ex / 2) % 8;
  if (wid <= 1) {
    const int j = wid;  // 0 / 1: accepted sizes, then PM sums 4 / 5 and their squares 6 / 7
    if (k > 0) big_sum_job(p, T, base, j, n_ex, 0, k, res + j, spill);
    big_sum_job(p, T, base, 4 + j, n_ex, 0, p.P, res + 4 + j, spill);
    big_sum_job(p, T, base, 6 + j, n_ex, 0, p.P, res + 6 + j, spill);
    if (split) {
      while (__hip_atomic_load(&B.klflag[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != mark)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      big_sum_job(p, T, base, 8 + j, n_ex, n2, n_ex - n2, (double LDSP *)&B.half[2 * (8 + j) + 1],
                  spill);
    }
  } else if (wid <= 3) {
    const int j = wid - 2;  // existing-VM sums 2 / 3, then their squared deviations 8 / 9
    big_sum_job(p, T, base, 2 + j, n_ex, 0, n_ex, res + 2 + j, spill);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(&B.klflag[j], mark, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (split)
      big_sum_job(p, T, base, 8 + j, n_ex, 0, n2, (double LDSP *)&B.half[2 * (8 + j)], spill);
    else
      big_sum_job(p, T, base, 8 + j, n_ex, 0, n_ex, res + 8 + j, spill);
  }
  __syncthreads();
  if (split && wid == 0) {
    if (lane == 0) {
      res[8] = B.half[16] + B.half[17];
      res[9] = B.half[18] + B.half[19];
    }
    wsync();
  }
}

// Wave 0 of k_env_big after the sums: reward, counters and termination.
__device__ VMP_BIG_CALL void big_stats_final(const EnvParams &p, BigShared &B, char LDSP *base,
                                             int64_t k, int n_ex, int n_w, int64_t n_term,
                                             int64_t arrivals) {
  const Lds L = make_lds(p, base);
  const int lane = lane_id();
  const int P = p.P;
  const bool kl = p.reward == 2;
  EnvHdr LDSP *H = L.hdr;
  double LDSP *res = L.jobres;
  double reward = 0.0;
  const double wr = n_ex > 0 ? (double)n_w / (double)n_ex : 0.0;
  const double r2 = kl ? res[2] : 0.0, r3 = kl ? res[3] : 0.0;
  double tcm = r2 / (double)P;
  if (p.cap_target_util && tcm > 1) tcm = 1.0;
  double tmm = r3 / (double)P;
  if (p.cap_target_util && tmm > 1) tmm = 1.0;
  if (n_ex > 0) {
    if (p.reward == 2) {
      double cv = res[6] / (double)P, mv = res[7] / (double)P;
      if (cv == 0) cv = 1e-6;
      if (mv == 0) mv = 1e-6;
      double tcv = res[8] / (double)n_ex, tmv = res[9] / (double)n_ex;
      if (tcv == 0) tcv = 1e-6;
      if (tmv == 0) tmv = 1e-6;
      reward = (tcm == 0 || tmm == 0)
                   ? 0.0
                   : kl_reward(tcm, tmm, tcv, tmv, res[4] / (double)P, res[5] / (double)P, cv, mv);
    } else if (p.reward == 1) {
      reward = p.beta * res[4] + (1 - p.beta) * res[5];
    } else {
      reward = -wr;
    }
  }
  const int64_t ts = H->timestep;
  const bool term = ts >= p.limit;
  const double a0 = k > 0 ? res[0] : 0.0, a1 = k > 0 ? res[1] : 0.0;
  wsync();
  if (lane == 0) {
    H->timestep = ts + 1;
    H->total_requests += arrivals;
    H->served += n_term;
    H->dropped += arrivals - k;
    H->waiting_ratio = wr;
    if (kl) {
      H->tcm = tcm;
      H->tmm = tmm;
    }
    if (k > 0) {
      H->total_cpu_req = H->total_cpu_req + a0;
      H->total_mem_req = H->total_mem_req + a1;
    }
    B.b64[0] = __double_as_longlong(reward);
    B.bc[6] = term;
  }
  wsync();
}

__device__ VMP_BIG_CALL void big_predraw(const EnvParams &p, const Tables &T, char LDSP *base,
                                         int K, const uint64_t *jt) {
  const Lds L = make_lds(p, base);
  const uint64_t GLBP *g = gptr(jt);
  const U128 JA{g[0], g[1]}, JM{g[2], g[3]};
  predraw(p, L, T, K, p.V, JA, JM);
}

// The env's outputs of the launch that are final once the step's accept
// phase is done: obs (VM part and PM part, env.py:295-296) and, with `state`,
// the VM words and PM resources. Issued before the stats so the stores drain
// while the pairwise sums run (the header follows at the end of the launch).
// With `state`: the low halves (placement, sizes) of the VM words that
// changed (the time words were written by big_tail as they changed).
template <int SPT>
__device__ __forceinline__ void big_store(const EnvParams &p, const Lds &L, const Tables &T,
                                          const uint32_t LDSP *W, SMask dirty, float *obs,
                                          bool state, int e) {
  const int t = threadIdx.x, NT = kBigNT;
  const int V = p.V, P = p.P;
  uint32_t *vmo = p.vmw + (int64_t)e * vm_pitch(V);
VMP_SLOOP
  for (int s = 0; s < SPT; s++) {
    const int v = s * NT + t;
    const uint32_t w = W[v];
    if (live(w)) {
      if (obs) {
        ST_NT(obs + v, (float)w_pl(w));
        ST_NT(obs + V + v, T.fcent[w_cc(w)]);
        ST_NT(obs + 2 * V + v, T.fcent[w_cm(w)]);
      }
      if (state && ((dirty >> s) & 1u)) ST_NT(vmo + vm_slot_idx(v), w);
    }
  }
  if (obs)
    for (int i = t; i < P; i += NT) {
      ST_NT(obs + 3 * V + i, (float)L.cpu[i]);
      ST_NT(obs + 3 * V + P + i, (float)L.mem[i]);
    }
  if (state) {  // the PM words written this launch (as env_body's store)
    double *pmo = p.pm + (int64_t)e * 2 * P;
    for (int i = t; i < 2 * P; i += NT)
      if ((L.pdirty[i >> 6] >> (i & 63)) & 1ull) ST_NT(pmo + i, (double)L.cpu[i]);
  }
}

// The state part of big_store from the owner's copy of its VM words (WR is a
// register array or the LDS words W, see big_tail).
template <int SPT, class WR>
__device__ __forceinline__ void big_store_words(const EnvParams &p, const Lds &L, const WR &wr,
                                                SMask dirty, int e) {
  const int t = threadIdx.x, NT = kBigNT;
  const int V = p.V, P = p.P;
  uint32_t *vmo = p.vmw + (int64_t)e * vm_pitch(V);
#pragma unroll
  for (int s = 0; s < SPT; s++)
    if (((dirty >> s) & 1u) && live(wr[s])) ST_NT(vmo + vm_slot_idx(s * NT + t), wr[s]);
  double *pmo = p.pm + (int64_t)e * 2 * P;
  for (int i = t; i < 2 * P; i += NT)
    if ((L.pdirty[i >> 6] >> (i & 63)) & 1ull) ST_NT(pmo + i, (double)L.cpu[i]);
}

// obs (env.py:295-296) from the LDS state by the threads [0, n) of a subset
// of the block's waves (thread i of them: slots i, i + n, ...).
__device__ __forceinline__ void big_store_obs(const EnvParams &p, const Lds &L, const Tables &T,
                                              const uint32_t LDSP *W, float *obs, int i, int n) {
  const int V = p.V, P = p.P;
  if (((uintptr_t)obs & 15) == 0 && (V & 3) == 0 && (P & 3) == 0) {
    // 4 consecutive VMs / PMs per thread: one 16-B LDS read of the VM words
    // and three 16-B streaming stores (a quarter of the store instructions)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    typedef double f64x2 __attribute__((ext_vector_type(2)));
#pragma unroll 2
    for (int g = i; g < V / 4; g += n) {
      const u32x4 w = *reinterpret_cast<const u32x4 LDSP *>(W + 4 * g);
      f32x4 pl, cc, cm;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        pl[j] = (float)w_pl(w[j]);
        cc[j] = T.fcent[w_cc(w[j])];
        cm[j] = T.fcent[w_cm(w[j])];
      }
      __builtin_nontemporal_store(pl, reinterpret_cast<f32x4 GLBP *>(gptr(obs + 4 * g)));
      __builtin_nontemporal_store(cc, reinterpret_cast<f32x4 GLBP *>(gptr(obs + V + 4 * g)));
      __builtin_nontemporal_store(cm, reinterpret_cast<f32x4 GLBP *>(gptr(obs + 2 * V + 4 * g)));
    }
    for (int g = i; g < P / 4; g += n) {
      const f64x2 c0 = *reinterpret_cast<const f64x2 LDSP *>(L.cpu + 4 * g);
      const f64x2 c1 = *reinterpret_cast<const f64x2 LDSP *>(L.cpu + 4 * g + 2);
      const f64x2 m0 = *reinterpret_cast<const f64x2 LDSP *>(L.mem + 4 * g);
      const f64x2 m1 = *reinterpret_cast<const f64x2 LDSP *>(L.mem + 4 * g + 2);
      const f32x4 fc = {(float)c0[0], (float)c0[1], (float)c1[0], (float)c1[1]};
      const f32x4 fm = {(float)m0[0], (float)m0[1], (float)m1[0], (float)m1[1]};
      __builtin_nontemporal_store(fc, reinterpret_cast<f32x4 GLBP *>(gptr(obs + 3 * V + 4 * g)));
      __builtin_nontemporal_store(fm, reinterpret_cast<f32x4 GLBP *>(gptr(obs + 3 * V + P + 4 * g)));
    }
    return;
  }
#pragma unroll 4
  for (int v = i; v < V; v += n) {
    const uint32_t w = W[v];
    ST_NT(obs + v, (float)w_pl(w));
    ST_NT(obs + V + v, T.fcent[w_cc(w)]);
    ST_NT(obs + 2 * V + v, T.fcent[w_cm(w)]);
  }
  for (int q = i; q < P; q += n) {
    ST_NT(obs + 3 * V + q, (float)L.cpu[q]);
    ST_NT(obs + 3 * V + P + q, (float)L.mem[q]);
  }
}

// _run_vms, _accept_vm_requests, stats + reward, termination (env_tail, block form).
// out_obs / store_state: big_store right after the accept phase (last step of
// the launch only).
// The time words (high halves of the VM words: finish keys of running VMs,
// remaining runtimes of waiting ones, §2) are read from HBM at the start of
// each step and written back as they change (placed, suspended, finished,
// accepted), so no per-slot time registers live across the step; the low
// halves live in LDS (W) and are stored by big_store (`dirty`).
template <int SPT>
__device__ __forceinline__ double big_tail(const EnvParams &p, const Lds &L, const Tables &T,
                                           BigShared &B, uint32_t LDSP *W, SMask run0,
                                           SMask &dirty, int kstep, bool &terminated,
                                           float *out_obs, bool store_state, bool heur,
                                           int e STAMP_PARAMS) {
  const int t = threadIdx.x, NT = kBigNT, lane = lane_id();
  const bool w0 = t < 64;
  const int P = p.P, WAIT = p.P, NUL = p.P + 1;
  EnvHdr LDSP *H = L.hdr;
  uint32_t *vw32 = p.vmw + (int64_t)e * vm_pitch(p.V);
  // ---- _run_vms: finish keys (env_tail), then free the finishers in ascending VM order ----
  const uint32_t t32 = (uint32_t)H->timestep;
  SMask fterm = 0;
  // this thread's VM words, in registers for the tail's per-slot passes (the
  // LDS copy W stays current for the cross-thread readers: frees, obs, mask)
  // (the tail reads its words from LDS: a 40-register copy pushed the kernel
  // to 256 VGPRs and spilled SGPRs to scratch, ~49 KB of scratch traffic
  // each way per env-step, 2 % slower)
  struct {
    uint32_t LDSP *W;
    int t;
    __device__ __forceinline__ uint32_t LDSP &operator[](int s) const { return W[s * kBigNT + t]; }
  } wr{W, t};
  {
    uint32_t hw[SPT];  // the time words, issued together, dead after this loop
#pragma unroll
    for (int s = 0; s < SPT; s++) hw[s] = gptr(vw32)[vm_time_idx(min(s * NT + t, p.V - 1))];
#pragma unroll
    for (int s = 0; s < SPT; s++) {
      const int v = s * NT + t;
      const bool running = w_pl(wr[s]) < P;
      uint32_t h = hw[s];
      if (running != (bool)((run0 >> s) & 1u)) {
        h = running ? h + t32 : h - t32;
        dirty |= SBIT(s);
      }
      if (running && (int32_t)(h - t32) <= 1) {
        fterm |= SBIT(s);
        h = 0;  // the word becomes NULL (below)
      }
      if (h != hw[s]) ST_NT(vw32 + vm_time_idx(v), h);  // padded slots never change
    }
  }
  dirty |= fterm;
  STAMP(8);
  const int n_term = row_counts<SPT>(fterm, B);
  STAMP(9);
  // heuristic actions never suspend, so only the PMs freed here can fall under
  // the precision clamp: they are clamped as they are freed (equal to the
  // reference's clamp after all frees: once a PM's value is < 1e-7 every
  // further free leaves it < 1e-7, and the clamp maps both to 0); external
  // actions keep the full clamp pass below
  const bool clamp_inline = heur;
#pragma unroll 1
  for (int j0 = 0; j0 < n_term; j0 += 512) {
    if (ballot(fterm != 0)) {  // waves without finishers skip the ranking
      int rb;
      const int pre = row_prefix<SPT>(B, rb);
VMP_SLOOP
      for (int s = 0; s < SPT; s++) {
        const int r = __builtin_amdgcn_readlane(pre, s) + below(ballot((fterm >> s) & 1u), lane);
        if (((fterm >> s) & 1u) && r >= j0 && r < j0 + 512) L.evw[r - j0] = wr[s];
      }
    }
    __syncthreads();
    if (w0) {
      const int nt = n_term - j0 < 512 ? n_term - j0 : 512;
#pragma unroll 1
      for (int i = 0; i < nt; i++) {  // frees in ascending VM order
        const uint32_t ew = L.evw[i];
        const int q = w_pl(ew);
        double cq = L.cpu[q] - T.cent[w_cc(ew)];
        double mq = L.mem[q] - T.cent[w_cm(ew)];
        if (clamp_inline) {
          if (cq < 1e-7) cq = 0;
          if (mq < 1e-7) mq = 0;
        }
        wsync();
        if (lane == 0) {
          L.cpu[q] = cq;
          L.mem[q] = mq;
          mark_pm(L, P, q);
        }
        wsync();
      }
    }
    __syncthreads();
  }
  STAMP(10);
#pragma unroll
  for (int s = 0; s < SPT; s++)
    if ((fterm >> s) & 1u) {
      wr[s] = w_make(NUL, 0, 0);
    }
  STAMP(2);
  if (w0 && !clamp_inline)
    for (int i = lane; i < P; i += 64) {  // precision clamp
      if (L.cpu[i] < 1e-7) L.cpu[i] = 0;
      if (L.mem[i] < 1e-7) L.mem[i] = 0;
    }
  // ---- _accept_vm_requests: the first k NULL slots in VM order ----
  SMask fnull = 0;
#pragma unroll
  for (int s = 0; s < SPT; s++)
    if (w_pl(wr[s]) == NUL) fnull |= SBIT(s);
  const int n_null = row_counts<SPT>(fnull, B);
  STAMP(14);
  const int64_t arrivals = L.arr[kstep];
  const int64_t k = arrivals < n_null ? arrivals : n_null;
  // accepted sizes: LDS up to acc_cap, else the env's HBM spill (bigscr)
  const bool acc_g = k > p.acc_cap;
  uint8_t GLBP *gsc = gptr(p.bigscr) + (int64_t)e * 4 * p.V;
  if (k > 0) {
    Pcg r1 = ld_pcg(H, 0), r2 = ld_pcg(H, 1);
#pragma unroll 1
    for (int64_t j0 = 0; j0 < k; j0 += 512) {
      const int64_t j1 = j0 + 512 < k ? j0 + 512 : k;
      if (w0) {
#pragma unroll 1
        for (int64_t j = j0; j < j1; j++) {
          const int cc = (int)rint((p.seq_lo + p.seq_range * next_double(r1)) * 100.0);
          const int cm = (int)rint((p.seq_lo + p.seq_range * next_double(r2)) * 100.0);
          const uint32_t rr = svc_take(p, L);
          if (lane == 0) {
            if (acc_g) {
              gsc[j] = (uint8_t)cc;
              gsc[p.V + j] = (uint8_t)cm;
            } else {
              L.accc[j] = (uint8_t)cc;
              L.accm[j] = (uint8_t)cm;
            }
            L.evt[j - j0] = (int32_t)rr;
          }
        }
      }
      __syncthreads();
      int rb;
      const int pre = row_prefix<SPT>(B, rb);
#pragma unroll
      for (int s = 0; s < SPT; s++) {  // wr[] statically indexed
        if (__builtin_amdgcn_readlane(rb, s) >= j1) break;  // later rows rank past the accepted
        const int j = __builtin_amdgcn_readlane(pre, s) + below(ballot((fnull >> s) & 1u), lane);
        if (((fnull >> s) & 1u) && j >= j0 && j < j1) {
          const int cc = acc_g ? gsc[j] : L.accc[j], cm = acc_g ? gsc[p.V + j] : L.accm[j];
          wr[s] = w_make(WAIT, cc, cm);
          ST_NT(vw32 + vm_time_idx(s * NT + t), (uint32_t)L.evt[j - j0]);
          dirty |= SBIT(s);
        }
      }
      __syncthreads();
    }
    if (w0) {
      st_pcg(H, 0, r1);
      st_pcg(H, 1, r2);
    }
  }
  __syncthreads();
  STAMP(15);
  // the VM words and PM resources are final: their owners store them now
  if (store_state) big_store_words<SPT>(p, L, wr, dirty, e);
  STAMP(3);
  // ---- stats + reward ----
  const bool kl = p.reward == 2;
  SMask fex = 0;
  int n_w = 0;
#pragma unroll
  for (int s = 0; s < SPT; s++) {
    const int c = w_pl(wr[s]);
    if (c <= WAIT) fex |= SBIT(s);
    n_w += c == WAIT;
  }
  const int n_ex = row_counts<SPT>(fex, B, &n_w);
  // existing-VM sizes: LDS up to ccomp_cap, else the env's HBM spill
  const bool cc_g = n_ex > p.ccomp_cap;
  if (kl) {
    int rb;
    const int pre = row_prefix<SPT>(B, rb);
    uint8_t LDSP *lc = L.ccomp, *lm = L.mcomp;
    uint8_t GLBP *gc = gsc + 2 * p.V, *gm = gsc + 3 * p.V;
#pragma unroll
    for (int s = 0; s < SPT; s++) {
      const int r = __builtin_amdgcn_readlane(pre, s) + below(ballot((fex >> s) & 1u), lane);
      if ((fex >> s) & 1u) {
        const uint32_t w = wr[s];
        if (cc_g) {
          gc[r] = (uint8_t)w_cc(w);
          gm[r] = (uint8_t)w_cm(w);
        } else {
          lc[r] = (uint8_t)w_cc(w);
          lm[r] = (uint8_t)w_cm(w);
        }
      }
    }
  }
  const uint32_t spill = (acc_g ? 1u : 0u) | (cc_g ? 2u : 0u);
  __syncthreads();
  STAMP(11);
  {  // phase A: plain sums; phase B (kl): squared deviations about their means
    const uint32_t ja = (k > 0 ? 0x3u : 0u) | (kl ? 0xCu : 0u) | (p.reward >= 1 ? 0x30u : 0u);
    // the observation is written by the waves that get no phase-A sum task
    // (task i runs on wave i), so its stores drain while the sums run
    const int nwv = NT >> 6, nj = big_sum_ntask(p, ja, (int)k, n_ex, kBigSplitA);
    if (out_obs) {
      const int ws = nj < nwv ? nj : 0;
      if ((t >> 6) >= ws) big_store_obs(p, L, T, W, out_obs, t - 64 * ws, NT - 64 * ws);
    }
#ifdef VMP_WGTIME
    STAMP(17);  // wave 0: obs issued
#endif
    // kl on four waves: chained, no phase barrier. Only wave 0 owns the LDS
    // plan of the deep pairwise sums, so the chains need every job of waves
    // 1-3 within the register plan (n <= pw_reg_cap): at P1000 / V10000
    // under 2 000 arrivals per step n_ex reaches ~10 000 and the block falls
    // back to the two phases (big_sum_phase sends those jobs to wave 0)
    constexpr int kCap = pw_reg_cap(kBigPwDepth);
    if (kl && kBigNT == 256 && n_ex <= kCap && (int)k <= kCap && p.P <= kCap) {
      big_kl_sums(p, T, L.base, B, (int)k, n_ex, spill, kstep + 1);
      STAMP(20);
      STAMP(21);
    } else {
      if (ja) big_sum_phase(p, T, L.base, B, ja, (int)k, n_ex, kBigSplitA, true, spill);
      STAMP(20);
      if (kl) big_sum_phase(p, T, L.base, B, 0x3C0u, (int)k, n_ex, true, false, spill);
      STAMP(21);
    }
  }
  if (w0) big_stats_final(p, B, L.base, k, n_ex, n_w, n_term, arrivals);
  __syncthreads();
  STAMP(12);
  const double reward = __longlong_as_double(B.b64[0]);
  terminated = B.bc[6] != 0;
  __syncthreads();
  return reward;
}

// ONE = true: the per-step launch (k_steps == 1), its own instantiation so the
// step's registers (rem[] above all) are dead after the state store instead of
// live around the K-step loop's back edge, which spilled them around the sums.
template <int SPT, bool ONE>
#ifndef VMP_BIG_WPE_ONE  // waves/SIMD the per-step instantiation is allocated for
#define VMP_BIG_WPE_ONE 2
#endif
__global__ __launch_bounds__(kBigNT, ONE ? VMP_BIG_WPE_ONE : 2) void k_env_big(EnvParams p, StepOut o) {
  extern __shared__ __align__(16) char lds[];
  __shared__ Tables T;
  __shared__ BigShared B;
  const int t = threadIdx.x, NT = kBigNT, lane = lane_id();
  const bool w0 = t < 64;
  const int e = blockIdx.x;
  const Lds L = make_lds(p, (char LDSP *)lds);
  uint32_t LDSP *W = reinterpret_cast<uint32_t LDSP *>((char LDSP *)lds + p.lds_wave_bytes);
  const int V = p.V, P = p.P;
#ifdef VMP_STAMPS
  __shared__ uint64_t st_lds[kStamps];
#endif
  STAMP_DECL_AT(w0 ? (uint64_t LDSP *)st_lds : nullptr)  // thread 0's clock
#ifdef VMP_WGTIME  // diagnostic: workgroup start / end (100 MHz) and its CU
  const uint64_t wg_t0 = __builtin_amdgcn_s_memrealtime();
  if (t < 24) wg_marks[t] = 0;
#endif
  for (int i = t; i < 128; i += NT) {
    T.cent[i] = (double)i / 100.0;
    T.fcent[i] = (float)((double)i / 100.0);
  }
  constexpr int kPoisWords = (int)(2 * sizeof(PoisConst) / 4);
  if (t < kPoisWords) reinterpret_cast<uint32_t *>(T.pois)[t] = gptr(reinterpret_cast<const uint32_t *>(p.pois))[t];
  // every global load of the env's state is issued before the first LDS store
  // (indices clamped, not branched on, so the loads are unconditional):
  // header, the first 4*NT PM words, the VM words
  const uint64_t hv = gptr(reinterpret_cast<const uint64_t *>(p.hdr + e))[t & 31];
  const double GLBP *pm = gptr(p.pm + (int64_t)e * 2 * P);
  const int n_pm = 2 * P;
  double pv[4];
#pragma unroll
  for (int j = 0; j < 4; j++) pv[j] = pm[min(j * NT + t, n_pm - 1)];
  const uint32_t GLBP *vmw = gptr(p.vmw + (int64_t)e * vm_pitch(V));
  __asm__ volatile("" ::: "memory");
  if (t < 32) reinterpret_cast<uint64_t LDSP *>(L.hdr)[t] = hv;
  if (w0) {
    // the random draws need only the header: wave 0 takes them while the
    // other waves load the VM words (the two never hold registers at once)
    if (o.k_steps > 0) {
      wsync();
      big_predraw(p, T, L.base, o.k_steps, p.jump + 4 * lane);
    }
  } else {
    // waves 1.. load the low halves of all VM words (placement, sizes) into W;
    // the time words are read by big_tail
    constexpr int kLd = kBigNT - 64, kLPT = (SPT * kBigNT + kLd - 1) / kLd;
    const int tl = t - 64;
    uint32_t wl[kLPT];
#pragma unroll
    for (int j = 0; j < kLPT; j++) wl[j] = vmw[vm_slot_idx(min(j * kLd + tl, V - 1))];
#pragma unroll
    for (int j = 0; j < kLPT; j++) {
      const int v = j * kLd + tl;
      if (v < SPT * kBigNT) W[v] = v < V ? wl[j] : (uint32_t)kPad;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; j++)
    if (j * NT + t < n_pm) L.cpu[j * NT + t] = pv[j];
  for (int i = 4 * NT + t; i < n_pm; i += NT) L.cpu[i] = pm[i];  // P > 2 * NT
  for (int i = t; i < (n_pm + 63) / 64; i += NT) L.pdirty[i] = 0;
  for (int i = t; i < kBigMaxSPT * kBigMaxWaves; i += NT) B.rc[i] = 0;
  if (t < 2) B.klflag[t] = 0;
  __syncthreads();
  STAMP(13);
  bool term = false;
  int64_t ndone = 0;
  SMask dirty = 0;  // bit s: this thread's VM word s changed (stored by big_store)
  const int k_steps = ONE ? 1 : o.k_steps;
#pragma unroll 1
  for (int k = 0; k < k_steps; k++) {
    const bool last = k == k_steps - 1;
    uint8_t *valid_row = (last && o.valid) ? o.valid + (int64_t)e * V : nullptr;
    int32_t *act_row = (last && o.act_out) ? o.act_out + (int64_t)e * V : nullptr;
    int64_t n_place = 0, n_susp = 0;
    SMask run0 = 0;
VMP_SLOOP
    for (int s = 0; s < SPT; s++) run0 |= (SMask)(w_pl(W[s * NT + t]) < P) << s;
    if (o.policy >= 0)
      n_place = big_heuristic<SPT>(p, L, T, B, W, o.policy, act_row, valid_row STAMP_ARGS);
    else
      big_external<SPT>(p, L, T, B, W, o.actions + (int64_t)e * V, valid_row, n_place, n_susp);
    __syncthreads();
    STAMP(16);
    if (t == 0) {
      L.hdr->place_action += n_place;
      L.hdr->suspend_action += n_susp;
    }
    __syncthreads();
    const double r = big_tail<SPT>(p, L, T, B, W, run0, dirty, k, term,
                                   last && o.obs ? o.obs + (int64_t)e * p.D : nullptr, last,
                                   o.policy >= 0, e
                                   STAMP_ARGS);
    if (o.reward && t == 0) gptr(o.reward)[(int64_t)k * p.N + e] = r;
    ndone += term;
  }
  if (o.k_steps > 0) {
    if (w0) svc_commit(L);
  }
  if (o.k_steps == 0 && o.policy >= 0 && o.act_out) {
    big_heuristic<SPT>(p, L, T, B, W, o.policy, o.act_out + (int64_t)e * V, nullptr STAMP_ARGS);
    __syncthreads();
    for (int v = t; v < V; v += NT) W[v] = vmw[vm_slot_idx(v)];  // act only: placements unchanged
  }
  __syncthreads();
  STAMP(4);
  // a stepping launch stored obs and state after its last accept phase
  if (o.obs && o.k_steps == 0) big_store<SPT>(p, L, T, W, 0u, o.obs + (int64_t)e * p.D, false, e);
  if (o.mask_bits) {
    uint32_t *bits = o.mask_bits + (int64_t)e * V * p.W32;
    const int A = p.A, NW32 = p.W32, WAIT = p.P, NUL = p.P + 1;
VMP_SLOOP
    for (int s = 0; s < SPT; s++) {
      const int v = s * NT + t;
      const uint32_t wv = W[v];
      const bool in = live(wv);
      const int c = in ? w_pl(wv) : NUL;
      const double vc = T.cent[w_cc(wv)], vm = T.cent[w_cm(wv)];
      const bool waiting = in && c == WAIT;
#pragma unroll 1
      for (int w = 0; w < NW32; w++) {
        uint32_t word = 0xFFFFFFFFu;
        const int a0 = w * 32;
        if (c >= a0 && c < a0 + 32 && c < A) word &= ~(1u << (c - a0));
        if (c < P && WAIT >= a0 && WAIT < a0 + 32) word &= ~(1u << (WAIT - a0));
        if (waiting) {
          const int hi = min(a0 + 32, P);
#pragma unroll 1
          for (int q = a0; q < hi; q++) {
            const bool fit = (L.cpu[q] + vc <= 1) && (L.mem[q] + vm <= 1);
            if (fit) word &= ~(1u << (q - a0));
          }
        }
        if (in) bits[(int64_t)v * NW32 + w] = word;
      }
    }
  }
  if (o.k_steps > 0) {
    if (o.done && t == 0) gptr(o.done)[e] = (uint8_t)term;
    if (o.done_count && t == 0) gptr(o.done_count)[e] += ndone;
    if (t < 32)  // (no draw hint: EnvHdr::pad = 0)
      gptr(reinterpret_cast<uint64_t *>(p.hdr + e))[t] = t == 31 ? 0ull : reinterpret_cast<uint64_t LDSP *>(L.hdr)[t];
  }
  STAMP(6);
  STAMP_FLUSH();
#ifdef VMP_WGTIME
  __syncthreads();
  if (t == 0 && p.stamps) {
    // slots: 0 start, 1 end, 5 HW_ID, 7 XCC_ID, else the clock at STAMP(slot)
    uint64_t *o = p.stamps + (int64_t)e * 24;
    for (int i = 2; i < 24; i++) o[i] = wg_marks[i];
    o[0] = wg_t0;
    o[1] = __builtin_amdgcn_s_memrealtime();
    o[5] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    o[7] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
#endif
}
template <bool ONE>
static void launch_big_one(int spt, int n_env, size_t lds, hipStream_t s, const EnvParams &p,
                           const StepOut &o) {
  const dim3 grid(n_env), block(kBigNT);
  if (spt == 4) hipLaunchKernelGGL((k_env_big<4, ONE>), grid, block, lds, s, p, o);
  else if (spt == 8) hipLaunchKernelGGL((k_env_big<8, ONE>), grid, block, lds, s, p, o);
  else if (spt == 16) hipLaunchKernelGGL((k_env_big<16, ONE>), grid, block, lds, s, p, o);
  else
  hipLaunchKernelGGL((k_env_big<kBigMaxSPT, ONE>), grid, block, lds, s, p, o);
}
// host side: the block kernel's geometry and launcher (vmp_capi.cpp)
void big_geometry(int *nt, int *spt_max) {
  *nt = kBigNT;
  *spt_max = kBigMaxSPT;
}
void launch_big_env(int spt, bool one, int n_env, size_t lds, hipStream_t s, const EnvParams &p,
                    const StepOut &o) {
  if (one) launch_big_one<true>(spt, n_env, lds, s, p, o);
  else launch_big_one<false>(spt, n_env, lds, s, p, o);
}
// workgroups per CU of the per-step block kernel at `lds` dynamic bytes, and
// its static LDS
int big_occupancy(int spt, size_t lds, int *static_lds) {
  const void *f = reinterpret_cast<const void *>(&k_env_big<kBigMaxSPT, true>);
  if (spt == 4) f = reinterpret_cast<const void *>(&k_env_big<4, true>);
  else if (spt == 8) f = reinterpret_cast<const void *>(&k_env_big<8, true>);
  else if (spt == 16) f = reinterpret_cast<const void *>(&k_env_big<16, true>);
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, f) == hipSuccess) *static_lds = (int)a.sharedSizeBytes;
  int nb = -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, kBigNT, lds) != hipSuccess) nb = -1;
  return nb;
}

// _get_rank for any V: one wave per env, LDS bitmap of used PMs.
__global__ __launch_bounds__(64) void k_rank(EnvParams p, int64_t *rank) {
  extern __shared__ unsigned long long used[];
  const int lane = lane_id(), e = blockIdx.x;
  const int NWP = (p.P + 63) / 64;
  for (int i = lane; i < NWP; i += 64) used[i] = 0ull;
  __syncthreads();
  const uint32_t *row = p.vmw + (int64_t)e * vm_pitch(p.V);
  for (int v = lane; v < p.V; v += 64) {
    const int st = (int)(row[vm_slot_idx(v)] & 0xFFFFu);
    if (st < p.P) atomicOr(used + (st >> 6), 1ull << (st & 63));
  }
  __syncthreads();
  int64_t r = 0;
  for (int i = lane; i < NWP; i += 64) r += __popcll(used[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
  if (lane == 0) rank[e] = r;
}

// target means for any V: one wave per env on the env's LDS carve (ccomp /
// mcomp and the pairwise-sum plan of make_lds).
__global__ __launch_bounds__(64) void k_target_means_lds(EnvParams p) {
  extern __shared__ __align__(16) char lds[];
  __shared__ double cent[128];
  for (int i = threadIdx.x; i < 128; i += 64) cent[i] = (double)i / 100.0;
  __syncthreads();
  const int lane = lane_id(), e = blockIdx.x;
  const Lds L = make_lds(p, (char LDSP *)lds);
  const int V = p.V, P = p.P;
  const uint32_t *row = p.vmw + (int64_t)e * vm_pitch(V);
  int n_ex = 0;
  for (int b = 0; b < V; b += 64) {
    const int v = b + lane;
    const uint32_t w = v < V ? row[vm_slot_idx(v)] : (uint32_t)(P + 1);
    const bool ex = v < V && (int)(w & 0xFFFFu) <= P;
    const uint64_t m = ballot(ex);
    if (ex) {
      const int rk = n_ex + below(m, lane);
      L.ccomp[rk] = (uint8_t)((w >> 16) & 0xFFu);
      L.mcomp[rk] = (uint8_t)((w >> 24) & 0xFFu);
    }
    n_ex += __popcll(m);
  }
  wsync();
  const double *ct = cent;
  const uint8_t LDSP *cc = L.ccomp;
  const uint8_t LDSP *cm = L.mcomp;
  const double sc = wave_pw_sum(n_ex, [=](int i) { return ct[cc[i]]; }, L.pw);
  const double sm = wave_pw_sum(n_ex, [=](int i) { return ct[cm[i]]; }, L.pw);
  if (lane == 0) {
    double tcm = sc / (double)P, tmm = sm / (double)P;
    if (p.cap_target_util && tcm > 1) tcm = 1.0;
    if (p.cap_target_util && tmm > 1) tmm = 1.0;
    p.hdr[e].tcm = tcm;
    p.hdr[e].tmm = tmm;
  }
}

// ---- FirstFitAgent.act / BestFitAgent.act on a caller's observation --------
// firstfit.py:21-38 / bestfit.py:21-40 exactly as written: the agent reads
// only the f32 observation it is passed (convert_obs_to_dict, utils.py:37-47),
// so this kernel takes obs f32[n_env][3V + 2P] and nothing of the env state.
// The obs need not be one the env produced (an edited or stale observation):
// fits are the f32 sums cpu[p] + vm_cpu[v] <= 1 and memory[p] + vm_memory[v]
// <= 1, FirstFit updates only cpu[p], BestFit both, and BestFit visits the PMs
// in flip(argsort(cpu + memory)) with numpy's scalar introsort tie order
// (wave_aquicksort). One wave per env; the waiting VMs are
// taken in index order, one PM scan (P/64 compares per lane) each. LDS:
// cpu, memory, keys f32[P], order u16[P], sort stack i32[256] + scratch
// u16[2P]. Not the hot path (the Base.test loop and the bench act on the
// env's own state, k_env); this is the contract of act(observation).
__device__ __forceinline__ int act_obs_bf(const float LDSP *fc, const float LDSP *fm,
                                          float LDSP *key, uint16_t LDSP *ord,
                                          int32_t LDSP *stk, int P, float vc, float vm) {
  const int lane = lane_id();
  float best = -INFINITY;
  int cnt = 0, bi = -1;
  for (int i = lane; i < P; i += 64) {
    if (fc[i] + vc <= 1.0f && fm[i] + vm <= 1.0f) {
      const float k = fc[i] + fm[i];
      if (k > best) {
        best = k;
        cnt = 1;
        bi = i;
      } else if (k == best) {
        cnt++;
      }
    }
  }
  float m = best;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  int tot = (best == m) ? cnt : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
  if (tot == 0) return -1;
  if (tot == 1) {
    const uint64_t who = ballot(best == m && cnt == 1);
    return __builtin_amdgcn_readlane(bi, __ffsll((unsigned long long)who) - 1);
  }
  int above = 0, eq = 0;
  for (int i = lane; i < P; i += 64) {
    const float k = fc[i] + fm[i];
    key[i] = k;
    ord[i] = (uint16_t)i;
    above += fless(m, k);
    eq += k == m;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    above += __shfl_xor(above, o);
    eq += __shfl_xor(eq, o);
  }
  const int hi = P - above - 1, lo = P - above - eq;
  wsync();
  wave_aquicksort(KeyArr{key}, ord, P, stk, lo, hi, reinterpret_cast<uint16_t LDSP *>(stk + 256));
  wsync();
  for (int b = hi; b >= lo; b -= 64) {  // visiting order: descending positions
    const int pos = b - lane;
    const int q = pos >= lo ? (int)ord[pos] : 0;
    const uint64_t f = ballot(pos >= lo && fc[q] + vc <= 1.0f && fm[q] + vm <= 1.0f);
    if (f) return __builtin_amdgcn_readlane(q, __ffsll((unsigned long long)f) - 1);
  }
  return -1;
}

__global__ __launch_bounds__(64) void k_act_obs(int P, int V, int policy, const float *obs,
                                                int32_t *act) {
  extern __shared__ __align__(16) char lds[];
  float LDSP *fc = reinterpret_cast<float LDSP *>((char LDSP *)lds);
  float LDSP *fm = fc + P;
  float LDSP *key = fm + P;
  int32_t LDSP *stk = reinterpret_cast<int32_t LDSP *>(key + P);
  uint16_t LDSP *ord = reinterpret_cast<uint16_t LDSP *>(stk + 256 + P);  // after the scratch
  const int lane = lane_id(), e = blockIdx.x;
  const int D = 3 * V + 2 * P;
  const float *o = obs + (int64_t)e * D;
  int32_t *a = act + (int64_t)e * V;
  for (int i = lane; i < P; i += 64) {
    fc[i] = o[3 * V + i];
    fm[i] = o[3 * V + P + i];
  }
  wsync();
  for (int b = 0; b < V; b += 64) {
    const int v = b + lane;
    const float pl = v < V ? o[v] : 0.f;
    const float vc = v < V ? o[V + v] : 0.f, vm = v < V ? o[2 * V + v] : 0.f;
    // observation[:V].astype(int) (utils.py:41) truncates before the
    // WAIT_STATUS compare: P + 0.4 waits (C++ truncation = numpy astype(int))
    int out = (int)pl;  // action = np.copy(vm_placement)
    uint64_t todo = ballot(v < V && out == P);
    while (todo) {
      const int l = __ffsll((unsigned long long)todo) - 1;
      todo &= todo - 1;
      const float c = __shfl(vc, l), m = __shfl(vm, l);
      int q = -1;
      if (policy == 0) {  // firstfit.py:33-37: first PM in index order
        for (int i0 = 0; i0 < P && q < 0; i0 += 64) {
          const int i = i0 + lane;
          const uint64_t f = ballot(i < P && fc[i] + c <= 1.0f && fm[i] + m <= 1.0f);
          if (f) q = i0 + __ffsll((unsigned long long)f) - 1;
        }
      } else {  // bestfit.py:33-39
        q = act_obs_bf(fc, fm, key, ord, stk, P, c, m);
      }
      if (q >= 0) {
        if (lane == l) out = q;
        wsync();
        if (lane == 0) {
          fc[q] = fc[q] + c;
          if (policy != 0) fm[q] = fm[q] + m;  // FirstFit leaves memory (firstfit.py:36)
        }
        wsync();
      }
    }
    if (v < V) a[v] = out;
  }
}

}  // namespace vmp
