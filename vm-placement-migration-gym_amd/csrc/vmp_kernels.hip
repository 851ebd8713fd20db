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

// Minimum waves per SIMD the env kernel is register-allocated for
// (__launch_bounds__ 2nd argument); measured choice, see DESIGN.md.
#ifndef VMP_WAVES_PER_EU
#define VMP_WAVES_PER_EU 1
#endif

namespace vmp {

// ------------------------------------------------------------ wave utils --
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
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
__device__ __forceinline__ double loggam_dev(double x) {
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

// random_poisson (distributions.c): mult method (lam < 10) / PTRS (lam >= 10).
__device__ __forceinline__ int64_t poisson(Pcg &r, const PoisConst &c) {
  if (c.kind == 2) {
    for (;;) {
      double U = next_double(r) - 0.5;
      double V = next_double(r);
      double us = 0.5 - fabs(U);
      int64_t k = (int64_t)floor((2 * c.a / us + c.b) * U + c.lam + 0.43);
      if ((us >= 0.07) && (V <= c.vr)) return k;
      if ((k < 0) || ((us < 0.013) && (V > us))) continue;
      double lg = (k + 1 < c.tab_n) ? c.loggam_tab[k + 1] : loggam_dev((double)(k + 1));
      if ((log(V) + c.log_invalpha - log(c.a / (us * us) + c.b)) <= (-c.lam + k * c.loglam - lg))
        return k;
    }
  } else if (c.kind == 0) {
    return 0;
  }
  double prod = 1.0;
  int64_t X = 0;
  for (;;) {
    prod *= next_double(r);
    if (prod > c.enlam)
      X += 1;
    else
      return X;
  }
}

// Out of line: one Poisson draw from stream k of the wave's LDS header (all
// lanes call it with identical state; lane 0 writes the advanced state back).
__device__ __forceinline__ int64_t poisson_lds(uint64_t *hdr_rng, const PoisConst *c) {
  Pcg r;
  r.s = U128{hdr_rng[0], hdr_rng[1]};
  r.inc = U128{hdr_rng[2], hdr_rng[3]};
  const int64_t x = poisson(r, *c);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if ((threadIdx.x & 63) == 0) {
    hdr_rng[0] = r.s.hi;
    hdr_rng[1] = r.s.lo;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return x;
}

// ---------------------------------------------------- pairwise summation --
// numpy DOUBLE_pairwise_sum (loops_utils.h.src, PW_BLOCKSIZE 128) of
// f(0..n-1) by one wave. Leaves (<= 128 elements: 8 interleaved accumulator
// chains, an ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) combine, a sequential tail)
// run lane-parallel (8 lanes per leaf); the split n2 = n/2 - (n/2)%8 is
// enumerated and the partial sums combined by lane 0 alone on small LDS
// stacks, so no cross-lane hand-off happens inside the recursion.
struct PwLds {
  int32_t *lo, *len;  // leaf list (DFS order), n_leaf entries
  int32_t *stk;       // lane-0 stack, 3 * 64 ints
  double *acc;        // 8 accumulators per leaf
  double *val;        // leaf sums, + value stack
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
  double *vs = S.val + nl;  // value stack after the leaf sums
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

template <class F>
__device__ __forceinline__ double wave_pw_sum(int n, F f, const PwLds &S) {
  const int lane = lane_id();
  int nl = 1;
  if (n > 128) {
    if (lane == 0) S.stk[191] = pw_plan(n, S);
    wsync();
    nl = S.stk[191];
  }
  const int j = lane & 7;
  for (int b = 0; b < nl; b += 8) {  // accumulator chains, 8 leaves per pass
    const int l = b + (lane >> 3);
    if (l < nl) {
      const int o = nl == 1 ? 0 : S.lo[l], m = nl == 1 ? n : S.len[l];
      const int full = m - (m % 8);
      double r = 0.0;
      if (m >= 8) {
        r = f(o + j);
        for (int i = o + j + 8; i < o + full; i += 8) r += f(i);
      }
      S.acc[l * 8 + j] = r;
    }
  }
  wsync();
  for (int l = lane; l < nl; l += 64) {  // leaf combine + sequential tail
    const int o = nl == 1 ? 0 : S.lo[l], m = nl == 1 ? n : S.len[l];
    const double *a = S.acc + l * 8;
    double res;
    int i0;
    if (m < 8) {
      res = 0.0;
      i0 = o;
    } else {
      res = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
      i0 = o + m - (m % 8);
    }
    for (int i = i0; i < o + m; i++) res += f(i);
    S.val[l] = res;
  }
  wsync();
  if (nl > 1) {
    if (lane == 0) S.val[nl] = pw_combine(n, S, nl);
    wsync();
  }
  const double r = S.val[nl > 1 ? nl : 0];
  wsync();
  return r;
}

// ------------------------------------------- numpy scalar argsort (BF) ----
// aquicksort_<float_tag> / aheapsort_ (npysort), run by ONE lane on LDS
// arrays (index form of the pointer algorithm); stack arrays live in LDS.
__device__ __forceinline__ bool fless(float a, float b) { return a < b || (b != b && a == a); }

__device__ void aheapsort_lds(const float *v, uint16_t *tosort, int n) {
  uint16_t *a = tosort - 1;
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

__device__ __noinline__ void aquicksort_lds(const float *v, uint16_t *t, int num, int32_t *stack) {
  int32_t *depth = stack + 128;
  int pl = 0, pr = num - 1;
  int sp = 0, dp = 0;
  int cdepth = 0;
  for (int u = num; u >>= 1;) cdepth++;
  cdepth *= 2;
  for (;;) {
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

// --------------------------------------------------------- env kernel ----
// Per-wave LDS carve (offsets from EnvParams, computed by the host).
struct Lds {
  EnvHdr *hdr;             // the env's 256-B header (scalars, RNG streams)
  double *cpu, *mem;       // f64[P] PM resources (the env state)
  float *fcpu, *fmem;      // f32[P] observation view used by the heuristics
  float *fkey;             // BF keys fcpu + fmem
  uint8_t *tc, *tm;        // per-PM largest fitting size (hundredths), f32 semantics
  uint16_t *ord;           // BF ascending argsort, then reversed into visiting order
  uint64_t *bc, *bm;       // [101][NW] fit bitmaps by size (bit = visiting position)
  int32_t *sortstk;        // introsort stacks
  uint64_t *stage;         // 64 staged accepted-VM words
  uint8_t *ccomp, *mcomp;  // compressed sizes of existing VMs [V]
  PwLds pw;
};

// Exact k/100 for k = 0..127 (np.around(., 2) values), per block.
struct Tables {
  double cent[128];
  float fcent[128];
};

__device__ __forceinline__ int w_pl(uint32_t w) { return (int)(w & 0xFFFFu); }
__device__ __forceinline__ int w_cc(uint32_t w) { return (int)((w >> 16) & 0xFFu); }
__device__ __forceinline__ int w_cm(uint32_t w) { return (int)(w >> 24); }
__device__ __forceinline__ uint32_t w_make(int pl, int cc, int cm) {
  return (uint32_t)pl | ((uint32_t)cc << 16) | ((uint32_t)cm << 24);
}

__device__ __forceinline__ Pcg ld_pcg(const EnvHdr *h, int k) {
  Pcg r;
  r.s = U128{h->rng[k][0], h->rng[k][1]};
  r.inc = U128{h->rng[k][2], h->rng[k][3]};
  return r;
}
__device__ __forceinline__ void st_pcg(EnvHdr *h, int k, const Pcg &r) {
  if (lane_id() == 0) {
    h->rng[k][0] = r.s.hi;
    h->rng[k][1] = r.s.lo;
  }
}

// Largest k in [0, 100] with f + FC[k] <= 1 in f32 (monotone in k), or -1.
__device__ __forceinline__ int fit_threshold(float f, const float *fc) {
  if (!(f + fc[0] <= 1.0f)) return -1;
  int lo = 0, hi = 101;
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (f + fc[mid] <= 1.0f) lo = mid; else hi = mid;
  }
  return lo;
}

// Rebuild the fit bitmaps: bit i of bc[k][w] is set iff the PM at visiting
// position w*64+i accepts a VM of cpu size k/100 (f32 obs arithmetic).
__device__ __forceinline__ void build_bitmaps(const EnvParams &p, const Lds &L, bool bf) {
  const int lane = lane_id();
  const int P = p.P, NW = p.NW;
  for (int w = 0; w < NW; w++) {
    int pos = w * 64 + lane;
    int q = pos < P ? (bf ? (int)L.ord[pos] : pos) : 0;
    int tcq = pos < P ? (int)L.tc[q] - 1 : -1;
    int tmq = pos < P ? (int)L.tm[q] - 1 : -1;
    uint64_t c0 = 0, c1 = 0, m0 = 0, m1 = 0;
    for (int k = 0; k < 101; k++) {
      uint64_t bcw = ballot(tcq >= k), bmw = ballot(tmq >= k);
      if ((k & 63) == lane) {
        if (k < 64) { c0 = bcw; m0 = bmw; } else { c1 = bcw; m1 = bmw; }
      }
    }
    L.bc[lane * NW + w] = c0;
    L.bm[lane * NW + w] = m0;
    if (lane + 64 < 101) {
      L.bc[(lane + 64) * NW + w] = c1;
      L.bm[(lane + 64) * NW + w] = m1;
    }
  }
  wsync();
}

// First visiting position accepting sizes (kc, km), or -1.
__device__ __forceinline__ int bm_query(const Lds &L, int NW, int kc, int km) {
  for (int w = 0; w < NW; w++) {
    uint64_t m = L.bc[kc * NW + w] & L.bm[km * NW + w];
    if (m) return w * 64 + __ffsll((unsigned long long)m) - 1;
  }
  return -1;
}

__device__ __forceinline__ void bf_sort(const EnvParams &p, const Lds &L) {
  const int lane = lane_id();
  const int P = p.P;
  for (int i = lane; i < P; i += 64) L.fkey[i] = L.fcpu[i] + L.fmem[i];
  wsync();
  if (lane == 0) {
    for (int i = 0; i < P; i++) L.ord[i] = (uint16_t)i;
    aquicksort_lds(L.fkey, L.ord, P, L.sortstk);
    // reverse in place: np.flip(argsort) = visiting order
    for (int i = 0, j = P - 1; i < j; i++, j--) {
      uint16_t x = L.ord[i];
      L.ord[i] = L.ord[j];
      L.ord[j] = x;
    }
  }
  wsync();
}

// One VM placement event of the env (env.py:74-84 for a WAIT -> PM move):
// _resource_valid in f64, then _place_vm. Returns validity (wave-uniform).
__device__ __forceinline__ bool env_place(const Lds &L, const Tables &T, int q, int kc, int km) {
  double cq = L.cpu[q], mq = L.mem[q];
  double vc = T.cent[kc], vm = T.cent[km];
  bool ok = (cq + vc <= 1) && (mq + vm <= 1);
  wsync();
  if (ok && lane_id() == 0) {
    L.cpu[q] = cq + vc;
    L.mem[q] = mq + vm;
  }
  wsync();
  return ok;
}

// FirstFitAgent.act / BestFitAgent.act (firstfit.py:21-38, bestfit.py:21-40)
// on the pre-step f32 observation, fused with the action phase of step().
// Exact w.r.t. the reference's sequential loop because:
//  - a waiting VM's choice is "first visiting position whose PM fits", answered
//    in O(P/64) from per-size fit bitmaps; the earliest VM (index order) with a
//    fit wins; VMs before it never fit again (loads only grow);
//  - the heuristic's state (f32 view) and the env's state (f64) are disjoint,
//    so applying each winner's env event as soon as it is decided equals
//    deciding every action first and stepping afterwards (env.py:68-88).
template <int VPT>
__device__ __forceinline__ int64_t heuristic_apply(const EnvParams &p, const Lds &L, const Tables &T,
                                   uint32_t (&wa)[VPT], int policy, int32_t *act_out,
                                   uint8_t *valid_out) {
  const int lane = lane_id();
  const int P = p.P, V = p.V, WAIT = p.P, NW = p.NW;
  const bool bf = policy == 1;
  uint32_t pend = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++)
    if (s * 64 + lane < V && w_pl(wa[s]) == WAIT) pend |= 1u << s;
  uint32_t won = 0, bad = 0;
  int64_t n_place = 0;
  if (ballot(pend != 0)) {
    for (int i = lane; i < P; i += 64) {
      float fcv = (float)L.cpu[i], fmv = (float)L.mem[i];
      L.fcpu[i] = fcv;
      L.fmem[i] = fmv;
      L.tc[i] = (uint8_t)(fit_threshold(fcv, T.fcent) + 1);
      L.tm[i] = (uint8_t)(fit_threshold(fmv, T.fcent) + 1);
    }
    wsync();
    if (bf) bf_sort(p, L);
    build_bitmaps(p, L, bf);
    for (;;) {
      int ws = -1, wl = 0, wpos = 0;
#pragma unroll
      for (int s = 0; s < VPT; s++) {
        bool pd = (pend >> s) & 1u;
        int pos = pd ? bm_query(L, NW, w_cc(wa[s]), w_cm(wa[s])) : -1;
        uint64_t m = ballot(pos >= 0);
        if (ws < 0 && m) {
          ws = s;
          wl = __ffsll((unsigned long long)m) - 1;
          wpos = __builtin_amdgcn_readlane(pos, wl);
        }
      }
      if (ws < 0) break;
      // everything up to and including the winner is decided
#pragma unroll
      for (int s = 0; s < VPT; s++)
        if (s < ws || (s == ws && lane <= wl)) pend &= ~(1u << s);
      uint32_t ww = 0;
#pragma unroll
      for (int s = 0; s < VPT; s++)
        if (s == ws) ww = rdlane(wa[s], wl);
      const int kc = w_cc(ww), km = w_cm(ww);
      const int q = bf ? (int)L.ord[wpos] : wpos;
      // env event, f64 (env.py:55-56, 58-64)
      bool ok = env_place(L, T, q, kc, km);
      n_place += ok;
      if (lane == wl) {
#pragma unroll
        for (int s = 0; s < VPT; s++)
          if (s == ws) {
            won |= 1u << s;
            if (ok) wa[s] = (wa[s] & 0xFFFF0000u) | (uint32_t)q;
            else bad |= 1u << s;
          }
        if (act_out) act_out[ws * 64 + wl] = q;
      }
      // heuristic state update (f32): FF updates cpu only (firstfit.py:36)
      if (lane == 0) {
        float nc = L.fcpu[q] + T.fcent[kc];
        L.fcpu[q] = nc;
        L.tc[q] = (uint8_t)(fit_threshold(nc, T.fcent) + 1);
        if (bf) {
          float nm = L.fmem[q] + T.fcent[km];
          L.fmem[q] = nm;
          L.tm[q] = (uint8_t)(fit_threshold(nm, T.fcent) + 1);
        }
      }
      wsync();
      if (bf) {
        bf_sort(p, L);
        build_bitmaps(p, L, true);
      } else {  // only PM q's bit changes, for sizes above its new threshold
        const int t = (int)L.tc[q] - 1;
        const int w = q >> 6;
        const uint64_t bit = 1ull << (q & 63);
        for (int k = lane; k < 101; k += 64) {
          uint64_t x = L.bc[k * NW + w];
          L.bc[k * NW + w] = (t >= k) ? (x | bit) : (x & ~bit);
        }
        wsync();
      }
    }
  }
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    int v = s * 64 + lane;
    if (v < V) {
      if (act_out && !((won >> s) & 1u)) act_out[v] = (int32_t)w_pl(wa[s]);
      if (valid_out) valid_out[v] = (uint8_t)!((bad >> s) & 1u);
    }
  }
  return n_place;
}

// Action phase of step() for external actions (env.py:68-88): per slot of 64
// VMs, the events (WAIT -> PM place attempts, PM -> WAIT suspends) are applied
// in ascending VM order by a wave-uniform loop over the ballot.
template <int VPT>
__device__ __forceinline__ void external_apply(const EnvParams &p, const Lds &L, const Tables &T,
                               uint32_t (&wa)[VPT], const int32_t *act_row, uint8_t *valid_out,
                               int64_t &n_place, int64_t &n_susp) {
  const int lane = lane_id();
  const int P = p.P, V = p.V, WAIT = p.P;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const int v = s * 64 + lane;
    const bool in = v < V;
    const int c = w_pl(wa[s]);
    const int t = in ? act_row[v] : c;
    const bool isplace = in && c == WAIT && t >= 0 && t < P;
    const bool issusp = in && c < P && t == WAIT;
    uint64_t evm = ballot(isplace || issusp);
    uint64_t okm = 0;
    const uint32_t me = wa[s];
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
      }
      okm |= (uint64_t)eok << l;
      wsync();
    }
    bool ok = (t == c) || issusp;
    if (isplace) ok = (okm >> lane) & 1ull;
    n_place += __popcll(okm & ballot(isplace));
    n_susp += __popcll(ballot(issusp));
    if (ok && t != c && in) wa[s] = (wa[s] & 0xFFFF0000u) | (uint32_t)t;
    if (valid_out && in) valid_out[v] = (uint8_t)ok;
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

// kl reward branch (env.py:124-149), out of line: it runs only for
// reward_function == "kl" and is register-heavy (six reductions, log/exp).
__device__ __forceinline__ double kl_block(const double *cpu, const double *mem, int P,
                                        const uint8_t *ccp, const uint8_t *cmp,
                                        const double *cent, int n_ex, double sum_c,
                                        double sum_m, double tcm, double tmm, PwLds S) {
  const double cm_ = wave_pw_sum(P, [=](int i) { return cpu[i]; }, S) / (double)P;
  const double mm_ = wave_pw_sum(P, [=](int i) { return mem[i]; }, S) / (double)P;
  double cv = wave_pw_sum(P, [=](int i) { double d = cpu[i] - cm_; return d * d; }, S) /
              (double)P;
  double mv = wave_pw_sum(P, [=](int i) { double d = mem[i] - mm_; return d * d; }, S) /
              (double)P;
  if (cv == 0) cv = 1e-6;
  if (mv == 0) mv = 1e-6;
  const double mc = sum_c / (double)n_ex, mmv = sum_m / (double)n_ex;
  double tcv = wave_pw_sum(n_ex, [=](int i) { double d = cent[ccp[i]] - mc; return d * d; }, S) /
               (double)n_ex;
  double tmv = wave_pw_sum(n_ex, [=](int i) { double d = cent[cmp[i]] - mmv; return d * d; }, S) /
               (double)n_ex;
  if (tcv == 0) tcv = 1e-6;
  if (tmv == 0) tmv = 1e-6;
  return (tcm == 0 || tmm == 0) ? 0.0 : kl_reward(tcm, tmm, tcv, tmv, cm_, mm_, cv, mv);
}

// Everything of step() after the action phase: _run_vms, _accept_vm_requests,
// stats + reward, termination (env.py:101, 108-163, 244-293).
template <int VPT>
__device__ __forceinline__ double env_tail(const EnvParams &p, const Lds &L, const Tables &T,
                           uint32_t (&wa)[VPT], uint32_t (&rem)[VPT], bool &terminated) {
  const int lane = lane_id();
  const int P = p.P, V = p.V, WAIT = p.P, NUL = p.P + 1;
  EnvHdr *H = L.hdr;
  // ---- _run_vms (env.py:244-268) ----
  int64_t n_term = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const bool in = s * 64 + lane < V;
    const bool running = in && w_pl(wa[s]) < P;
    if (running && rem[s] > 0) rem[s] -= 1;
    const bool term = running && rem[s] == 0;
    uint64_t it = ballot(term);
    n_term += __popcll(it);
    const uint32_t me = wa[s];
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
      }
      wsync();
    }
    if (term) {
      wa[s] = w_make(NUL, 0, 0);
      rem[s] = 0;
    }
  }
  for (int i = lane; i < P; i += 64) {  // precision clamp (env.py:267-268)
    if (L.cpu[i] < 1e-7) L.cpu[i] = 0;
    if (L.mem[i] < 1e-7) L.mem[i] = 0;
  }
  // ---- _accept_vm_requests (env.py:271-293) ----
  const int64_t arrivals = poisson_lds(H->rng[2], p.pois + 0);
  int n_null = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++)
    n_null += __popcll(ballot(s * 64 + lane < V && w_pl(wa[s]) == NUL));
  const int64_t k = arrivals < n_null ? arrivals : n_null;
  wsync();
  if (k > 0) {
    // ranks of the NULL slots in ascending VM order (to_accept, env.py:276-277)
    int rk[VPT];
    int base = 0;
#pragma unroll
    for (int s = 0; s < VPT; s++) {
      const bool isnull = s * 64 + lane < V && w_pl(wa[s]) == NUL;
      const uint64_t nm = ballot(isnull);
      rk[s] = isnull ? base + below(nm, lane) : -1;
      base += __popcll(nm);
    }
    // draws in to_accept order, 64 per chunk: sizes from rng1/rng2 (the popped
    // sequences, env.py:279-287) and planned runtimes from rng4 (env.py:289)
    for (int c0 = 0; c0 < k; c0 += 64) {
      const int cn = (int)(k - c0 < 64 ? k - c0 : 64);
      Pcg r1 = ld_pcg(H, 0), r2 = ld_pcg(H, 1);
      for (int j = 0; j < cn; j++) {
        const int cc = (int)rint((p.seq_lo + p.seq_range * next_double(r1)) * 100.0);
        const int cm = (int)rint((p.seq_lo + p.seq_range * next_double(r2)) * 100.0);
        const uint32_t rr = (uint32_t)(poisson_lds(H->rng[3], p.pois + 1) + 1);
        if (lane == 0) {
          L.stage[j] = (uint64_t)w_make(WAIT, cc, cm) | ((uint64_t)rr << 32);
          L.ccomp[c0 + j] = (uint8_t)cc;
          L.mcomp[c0 + j] = (uint8_t)cm;
        }
      }
      st_pcg(H, 0, r1);
      st_pcg(H, 1, r2);
      wsync();
#pragma unroll
      for (int s = 0; s < VPT; s++) {
        if (rk[s] >= c0 && rk[s] < c0 + cn) {
          const uint64_t w = L.stage[rk[s] - c0];
          wa[s] = (uint32_t)w;
          rem[s] = (uint32_t)(w >> 32);
        }
      }
      wsync();
    }
    const uint8_t *ccp = L.ccomp, *cmp = L.mcomp;
    const double *cent = T.cent;
    const double sc = wave_pw_sum((int)k, [=](int i) { return cent[ccp[i]]; }, L.pw);
    const double sm = wave_pw_sum((int)k, [=](int i) { return cent[cmp[i]]; }, L.pw);
    if (lane == 0) {
      H->total_cpu_req = H->total_cpu_req + sc;
      H->total_mem_req = H->total_mem_req + sm;
    }
  }
  // ---- stats + reward (env.py:112-156) ----
  int n_ex = 0, n_w = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const bool in = s * 64 + lane < V;
    const int c = w_pl(wa[s]);
    const uint64_t em = ballot(in && c <= WAIT);
    if (in && c <= WAIT) {
      const int rk = n_ex + below(em, lane);
      L.ccomp[rk] = (uint8_t)w_cc(wa[s]);
      L.mcomp[rk] = (uint8_t)w_cm(wa[s]);
    }
    n_ex += __popcll(em);
    n_w += __popcll(ballot(in && c == WAIT));
  }
  wsync();
  const double wr = n_ex > 0 ? (double)n_w / (double)n_ex : 0.0;
  const uint8_t *ccp = L.ccomp, *cmp = L.mcomp;
  const double *cent = T.cent;
  const double sum_c = wave_pw_sum(n_ex, [=](int i) { return cent[ccp[i]]; }, L.pw);
  const double sum_m = wave_pw_sum(n_ex, [=](int i) { return cent[cmp[i]]; }, L.pw);
  double tcm = sum_c / (double)P;
  if (p.cap_target_util && tcm > 1) tcm = 1.0;
  double tmm = sum_m / (double)P;
  if (p.cap_target_util && tmm > 1) tmm = 1.0;
  double reward = 0.0;
  if (n_ex > 0) {
    const double *cpu = L.cpu, *mem = L.mem;
    if (p.reward == 2) {  // kl
      reward = kl_block(cpu, mem, P, ccp, cmp, cent, n_ex, sum_c, sum_m, tcm, tmm, L.pw);
    } else if (p.reward == 1) {  // ut
      const double sc = wave_pw_sum(P, [=](int i) { return cpu[i]; }, L.pw);
      const double sm = wave_pw_sum(P, [=](int i) { return mem[i]; }, L.pw);
      reward = p.beta * sc + (1 - p.beta) * sm;
    } else {  // wr
      reward = -wr;
    }
  }
  // ---- counters, termination (env.py:160-163, 101) ----
  const int64_t ts = H->timestep;
  terminated = ts >= p.limit;
  wsync();
  if (lane == 0) {
    H->timestep = ts + 1;
    H->total_requests += arrivals;
    H->served += n_term;
    H->dropped += arrivals - k;
    H->waiting_ratio = wr;
    H->tcm = tcm;
    H->tmm = tmm;
  }
  wsync();
  return reward;
}

template <int VPT>
__device__ __forceinline__ void write_obs(const EnvParams &p, const Lds &L, const Tables &T,
                          const uint32_t (&wa)[VPT], float *obs) {
  const int lane = lane_id();
  const int V = p.V, P = p.P;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const int v = s * 64 + lane;
    if (v < V) {
      obs[v] = (float)w_pl(wa[s]);
      obs[V + v] = T.fcent[w_cc(wa[s])];
      obs[2 * V + v] = T.fcent[w_cm(wa[s])];
    }
  }
  for (int i = lane; i < P; i += 64) {
    obs[3 * V + i] = (float)L.cpu[i];
    obs[3 * V + P + i] = (float)L.mem[i];
  }
}

// get_invalid_action_mask(masked=True) (env.py:45-53), bit-packed, 1 = invalid.
template <int VPT>
__device__ __forceinline__ void write_mask(const EnvParams &p, const Lds &L, const Tables &T,
                           const uint32_t (&wa)[VPT], uint32_t *bits) {
  const int lane = lane_id();
  const int V = p.V, P = p.P, A = p.A, W = p.W32, WAIT = p.P, NUL = p.P + 1;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const int v = s * 64 + lane;
    const bool in = v < V;
    const int c = in ? w_pl(wa[s]) : NUL;
    const double vc = T.cent[w_cc(wa[s])], vm = T.cent[w_cm(wa[s])];
    const bool waiting = in && c == WAIT;
    const bool anyw = ballot(waiting) != 0;
    for (int w = 0; w < W; w++) {
      uint32_t word = 0xFFFFFFFFu;
      const int a0 = w * 32;
      if (c >= a0 && c < a0 + 32 && c < A) word &= ~(1u << (c - a0));  // stay
      if (c < P && WAIT >= a0 && WAIT < a0 + 32) word &= ~(1u << (WAIT - a0));  // suspend
      if (anyw) {
        const int hi = min(a0 + 32, P);
        for (int q = a0; q < hi; q++) {  // uniform q: LDS broadcast reads
          const bool fit = (L.cpu[q] + vc <= 1) && (L.mem[q] + vm <= 1);
          if (waiting && fit) word &= ~(1u << (q - a0));
        }
      }
      if (in) bits[(int64_t)v * W + w] = word;
    }
  }
}

template <int VPT>
__global__ __launch_bounds__(256, VMP_WAVES_PER_EU) void k_env(EnvParams p, StepOut o) {
  extern __shared__ __align__(16) char lds[];
  __shared__ Tables T;
  for (int i = threadIdx.x; i < 128; i += blockDim.x) {
    T.cent[i] = (double)i / 100.0;
    T.fcent[i] = (float)((double)i / 100.0);
  }
  __syncthreads();  // the only block-wide barrier: waves are independent below
  const int lane = lane_id();
  const int wid = threadIdx.x >> 6;
  const int e = uni(blockIdx.x * kWavesPerBlock + wid);
  if (e >= p.N) return;
  char *base = lds + wid * p.lds_wave_bytes;
  Lds L;
  L.hdr = reinterpret_cast<EnvHdr *>(base + p.off_hdr);
  L.cpu = reinterpret_cast<double *>(base + p.off_pm);
  L.mem = L.cpu + p.P;
  L.fcpu = reinterpret_cast<float *>(base + p.off_fpm);
  L.fmem = L.fcpu + p.P;
  L.fkey = L.fmem + p.P;
  L.tc = reinterpret_cast<uint8_t *>(base + p.off_thr);
  L.tm = L.tc + p.P;
  L.ord = reinterpret_cast<uint16_t *>(base + p.off_ord);
  L.bc = reinterpret_cast<uint64_t *>(base + p.off_bits);
  L.bm = L.bc + 101 * p.NW;
  L.sortstk = reinterpret_cast<int32_t *>(base + p.off_sort);
  L.stage = reinterpret_cast<uint64_t *>(base + p.off_stage);
  L.ccomp = reinterpret_cast<uint8_t *>(base + p.off_ccomp);
  L.mcomp = L.ccomp + p.V;
  L.pw.lo = reinterpret_cast<int32_t *>(base + p.off_leaf);
  L.pw.len = L.pw.lo + p.n_leaf;
  L.pw.stk = L.pw.len + p.n_leaf;
  L.pw.acc = reinterpret_cast<double *>(base + p.off_leafval);
  L.pw.val = L.pw.acc + 8 * p.n_leaf;
  const int V = p.V, P = p.P;
  // ---- load: VM words to registers, PM resources + header to LDS ----
  const uint64_t *vmw = p.vmw + (int64_t)e * V;
  uint32_t wa[VPT], rem[VPT];
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    const int v = s * 64 + lane;
    const uint64_t w = v < V ? vmw[v] : (uint64_t)(P + 1);
    wa[s] = (uint32_t)w;
    rem[s] = (uint32_t)(w >> 32);
  }
  const double *pm = p.pm + (int64_t)e * 2 * P;
  for (int i = lane; i < 2 * P; i += 64) L.cpu[i] = pm[i];
  if (lane < 32)
    reinterpret_cast<uint64_t *>(L.hdr)[lane] = reinterpret_cast<const uint64_t *>(p.hdr + e)[lane];
  wsync();
  bool term = false;
  int64_t ndone = 0;
  for (int k = 0; k < o.k_steps; k++) {
    const bool last = k == o.k_steps - 1;
    uint8_t *valid_row = (last && o.valid) ? o.valid + (int64_t)e * V : nullptr;
    int32_t *act_row = (last && o.act_out) ? o.act_out + (int64_t)e * V : nullptr;
    int64_t n_place = 0, n_susp = 0;
    if (o.policy >= 0)
      n_place = heuristic_apply<VPT>(p, L, T, wa, o.policy, act_row, valid_row);
    else
      external_apply<VPT>(p, L, T, wa, o.actions + (int64_t)e * V, valid_row, n_place, n_susp);
    wsync();
    if (lane == 0) {
      L.hdr->place_action += n_place;
      L.hdr->suspend_action += n_susp;
    }
    wsync();
    const double r = env_tail<VPT>(p, L, T, wa, rem, term);
    if (o.reward && lane == 0) o.reward[(int64_t)k * p.N + e] = r;
    ndone += term;
  }
  if (o.k_steps == 0 && o.policy >= 0 && o.act_out) {
    // act only: decide on a scratch copy, the state is not stored
    uint32_t wt[VPT];
#pragma unroll
    for (int s = 0; s < VPT; s++) wt[s] = wa[s];
    heuristic_apply<VPT>(p, L, T, wt, o.policy, o.act_out + (int64_t)e * V, nullptr);
    for (int i = lane; i < 2 * P; i += 64) L.cpu[i] = pm[i];  // undo env events
    wsync();
  }
  if (o.obs) write_obs<VPT>(p, L, T, wa, o.obs + (int64_t)e * p.D);
  if (o.mask_bits) write_mask<VPT>(p, L, T, wa, o.mask_bits + (int64_t)e * V * p.W32);
  if (o.k_steps > 0) {
    if (o.done && lane == 0) o.done[e] = (uint8_t)term;
    if (o.done_count && lane == 0) o.done_count[e] += ndone;
    uint64_t *vmo = p.vmw + (int64_t)e * V;
#pragma unroll
    for (int s = 0; s < VPT; s++) {
      const int v = s * 64 + lane;
      if (v < V) vmo[v] = (uint64_t)wa[s] | ((uint64_t)rem[s] << 32);
    }
    double *pmo = p.pm + (int64_t)e * 2 * P;
    for (int i = lane; i < 2 * P; i += 64) pmo[i] = L.cpu[i];
    if (lane < 32)
      reinterpret_cast<uint64_t *>(p.hdr + e)[lane] = reinterpret_cast<uint64_t *>(L.hdr)[lane];
  }
}

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
  uint64_t nul = (uint64_t)(P + 1);
  for (int v = lane; v < V; v += 64) p.vmw[(int64_t)e * V + v] = nul;
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
    uint64_t w = p.vmw[i];
    if (placement) placement[i] = (int64_t)(w & 0xFFFF);
    if (vm_cpu) vm_cpu[i] = (double)((w >> 16) & 0xFF) / 100.0;
    if (vm_mem) vm_mem[i] = (double)((w >> 24) & 0xFF) / 100.0;
    if (remaining) remaining[i] = (int64_t)(w >> 32);
  }
  int64_t np_ = (int64_t)p.N * p.P;
  if (i < np_) {
    int64_t e = i / p.P, q = i % p.P;
    if (cpu) cpu[i] = p.pm[e * 2 * p.P + q];
    if (mem) mem[i] = p.pm[e * 2 * p.P + p.P + q];
  }
  if (rank && i < p.N) {  // _get_rank (env.py:320-325): distinct PMs hosting a VM
    int64_t r = 0;
    const uint64_t *row = p.vmw + i * p.V;
    for (int q = 0; q < p.P; q++) {
      bool used = false;
      for (int v = 0; v < p.V && !used; v++) used = (int)(row[v] & 0xFFFF) == q;
      r += used;
    }
    rank[i] = r;
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

// ----------------------------------------------------------------- GAE ---
// PPOAgent.update advantage scan (ppo.py:232-243), one lane per env column.
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

// ------------------------------------------------ masked categorical -----
// One wave per (sample, VM) row of A logits: mask to -1e7 (ppo.py:119),
// log-softmax, Gumbel-max sample, log_prob and entropy; per-sample sums by
// atomics on the row's sample. Philox-free counter hash for the uniforms.
__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void k_masked_sample(int B, int V, int A, int W,
                                                       const float *logits,
                                                       const uint32_t *bits, uint64_t seed,
                                                       uint64_t offset, int32_t *action,
                                                       float *lp_row, float *ent_row) {
  const int lane = lane_id();
  const int64_t row = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (row >= (int64_t)B * V) return;
  const float *lg = logits + row * A;
  const uint32_t *mb = bits ? bits + row * W : nullptr;
  float mx = -INFINITY;
  for (int a = lane; a < A; a += 64) {
    float x = lg[a];
    if (mb && ((mb[a >> 5] >> (a & 31)) & 1u)) x = -1e7f;
    mx = fmaxf(mx, x);
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float se = 0.f;
  float best = -INFINITY;
  int bi = 0;
  for (int a = lane; a < A; a += 64) {
    float x = lg[a];
    if (mb && ((mb[a >> 5] >> (a & 31)) & 1u)) x = -1e7f;
    se += expf(x - mx);
    uint64_t h = splitmix(seed ^ splitmix(offset + (uint64_t)row * (uint64_t)A + a));
    float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
    float g = x - logf(-logf(u));
    if (g > best) {
      best = g;
      bi = a;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    se += __shfl_xor(se, o);
    float ob = __shfl_xor(best, o);
    int oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  float lse = mx + logf(se);
  float ent = 0.f;
  for (int a = lane; a < A; a += 64) {
    float x = lg[a];
    if (mb && ((mb[a >> 5] >> (a & 31)) & 1u)) x = -1e7f;
    float lp = x - lse;
    ent -= expf(lp) * lp;
  }
  for (int o = 32; o > 0; o >>= 1) ent += __shfl_xor(ent, o);
  if (lane == 0) {
    float xs = lg[bi];
    if (mb && ((mb[bi >> 5] >> (bi & 31)) & 1u)) xs = -1e7f;
    action[row] = bi;
    lp_row[row] = xs - lse;
    ent_row[row] = ent;
  }
}

// Explicit instantiations used by the host dispatcher.
template __global__ void k_env<1>(EnvParams, StepOut);
template __global__ void k_env<2>(EnvParams, StepOut);
template __global__ void k_env<4>(EnvParams, StepOut);
template __global__ void k_env<8>(EnvParams, StepOut);
template __global__ void k_env<16>(EnvParams, StepOut);

}  // namespace vmp
