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

// random_poisson (distributions.c): mult method (lam < 10) / PTRS (lam >= 10).
__device__ int64_t poisson(Pcg &r, const PoisConst &c) {
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

// ---------------------------------------------------- pairwise summation --
// numpy DOUBLE_pairwise_sum (loops_utils.h.src, PW_BLOCKSIZE 128) over
// f(0..n-1), evaluated by one wave. Leaves (<= 128 elements, 8 interleaved
// accumulators + sequential tail) are computed 8 per pass by lane groups of 8;
// the recursion n2 = n/2 - (n/2)%8 is replayed by a wave-uniform stack
// machine. `scr` is a per-wave LDS scratch of >= 3*(#leaves + 64) words.
struct PwScratch {
  int32_t *lo, *len;  // leaf list
  double *val;        // leaf sums
  int32_t *stk;       // DFS stack (o, n, phase) triples
  double *vstk;       // value stack
};

template <class F>
__device__ __forceinline__ double pw_leaf_group(int o, int m, int j, F &f, int lane) {
  // lanes j = lane&7 of a group: accumulator chain j, then lane j==0 combines.
  double r = 0.0;
  int full = m - (m % 8);
  if (m >= 8) {
    r = f(o + j);
    for (int i = o + j + 8; i < o + full; i += 8) r += f(i);
  }
  int base = lane & ~7;
  double r0 = __shfl(r, base + 0), r1 = __shfl(r, base + 1), r2 = __shfl(r, base + 2),
         r3 = __shfl(r, base + 3), r4 = __shfl(r, base + 4), r5 = __shfl(r, base + 5),
         r6 = __shfl(r, base + 6), r7 = __shfl(r, base + 7);
  double res;
  int i0;
  if (m < 8) {
    res = 0.0;
    i0 = o;
  } else {
    res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    i0 = o + full;
  }
  for (int i = i0; i < o + m; i++) res += f(i);
  return res;
}

template <class F>
__device__ double wave_pw_sum(int n, F f, const PwScratch &S) {
  const int lane = lane_id();
  if (n <= 128) {
    // single leaf: every group computes it, all lanes hold the result
    return pw_leaf_group(0, n, lane & 7, f, lane);
  }
  // 1) enumerate leaves in DFS (left-first) order
  int nleaf = 0, sp = 0;
  S.stk[0] = 0;
  S.stk[1] = n;
  sp = 1;
  wsync();
  while (sp > 0) {
    sp--;
    int o = S.stk[2 * sp], m = S.stk[2 * sp + 1];
    wsync();
    if (m <= 128) {
      if (lane == 0) {
        S.lo[nleaf] = o;
        S.len[nleaf] = m;
      }
      nleaf++;
    } else {
      int n2 = m / 2;
      n2 -= n2 % 8;
      if (lane == 0) {  // push right then left: left is popped first
        S.stk[2 * sp] = o + n2;
        S.stk[2 * sp + 1] = m - n2;
        S.stk[2 * sp + 2] = o;
        S.stk[2 * sp + 3] = n2;
      }
      sp += 2;
    }
    wsync();
  }
  // 2) leaf sums, 8 leaves per pass
  for (int b = 0; b < nleaf; b += 8) {
    int l = b + (lane >> 3);
    int o = 0, m = 0;
    if (l < nleaf) {
      o = S.lo[l];
      m = S.len[l];
    }
    double v = pw_leaf_group(o, m, lane & 7, f, lane);
    if (l < nleaf && (lane & 7) == 0) S.val[l] = v;
  }
  wsync();
  // 3) replay the recursion combining leaf sums: stack of (o, n, phase)
  int leaf = 0, vsp = 0;
  sp = 0;
  S.stk[0] = 0;
  S.stk[1] = n;
  S.stk[2] = 0;
  sp = 1;
  wsync();
  while (sp > 0) {
    sp--;
    int o = S.stk[3 * sp], m = S.stk[3 * sp + 1], ph = S.stk[3 * sp + 2];
    wsync();
    if (m <= 128) {
      double v = S.val[leaf++];
      if (lane == 0) S.vstk[vsp] = v;
      vsp++;
    } else if (ph == 0) {
      int n2 = m / 2;
      n2 -= n2 % 8;
      if (lane == 0) {
        S.stk[3 * sp + 2] = 1;                // revisit after both children
        S.stk[3 * sp + 3] = o + n2;           // right
        S.stk[3 * sp + 4] = m - n2;
        S.stk[3 * sp + 5] = 0;
        S.stk[3 * sp + 6] = o;                // left (popped first)
        S.stk[3 * sp + 7] = n2;
        S.stk[3 * sp + 8] = 0;
      }
      sp += 3;
    } else {
      wsync();
      double b2 = S.vstk[vsp - 1], a2 = S.vstk[vsp - 2];
      wsync();
      if (lane == 0) S.vstk[vsp - 2] = a2 + b2;
      vsp--;
    }
    wsync();
  }
  return S.vstk[0];
}

// ------------------------------------------- numpy scalar argsort (BF) ----
// aquicksort_<float_tag> / aheapsort_ (npysort), run by ONE lane on LDS.
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

__device__ void aquicksort_lds(const float *v, uint16_t *t, int num) {
  // index-based restatement of the pointer algorithm
  int pl = 0, pr = num - 1;
  int stack[64];
  int depth[32];
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
struct WaveLds {
  double *cpu, *mem;       // f64[P] each
  float *fcpu, *fmem;      // f32 copies (obs view) for the heuristics
  float *fkey;             // BF keys
  uint16_t *ord;           // BF visiting order (ascending argsort)
  uint16_t *acts;          // heuristic actions [V]
  uint32_t *list;          // compacted waiting VMs [V]
  uint8_t *ccomp, *mcomp;  // compressed sizes (hundredths) [V]
  PwScratch pw;
};

struct Scal {  // per-env scalars (wave-uniform)
  Pcg rng[4];
  Pcg seqbase[2];
  int64_t timestep, total_requests, served, suspend_action, place_action, dropped;
  double total_cpu_req, total_mem_req, waiting_ratio, tcm, tmm;
};

__device__ __forceinline__ int w_pl(uint32_t w) { return (int)(w & 0xFFFFu); }
__device__ __forceinline__ int w_cc(uint32_t w) { return (int)((w >> 16) & 0xFFu); }
__device__ __forceinline__ int w_cm(uint32_t w) { return (int)(w >> 24); }
__device__ __forceinline__ uint32_t w_make(int pl, int cc, int cm) {
  return (uint32_t)pl | ((uint32_t)cc << 16) | ((uint32_t)cm << 24);
}

__device__ __forceinline__ void load_scal(const EnvHdr *h, Scal &S) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    S.rng[k].s = U128{h->rng[k][0], h->rng[k][1]};
    S.rng[k].inc = U128{h->rng[k][2], h->rng[k][3]};
  }
#pragma unroll
  for (int k = 0; k < 2; k++) {
    S.seqbase[k].s = U128{h->seqbase[k][0], h->seqbase[k][1]};
    S.seqbase[k].inc = S.rng[k].inc;
  }
  S.timestep = h->timestep;
  S.total_requests = h->total_requests;
  S.served = h->served;
  S.suspend_action = h->suspend_action;
  S.place_action = h->place_action;
  S.dropped = h->dropped;
  S.total_cpu_req = h->total_cpu_req;
  S.total_mem_req = h->total_mem_req;
  S.waiting_ratio = h->waiting_ratio;
  S.tcm = h->tcm;
  S.tmm = h->tmm;
}

__device__ __forceinline__ void store_scal(EnvHdr *h, const Scal &S, int lane) {
  // lane-parallel store of the 256-B header
  uint64_t w = 0;
  int k = lane >> 2, q = lane & 3;
  if (lane < 16) {
    const Pcg &r = S.rng[lane >> 2];
    w = q == 0 ? r.s.hi : q == 1 ? r.s.lo : q == 2 ? r.inc.hi : r.inc.lo;
  } else if (lane < 20) {
    const Pcg &r = S.seqbase[(lane - 16) >> 1];
    w = ((lane - 16) & 1) ? r.s.lo : r.s.hi;
  } else if (lane < 32) {
    int f = lane - 20;
    double d = 0.0;
    switch (f) {
      case 0: w = (uint64_t)S.timestep; break;
      case 1: w = (uint64_t)S.total_requests; break;
      case 2: w = (uint64_t)S.served; break;
      case 3: w = (uint64_t)S.suspend_action; break;
      case 4: w = (uint64_t)S.place_action; break;
      case 5: w = (uint64_t)S.dropped; break;
      case 6: d = S.total_cpu_req; w = __double_as_longlong(d); break;
      case 7: d = S.total_mem_req; w = __double_as_longlong(d); break;
      case 8: d = S.waiting_ratio; w = __double_as_longlong(d); break;
      case 9: d = S.tcm; w = __double_as_longlong(d); break;
      case 10: d = S.tmm; w = __double_as_longlong(d); break;
      default: w = 0;
    }
  }
  (void)k;
  if (lane < 32) reinterpret_cast<uint64_t *>(h)[lane] = w;
}

// Exact k/100 for k = 0..100 (np.around(., 2) values), built per block.
struct Tables {
  double cent[128];
  float fcent[128];
};

// The heuristic act (firstfit.py:21-38 / bestfit.py:21-40) on the current
// state's f32 observation view, exact w.r.t. the reference's sequential loop:
//  - every waiting VM's first feasible PM in scan order is found lane-parallel;
//  - the earliest VM (index order) with a feasible PM wins and is applied;
//    VMs before it stay infeasible forever (loads only grow), VMs after it
//    keep their choice unless it was the winner's PM (FF) / always rescan (BF,
//    whose order depends on every key);
//  - repeat until no pending VM has a feasible PM.
// Output: acts[v] in LDS (stay = current placement).
template <int VPT>
__device__ void heuristic_act(const EnvParams &p, const WaveLds &L, const Tables &T,
                              const uint32_t (&wa)[VPT], int policy) {
  const int lane = lane_id();
  const int P = p.P, V = p.V, WAIT = p.P;
  for (int i = lane; i < P; i += 64) {
    L.fcpu[i] = (float)L.cpu[i];
    L.fmem[i] = (float)L.mem[i];
  }
  // compact the waiting VMs in index order; stays for everyone
  int nW = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    int v = s * 64 + lane;
    bool in = v < V;
    int pl = w_pl(wa[s]);
    if (in) L.acts[v] = (uint16_t)pl;
    uint64_t m = ballot(in && pl == WAIT);
    if (in && pl == WAIT) L.list[nW + below(m, lane)] = (uint32_t)v | (wa[s] & 0xFFFF0000u);
    nW += __popcll(m);
  }
  wsync();
  if (nW == 0) return;
  const bool bf = policy == 1;
  // per-lane compacted entries j: idx = j*64 + lane
  int pos[VPT];    // scan position (index into visiting order); P = none
  int stat[VPT];   // 0 = needs scan, 1 = found, 2 = no fit, 3 = won
  float fc[VPT], fm[VPT];
#pragma unroll
  for (int j = 0; j < VPT; j++) {
    int idx = j * 64 + lane;
    uint32_t ent = idx < nW ? L.list[idx] : 0u;
    fc[j] = T.fcent[(ent >> 16) & 0xFF];
    fm[j] = T.fcent[ent >> 24];
    pos[j] = 0;
    stat[j] = idx < nW ? 0 : 3;
  }
  if (bf) {
    for (int i = lane; i < P; i += 64) L.fkey[i] = L.fcpu[i] + L.fmem[i];
    wsync();
    if (lane == 0) {
      for (int i = 0; i < P; i++) L.ord[i] = (uint16_t)i;
      aquicksort_lds(L.fkey, L.ord, P);
    }
    wsync();
  }
  for (;;) {
    // scan pending entries from pos
#pragma unroll
    for (int j = 0; j < VPT; j++) {
      if (stat[j] == 0) {
        int i = pos[j];
        for (; i < P; i++) {
          int q = bf ? (int)L.ord[P - 1 - i] : i;
          if (L.fcpu[q] + fc[j] <= 1.0f && L.fmem[q] + fm[j] <= 1.0f) break;
        }
        pos[j] = i;
        stat[j] = i < P ? 1 : 2;
      }
    }
    // earliest found entry
    int wj = -1, wl = 0;
#pragma unroll
    for (int j = 0; j < VPT; j++) {
      uint64_t m = ballot(stat[j] == 1);
      if (wj < 0 && m) {
        wj = j;
        wl = __ffsll((unsigned long long)m) - 1;
      }
    }
    if (wj < 0) break;
    // winner data to every lane
    int wpos = 0, widx = wj * 64 + wl;
    float wfc = 0.f, wfm = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; j++)
      if (j == wj) {
        wpos = __shfl(pos[j], wl);
        wfc = __shfl(fc[j], wl);
        wfm = __shfl(fm[j], wl);
      }
    int q = bf ? (int)L.ord[P - 1 - wpos] : wpos;
    uint32_t went = L.list[widx];
    wsync();
    if (lane == 0) {
      L.acts[went & 0xFFFF] = (uint16_t)q;
      L.fcpu[q] = L.fcpu[q] + wfc;
      if (bf) L.fmem[q] = L.fmem[q] + wfm;  // FF leaves memory stale (firstfit.py:36)
    }
    wsync();
#pragma unroll
    for (int j = 0; j < VPT; j++) {
      int idx = j * 64 + lane;
      if (idx == widx) stat[j] = 3;
      else if (stat[j] == 1 && idx > widx) {
        if (bf)
          { stat[j] = 0; pos[j] = 0; }
        else if (pos[j] == q)
          stat[j] = 0;  // rescan from the winner's PM on
      }
    }
    if (bf) {
      for (int i = lane; i < P; i += 64) L.fkey[i] = L.fcpu[i] + L.fmem[i];
      wsync();
      if (lane == 0) {
        for (int i = 0; i < P; i++) L.ord[i] = (uint16_t)i;
        aquicksort_lds(L.fkey, L.ord, P);
      }
      wsync();
    }
  }
  wsync();
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

// One VmEnv.step (env.py:66-103) on the wave's env. act_row: external
// actions (global) or null (use L.acts from heuristic_act).
template <int VPT>
__device__ double env_step(const EnvParams &p, const WaveLds &L, const Tables &T, Scal &S,
                           uint32_t (&wa)[VPT], uint32_t (&rem)[VPT], const int32_t *act_row,
                           uint8_t *valid_row, int32_t *act_out_row, bool &terminated) {
  const int lane = lane_id();
  const int P = p.P, V = p.V, WAIT = p.P, NUL = p.P + 1;
  // ---- 1. per-VM validation + apply, VM order (env.py:68-88) ------------
  int64_t n_place = 0, n_susp = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    int v = s * 64 + lane;
    bool in = v < V;
    int c = w_pl(wa[s]);
    int t = c;
    if (in) t = act_row ? act_row[v] : (int)L.acts[v];
    if (act_out_row && in) act_out_row[v] = t;
    bool isplace = in && c == WAIT && t >= 0 && t < P;
    bool issusp = in && c < P && t == WAIT;
    bool ok = (t == c) || issusp;
    uint64_t evm = ballot(isplace || issusp);
    uint64_t okm = 0;
    uint32_t me = wa[s];
    while (evm) {  // wave-uniform, ascending lane = ascending VM index
      int l = __ffsll((unsigned long long)evm) - 1;
      evm &= evm - 1;
      uint32_t ew = rdlane(me, l);
      int et = __builtin_amdgcn_readlane(t, l);
      int ec = w_pl(ew);
      double vc = T.cent[w_cc(ew)], vm = T.cent[w_cm(ew)];
      int q = (ec == WAIT) ? et : ec;
      double cq = L.cpu[q], mq = L.mem[q];
      bool eok = true;
      if (ec == WAIT) {  // place: _resource_valid (env.py:55-56), then _place_vm
        eok = (cq + vc <= 1) && (mq + vm <= 1);
        if (eok) {
          cq = cq + vc;
          mq = mq + vm;
        }
      } else {  // suspend: _free_pm
        cq = cq - vc;
        mq = mq - vm;
      }
      if (lane == 0) {
        L.cpu[q] = cq;
        L.mem[q] = mq;
      }
      okm |= (uint64_t)eok << l;
      wsync();
    }
    if (isplace) ok = (okm >> lane) & 1ull;
    n_place += __popcll(okm & ballot(isplace));
    n_susp += __popcll(ballot(issusp));
    if (ok && t != c && in) wa[s] = (wa[s] & 0xFFFF0000u) | (uint32_t)t;
    if (valid_row && in) valid_row[v] = (uint8_t)ok;
  }
  S.place_action += n_place;
  S.suspend_action += n_susp;
  // ---- 2. _run_vms (env.py:244-268) --------------------------------------
  int64_t n_term = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    int v = s * 64 + lane;
    bool in = v < V;
    int c = w_pl(wa[s]);
    bool running = in && c < P;
    if (running && rem[s] > 0) rem[s] -= 1;
    bool term = running && rem[s] == 0;
    uint64_t tm = ballot(term);
    uint32_t me = wa[s];
    uint64_t it = tm;
    while (it) {
      int l = __ffsll((unsigned long long)it) - 1;
      it &= it - 1;
      uint32_t ew = rdlane(me, l);
      int q = w_pl(ew);
      double cq = L.cpu[q] - T.cent[w_cc(ew)];
      double mq = L.mem[q] - T.cent[w_cm(ew)];
      if (lane == 0) {
        L.cpu[q] = cq;
        L.mem[q] = mq;
      }
      wsync();
    }
    n_term += __popcll(tm);
    if (term) {
      wa[s] = w_make(NUL, 0, 0);
      rem[s] = 0;
    }
  }
  S.served += n_term;
  for (int i = lane; i < P; i += 64) {  // precision clamp (env.py:267-268)
    if (L.cpu[i] < 1e-7) L.cpu[i] = 0;
    if (L.mem[i] < 1e-7) L.mem[i] = 0;
  }
  wsync();
  // ---- 3. _accept_vm_requests (env.py:271-293) ---------------------------
  int64_t arrivals = poisson(S.rng[2], p.arr);
  S.total_requests += arrivals;
  int n_null = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    int v = s * 64 + lane;
    n_null += __popcll(ballot(v < V && w_pl(wa[s]) == NUL));
  }
  int64_t k = arrivals < n_null ? arrivals : n_null;
  if (k > 0) {
    int base = 0;
#pragma unroll
    for (int s = 0; s < VPT; s++) {
      int v = s * 64 + lane;
      bool isnull = v < V && w_pl(wa[s]) == NUL;
      uint64_t nm = ballot(isnull);
      int r = base + below(nm, lane);
      uint64_t am = ballot(isnull && r < k);
      while (am) {  // ascending slot order (rng4 draws in to_accept order)
        int l = __ffsll((unsigned long long)am) - 1;
        am &= am - 1;
        int cc = (int)rint((p.seq_lo + p.seq_range * next_double(S.rng[0])) * 100.0);
        int cm = (int)rint((p.seq_lo + p.seq_range * next_double(S.rng[1])) * 100.0);
        uint32_t rr = (uint32_t)(poisson(S.rng[3], p.svc) + 1);
        if (lane == l) {
          wa[s] = w_make(WAIT, cc, cm);
          rem[s] = rr;
          L.ccomp[r] = (uint8_t)cc;
          L.mcomp[r] = (uint8_t)cm;
        }
      }
      base += __popcll(nm);
    }
    wsync();
    const uint8_t *cc = L.ccomp, *cm = L.mcomp;
    const double *cent = T.cent;
    S.total_cpu_req += wave_pw_sum((int)k, [&](int i) { return cent[cc[i]]; }, L.pw);
    S.total_mem_req += wave_pw_sum((int)k, [&](int i) { return cent[cm[i]]; }, L.pw);
    wsync();
  }
  S.dropped += arrivals - k;
  // ---- 4. stats + reward (env.py:112-156) --------------------------------
  int n_ex = 0, n_w = 0;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    int v = s * 64 + lane;
    bool in = v < V;
    int c = w_pl(wa[s]);
    uint64_t em = ballot(in && c <= WAIT);
    if (in && c <= WAIT) {
      int r = n_ex + below(em, lane);
      L.ccomp[r] = (uint8_t)w_cc(wa[s]);
      L.mcomp[r] = (uint8_t)w_cm(wa[s]);
    }
    n_ex += __popcll(em);
    n_w += __popcll(ballot(in && c == WAIT));
  }
  wsync();
  S.waiting_ratio = n_ex > 0 ? (double)n_w / (double)n_ex : 0.0;
  const uint8_t *ccp = L.ccomp, *cmp = L.mcomp;
  const double *cent = T.cent;
  auto fx = [&](int i) { return cent[ccp[i]]; };
  auto fy = [&](int i) { return cent[cmp[i]]; };
  double sum_c = wave_pw_sum(n_ex, fx, L.pw);
  double sum_m = wave_pw_sum(n_ex, fy, L.pw);
  S.tcm = sum_c / (double)P;
  if (p.cap_target_util && S.tcm > 1) S.tcm = 1.0;
  S.tmm = sum_m / (double)P;
  if (p.cap_target_util && S.tmm > 1) S.tmm = 1.0;
  double reward = 0.0;
  if (n_ex > 0) {
    const double *cpu = L.cpu, *mem = L.mem;
    if (p.reward == 2) {  // kl
      double cm_ = wave_pw_sum(P, [&](int i) { return cpu[i]; }, L.pw) / (double)P;
      double mm_ = wave_pw_sum(P, [&](int i) { return mem[i]; }, L.pw) / (double)P;
      double cv = wave_pw_sum(P, [&](int i) { double d = cpu[i] - cm_; return d * d; }, L.pw) /
                  (double)P;
      double mv = wave_pw_sum(P, [&](int i) { double d = mem[i] - mm_; return d * d; }, L.pw) /
                  (double)P;
      if (cv == 0) cv = 1e-6;
      if (mv == 0) mv = 1e-6;
      double mc = sum_c / (double)n_ex, mmv = sum_m / (double)n_ex;
      double tcv = wave_pw_sum(n_ex, [&](int i) { double d = cent[ccp[i]] - mc; return d * d; },
                               L.pw) / (double)n_ex;
      double tmv = wave_pw_sum(n_ex, [&](int i) { double d = cent[cmp[i]] - mmv; return d * d; },
                               L.pw) / (double)n_ex;
      if (tcv == 0) tcv = 1e-6;
      if (tmv == 0) tmv = 1e-6;
      if (S.tcm == 0 || S.tmm == 0)
        reward = 0.0;
      else
        reward = kl_reward(S.tcm, S.tmm, tcv, tmv, cm_, mm_, cv, mv);
    } else if (p.reward == 1) {  // ut
      double sc = wave_pw_sum(P, [&](int i) { return cpu[i]; }, L.pw);
      double sm = wave_pw_sum(P, [&](int i) { return mem[i]; }, L.pw);
      reward = p.beta * sc + (1 - p.beta) * sm;
    } else {  // wr
      reward = -S.waiting_ratio;
    }
  }
  wsync();
  // ---- 5. termination (env.py:160-163, 101) ------------------------------
  terminated = S.timestep >= p.limit;
  S.timestep += 1;
  return reward;
}

template <int VPT>
__device__ void write_obs(const EnvParams &p, const WaveLds &L, const Tables &T,
                          const uint32_t (&wa)[VPT], float *obs) {
  const int lane = lane_id();
  const int V = p.V, P = p.P;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    int v = s * 64 + lane;
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
__device__ void write_mask(const EnvParams &p, const WaveLds &L, const Tables &T,
                           const uint32_t (&wa)[VPT], uint32_t *bits) {
  const int lane = lane_id();
  const int V = p.V, P = p.P, A = p.A, W = p.W32, WAIT = p.P, NUL = p.P + 1;
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    int v = s * 64 + lane;
    bool in = v < V;
    int c = in ? w_pl(wa[s]) : NUL;
    double vc = T.cent[w_cc(wa[s])], vm = T.cent[w_cm(wa[s])];
    bool waiting = in && c == WAIT;
    bool anyw = ballot(waiting) != 0;
    for (int w = 0; w < W; w++) {
      uint32_t word = 0xFFFFFFFFu;  // all invalid
      int a0 = w * 32;
      // statically valid entries: stay, and running -> WAIT
      if (c >= a0 && c < a0 + 32 && c < A) word &= ~(1u << (c - a0));
      if (c < P && WAIT >= a0 && WAIT < a0 + 32) word &= ~(1u << (WAIT - a0));
      if (anyw) {
        int hi = min(a0 + 32, P);
        for (int q = a0; q < hi; q++) {  // uniform q: LDS broadcast reads
          bool fit = (L.cpu[q] + vc <= 1) && (L.mem[q] + vm <= 1);
          if (waiting && fit) word &= ~(1u << (q - a0));
        }
      }
      // bits beyond A stay set (never valid)
      if (in) bits[(int64_t)v * W + w] = word;
    }
  }
}

template <int VPT>
__global__ __launch_bounds__(256) void k_env(EnvParams p, StepOut o) {
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
  WaveLds L;
  L.cpu = reinterpret_cast<double *>(base + p.off_pm);
  L.mem = L.cpu + p.P;
  L.fcpu = reinterpret_cast<float *>(base + p.off_fpm);
  L.fmem = L.fcpu + p.P;
  L.fkey = L.fmem + p.P;
  L.ord = reinterpret_cast<uint16_t *>(base + p.off_ord);
  L.acts = L.ord + p.P;
  L.list = reinterpret_cast<uint32_t *>(base + p.off_list);
  L.ccomp = reinterpret_cast<uint8_t *>(base + p.off_ccomp);
  L.mcomp = reinterpret_cast<uint8_t *>(base + p.off_mcomp);
  {
    int32_t *lf = reinterpret_cast<int32_t *>(base + p.off_leaf);
    int nl = (p.V + 63) / 64 + 8;
    L.pw.lo = lf;
    L.pw.len = lf + nl;
    L.pw.stk = lf + 2 * nl;
    L.pw.val = reinterpret_cast<double *>(base + p.off_tmp);
    L.pw.vstk = L.pw.val + nl;
  }
  const int V = p.V, P = p.P;
  const uint64_t *vmw = p.vmw + (int64_t)e * V;
  const double *pm = p.pm + (int64_t)e * 2 * P;
  // ---- load state: VM words to registers, PM resources to LDS ----
  uint32_t wa[VPT], rem[VPT];
#pragma unroll
  for (int s = 0; s < VPT; s++) {
    int v = s * 64 + lane;
    uint64_t w = v < V ? vmw[v] : (uint64_t)(P + 1);
    wa[s] = (uint32_t)w;
    rem[s] = (uint32_t)(w >> 32);
  }
  for (int i = lane; i < 2 * P; i += 64) L.cpu[i] = pm[i];
  Scal S;
  load_scal(p.hdr + e, S);
  wsync();
  bool term = false;
  int64_t ndone = 0;
  for (int k = 0; k < o.k_steps; k++) {
    const bool last = k == o.k_steps - 1;
    const int32_t *act_row = nullptr;
    if (o.policy >= 0)
      heuristic_act<VPT>(p, L, T, wa, o.policy);
    else
      act_row = o.actions + (int64_t)e * V;
    double r = env_step<VPT>(p, L, T, S, wa, rem, act_row,
                             (last && o.valid) ? o.valid + (int64_t)e * V : nullptr,
                             (last && o.act_out) ? o.act_out + (int64_t)e * V : nullptr, term);
    if (o.reward && lane == 0) o.reward[(int64_t)k * p.N + e] = r;
    ndone += term;
  }
  if (o.k_steps == 0 && o.policy >= 0 && o.act_out) {  // act only (no step)
    heuristic_act<VPT>(p, L, T, wa, o.policy);
    for (int v = lane; v < V; v += 64) o.act_out[(int64_t)e * V + v] = L.acts[v];
  }
  if (o.obs) write_obs<VPT>(p, L, T, wa, o.obs + (int64_t)e * p.D);
  if (o.mask_bits) write_mask<VPT>(p, L, T, wa, o.mask_bits + (int64_t)e * V * p.W32);
  if (o.k_steps > 0) {
    if (o.done && lane == 0) o.done[e] = (uint8_t)term;
    if (o.done_count && lane == 0) o.done_count[e] += ndone;
    uint64_t *vmo = p.vmw + (int64_t)e * V;
#pragma unroll
    for (int s = 0; s < VPT; s++) {
      int v = s * 64 + lane;
      if (v < V) vmo[v] = (uint64_t)wa[s] | ((uint64_t)rem[s] << 32);
    }
    double *pmo = p.pm + (int64_t)e * 2 * P;
    for (int i = lane; i < 2 * P; i += 64) pmo[i] = L.cpu[i];
    store_scal(p.hdr + e, S, lane);
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
