// vmp_record.hip — eval-mode Record metrics on the device (src/record.py:34-134
// fed by Base.record_testing_step, src/agents/base.py:131-148), for every env
// of a handle, updated after each recorded step; no per-step host copies.
//
// Per VM slot the recorder keeps the slot's previous placement and the running
// "life" of its current VM: the length n of its status sequence (post-step
// placements <= WAIT since its arrival), the index of its first running status
// (allocated_at, -1 = never) and the WAIT statuses after that index. A life is
// closed when the next VM arrives in the slot (or when metrics are read):
//   pending  = around((allocated_at + 1) / n, 3)   (1.0 if not allocated_at)
//   slowdown = around(waits / (n - allocated_at - 1), 3), 0 if that life is 0
//              (only lives with allocated_at, record.py:67-82)
//   lifetime = n - allocated_at - 1                 (0 if not allocated_at)
// which is record.py's unique_vms_placement split at vm_arrival_steps
// (record.py:33-51): a segment runs from a VM's arrival step to the step
// before the slot's next arrival, NULL statuses filtered out. Rounded rates
// are binned by their integer x1000 value (exact), so means, medians and
// maxima over lives are exact up to the summation order of the mean.
//
// Arrivals are derived, not stored by the env kernel: a slot is a new arrival
// iff its post-step placement is WAIT and it was neither a WAIT VM that stayed
// unplaced nor a running VM that was suspended this step (env.py:68-88,
// 271-293), from the previous placement, the action and its validity.
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/vmp.h"
#include "vmp_layout.h"
#include "vmp_record.h"

namespace vmp {

constexpr int kRecBins = VMP_REC_BINS;  // rates rounded to 3 decimals: 0.000 .. 1.000

__device__ __forceinline__ int rate_bin(double x) { return (int)rint(x * 1000.0); }

// Close one life into (hist, life sum/count); a "not allocated_at" life
// (None or 0, record.py's truthiness test) has pending 1.0 and lifetime 0.
__device__ __forceinline__ void close_life(uint32_t n, int32_t al, uint32_t w, uint32_t *hp,
                                           uint32_t *hs, double &life_sum, double &life_cnt) {
  if (n == 0) return;
  life_cnt += 1.0;
  if (al > 0) {
    atomicAdd(hp + rate_bin((al + 1.0) / (double)n), 1u);
    const int64_t life = (int64_t)n - al - 1;
    life_sum += (double)life;
    atomicAdd(hs + (life == 0 ? 0 : rate_bin((double)w / (double)life)), 1u);
  } else {
    atomicAdd(hp + 1000, 1u);
  }
}

__device__ __forceinline__ double wsum(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// One wave per env, after its step.
__global__ __launch_bounds__(256) void k_record(EnvParams p, RecArgs r) {
  extern __shared__ __align__(8) unsigned long long used_lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int e = blockIdx.x * 4 + wid;
  const int NWP = (p.P + 63) / 64;
  unsigned long long *used = used_lds + wid * NWP;
  for (int i = lane; i < NWP; i += 64) used[i] = 0ull;
  __syncthreads();
  if (e >= p.N) return;
  const int V = p.V, P = p.P, WAIT = p.P;
  const int64_t base = (int64_t)e * V;
  uint32_t *hp = r.hist + (int64_t)e * 2 * kRecBins, *hs = hp + kRecBins;
  double life_sum = 0.0, life_cnt = 0.0, sc = 0.0, sm = 0.0;
  for (int v = lane; v < V; v += 64) {
    const uint32_t w = p.vmw[(int64_t)e * vm_pitch(V) + vm_slot_idx(v)];
    const int st = (int)(w & 0xFFFFu);
    const int pv = r.prev[base + v];
    const int a = r.act[base + v];
    const bool ok = r.valid[base + v] != 0;
    const bool placed = pv == WAIT && ok && a < P && a >= 0;
    const bool susp = pv < P && ok && a == WAIT;
    const bool arrival = st == WAIT && !(pv == WAIT && !placed) && !susp;
    uint32_t n = r.life_n[base + v], wt = r.waits[base + v];
    int32_t al = r.alloc[base + v];
    if (arrival) {
      close_life(n, al, wt, hp, hs, life_sum, life_cnt);
      n = 1;
      al = -1;
      wt = 0;
    } else if (st <= WAIT) {
      const uint32_t idx = n++;
      if (st < WAIT) {
        if (al < 0) al = (int32_t)idx;
      } else if (al >= 0) {
        wt++;
      }
    }
    r.life_n[base + v] = n;
    r.alloc[base + v] = al;
    r.waits[base + v] = wt;
    r.prev[base + v] = (uint16_t)st;
    if (st < P) atomicOr(used + (st >> 6), 1ull << (st & 63));
    if (st <= WAIT) {  // env.py:111-121 vms_existing
      sc += (double)((w >> 16) & 0xFFu) / 100.0;
      sm += (double)((w >> 24) & 0xFFu) / 100.0;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  double rank = 0.0;
  for (int i = lane; i < NWP; i += 64) rank += (double)__popcll(used[i]);
  double c1 = 0.0, c2 = 0.0, m1 = 0.0, m2 = 0.0;
  const double *pm = p.pm + (int64_t)e * 2 * P;
  for (int i = lane; i < P; i += 64) {
    const double c = pm[i], m = pm[P + i];
    c1 += c;
    c2 += c * c;
    m1 += m;
    m2 += m * m;
  }
  rank = wsum(rank);
  c1 = wsum(c1);
  c2 = wsum(c2);
  m1 = wsum(m1);
  m2 = wsum(m2);
  // per-step variance over PMs, two-pass as np.var (the PM rows are L2-hot);
  // the cross-env product for exp_performance's variance over seeds reads the
  // other envs' post-step memory rows (all envs have stepped before this launch)
  const double cmean = c1 / P, mmean = m1 / P;
  const bool cross = p.N <= VMP_REC_XMAX;
  double cv = 0.0, mv = 0.0, xm = 0.0;
  for (int i = lane; i < P; i += 64) {
    const double dc = pm[i] - cmean, dm = pm[P + i] - mmean;
    cv += dc * dc;
    mv += dm * dm;
    if (cross) {
      double col = 0.0;
      for (int s = 0; s < p.N; s++) col += p.pm[(int64_t)s * 2 * P + P + i];
      xm += pm[P + i] * col;
    }
  }
  cv = wsum(cv);
  mv = wsum(mv);
  xm = wsum(xm);
  sc = wsum(sc);
  sm = wsum(sm);
  life_sum = wsum(life_sum);
  life_cnt = wsum(life_cnt);
  if (lane == 0) {
    const EnvHdr &h = p.hdr[e];
    double *s = r.sums + (int64_t)e * VMP_NREC;
    double tcm = sc / P, tmm = sm / P;
    if (p.cap_target_util) {
      if (tcm > 1) tcm = 1.0;
      if (tmm > 1) tmm = 1.0;
    }
    s[VMP_REC_STEPS] += 1.0;
    s[VMP_REC_REWARD] += r.reward[e];
    s[VMP_REC_CPU] += c1;
    s[VMP_REC_CPU2] += c2;
    s[VMP_REC_MEM] += m1;
    s[VMP_REC_MEM2] += m2;
    s[VMP_REC_RANK] += rank;
    s[VMP_REC_CPUVAR] += cv / P;
    s[VMP_REC_MEMVAR] += mv / P;
    s[VMP_REC_XMEM] += xm;
    s[VMP_REC_DROP] += h.total_requests ? (double)h.dropped / (double)h.total_requests : 0.0;
    s[VMP_REC_TCM] += tcm;
    s[VMP_REC_TMM] += tmm;
    s[VMP_REC_WAITING] += h.waiting_ratio;
    s[VMP_REC_LIFE_SUM] += life_sum;
    s[VMP_REC_LIVES] += life_cnt;
    const double rw = r.reward[e];  // Record.total_rewards' -1e7 rule (record.py:105-108)
    if (rw > -1e7) {
      s[VMP_REC_REWARD_OK] += rw;
      s[VMP_REC_N_OK] += 1.0;
    } else if (rw < -1e7) {
      s[VMP_REC_N_BAD] += 1.0;
    }
  }
}

// Start recording: previous placement = current, no open lives, zero sums.
__global__ void k_record_init(EnvParams p, RecArgs r) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nv = (int64_t)p.N * p.V;
  if (i < nv) {
    r.prev[i] = (uint16_t)(p.vmw[(i / p.V) * vm_pitch(p.V) + vm_slot_idx((int)(i % p.V))] & 0xFFFFu);
    r.life_n[i] = 0;
    r.alloc[i] = -1;
    r.waits[i] = 0;
  }
  if (i < (int64_t)p.N * 2 * kRecBins) r.hist[i] = 0;
  if (i < (int64_t)p.N * VMP_NREC) r.sums[i] = 0.0;
}

// Read-out (after vmp_record_read copied hist/sums into the caller's buffers):
// close every open life into the copies; the recorder itself is untouched.
__global__ __launch_bounds__(256) void k_record_close(EnvParams p, RecArgs r, uint32_t *hist,
                                                      double *sums) {
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= p.N) return;
  uint32_t *hp = hist + (int64_t)e * 2 * kRecBins, *hs = hp + kRecBins;
  double life_sum = 0.0, life_cnt = 0.0;
  const int64_t base = (int64_t)e * p.V;
  for (int v = lane; v < p.V; v += 64)
    close_life(r.life_n[base + v], r.alloc[base + v], r.waits[base + v], hp, hs, life_sum,
               life_cnt);
  life_sum = wsum(life_sum);
  life_cnt = wsum(life_cnt);
  if (lane == 0) {
    double *s = sums + (int64_t)e * VMP_NREC;
    s[VMP_REC_LIFE_SUM] += life_sum;
    s[VMP_REC_LIVES] += life_cnt;
  }
}

}  // namespace vmp
