// vmp_layout.h — device-resident state layout and launch parameters shared by
// the HIP kernels (vmp_kernels.hip) and the C-ABI host side (vmp_capi.cpp).
//
// HBM layout, env-major so one wavefront streams one env's state with
// coalesced 64-lane accesses (one wave per env):
//
//   vmw  u32 [N][VB][2][64]  two 32-bit words per VM slot (env.py:186-196
//                       state, 8 B/VM), in blocks of 64 slots (VB = ceil(V/64)):
//                       block b holds the SLOT words of slots 64b..64b+63,
//                       then their TIME words, so a kernel that reads only
//                       one kind touches only that kind's cache lines.
//                       slot word: bits  0..15 placement (0..P-1 PM, P = WAIT,
//                                             P+1 = NULL)
//                                  bits 16..23 vm_cpu in hundredths (np.around
//                                             (.,2) makes every size k/100
//                                             exactly, env.py:212-219)
//                                  bits 24..31 vm_memory in hundredths
//                       time word: waiting VM: remaining runtime (env.py:290);
//                                  running VM: finish key F = timestep +
//                                  remaining, so a running VM's words do not
//                                  change while it runs (the step kernels
//                                  store only the words that changed)
//   pm   f64 [N][2][P] cpu[P] then memory[P]; kept in f64 because their values
//                       carry the reference's accumulated rounding history
//   hdr  EnvHdr [N]    256 B: 4 PCG64 streams, sequence bases, counters, stats
//
// vm_suspended / vm_planned_runtime are never read on the path (SURVEY App. B
// item 14) and are not stored.
#pragma once
#include <stdint.h>

namespace vmp {

constexpr int kWaveSize = 64;
constexpr int kWavesPerBlock = 4;
// envs (waves) per workgroup of the env kernel k_env
#ifndef VMP_ENV_WPB
#define VMP_ENV_WPB 1
#endif
constexpr int kEnvWavesPerBlock = VMP_ENV_WPB;
constexpr int kMaxVPT = 16;  // VM slots per lane held in registers: V <= 1024
constexpr int kMaxStepsPerLaunch = 256;  // rollout launches are split by the host
constexpr int kSpecDraws = 64;           // speculative service draws per launch

// VM words (see vmw above): u32 elements per env, and the slot / time word of
// slot v inside an env's block array
// (V <= 1024, the wave kernels: the block count is rounded up to the kernel's
// slot rows per lane, 1 / 2 / 4 / 8 / 16, so row s of every lane lies inside
// the env's pitch and the loads need no clamp)
__host__ __device__ inline int64_t vm_pitch(int V) {
  int b = (V + 63) >> 6;
  if (V <= 1024) {
    int q = 1;
    while (q < b) q <<= 1;
    b = q;
  }
  return (int64_t)b << 7;
}
__host__ __device__ inline int vm_slot_idx(int v) { return ((v >> 6) << 7) | (v & 63); }
__host__ __device__ inline int vm_time_idx(int v) { return ((v >> 6) << 7) | 64 | (v & 63); }

struct alignas(16) EnvHdr {
  uint64_t rng[4][4];      // [stream][state_hi, state_lo, inc_hi, inc_lo]; rng1..rng4
  uint64_t seqbase[2][2];  // rng1/rng2 state at the last reset (sequence element 0)
  int64_t timestep;
  int64_t total_requests, served, suspend_action, place_action, dropped;
  double total_cpu_req, total_mem_req, waiting_ratio, tcm, tmm;
  // per-step kernels' hint for the next launch's draws (predraw): bit 63
  // valid, bit 32 some NULL slot after the step, bits 0..31 the smallest
  // finish key of the VMs still running (0: no hint). Bit 62 (any k_env
  // launch): "quiet" - no pending VM fit any PM at the last step and no VM
  // finished or arrived in it, so the next heuristic pass places nothing.
  // Bit 60 (round 6): the last step's heuristic placements were ALL invalid
  // in f64 and no VM finished or arrived, so the next step repeats the same
  // decisions and rejections (skipped where no actions / validity flags are
  // returned). Both written 0 by k_reset, k_env_ext and k_env_big. Bit 61,
  // read only with bit 62 / 60: some VM existed after the step (the wr
  // reward's n_ex > 0)
  // INVARIANT: any new code path that changes an env's hdr / vmw / pm words
  // must either write this word as 0 or keep every bit exact for the state it
  // leaves (vmp_restore copies it with the state it belongs to). A stale bit
  // 62 silently skips placements: the -DVMP_CHECK_QUIET build counts such
  // steps (vmp_debug_quiet_violations, tests/test_gpu_env.py).
  uint64_t pad;
};
static_assert(sizeof(EnvHdr) == 256, "EnvHdr must be 256 B");

// Poisson(lam) constants (distributions.c random_poisson), computed on the host
// with glibc so the device only evaluates per-draw terms.
struct PoisConst {
  double lam, enlam;                         // mult method (lam < 10)
  double loglam, b, a, invalpha, vr, log_invalpha;  // PTRS (lam >= 10)
  const double *loggam_tab;                  // loggam(k+1) for k in [0, tab_n)
  int32_t kind;                              // 0: lam == 0, 1: mult, 2: PTRS
  int32_t tab_n;
};

struct EnvParams {
  int32_t N, P, V, A, D, W32;  // W32 = ceil(A/32) mask words per VM row
  int32_t reward, cap_target_util, eval_mode, pad0;
  int64_t limit;          // eval_steps if eval_mode else training_steps
  int64_t M2;             // 2 * max(training_steps, eval_steps)
  double beta, seq_lo, seq_range;
  const PoisConst *pois;  // device copy: [0] arrivals, [1] service lengths
  uint64_t *stamps;       // [N][8] phase clocks (diagnostic builds only)
  uint32_t *vmw;          // [N][vm_pitch(V)] (slot words | time words per 64-slot block)
  double *pm;
  EnvHdr *hdr;
  // per-wave LDS carve (bytes); offsets inside one wave's region
  int32_t lds_wave_bytes;
  int32_t NW;      // ceil(P/64) words per fit bitmap row
  int32_t n_leaf;  // capacity of the pairwise-sum leaf list
  int32_t off_hdr, off_pm, off_fpm, off_thr, off_ord, off_bits, off_sort, off_ccomp;
  int32_t off_leaf, off_leafval, off_stage, off_pre;
  int32_t scap;    // speculative service draws per launch
  int32_t off_pdirty;  // u64[ceil(2P/64)]: PM doubles (cpu then memory) changed this launch
  // accepted sizes accc/accm (u8 [acc_cap] each) and the existing-VM sizes
  // ccomp/mcomp (u8 [ccomp_cap] each); k_env_big's event lists (off_ev:
  // u32 [512] VM words, i32 [512] targets, u8 [512] results)
  int32_t off_acc, acc_cap, ccomp_cap, off_ev;
  int32_t fmem_off, tm_off;  // fmem - fcpu, tm - tc (elements): P, or 16-B aligned in k_env_big
  // PCG64 jump table: entry j = (A, M) with state after j+1 draws = A*s + M*inc
  // (A = a^(j+1), M = sum_{i<=j} a^i mod 2^128), u64 [64][4] {A.hi, A.lo, M.hi, M.lo}
  const uint64_t *jump;
  // k_env_big: u8 [N][4V] HBM spill of accc | accm | ccomp | mcomp for a step
  // whose accepted (> acc_cap) or existing (> ccomp_cap) VMs exceed the LDS copy
  uint8_t *bigscr;
};

struct StepOut {
  const int32_t *actions;  // external actions [N][V] or null (heuristic)
  int32_t *act_out;        // [N][V] nullable
  float *obs;              // [N][D] nullable (final state)
  double *reward;          // [K][N] nullable
  uint8_t *done;           // [N] nullable (last step)
  int64_t *done_count;     // [N] nullable
  uint8_t *valid;          // [N][V] nullable (last step)
  uint32_t *mask_bits;     // [N][V][W32] nullable (final state)
  int32_t policy;          // -1 external, 0 first-fit, 1 best-fit
  int32_t k_steps;
};

}  // namespace vmp
