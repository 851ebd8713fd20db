// vmp_capi.cpp — extern "C" entry points of libvmp.so (declared in include/vmp.h).
// Host-side: argument checks, device allocation, per-config constants
// (Poisson setup evaluated with glibc exactly as numpy's C code does), LDS
// carve-out, and kernel dispatch on the handle's stream.
#include <hip/hip_runtime.h>

#include <atomic>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vmp.h"
#include "vmp_layout.h"
#include "vmp_record.h"

namespace vmp {
constexpr int kStamps = 24;  // per-env phase clocks (diagnostic builds)
template <int VPT, bool ONE>
__global__ void k_env(EnvParams p, StepOut o);
template <int VPT>
__global__ void k_env_ext(EnvParams p, StepOut o);
__global__ void k_rank(EnvParams p, int64_t *rank);
__global__ void k_target_means_lds(EnvParams p);
// k_env_big: one workgroup per env; its geometry (threads, slots per thread)
// and launcher live with the kernel (vmp_kernels.hip)
void big_geometry(int *nt, int *spt_max);
void launch_big_env(int spt, bool one, int n_env, size_t lds, hipStream_t s, const EnvParams &p,
                    const StepOut &o);
int big_occupancy(int spt, size_t lds, int *static_lds);
constexpr int kBigStaticLds = 4 * 1024;  // Tables + BigShared (static LDS of k_env_big)
constexpr int kBigAccLds = 512;          // accepted sizes held in LDS
__global__ void k_reset(EnvParams p, const int64_t *seeds, const uint8_t *env_mask, float *obs);
__global__ void k_export(EnvParams p, int64_t *placement, double *vm_cpu, double *vm_mem,
                         double *cpu, double *mem, int64_t *remaining, int64_t *rank);
__global__ void k_counters(EnvParams p, int64_t *ctr, double *st);
__global__ void k_target_means(EnvParams p);
__global__ void k_record(EnvParams p, RecArgs r);
__global__ void k_record_init(EnvParams p, RecArgs r);
__global__ void k_record_close(EnvParams p, RecArgs r, uint32_t *hist, double *sums);
__global__ void k_mask_bool(int64_t rows, int A, int W, const uint32_t *bits, uint8_t *mask);
__global__ void k_act_obs(int P, int V, int policy, const float *obs, int32_t *act);
int64_t quiet_violations_take();
}  // namespace vmp

using namespace vmp;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess)                                                          \
      return fail(_e == hipErrorOutOfMemory ? VMP_EOOM : VMP_EDEVICE,              \
                  std::string(#expr) + ": " + hipGetErrorString(_e));              \
  } while (0)

// Device allocations of the handle go through here, so the failure paths can
// be exercised (vmp_debug_fail_alloc: the n-th allocation from now fails as
// out-of-memory; tests/test_sanitizers_cpu.py, tests/native/capi_faults.cpp).
// g_live counts the library's live device allocations (vmp_debug_live_allocs),
// so a leak on a failure path is seen exactly, whatever the runtime caches.
std::atomic<int64_t> g_fail_alloc{0};
std::atomic<int64_t> g_live{0};
template <class T>
hipError_t dev_malloc(T **p, size_t bytes) {
  int64_t n = g_fail_alloc.load();
  while (n > 0 && !g_fail_alloc.compare_exchange_weak(n, n - 1)) {
  }
  if (n == 1) {
    *p = nullptr;
    return hipErrorOutOfMemory;
  }
  const hipError_t e = hipMalloc(reinterpret_cast<void **>(p), bytes);
  if (e == hipSuccess && *p) g_live++;
  else *p = nullptr;
  return e;
}
void dev_free(void *p) {
  if (!p) return;
  (void)hipFree(p);
  g_live--;
}

// random_loggam (numpy distributions.c), host copy for the PTRS table.
double loggam_host(double x) {
  static const double a[10] = {8.333333333333333e-02, -2.777777777777778e-03,
                               7.936507936507937e-04, -5.952380952380952e-04,
                               8.417508417508418e-04, -1.917526917526918e-03,
                               6.410256410256410e-03, -2.955065359477124e-02,
                               1.796443723688307e-01, -1.39243221690590e+00};
  if (x == 1.0 || x == 2.0) return 0.0;
  int64_t n = (x < 7.0) ? (int64_t)(7 - x) : 0;
  double x0 = x + n;
  double x2 = (1.0 / x0) * (1.0 / x0);
  double gl0 = a[9];
  for (int k = 8; k >= 0; k--) {
    gl0 *= x2;
    gl0 += a[k];
  }
  double gl = gl0 / x0 + 0.5 * 1.8378770664093453e+00 + (x0 - 0.5) * std::log(x0) - x0;
  if (x < 7.0)
    for (int64_t k = 1; k <= n; k++) {
      gl -= std::log(x0 - 1.0);
      x0 -= 1.0;
    }
  return gl;
}

}  // namespace

namespace vmp {
// error reporting for the policy kernels (vmp_policy.hip) through vmp_last_error()
int policy_fail(int code, const char *msg) { return fail(code, msg); }
}  // namespace vmp

struct vmp_handle {
  vmp_config cfg;
  int32_t N, P, V, A, D, W32;
  int32_t device;
  int32_t eval_mode;
  hipStream_t stream;
  uint32_t *vmw;  // [N][vm_pitch(V)]
  double *pm;
  EnvHdr *hdr;
  double *lg_arr, *lg_svc;
  PoisConst arr, svc;
  EnvParams prm;
  uint32_t *scratch_bits;  // for vmp_mask_bool
  PoisConst *pois_dev;
  uint64_t *stamps;
  uint64_t *jump_dev;
  uint8_t *bigscr;  // k_env_big's HBM spill of the accepted / existing VM sizes
  bool big;  // k_env_big (V > 1024, or VMP_BIG_KERNEL=1)
  // eval-mode Record metrics (vmp_record.hip), allocated by vmp_record_enable
  bool rec_on;
  RecArgs rec;
  int32_t *rec_act;   // scratch action / validity / reward when the caller passes none
  uint8_t *rec_valid;
  double *rec_reward;
};

namespace {

int setup_pois(double lam, PoisConst &c, double **dev_tab, std::vector<double> &host_tab) {
  std::memset(&c, 0, sizeof(c));
  c.lam = lam;
  if (lam == 0) {
    c.kind = 0;
  } else if (lam < 10) {
    c.kind = 1;
    c.enlam = std::exp(-lam);
  } else {
    c.kind = 2;
    double slam = std::sqrt(lam);
    c.loglam = std::log(lam);
    c.b = 0.931 + 2.53 * slam;
    c.a = -0.059 + 0.02483 * c.b;
    c.invalpha = 1.1239 + 1.1328 / (c.b - 3.4);
    c.vr = 0.9277 - 3.6224 / (c.b - 2);
    c.log_invalpha = std::log(c.invalpha);
    int64_t n = (int64_t)(lam + 16.0 * slam + 64.0);
    if (n > (1 << 22)) n = 1 << 22;
    host_tab.resize((size_t)n);
    for (int64_t k = 0; k < n; k++) host_tab[(size_t)k] = loggam_host((double)k);
    c.tab_n = (int32_t)n;
    HIP_TRY(dev_malloc(dev_tab, sizeof(double) * n));
    HIP_TRY(hipMemcpy(*dev_tab, host_tab.data(), sizeof(double) * n, hipMemcpyHostToDevice));
    c.loggam_tab = *dev_tab;
  }
  return VMP_OK;
}

inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

// Max recursion depth of numpy's pairwise split for n <= V (kernel limit 5).
int pw_depth(int n) {
  if (n <= 128) return 0;
  int n2 = n / 2;
  n2 -= n2 % 8;
  int a = pw_depth(n2), b = pw_depth(n - n2);
  return 1 + (a > b ? a : b);
}
int pw_leaves(int n) {
  if (n <= 128) return 1;
  int n2 = n / 2;
  n2 -= n2 % 8;
  return pw_leaves(n2) + pw_leaves(n - n2);
}

void carve_big(vmp_handle *h);

void carve(vmp_handle *h) {
  EnvParams &p = h->prm;
  const int64_t P = h->P, V = h->V;
  int max_leaves = 1;
  bool deep = (V > 1928 || P > 1928);  // only deeper recursions use the LDS plan
  if (deep)
    for (int n = 0; n <= V || n <= P; n++) {
      int l = pw_leaves(n);
      if (l > max_leaves) max_leaves = l;
    }
  p.NW = (int32_t)((P + 63) / 64);
  p.n_leaf = deep ? max_leaves + 8 : 1;
  int64_t off = 0;
  p.off_hdr = (int32_t)off;
  off = align16(off + (int64_t)sizeof(EnvHdr));
  p.off_pm = (int32_t)off;
  off = align16(off + 16 * P);           // cpu, mem f64
  p.off_fpm = (int32_t)off;
  off = align16(off + 12 * P);           // fcpu, fmem f32 (+ P spare: the wave kernel's
  p.off_thr = (int32_t)off;              // measured layout; BF keys are formed on the fly)
  off = align16(off + 2 * P);            // tc, tm u8
  p.fmem_off = (int32_t)P;
  p.tm_off = (int32_t)P;
  p.off_ord = (int32_t)off;
  off = align16(off + 2 * P);            // BF visiting order u16
  p.off_bits = (int32_t)off;  // any-fit table (u32[128]); after the heuristic: NULL list + accepted sizes
  off = align16(off + (4 * V > 512 ? 4 * V : 512));
  p.off_stage = (int32_t)off;
  off = align16(off + 8 * 16);           // reduction results + draw bookkeeping
  // ccomp, mcomp u8 (stats, after the action phase) share their region with
  // the BF introsort stacks + partition lists (action phase only)
  p.off_ccomp = (int32_t)off;
  p.off_sort = (int32_t)off;
  off = align16(off + (2 * V > 4 * 256 + 4 * P ? 2 * V : 4 * 256 + 4 * P));
  // the LDS plan of the pairwise sums exists only for n > 1928 (wave_pw_sum)
  p.off_leaf = (int32_t)off;
  if (deep) off = align16(off + 8 * (int64_t)p.n_leaf + 4 * 192);  // lo, len, lane-0 stack
  p.off_leafval = (int32_t)off;
  if (deep) off = align16(off + 8 * (2 * (int64_t)p.n_leaf + 64));  // leaf sums + value stack
  // changed-PM bitmap (bit i: double i of cpu[P] | memory[P] was written this
  // launch): only those PM words are stored back
  p.off_pdirty = (int32_t)off;
  off = align16(off + 8 * ((2 * P + 63) / 64));
  p.off_acc = p.off_bits + (int32_t)(2 * V);  // after the NULL list
  p.acc_cap = (int32_t)V;
  p.ccomp_cap = (int32_t)V;
  p.off_ev = 0;  // k_env_big only
  p.off_pre = (int32_t)off;   // per-launch random draws follow (launch_env)
  p.lds_wave_bytes = (int32_t)off;
  if (h->big) carve_big(h);
}

// k_env_big's carve, sized for two workgroups per CU at P1000 / V10000 (≤ 80 KB
// with the VM words): the regions of the action phase and of the tail share
// one union. Heuristic side: the f32 view fcpu/fmem, thresholds tc/tm, the BF
// tie sort's order and stacks. Tail side: the pairwise-sum LDS plan, the
// event lists, the accepted sizes (≤ 512 in LDS) and the existing-VM sizes
// (as many as the rest of the union holds). Steps with more accepted or
// existing VMs than that use the handle's HBM spill (p.bigscr).
void carve_big(vmp_handle *h) {
  EnvParams &p = h->prm;
  const int64_t P = h->P, V = h->V;
  const bool deep = p.n_leaf > 1;
  int64_t off = 0;
  p.off_hdr = 0;
  off = align16((int64_t)sizeof(EnvHdr));
  p.off_pm = (int32_t)off;
  off = align16(off + 16 * P);
  p.off_stage = (int32_t)off;
  off = align16(off + 8 * 16);
  p.off_pdirty = (int32_t)off;
  off = align16(off + 8 * ((2 * P + 63) / 64));
  const int64_t u0 = off;
  // heuristic side
  p.off_fpm = (int32_t)off;
  off = align16(off + 8 * ((P + 3) & ~3));  // fcpu, fmem f32, 16-B aligned rows (BF keys are formed on the fly)
  p.off_thr = (int32_t)off;
  off = align16(off + 2 * align16(P));      // tc, tm u8, 16-B aligned rows (big_choose)
  p.fmem_off = (int32_t)((P + 3) & ~3);
  p.tm_off = (int32_t)align16(P);
  p.off_ord = (int32_t)off;
  off = align16(off + 2 * P);
  p.off_sort = (int32_t)off;
  off = align16(off + 4 * 256 + 4 * P);
  const int64_t heur_end = off;
  p.off_bits = p.off_fpm;  // the wave kernel's any-fit table / NULL list: unused here
  // tail side
  off = u0;
  p.off_leaf = (int32_t)off;
  if (deep) off = align16(off + 8 * (int64_t)p.n_leaf + 4 * 192);
  p.off_leafval = (int32_t)off;
  if (deep) off = align16(off + 8 * (2 * (int64_t)p.n_leaf + 64));
  p.off_ev = (int32_t)off;
  off = align16(off + 512 * (4 + 4 + 1));
  p.acc_cap = (int32_t)(V < kBigAccLds ? V : kBigAccLds);
  p.off_acc = (int32_t)off;
  off = align16(off + 2 * (int64_t)p.acc_cap);
  p.off_ccomp = (int32_t)off;
  int64_t cap = (heur_end - off) / 2;
  const int64_t cap_min = V < 1024 ? V : 1024;
  if (cap < cap_min) cap = cap_min;
  if (cap > V) cap = V;
  p.ccomp_cap = (int32_t)cap;
  off = align16(off + 2 * cap);
  if (off < heur_end) off = heur_end;
  p.off_pre = (int32_t)off;
  p.lds_wave_bytes = (int32_t)off;
}

void launch_ext(int need, dim3 grid, dim3 block, size_t lds, hipStream_t s, const EnvParams &p,
                const StepOut &o) {
  if (need <= 1) hipLaunchKernelGGL((k_env_ext<1>), grid, block, lds, s, p, o);
  else if (need <= 2) hipLaunchKernelGGL((k_env_ext<2>), grid, block, lds, s, p, o);
  else if (need <= 4) hipLaunchKernelGGL((k_env_ext<4>), grid, block, lds, s, p, o);
  else if (need <= 8) hipLaunchKernelGGL((k_env_ext<8>), grid, block, lds, s, p, o);
  else hipLaunchKernelGGL((k_env_ext<16>), grid, block, lds, s, p, o);
}

template <bool ONE>
void launch_vpt(int need, dim3 grid, dim3 block, size_t lds, hipStream_t s, const EnvParams &p,
                const StepOut &o) {
  if (need <= 1) hipLaunchKernelGGL((k_env<1, ONE>), grid, block, lds, s, p, o);
  else if (need <= 2) hipLaunchKernelGGL((k_env<2, ONE>), grid, block, lds, s, p, o);
  else if (need <= 4) hipLaunchKernelGGL((k_env<4, ONE>), grid, block, lds, s, p, o);
  else if (need <= 8) hipLaunchKernelGGL((k_env<8, ONE>), grid, block, lds, s, p, o);
  else hipLaunchKernelGGL((k_env<16, ONE>), grid, block, lds, s, p, o);
}

// k_env_big's shape: the fewest slots per thread that fit 384 threads, and the
// thread count (whole waves). The block's VM words live in LDS (4 B per slot).
void big_shape(int64_t V, int &spt, int &nt) {
  int mx;
  big_geometry(&nt, &mx);  // nt: the kernel's compile-time workgroup size (kBigNT)
  spt = V <= 4 * nt ? 4 : V <= 8 * nt ? 8 : V <= 16 * nt ? 16 : mx;
}

int launch_env(vmp_handle *h, const StepOut &o) {
  dim3 grid((h->N + kEnvWavesPerBlock - 1) / kEnvWavesPerBlock), block(64 * kEnvWavesPerBlock);
  EnvParams p = h->prm;
  // per-launch region: speculative service draws (state + value) and arrivals
  p.scap = kSpecDraws;
  const int64_t pre = 20 * (int64_t)p.scap + 4 * (int64_t)(o.k_steps > 0 ? o.k_steps : 1);
  p.lds_wave_bytes = (int32_t)align16(p.off_pre + pre);
  size_t lds = (size_t)p.lds_wave_bytes * kEnvWavesPerBlock;
  if (!h->big && lds > 160 * 1024 - 2048) return fail(VMP_EINVAL, "config too large for the LDS carve");
  if (h->big) {
    // one workgroup per env; the VM words follow the wave carve
    int spt, nt;
    big_shape(h->V, spt, nt);
    const size_t lds1 = (size_t)p.lds_wave_bytes + 4 * (size_t)spt * nt;
    launch_big_env(spt, o.k_steps == 1, h->N, lds1, h->stream, p, o);
    HIP_TRY(hipGetLastError());
    return VMP_OK;
  }
  const int need = (h->V + 63) / 64;
  if (o.actions) {  // external actions: vmp_step, one step
    if (o.k_steps != 1) return fail(VMP_EINVAL, "external actions take one step per launch");
    launch_ext(need, grid, block, lds, h->stream, p, o);
  } else if (o.k_steps == 1) launch_vpt<true>(need, grid, block, lds, h->stream, p, o);
  else launch_vpt<false>(need, grid, block, lds, h->stream, p, o);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

StepOut empty_out() {
  StepOut o;
  std::memset(&o, 0, sizeof(o));
  o.policy = -1;
  return o;
}

void refresh_params(vmp_handle *h) {
  h->prm.eval_mode = h->eval_mode;
  h->prm.limit = h->eval_mode ? h->cfg.eval_steps : h->cfg.training_steps;
}

}  // namespace

extern "C" {

int vmp_abi_version(void) { return VMP_ABI_VERSION; }
const char *vmp_last_error(void) { return g_err.c_str(); }

static int create_rest(vmp_handle *h, const vmp_config *cfg, int32_t n_env, const int64_t *seeds);

int vmp_create(const vmp_config *cfg, int32_t n_env, const int64_t *seeds, int32_t device,
               vmp_handle **out) {
  if (!cfg || !out || n_env <= 0 || !seeds) return fail(VMP_EINVAL, "null argument or n_env <= 0");
  if (cfg->pms < 1 || cfg->pms > 65533) return fail(VMP_EINVAL, "pms must be in [1, 65533]");
  int big_nt, big_spt;
  big_geometry(&big_nt, &big_spt);
  if (cfg->vms < 1 || cfg->vms > big_nt * big_spt)
    return fail(VMP_EINVAL, "vms must be in [1, 10240] on this build");
  if (cfg->reward_function < 0 || cfg->reward_function > 2)
    return fail(VMP_EINVAL, "Function does not exist: reward_function");  // env.py:156
  if (cfg->sequence < 0 || cfg->sequence > 2) return fail(VMP_EINVAL, "unknown sequence");
  if (!(cfg->arrival_rate >= 0) || !(cfg->service_length >= 0))
    return fail(VMP_EINVAL, "arrival_rate and service_length must be >= 0");
  for (int32_t i = 0; i < n_env; i++)
    if (seeds[i] < 0) return fail(VMP_EINVAL, "seeds must be non-negative");
  HIP_TRY(hipSetDevice(device));
  vmp_handle *h = new vmp_handle();
  std::memset(h, 0, sizeof(*h));
  h->cfg = *cfg;
  h->N = n_env;
  h->P = cfg->pms;
  h->V = cfg->vms;
  h->A = cfg->allow_null_action ? cfg->pms + 2 : cfg->pms + 1;
  h->D = 3 * cfg->vms + 2 * cfg->pms;
  h->W32 = (h->A + 31) / 32;
  {
    const char *force = getenv("VMP_BIG_KERNEL");
    h->big = cfg->vms > kMaxVPT * kWaveSize || (force && force[0] == '1');
  }
  h->device = device;
  h->stream = nullptr;
  std::vector<double> t1, t2;
  int rc = setup_pois(cfg->arrival_rate, h->arr, &h->lg_arr, t1);
  if (rc == VMP_OK) rc = setup_pois(cfg->service_length, h->svc, &h->lg_svc, t2);
  if (rc != VMP_OK) {
    const std::string msg = g_err;
    vmp_destroy(h);  // frees whatever the first setup_pois allocated
    return fail(rc, msg);
  }
  rc = create_rest(h, cfg, n_env, seeds);
  if (rc != VMP_OK) {
    const std::string msg = g_err;
    vmp_destroy(h);
    return fail(rc, msg);
  }
  *out = h;
  return VMP_OK;
}

// vmp_create after the handle exists: every failure returns a code and the
// caller destroys the handle (vmp_destroy tolerates what was not allocated).
static int create_rest(vmp_handle *h, const vmp_config *cfg, int32_t n_env, const int64_t *seeds) {
  hipError_t e1 = dev_malloc(&h->vmw, sizeof(uint32_t) * (size_t)n_env * vm_pitch(h->V));
  hipError_t e2 = dev_malloc(&h->pm, sizeof(double) * (size_t)n_env * 2 * h->P);
  hipError_t e3 = dev_malloc(&h->hdr, sizeof(EnvHdr) * (size_t)n_env);
  if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess)
    return fail(VMP_EOOM, "device allocation failed");
  HIP_TRY(hipMemset(h->hdr, 0, sizeof(EnvHdr) * (size_t)n_env));
  EnvParams &p = h->prm;
  p.N = h->N;
  p.P = h->P;
  p.V = h->V;
  p.A = h->A;
  p.D = h->D;
  p.W32 = h->W32;
  p.reward = cfg->reward_function;
  p.cap_target_util = cfg->cap_target_util;
  int64_t M = cfg->training_steps > cfg->eval_steps ? cfg->training_steps : cfg->eval_steps;
  p.M2 = 2 * M;
  p.beta = cfg->beta;
  p.seq_lo = cfg->sequence == VMP_SEQ_HIGHUNIFORM ? 0.25 : 0.1;
  double hi = cfg->sequence == VMP_SEQ_LOWUNIFORM ? 0.65 : 1.0;
  p.seq_range = hi - p.seq_lo;  // Generator.uniform: low + (high-low)*u
  {
    PoisConst pc[2] = {h->arr, h->svc};
    HIP_TRY(dev_malloc(&h->pois_dev, sizeof(pc)));
    HIP_TRY(hipMemcpy(h->pois_dev, pc, sizeof(pc), hipMemcpyHostToDevice));
    p.pois = h->pois_dev;
    // PCG64 jump table for the lane-parallel draws (k_env prologue)
    uint64_t jt[64 * 4];
    const unsigned __int128 a = ((unsigned __int128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;
    unsigned __int128 A = a, M = 1;
    for (int j = 0; j < 64; j++) {
      jt[4 * j + 0] = (uint64_t)(A >> 64);
      jt[4 * j + 1] = (uint64_t)A;
      jt[4 * j + 2] = (uint64_t)(M >> 64);
      jt[4 * j + 3] = (uint64_t)M;
      A *= a;
      M = M * a + 1;
    }
    HIP_TRY(dev_malloc(&h->jump_dev, sizeof(jt)));
    HIP_TRY(hipMemcpy(h->jump_dev, jt, sizeof(jt), hipMemcpyHostToDevice));
    p.jump = h->jump_dev;
  }
  p.vmw = h->vmw;
  p.pm = h->pm;
  p.hdr = h->hdr;
  carve(h);
  if (h->big) {
    HIP_TRY(dev_malloc(&h->bigscr, (size_t)n_env * 4 * (size_t)h->V));
    p.bigscr = h->bigscr;
  }
  // diagnostic per-env clocks: -DVMP_STAMPS builds, or VMP_STAMP_BUF=1 for the
  // workgroup timing build (-DVMP_WGTIME, tools/wgtime.py)
  bool want_stamps = getenv("VMP_STAMP_BUF") && getenv("VMP_STAMP_BUF")[0] == '1';
#ifdef VMP_STAMPS
  want_stamps = true;
#endif
  if (want_stamps) {
    HIP_TRY(dev_malloc(&h->stamps, sizeof(uint64_t) * kStamps * (size_t)n_env));
    HIP_TRY(hipMemset(h->stamps, 0, sizeof(uint64_t) * kStamps * (size_t)n_env));
    p.stamps = h->stamps;
  }
  int maxn = h->V > h->P ? h->V : h->P;
  int depth = 0;
  for (int n = 0; n <= maxn; n++) depth = pw_depth(n) > depth ? pw_depth(n) : depth;
  if (depth > 12)
    return fail(VMP_EINVAL, "config exceeds the pairwise-sum recursion depth of this build");
  {
    const int64_t per_env = p.lds_wave_bytes + 20 * kSpecDraws + 4 * kMaxStepsPerLaunch;
    int spt = 0, nt = 0;
    if (h->big) big_shape(h->V, spt, nt);
    const int64_t need = h->big ? per_env + kBigStaticLds + 4 * (int64_t)spt * nt
                                : per_env * kEnvWavesPerBlock + 2048;
    if (need > 160 * 1024)
      return fail(VMP_EINVAL, "config too large for the LDS carve of this build");
  }
  refresh_params(h);
  int64_t *dseeds = nullptr;
  HIP_TRY(dev_malloc(&dseeds, sizeof(int64_t) * n_env));
  hipError_t e = hipMemcpy(dseeds, seeds, sizeof(int64_t) * n_env, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    dim3 grid((n_env + kWavesPerBlock - 1) / kWavesPerBlock), block(64 * kWavesPerBlock);
    hipLaunchKernelGGL(k_reset, grid, block, 0, h->stream, h->prm, dseeds, nullptr, nullptr);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  }
  dev_free(dseeds);
  if (e != hipSuccess) return fail(VMP_EDEVICE, std::string("vmp_create reset: ") + hipGetErrorString(e));
  return VMP_OK;
}

int vmp_destroy(vmp_handle *h) {
  if (!h) return VMP_OK;
  dev_free(h->vmw);
  dev_free(h->pm);
  dev_free(h->hdr);
  dev_free(h->lg_arr);
  dev_free(h->lg_svc);
  dev_free(h->scratch_bits);
  dev_free(h->pois_dev);
  dev_free(h->jump_dev);
  dev_free(h->bigscr);
  dev_free(h->stamps);
  vmp_record_enable(h, 0);
  delete h;
  return VMP_OK;
}

int vmp_set_stream(vmp_handle *h, void *s) {
  if (!h) return fail(VMP_EINVAL, "null handle");
  h->stream = (hipStream_t)s;
  return VMP_OK;
}

int vmp_set_eval(vmp_handle *h, int32_t eval_mode) {
  if (!h) return fail(VMP_EINVAL, "null handle");
  h->eval_mode = eval_mode ? 1 : 0;
  refresh_params(h);
  return VMP_OK;
}

int vmp_dims(const vmp_handle *h, int32_t *n, int32_t *P, int32_t *V, int32_t *A, int32_t *D) {
  if (!h) return fail(VMP_EINVAL, "null handle");
  if (n) *n = h->N;
  if (P) *P = h->P;
  if (V) *V = h->V;
  if (A) *A = h->A;
  if (D) *D = h->D;
  return VMP_OK;
}

int vmp_reset(vmp_handle *h, const int64_t *seeds, const uint8_t *env_mask, float *obs) {
  if (!h) return fail(VMP_EINVAL, "null handle");
  dim3 grid((h->N + kWavesPerBlock - 1) / kWavesPerBlock), block(64 * kWavesPerBlock);
  hipLaunchKernelGGL(k_reset, grid, block, 0, h->stream, h->prm, seeds, env_mask, obs);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

static int record_after(vmp_handle *h, const int32_t *act, const uint8_t *valid,
                        const double *reward);

int vmp_step(vmp_handle *h, const int32_t *actions, float *obs, double *reward, uint8_t *done,
             uint8_t *valid) {
  return vmp_step_mask(h, actions, obs, reward, done, valid, nullptr);
}

int vmp_step_mask(vmp_handle *h, const int32_t *actions, float *obs, double *reward, uint8_t *done,
                  uint8_t *valid, uint32_t *next_mask_bits) {
  if (!h || !actions) return fail(VMP_EINVAL, "null handle or actions");
  StepOut o = empty_out();
  o.actions = actions;
  o.obs = obs;
  o.reward = reward;
  o.done = done;
  o.valid = valid;
  o.mask_bits = next_mask_bits;  // written from the post-step state, as vmp_mask would
  o.k_steps = 1;
  if (h->rec_on) {
    if (!o.reward) o.reward = h->rec_reward;
    if (!o.valid) o.valid = h->rec_valid;
  }
  int rc = launch_env(h, o);
  if (rc == VMP_OK && h->rec_on) rc = record_after(h, actions, o.valid, o.reward);
  return rc;
}

int vmp_heuristic_act(vmp_handle *h, int32_t policy, int32_t *actions) {
  if (!h || !actions) return fail(VMP_EINVAL, "null handle or actions");
  if (policy != VMP_POLICY_FIRSTFIT && policy != VMP_POLICY_BESTFIT)
    return fail(VMP_EINVAL, "unknown policy");
  StepOut o = empty_out();
  o.policy = policy;
  o.act_out = actions;
  o.k_steps = 0;
  return launch_env(h, o);
}

int vmp_heuristic_act_obs(vmp_handle *h, int32_t policy, const float *obs, int32_t *actions) {
  if (!h || !obs || !actions) return fail(VMP_EINVAL, "null handle, obs or actions");
  if (policy != VMP_POLICY_FIRSTFIT && policy != VMP_POLICY_BESTFIT)
    return fail(VMP_EINVAL, "unknown policy");
  const size_t lds = 18 * (size_t)h->P + 1024;  // cpu, memory, keys, order, sort stack
  // the whole PM view in one workgroup's LDS (gfx950: 160 KB per workgroup)
  if (lds > (size_t)160 * 1024) return fail(VMP_EINVAL, "act from observation supports P <= 9045");
  hipLaunchKernelGGL(k_act_obs, dim3(h->N), dim3(64), lds, h->stream, h->P, h->V, policy, obs,
                     actions);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

static int heuristic_step_impl(vmp_handle *h, int32_t policy, int32_t *actions_out, float *obs,
                               double *reward, uint8_t *done, uint8_t *valid,
                               int64_t *done_count) {
  if (!h) return fail(VMP_EINVAL, "null handle");
  if (policy != VMP_POLICY_FIRSTFIT && policy != VMP_POLICY_BESTFIT)
    return fail(VMP_EINVAL, "unknown policy");
  StepOut o = empty_out();
  o.policy = policy;
  o.act_out = actions_out;
  o.obs = obs;
  o.reward = reward;
  o.done = done;
  o.done_count = done_count;
  o.valid = valid;
  o.k_steps = 1;
  if (h->rec_on) {
    if (!o.act_out) o.act_out = h->rec_act;
    if (!o.reward) o.reward = h->rec_reward;
    if (!o.valid) o.valid = h->rec_valid;
  }
  int rc = launch_env(h, o);
  if (rc == VMP_OK && h->rec_on) rc = record_after(h, o.act_out, o.valid, o.reward);
  return rc;
}

int vmp_heuristic_step(vmp_handle *h, int32_t policy, int32_t *actions_out, float *obs,
                       double *reward, uint8_t *done, uint8_t *valid) {
  return heuristic_step_impl(h, policy, actions_out, obs, reward, done, valid, nullptr);
}

int vmp_rollout_heuristic(vmp_handle *h, int32_t policy, int32_t k_steps, double *rewards,
                          int64_t *done_count) {
  if (!h || k_steps < 1) return fail(VMP_EINVAL, "null handle or k_steps < 1");
  if (policy != VMP_POLICY_FIRSTFIT && policy != VMP_POLICY_BESTFIT)
    return fail(VMP_EINVAL, "unknown policy");
  if (h->rec_on) {  // recorded: one step per launch, the recorder after each
    for (int32_t k = 0; k < k_steps; k++) {
      int rc = heuristic_step_impl(h, policy, nullptr, nullptr,
                                   rewards ? rewards + (int64_t)k * h->N : nullptr, nullptr,
                                   nullptr, done_count);
      if (rc) return rc;
    }
    return VMP_OK;
  }
  // launches of at most kMaxStepsPerLaunch steps (the per-launch draw region)
  for (int32_t k0 = 0; k0 < k_steps; k0 += kMaxStepsPerLaunch) {
    StepOut o = empty_out();
    o.policy = policy;
    o.reward = rewards ? rewards + (int64_t)k0 * h->N : nullptr;
    o.done_count = done_count;
    o.k_steps = k_steps - k0 < kMaxStepsPerLaunch ? k_steps - k0 : kMaxStepsPerLaunch;
    int rc = launch_env(h, o);
    if (rc) return rc;
  }
  return VMP_OK;
}

static int record_after(vmp_handle *h, const int32_t *act, const uint8_t *valid,
                        const double *reward) {
  RecArgs r = h->rec;
  r.act = act;
  r.valid = valid;
  r.reward = reward;
  const size_t lds = (size_t)4 * ((h->P + 63) / 64) * sizeof(unsigned long long);
  hipLaunchKernelGGL(k_record, dim3((h->N + 3) / 4), dim3(256), lds, h->stream, h->prm, r);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

int vmp_record_enable(vmp_handle *h, int32_t on) {
  if (!h) return fail(VMP_EINVAL, "null handle");
  if (!on) {
    if (h->rec_on) (void)hipStreamSynchronize(h->stream);
    dev_free(h->rec.prev);
    dev_free(h->rec.life_n);
    dev_free(h->rec.alloc);
    dev_free(h->rec.waits);
    dev_free(h->rec.hist);
    dev_free(h->rec.sums);
    dev_free(h->rec_act);
    dev_free(h->rec_valid);
    dev_free(h->rec_reward);
    std::memset(&h->rec, 0, sizeof(h->rec));
    h->rec_act = nullptr;
    h->rec_valid = nullptr;
    h->rec_reward = nullptr;
    h->rec_on = false;
    return VMP_OK;
  }
  const size_t nv = (size_t)h->N * h->V;
  if (!h->rec.prev) {
    // all or nothing: a partial set would leave null buffers behind a
    // non-null `prev` for the next call's k_record_init to write through
    const hipError_t e[9] = {
        dev_malloc(&h->rec.prev, sizeof(uint16_t) * nv),
        dev_malloc(&h->rec.life_n, sizeof(uint32_t) * nv),
        dev_malloc(&h->rec.alloc, sizeof(int32_t) * nv),
        dev_malloc(&h->rec.waits, sizeof(uint32_t) * nv),
        dev_malloc(&h->rec.hist, sizeof(uint32_t) * (size_t)h->N * 2 * VMP_REC_BINS),
        dev_malloc(&h->rec.sums, sizeof(double) * (size_t)h->N * VMP_NREC),
        dev_malloc(&h->rec_act, sizeof(int32_t) * nv),
        dev_malloc(&h->rec_valid, nv),
        dev_malloc(&h->rec_reward, sizeof(double) * (size_t)h->N)};
    for (hipError_t x : e)
      if (x != hipSuccess) {
        vmp_record_enable(h, 0);
        return fail(x == hipErrorOutOfMemory ? VMP_EOOM : VMP_EDEVICE,
                    std::string("vmp_record_enable: ") + hipGetErrorString(x));
      }
  }
  size_t n = nv;
  if ((size_t)h->N * 2 * VMP_REC_BINS > n) n = (size_t)h->N * 2 * VMP_REC_BINS;
  if ((size_t)h->N * VMP_NREC > n) n = (size_t)h->N * VMP_NREC;
  hipLaunchKernelGGL(k_record_init, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream,
                     h->prm, h->rec);
  HIP_TRY(hipGetLastError());
  h->rec_on = true;
  return VMP_OK;
}

int vmp_record_read(vmp_handle *h, uint32_t *hist, double *sums) {
  if (!h || !hist || !sums) return fail(VMP_EINVAL, "null argument");
  if (!h->rec_on) return fail(VMP_ESTATE, "recording is not enabled (vmp_record_enable)");
  HIP_TRY(hipMemcpyAsync(hist, h->rec.hist, sizeof(uint32_t) * (size_t)h->N * 2 * VMP_REC_BINS,
                         hipMemcpyDeviceToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(sums, h->rec.sums, sizeof(double) * (size_t)h->N * VMP_NREC,
                         hipMemcpyDeviceToDevice, h->stream));
  hipLaunchKernelGGL(k_record_close, dim3((h->N + 3) / 4), dim3(256), 0, h->stream, h->prm,
                     h->rec, hist, sums);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

int vmp_mask(vmp_handle *h, uint32_t *bits) {
  if (!h || !bits) return fail(VMP_EINVAL, "null argument");
  StepOut o = empty_out();
  o.mask_bits = bits;
  return launch_env(h, o);
}

int vmp_mask_bool(vmp_handle *h, uint8_t *mask) {
  if (!h || !mask) return fail(VMP_EINVAL, "null argument");
  if (!h->scratch_bits)
    HIP_TRY(dev_malloc(&h->scratch_bits, sizeof(uint32_t) * (size_t)h->N * h->V * h->W32));
  int rc = vmp_mask(h, h->scratch_bits);
  if (rc) return rc;
  int64_t rows = (int64_t)h->N * h->V;
  int64_t n = rows * h->A;
  hipLaunchKernelGGL(k_mask_bool, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream,
                     rows, h->A, h->W32, h->scratch_bits, mask);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

int vmp_get_obs(vmp_handle *h, float *obs) {
  if (!h || !obs) return fail(VMP_EINVAL, "null argument");
  StepOut o = empty_out();
  o.obs = obs;
  return launch_env(h, o);
}

int vmp_get_counters(vmp_handle *h, int64_t *counters) {
  if (!h || !counters) return fail(VMP_EINVAL, "null argument");
  hipLaunchKernelGGL(k_counters, dim3((h->N + 255) / 256), dim3(256), 0, h->stream, h->prm,
                     counters, nullptr);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

int vmp_get_stats(vmp_handle *h, double *stats) {
  if (!h || !stats) return fail(VMP_EINVAL, "null argument");
  if (h->V > kMaxVPT * kWaveSize) {
    // beyond the static per-wave buffers: a private carve laid out from 0 for
    // this kernel alone (ccomp | mcomp of V bytes each, then the pairwise-sum
    // plan); the env's own carve (carve_big) places ccomp after regions this
    // kernel does not allocate and caps it below V
    EnvParams q = h->prm;
    q.off_ccomp = 0;
    q.ccomp_cap = h->V;
    q.off_leaf = (int32_t)align16(2 * (int64_t)h->V);
    q.off_leafval = (int32_t)(q.off_leaf + align16(8 * (int64_t)q.n_leaf + 4 * 192));
    const size_t lds = (size_t)q.off_leafval + 8 * (2 * (size_t)q.n_leaf + 64);
    hipLaunchKernelGGL(k_target_means_lds, dim3(h->N), dim3(64), lds, h->stream, q);
  } else
    hipLaunchKernelGGL(k_target_means, dim3((h->N + kWavesPerBlock - 1) / kWavesPerBlock),
                       dim3(64 * kWavesPerBlock), 0, h->stream, h->prm);
  hipLaunchKernelGGL(k_counters, dim3((h->N + 255) / 256), dim3(256), 0, h->stream, h->prm,
                     nullptr, stats);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

int vmp_get_state(vmp_handle *h, int64_t *placement, double *vm_cpu, double *vm_mem,
                  double *cpu, double *mem, int64_t *remaining) {
  if (!h) return fail(VMP_EINVAL, "null handle");
  int64_t n = (int64_t)h->N * (h->V > h->P ? h->V : h->P);
  hipLaunchKernelGGL(k_export, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream,
                     h->prm, placement, vm_cpu, vm_mem, cpu, mem, remaining, nullptr);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

int vmp_get_rank(vmp_handle *h, int64_t *rank) {
  if (!h || !rank) return fail(VMP_EINVAL, "null argument");
  hipLaunchKernelGGL(k_rank, dim3(h->N), dim3(64), sizeof(uint64_t) * ((h->P + 63) / 64),
                     h->stream, h->prm, rank);
  HIP_TRY(hipGetLastError());
  return VMP_OK;
}

// ---- checkpoint / resume of the batched env state ----
// Snapshot = a 256-B descriptor, then hdr[N] | pm[N][2P] | vmw[N][pitch] as the
// kernels keep them (PCG64 states, sequence bases, counters, step hints and
// finish keys included), so a restore is bit-exact by construction: the
// restored handle holds the very bytes every later kernel reads.
namespace {
constexpr uint64_t kSnapMagic = 0x31504e534d504d56ULL;  // "VMPMSNP1"
constexpr int64_t kSnapHead = 256;
struct SnapDesc {
  uint64_t magic;
  int32_t abi, hdr_bytes;
  int32_t N, P, V, A;
  vmp_config cfg;  // seed excluded from the compatibility check
};
static_assert(sizeof(SnapDesc) <= kSnapHead, "snapshot descriptor exceeds its header");
int64_t snap_bytes(const vmp_handle *h) {
  return kSnapHead + (int64_t)sizeof(EnvHdr) * h->N + 16 * (int64_t)h->N * h->P +
         4 * (int64_t)h->N * vm_pitch(h->V);
}
bool same_config(const vmp_config &a, const vmp_config &b) {
  vmp_config x = a, y = b;
  x.seed = y.seed = 0;
  return std::memcmp(&x, &y, sizeof(x)) == 0;
}
}  // namespace

int vmp_snapshot_bytes(const vmp_handle *h, int64_t *bytes) {
  if (!h || !bytes) return fail(VMP_EINVAL, "null argument");
  *bytes = snap_bytes(h);
  return VMP_OK;
}

int vmp_snapshot(vmp_handle *h, void *dst) {
  if (!h || !dst) return fail(VMP_EINVAL, "null argument");
  if (((uintptr_t)dst) & 15) return fail(VMP_EINVAL, "vmp_snapshot: dst must be 16-byte aligned");
  uint8_t head[kSnapHead];
  std::memset(head, 0, sizeof(head));
  SnapDesc d;
  std::memset(&d, 0, sizeof(d));
  d.magic = kSnapMagic;
  d.abi = VMP_ABI_VERSION;
  d.hdr_bytes = (int32_t)sizeof(EnvHdr);
  d.N = h->N, d.P = h->P, d.V = h->V, d.A = h->A;
  d.cfg = h->cfg;
  std::memcpy(head, &d, sizeof(d));
  uint8_t *o = (uint8_t *)dst;
  const size_t nh = sizeof(EnvHdr) * (size_t)h->N, np = 16 * (size_t)h->N * h->P;
  HIP_TRY(hipMemcpyAsync(o, head, kSnapHead, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(o + kSnapHead, h->hdr, nh, hipMemcpyDeviceToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(o + kSnapHead + nh, h->pm, np, hipMemcpyDeviceToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(o + kSnapHead + nh + np, h->vmw, 4 * (size_t)h->N * vm_pitch(h->V),
                         hipMemcpyDeviceToDevice, h->stream));
  // the descriptor's host copy is a stack buffer: the call returns after it is read
  HIP_TRY(hipStreamSynchronize(h->stream));
  return VMP_OK;
}

int vmp_restore(vmp_handle *h, const void *src) {
  if (!h || !src) return fail(VMP_EINVAL, "null argument");
  if (((uintptr_t)src) & 15) return fail(VMP_EINVAL, "vmp_restore: src must be 16-byte aligned");
  SnapDesc d;
  HIP_TRY(hipStreamSynchronize(h->stream));
  HIP_TRY(hipMemcpy(&d, src, sizeof(d), hipMemcpyDeviceToHost));
  if (d.magic != kSnapMagic || d.abi != VMP_ABI_VERSION || d.hdr_bytes != (int32_t)sizeof(EnvHdr))
    return fail(VMP_EINVAL, "vmp_restore: not a snapshot of this library version");
  if (d.N != h->N || d.P != h->P || d.V != h->V || d.A != h->A || !same_config(d.cfg, h->cfg))
    return fail(VMP_EINVAL, "vmp_restore: snapshot of another env count or config");
  const uint8_t *s = (const uint8_t *)src;
  const size_t nh = sizeof(EnvHdr) * (size_t)h->N, np = 16 * (size_t)h->N * h->P;
  HIP_TRY(hipMemcpyAsync(h->hdr, s + kSnapHead, nh, hipMemcpyDeviceToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(h->pm, s + kSnapHead + nh, np, hipMemcpyDeviceToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(h->vmw, s + kSnapHead + nh + np, 4 * (size_t)h->N * vm_pitch(h->V),
                         hipMemcpyDeviceToDevice, h->stream));
  return VMP_OK;
}

int64_t vmp_debug_live_allocs(void) { return g_live.load(); }

int vmp_debug_quiet_violations(int64_t *count) {
  if (!count) return fail(VMP_EINVAL, "null argument");
  const int64_t v = quiet_violations_take();
  if (v == -1) return fail(VMP_EINVAL, "library built without -DVMP_CHECK_QUIET");
  if (v < 0) return fail(VMP_EDEVICE, "vmp_debug_quiet_violations: device read failed");
  *count = v;
  return VMP_OK;
}

int vmp_debug_fail_alloc(int32_t n) {
  if (n < 0) return fail(VMP_EINVAL, "n must be >= 0");
  g_fail_alloc.store(n);
  return VMP_OK;
}

int vmp_debug_occupancy(vmp_handle *h, int32_t *blocks_per_cu, int32_t *lds_bytes) {
  if (!h || !blocks_per_cu || !lds_bytes) return fail(VMP_EINVAL, "null argument");
  if (!h->big) return fail(VMP_EINVAL, "occupancy query covers the block kernel (V > 1024) only");
  int spt, nt;
  big_shape(h->V, spt, nt);
  const size_t lds1 = (size_t)align16(h->prm.off_pre + 20 * (int64_t)kSpecDraws + 4) + 4 * (size_t)spt * nt;
  int st = 0;
  *blocks_per_cu = big_occupancy(spt, lds1, &st);
  *lds_bytes = (int32_t)lds1 + st;
  return VMP_OK;
}

int vmp_debug_stamps(vmp_handle *h, uint64_t *out) {
  if (!h || !out) return fail(VMP_EINVAL, "null argument");
  if (!h->stamps) return fail(VMP_EINVAL, "library built without -DVMP_STAMPS");
  HIP_TRY(hipMemcpyAsync(out, h->stamps, sizeof(uint64_t) * kStamps * (size_t)h->N,
                         hipMemcpyDeviceToDevice, h->stream));
  HIP_TRY(hipMemsetAsync(h->stamps, 0, sizeof(uint64_t) * kStamps * (size_t)h->N, h->stream));
  return VMP_OK;
}

}  // extern "C"
