// Host-sanitizer driver for the C ABI's argument checks and failure paths
// (TEST INFRASTRUCTURE). Linked against
// libvmp_san.so, whose host code (csrc/vmp_capi.cpp) is built with
// AddressSanitizer + UndefinedBehaviorSanitizer (`make -C
// vm-placement-migration-gym_amd sanitize`); the kernels are the normal
// gfx950 objects. Every check prints a line and the program exits non-zero
// on the first mismatch; the sanitizers abort on the first report.
//
//   without a device (the build container): every entry point rejects null
//   handles / arguments with VMP_EINVAL; vmp_create rejects each invalid
//   config field (env.py:156's unknown reward, an unknown sequence, P / V
//   out of range, negative rates and seeds, n_env <= 0) before touching the
//   device, and a valid config fails cleanly with VMP_EDEVICE;
//   with a device (`capi_faults --device`, the GPU box): for every n, the
//   n-th device allocation of vmp_create / vmp_record_enable / vmp_mask_bool
//   fails (vmp_debug_fail_alloc) and the call returns VMP_EOOM with nothing
//   leaked (host: LeakSanitizer; device: the library's live-allocation count,
//   vmp_debug_live_allocs, back to its value before the call), the
//   handle stays usable after a failed vmp_record_enable, and a full create /
//   step / record / destroy cycle runs clean.
#include <hip/hip_runtime.h>
#include <sanitizer/lsan_interface.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/vmp.h"

static int g_fail = 0;
#define CHECK(cond, what)                                          \
  do {                                                             \
    if (!(cond)) {                                                 \
      std::fprintf(stderr, "FAIL %s (%s:%d)\n", what, __FILE__, __LINE__); \
      g_fail = 1;                                                  \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

static vmp_config base_cfg() {
  vmp_config c;
  std::memset(&c, 0, sizeof(c));
  c.arrival_rate = 1.8182;
  c.service_length = 100;
  c.pms = 100;
  c.vms = 300;
  c.training_steps = 1000;
  c.eval_steps = 1000;
  c.seed = 0;
  c.reward_function = VMP_REWARD_KL;
  c.sequence = VMP_SEQ_UNIFORM;
  c.cap_target_util = 1;
  c.allow_null_action = 1;
  c.beta = 0.5;
  return c;
}

static void expect_einval(int rc, const char *what) {
  CHECK(rc == VMP_EINVAL, what);
  CHECK(vmp_last_error() && std::strlen(vmp_last_error()) > 0, what);
  std::printf("ok  EINVAL  %s: %s\n", what, vmp_last_error());
}

static void argument_checks() {
  std::vector<int64_t> seeds(8, 0);
  vmp_handle *h = nullptr;
  vmp_config c = base_cfg();
  expect_einval(vmp_create(nullptr, 8, seeds.data(), 0, &h), "create null cfg");
  expect_einval(vmp_create(&c, 0, seeds.data(), 0, &h), "create n_env 0");
  expect_einval(vmp_create(&c, 8, nullptr, 0, &h), "create null seeds");
  expect_einval(vmp_create(&c, 8, seeds.data(), 0, nullptr), "create null out");
  struct Bad { const char *what; void (*edit)(vmp_config &); } bad[] = {
      {"pms 0", [](vmp_config &x) { x.pms = 0; }},
      {"pms 70000", [](vmp_config &x) { x.pms = 70000; }},
      {"vms 0", [](vmp_config &x) { x.vms = 0; }},
      {"vms 20000", [](vmp_config &x) { x.vms = 20000; }},
      {"reward 7 (env.py:156)", [](vmp_config &x) { x.reward_function = 7; }},
      {"sequence 9", [](vmp_config &x) { x.sequence = 9; }},
      {"arrival_rate -1", [](vmp_config &x) { x.arrival_rate = -1; }},
      {"arrival_rate NaN", [](vmp_config &x) { x.arrival_rate = std::nan(""); }},
      {"service_length NaN", [](vmp_config &x) { x.service_length = std::nan(""); }},
  };
  for (auto &b : bad) {
    vmp_config x = base_cfg();
    b.edit(x);
    h = nullptr;
    expect_einval(vmp_create(&x, 8, seeds.data(), 0, &h), b.what);
    CHECK(h == nullptr, b.what);
  }
  seeds[5] = -3;
  expect_einval(vmp_create(&c, 8, seeds.data(), 0, &h), "negative seed");
  // every entry point on a null handle
  int32_t i32[4];
  float f[4];
  double d[4];
  uint8_t u8[4];
  int64_t i64[8];
  uint32_t u32[4];
  expect_einval(vmp_reset(nullptr, nullptr, nullptr, f), "reset null handle");
  expect_einval(vmp_step(nullptr, i32, f, d, u8, u8), "step null handle");
  expect_einval(vmp_heuristic_act(nullptr, 0, i32), "act null handle");
  expect_einval(vmp_heuristic_act_obs(nullptr, 0, f, i32), "act_obs null handle");
  expect_einval(vmp_heuristic_step(nullptr, 0, i32, f, d, u8, u8), "heuristic_step null handle");
  expect_einval(vmp_rollout_heuristic(nullptr, 0, 4, d, i64), "rollout null handle");
  expect_einval(vmp_mask(nullptr, u32), "mask null handle");
  expect_einval(vmp_mask_bool(nullptr, u8), "mask_bool null handle");
  expect_einval(vmp_get_obs(nullptr, f), "get_obs null handle");
  expect_einval(vmp_get_counters(nullptr, i64), "get_counters null handle");
  expect_einval(vmp_get_stats(nullptr, d), "get_stats null handle");
  expect_einval(vmp_get_rank(nullptr, i64), "get_rank null handle");
  expect_einval(vmp_set_eval(nullptr, 1), "set_eval null handle");
  expect_einval(vmp_set_stream(nullptr, nullptr), "set_stream null handle");
  expect_einval(vmp_record_enable(nullptr, 1), "record_enable null handle");
  expect_einval(vmp_record_read(nullptr, u32, d), "record_read null handle");
  expect_einval(vmp_debug_fail_alloc(-1), "fail_alloc negative");
  CHECK(vmp_destroy(nullptr) == VMP_OK, "destroy null");
  std::printf("ok  argument checks\n");
}

static size_t free_mem() {
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  return fr;
}

// One sweep: the n-th device allocation of vmp_create fails, for every n up to
// the first n past the last allocation. Returns the number of failure points.
static int create_sweep(const vmp_config &c, std::vector<int64_t> &seeds) {
  int n_fail = 0;
  for (int n = 1; n < 64; n++) {
    CHECK(vmp_debug_fail_alloc(n) == VMP_OK, "arm");
    vmp_handle *h = nullptr;
    const int64_t live = vmp_debug_live_allocs();
    const int rc = vmp_create(&c, (int32_t)seeds.size(), seeds.data(), 0, &h);
    vmp_debug_fail_alloc(0);
    if (rc != VMP_OK) CHECK(vmp_debug_live_allocs() == live, "no device allocation kept");
    if (rc == VMP_OK) {
      CHECK(h != nullptr, "handle");
      vmp_destroy(h);
      break;
    }
    CHECK(rc == VMP_EOOM, "create under injected OOM returns VMP_EOOM");
    CHECK(h == nullptr, "no handle on failure");
    n_fail++;
  }
  CHECK(hipDeviceSynchronize() == hipSuccess, "sync");
  return n_fail;
}

static void device_faults() {
  vmp_config c = base_cfg();
  // large enough that a leaked buffer shows in the free memory (vm words
  // 9.8 MB, PM state 6.6 MB, headers 1 MB at 4096 envs)
  std::vector<int64_t> seeds(4096);
  for (size_t i = 0; i < seeds.size(); i++) seeds[i] = 4 * (int64_t)i;
  vmp_handle *h = nullptr;
  // warm the runtime (code objects, pools) with one full sweep, then measure
  // the free device memory across three more: a leak on any failure path
  // grows it by at least one buffer per sweep
  const int n_fail = create_sweep(c, seeds);
  CHECK(n_fail >= 5, "vmp_create has its allocations behind dev_malloc");
  const size_t base = free_mem();
  const int64_t live0 = vmp_debug_live_allocs();
  for (int r = 0; r < 3; r++) CHECK(create_sweep(c, seeds) == n_fail, "same failure points");
  // exact: the library's own count of live device allocations; the runtime's
  // free-memory figure is printed for context (it keeps freed blocks cached)
  std::printf("ok  create: %d failure points; live device allocations %lld -> %lld; free device "
              "memory %zu -> %zu bytes over 3 sweeps\n", n_fail, (long long)live0,
              (long long)vmp_debug_live_allocs(), base, free_mem());
  CHECK(vmp_debug_live_allocs() == live0 && live0 == 0, "device allocations back to none");
  // record_enable / mask_bool on a live handle
  CHECK(vmp_create(&c, 64, seeds.data(), 0, &h) == VMP_OK, "create");
  for (int n = 1; n <= 9; n++) {  // warm: the recorder's first allocations
    vmp_debug_fail_alloc(n);
    (void)vmp_record_enable(h, 1);
    vmp_debug_fail_alloc(0);
  }
  const size_t with_handle = free_mem();
  const int64_t live_h = vmp_debug_live_allocs();
  for (int n = 1; n <= 9; n++) {
    vmp_debug_fail_alloc(n);
    CHECK(vmp_record_enable(h, 1) == VMP_EOOM, "record_enable under injected OOM");
    vmp_debug_fail_alloc(0);
    CHECK(vmp_debug_live_allocs() == live_h, "recorder buffers released after the failure");
  }
  CHECK(hipDeviceSynchronize() == hipSuccess, "sync");
  std::printf("ok  record_enable: 9 failure points; free device memory %zu -> %zu bytes\n",
              with_handle, free_mem());
  CHECK(vmp_record_enable(h, 1) == VMP_OK, "record_enable after the failures");
  float *obs = nullptr;
  double *rew = nullptr, *sums = nullptr;
  uint8_t *done = nullptr, *mask = nullptr;
  uint32_t *hist = nullptr;
  CHECK(hipMalloc(&obs, sizeof(float) * 64 * (3 * 300 + 2 * 100)) == hipSuccess, "obs");
  CHECK(hipMalloc(&rew, sizeof(double) * 64) == hipSuccess, "rew");
  CHECK(hipMalloc(&done, 64) == hipSuccess, "done");
  CHECK(hipMalloc(&mask, (size_t)64 * 300 * 102) == hipSuccess, "mask");
  CHECK(hipMalloc(&hist, sizeof(uint32_t) * 64 * 2 * VMP_REC_BINS) == hipSuccess, "hist");
  CHECK(hipMalloc(&sums, sizeof(double) * 64 * VMP_NREC) == hipSuccess, "sums");
  for (int t = 0; t < 20; t++)
    CHECK(vmp_heuristic_step(h, VMP_POLICY_BESTFIT, nullptr, obs, rew, done, nullptr) == VMP_OK,
          "heuristic_step");
  CHECK(vmp_record_read(h, hist, sums) == VMP_OK, "record_read");
  const int64_t live_r = vmp_debug_live_allocs();
  vmp_debug_fail_alloc(1);
  CHECK(vmp_mask_bool(h, mask) == VMP_EOOM, "mask_bool under injected OOM");
  vmp_debug_fail_alloc(0);
  CHECK(vmp_debug_live_allocs() == live_r, "mask_bool failure keeps nothing");
  CHECK(vmp_mask_bool(h, mask) == VMP_OK, "mask_bool after the failure");
  CHECK(hipDeviceSynchronize() == hipSuccess, "kernels ran");
  CHECK(vmp_destroy(h) == VMP_OK, "destroy");
  CHECK(vmp_debug_live_allocs() == 0, "destroy releases every device allocation");
  (void)hipFree(obs);
  (void)hipFree(rew);
  (void)hipFree(done);
  (void)hipFree(mask);
  (void)hipFree(hist);
  (void)hipFree(sums);
  std::printf("ok  device failure paths (%d vmp_create failure points)\n", n_fail);
}

int main(int argc, char **argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);  // every line out before a sanitizer abort
  argument_checks();
  const bool device = argc > 1 && std::strcmp(argv[1], "--device") == 0;
  if (!device) {
    vmp_config c = base_cfg();
    std::vector<int64_t> seeds(8, 0);
    vmp_handle *h = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
      const int rc = vmp_create(&c, 8, seeds.data(), 0, &h);
      CHECK(rc == VMP_EDEVICE && h == nullptr, "create without a device fails cleanly");
      std::printf("ok  create without a device: %s\n", vmp_last_error());
    }
  } else {
    device_faults();
  }
  // the leak check now, then leave without the HIP / HSA runtime teardown (its
  // static destructors trip ASan's device-allocator check at exit on ROCm 7.2,
  // a runtime / sanitizer interaction outside this library)
  const int leaks = __lsan_do_recoverable_leak_check();
  std::printf("leak check: %s\n", leaks ? "LEAKS" : "none");
  if (leaks) g_fail = 1;
  if (!g_fail) std::printf("capi faults ok\n");
  std::fflush(stdout);
  _exit(g_fail);
}
