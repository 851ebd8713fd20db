// HBM probe for the env-step access mix: each 64-lane wave
// owns one "env" and streams R bytes in (16-B loads) and W bytes out (16-B
// non-temporal stores), no compute — the memory-only bound of k_env's traffic
// (P100 / V1000: ~9.9 KB read, ~22.7 KB written per env-step), plus the pure
// read and pure write lines.
// `hbm_mix block N NT R W LDS`: the same with one workgroup per env (the
// k_env_big shape, LDS-limited residency).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/hbm_mix tools/probe/hbm_mix.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mix(const f4 *in, f4 *out, int r4, int w4, int n_env,
                                             float *sink) {
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= n_env) return;
  const f4 *src = in + (size_t)e * r4;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i = lane; i < r4; i += 64) acc += src[i];
  f4 *dst = out + (size_t)e * w4;
  const f4 v = acc * 0.5f;
  for (int i = lane; i < w4; i += 64) __builtin_nontemporal_store(v, dst + i);
  if (acc[0] == 12345.f) sink[0] = acc[1];
}

// One workgroup per env (k_env_big's shape): NT threads stream R bytes in and
// W bytes out as 8-B words, thread t taking words t, t + NT, ...
__global__ void k_block(const uint64_t *in, uint64_t *out, int r8, int w8, float *sink) {
  extern __shared__ char pad[];
  const int t = threadIdx.x, nt = blockDim.x, e = blockIdx.x;
  const uint64_t *src = in + (size_t)e * r8;
  uint64_t acc = 0;
  for (int i = t; i < r8; i += nt) acc += src[i];
  uint64_t *dst = out + (size_t)e * w8;
  for (int i = t; i < w8; i += nt) __builtin_nontemporal_store(acc + i, dst + i);
  if (acc == 12345u) sink[0] = (float)pad[0];
}

int block_mode(int argc, char **argv) {
  // block N NT R W LDS
  const int n = atoi(argv[2]), nt = atoi(argv[3]), rb = atoi(argv[4]), wb = atoi(argv[5]);
  const int lds = argc > 6 ? atoi(argv[6]) : 0;
  const int r8 = rb / 8, w8 = wb / 8;
  uint64_t *in, *out;
  float *sink;
  if (hipMalloc(&in, (size_t)n * r8 * 8 + 8) || hipMalloc(&out, (size_t)n * w8 * 8 + 8) ||
      hipMalloc(&sink, 4))
    return 1;
  if (hipMemset(in, 0, (size_t)n * r8 * 8)) return 1;
  hipEvent_t a, b;
  if (hipEventCreate(&a) || hipEventCreate(&b)) return 1;
  const int cases[3][2] = {{r8, w8}, {r8, 0}, {0, w8}};
  const char *names[3] = {"block read R + write W", "block read R", "block write W"};
  for (int c = 0; c < 3; c++) {
    for (int it = 0; it < 3; it++)
      hipLaunchKernelGGL(k_block, dim3(n), dim3(nt), lds, 0, in, out, cases[c][0], cases[c][1], sink);
    if (hipEventRecord(a, 0)) return 1;
    const int reps = 20;
    for (int it = 0; it < reps; it++)
      hipLaunchKernelGGL(k_block, dim3(n), dim3(nt), lds, 0, in, out, cases[c][0], cases[c][1], sink);
    float ms;
    if (hipEventRecord(b, 0) || hipEventSynchronize(b) || hipEventElapsedTime(&ms, a, b)) return 1;
    ms /= reps;
    const double bytes = (double)n * 8.0 * (cases[c][0] + cases[c][1]);
    printf("{\"case\": \"%s\", \"blocks\": %d, \"threads\": %d, \"read_B\": %d, \"write_B\": %d, \"lds_per_block\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
           names[c], n, nt, cases[c][0] * 8, cases[c][1] * 8, lds, ms, bytes / ms / 1e6);
  }
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && argv[1][0] == 'b') return block_mode(argc, argv);
  const int n_env = argc > 1 ? atoi(argv[1]) : 32768;
  const int rb = argc > 2 ? atoi(argv[2]) : 9920, wb = argc > 3 ? atoi(argv[3]) : 22640;
  // dynamic LDS per 4-wave block: caps the resident waves like k_env's carve
  // (43.6 KB -> 3 blocks = 12 waves per CU; 60 KB -> 2 blocks = 8 waves)
  const int lds = argc > 4 ? atoi(argv[4]) : 0;
  const int r4 = (rb + 15) / 16, w4 = (wb + 15) / 16;
  f4 *in, *out;
  float *sink;
  if (hipMalloc(&in, (size_t)n_env * r4 * 16) || hipMalloc(&out, (size_t)n_env * w4 * 16) ||
      hipMalloc(&sink, 4))
    return 1;
  if (hipMemset(in, 0, (size_t)n_env * r4 * 16)) return 1;
  hipEvent_t a, b;
  if (hipEventCreate(&a) || hipEventCreate(&b)) return 1;
  const int cases[3][2] = {{r4, w4}, {r4, 0}, {0, w4}};  // never read past the R-byte rows
  const char *names[3] = {"env mix (read R, write W)", "read only R", "write only W"};
  for (int c = 0; c < 3; c++) {
    const int rr = cases[c][0], ww = cases[c][1];
    for (int it = 0; it < 3; it++)
      hipLaunchKernelGGL(k_mix, dim3((n_env + 3) / 4), dim3(256), lds, 0, in, out, rr, ww, n_env, sink);
    if (hipEventRecord(a, 0)) return 1;
    const int n = 20;
    for (int it = 0; it < n; it++)
      hipLaunchKernelGGL(k_mix, dim3((n_env + 3) / 4), dim3(256), lds, 0, in, out, rr, ww, n_env, sink);
    float ms;
    if (hipEventRecord(b, 0) || hipEventSynchronize(b) || hipEventElapsedTime(&ms, a, b)) return 1;
    ms /= n;
    const double bytes = (double)n_env * 16.0 * (rr + ww);
    printf("{\"case\": \"%s\", \"envs\": %d, \"read_B\": %d, \"write_B\": %d, \"lds_per_block\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
           names[c], n_env, rr * 16, ww * 16, lds, ms, bytes / ms / 1e6);
  }
  return 0;
}
