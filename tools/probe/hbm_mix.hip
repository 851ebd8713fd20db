// HBM probe for the env-step access mix: each 64-lane wave
// owns one "env" and streams R bytes in (16-B loads) and W bytes out (16-B
// non-temporal stores), no compute — the memory-only bound of k_env's traffic
// (P100 / V1000: ~9.9 KB read, ~22.7 KB written per env-step), plus the pure
// read and pure write lines.
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

int main(int argc, char **argv) {
  const int n_env = argc > 1 ? atoi(argv[1]) : 32768;
  const int rb = argc > 2 ? atoi(argv[2]) : 9920, wb = argc > 3 ? atoi(argv[3]) : 22640;
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
      hipLaunchKernelGGL(k_mix, dim3((n_env + 3) / 4), dim3(256), 0, 0, in, out, rr, ww, n_env, sink);
    if (hipEventRecord(a, 0)) return 1;
    const int n = 20;
    for (int it = 0; it < n; it++)
      hipLaunchKernelGGL(k_mix, dim3((n_env + 3) / 4), dim3(256), 0, 0, in, out, rr, ww, n_env, sink);
    float ms;
    if (hipEventRecord(b, 0) || hipEventSynchronize(b) || hipEventElapsedTime(&ms, a, b)) return 1;
    ms /= n;
    const double bytes = (double)n_env * 16.0 * (rr + ww);
    printf("{\"case\": \"%s\", \"envs\": %d, \"read_B\": %d, \"write_B\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
           names[c], n_env, rr * 16, ww * 16, ms, bytes / ms / 1e6);
  }
  return 0;
}
