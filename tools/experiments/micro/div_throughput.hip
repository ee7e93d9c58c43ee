// Microbenchmark: wave64 issue cost of f64 division variants on gfx950 (tools/micro, not product).
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 8
#define ITERS 256
__device__ __forceinline__ double div_full(double x, double y) { return x / y; }
__device__ __forceinline__ double div_fast(double x, double y) {
  double r = __builtin_amdgcn_rcp(y);
  double e = __builtin_fma(-y, r, 1.0); r = __builtin_fma(r, e, r);
  e = __builtin_fma(-y, r, 1.0); r = __builtin_fma(r, e, r);
  double m = x * r; e = __builtin_fma(-y, m, x);
  return __builtin_fma(e, r, m);
}
template <int MODE>
__global__ void k(double* out, double seed) {
  double a[N], b[N];
  for (int i = 0; i < N; ++i) { a[i] = seed + threadIdx.x * 1e-3 + i; b[i] = 945.0 + i + threadIdx.x; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if (MODE == 0) { b[i] = b[i] + a[i]; a[i] = div_full(a[i], b[i]) + 1.0; }
      else if (MODE == 1) { b[i] = b[i] + a[i]; a[i] = div_fast(a[i], b[i]) + 1.0; }
      else if (MODE == 7) { b[i] = b[i] + a[i]; a[i] = a[i] * b[i] + 1.0; }
      else if (MODE == 2) a[i] = __builtin_fma(a[i], b[i], 1.0);
      else if (MODE == 3) a[i] = __builtin_amdgcn_rcp(a[i]) + 1.0;
      else if (MODE == 4) { bool f; a[i] = __builtin_amdgcn_div_scale(a[i], b[i], true, &f) + 1.0; }
      else if (MODE == 5) a[i] = __builtin_amdgcn_div_fixup(a[i], b[i], 3.0) + 1.0;
      else if (MODE == 6) a[i] = __builtin_amdgcn_div_fmas(a[i], b[i], 1.0, threadIdx.x & 1) + 1.0;
    }
  }
  double s = 0; for (int i = 0; i < N; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int MODE> float run(double* d, int blocks, int threads) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, d, 1.5);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, d, 1.5);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); return ms / 5;
}
int main() {
  int blocks = 256 * 4 * 8, threads = 64;  // 8 waves per SIMD
  double* d; hipMalloc(&d, sizeof(double) * blocks * threads);
  const char* names[] = {"div_full(+2add)", "div_fast(+2add)", "fma", "rcp(+add)", "div_scale(+add)", "div_fixup(+add)", "div_fmas(+add)", "mul(+2add)"};
  float t[8] = {run<0>(d, blocks, threads), run<1>(d, blocks, threads), run<2>(d, blocks, threads), run<3>(d, blocks, threads),
                run<4>(d, blocks, threads), run<5>(d, blocks, threads), run<6>(d, blocks, threads), run<7>(d, blocks, threads)};
  // cycles per (wave, op) per SIMD: waves per SIMD * ops per wave
  double waves_per_simd = (double)blocks / 1024.0, ops = (double)ITERS * N;
  for (int m = 0; m < 8; ++m)
    printf("%-18s %8.3f ms  %7.2f SIMD-cycles per wave-op @2.4GHz\n", names[m], t[m], t[m] * 1e-3 * 2.4e9 / (waves_per_simd * ops));
  return 0;
}
