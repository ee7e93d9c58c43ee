// clock.hip -- the GPU's shader clock while a kernel runs: one wave spins a fixed dependent loop
// and reads the shader-clock counter (clock64) and the constant-rate wall clock (wall_clock64)
// before and after it.  Boxes of the pool run the same kernels at different clocks (same cycle
// counts, different times), so bench.py reports the clock it measured beside its numbers.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void k_clock(unsigned long long* out, int iters) {
  const unsigned long long c0 = clock64(), w0 = wall_clock64();
  float x = (float)threadIdx.x;
  for (int i = 0; i < iters; ++i) x = x * 1.000001f + 0.5f;  // dependent chain: the wave stays busy
  const unsigned long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
    out[2] = (unsigned long long)(x != x);  // keeps the loop
  }
}

// -> 0 and *ghz = shader-clock cycles / elapsed wall-clock time (GHz), else a HIP error code
extern "C" int ft8probe_clock_ghz(int device, double* ghz) {
  if (!ghz) return -1;
  hipError_t e = hipSetDevice(device);
  int wall_khz = 0;
  if (e == hipSuccess) e = hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, device);
  unsigned long long* d = nullptr;
  if (e == hipSuccess) e = hipMalloc(&d, 3 * sizeof(unsigned long long));
  unsigned long long h[3] = {0, 0, 0};
  double best = 0.0;
  for (int rep = 0; rep < 3 && e == hipSuccess; ++rep) {
    hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, d, 2000000);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    if (e == hipSuccess && h[1] > 0 && wall_khz > 0) {
      const double g = (double)h[0] / ((double)h[1] / ((double)wall_khz * 1e3)) / 1e9;
      if (g > best) best = g;
    }
  }
  if (d) (void)hipFree(d);
  if (e != hipSuccess) return (int)e;
  *ghz = best;
  return 0;
}
