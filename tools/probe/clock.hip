// clock.hip -- the GPU's shader clock while kernels run.  Boxes of the pool run the same kernels at
// different clocks (same cycle counts, different times), so bench.py reports what it measured:
//   light: one wave spins a dependent float32 loop (the clock a lightly loaded GPU boosts to);
//   loaded: four waves per SIMD on every CU spin float64 FMA chains, the issue load of k_bp (the
//           clock the power limit allows under the headline's dominant kernel).
// Each wave reads the shader-clock counter (clock64) and the constant-rate wall clock
// (wall_clock64) before and after its loop; the result is the median wave's cycles per second.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <vector>

__global__ void k_clock_light(unsigned long long* out, int iters) {
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

__global__ void k_clock_loaded(unsigned long long* out, int iters) {
  const unsigned long long c0 = clock64(), w0 = wall_clock64();
  double a = threadIdx.x, b = a + 1.0, c = a + 2.0, d = a + 3.0;
  for (int i = 0; i < iters; ++i) {  // four independent FP64 FMA chains per lane
    a = __builtin_fma(a, 0.999999, 1e-3);
    b = __builtin_fma(b, 0.999999, 1e-3);
    c = __builtin_fma(c, 0.999999, 1e-3);
    d = __builtin_fma(d, 0.999999, 1e-3);
  }
  const unsigned long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x] = c1 - c0;
    out[3 * blockIdx.x + 1] = w1 - w0;
    out[3 * blockIdx.x + 2] = (unsigned long long)((a + b + c + d) != (a + b + c + d));
  }
}

// loaded = 0: light, 1: loaded.  -> 0 and *ghz, else a HIP error code
extern "C" int ft8probe_clock_ghz(int device, int loaded, double* ghz) {
  if (!ghz) return -1;
  hipError_t e = hipSetDevice(device);
  int wall_khz = 0, cus = 0;
  if (e == hipSuccess) e = hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, device);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess || wall_khz <= 0 || cus <= 0) return e != hipSuccess ? (int)e : -2;
  const int waves = loaded ? 16 * cus : 1;  // four single-wave workgroups per SIMD
  unsigned long long* d = nullptr;
  e = hipMalloc(&d, 3 * sizeof(unsigned long long) * waves);
  std::vector<unsigned long long> h(3 * waves);
  double best = 0.0;
  for (int rep = 0; rep < (loaded ? 1 : 3) && e == hipSuccess; ++rep) {
    if (loaded) hipLaunchKernelGGL(k_clock_loaded, dim3(waves), dim3(64), 0, 0, d, 400000);
    else hipLaunchKernelGGL(k_clock_light, dim3(1), dim3(64), 0, 0, d, 2000000);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(h.data(), d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    if (e != hipSuccess) break;
    std::vector<double> g;
    for (int w = 0; w < waves; ++w)
      if (h[3 * w + 1] > 0) g.push_back((double)h[3 * w] / ((double)h[3 * w + 1] / ((double)wall_khz * 1e3)) / 1e9);
    if (g.empty()) continue;
    std::nth_element(g.begin(), g.begin() + g.size() / 2, g.end());
    best = std::max(best, g[g.size() / 2]);
  }
  if (d) (void)hipFree(d);
  if (e != hipSuccess) return (int)e;
  *ghz = best;
  return 0;
}
