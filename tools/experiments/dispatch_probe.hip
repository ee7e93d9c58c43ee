// Workgroup-dispatch floor on gfx950: how long a grid of N workgroups of T threads with L bytes
// of dynamic LDS takes when each workgroup does (almost) nothing -- one float store per thread,
// a barrier, and `work` dependent VALU steps per thread.  Compares k_score2's launch shape (15 360
// workgroups x 512 threads, 17 KB LDS) with fewer, larger workgroups and a persistent loop.
//   hipcc --offload-arch=gfx950 -O3 -o dispatch_probe dispatch_probe.hip && ./dispatch_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void k_probe(float* out, int tiles, int work) {
  extern __shared__ float lds[];
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    float x = (float)(t + threadIdx.x);
    lds[threadIdx.x] = x;
    __syncthreads();
    x += lds[(threadIdx.x + 1) & 511];
    for (int i = 0; i < work; ++i) x = x * 1.0001f + 0.5f;
    __syncthreads();
    if (x == -1.0f) out[t] = x;  // never true: keeps the loop alive
  }
}

int main() {
  float* d = nullptr;
  if (hipMalloc(&d, 1 << 20) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct Case { int grid, tiles, lds, work; const char* what; };
  const std::vector<Case> cases = {
      {15360, 15360, 17280, 0, "k_score2 shape, empty"},
      {15360, 15360, 17280, 64, "k_score2 shape, 64 steps"},
      {7680, 7680, 17280, 0, "half the workgroups, empty"},
      {1024, 15360, 17280, 0, "persistent 1024 x 15 tiles, empty"},
      {1024, 15360, 17280, 64, "persistent 1024, 64 steps"},
      {15360, 15360, 0, 0, "k_score2 shape, no LDS"},
  };
  for (const Case& c : cases) {
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_probe, dim3(c.grid), dim3(512), c.lds, 0, d, c.tiles, c.work);
    hipDeviceSynchronize();
    const int n = 50;
    hipEventRecord(e0, 0);
    for (int rep = 0; rep < n; ++rep) hipLaunchKernelGGL(k_probe, dim3(c.grid), dim3(512), c.lds, 0, d, c.tiles, c.work);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::printf("%-40s grid %6d tiles %6d lds %6d: %.4f ms per launch\n", c.what, c.grid, c.tiles, c.lds, ms / n);
  }
  hipFree(d);
  return 0;
}
