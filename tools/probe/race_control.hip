// race_control.hip -- positive control for the barrier-race check build (ft8_internal.h
// FT8_RACE_PROLOGUE, tools/build_race.sh).  Always compiled with -DFT8_RACE_CHECK.
//
// k_race_control: a 4-wave workgroup with `dyn` bytes of dynamic LDS on top of 1 KB static.  Every
// thread first checks that its slots of BOTH allocations read the sentinel the prologue wrote (so
// the prologue sized its fill from the dispatch packet's group_segment_size, dynamic part
// included), then writes its value, then -- with `barrier` = 0 deliberately WITHOUT a barrier --
// reads the value of the thread 64 places on (the next wave).  Under the prologue one wave of each
// workgroup starts ~64 k cycles late, so the wave before it reads the sentinel: the control must
// report races with barrier = 0 and none with barrier = 1.
#include <hip/hip_runtime.h>

#include "../../ft8_demodulator_amd/csrc/ft8_internal.h"

#ifndef FT8_RACE_CHECK
#error "race_control.hip is built with -DFT8_RACE_CHECK only"
#endif

__global__ __launch_bounds__(256) void k_race_control(int barrier, int dyn_words, unsigned* counts) {
  FT8_RACE_PROLOGUE();
  __shared__ unsigned st[256];
  extern __shared__ unsigned dl[];
  const int t = threadIdx.x;
  unsigned unfilled = 0;
  if (st[t] != 0xffffffffu) ++unfilled;
  for (int i = t; i < dyn_words; i += 256)
    if (dl[i] != 0xffffffffu) ++unfilled;
  st[t] = 1000u + (unsigned)t;
  if (barrier) __syncthreads();
  const unsigned v = st[(t + 64) & 255];
  const unsigned raced = (v != 1000u + (unsigned)((t + 64) & 255)) ? 1u : 0u;
  atomicAdd(&counts[0], raced);
  atomicAdd(&counts[1], unfilled);
}

// counts[0] = reads that saw another wave's slot unwritten, counts[1] = LDS words the prologue did
// not fill.  -> 0 or a HIP error code
extern "C" int ft8probe_race_control(int barrier, int workgroups, int dyn_bytes, unsigned* host_counts) {
  unsigned* d = nullptr;
  hipError_t e = hipMalloc(&d, 2 * sizeof(unsigned));
  if (e == hipSuccess) e = hipMemset(d, 0, 2 * sizeof(unsigned));
  if (e == hipSuccess && dyn_bytes > 48 * 1024)
    e = hipFuncSetAttribute((const void*)k_race_control, hipFuncAttributeMaxDynamicSharedMemorySize, dyn_bytes);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_race_control, dim3(workgroups), dim3(256), dyn_bytes, 0, barrier, dyn_bytes / 4, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(host_counts, d, 2 * sizeof(unsigned), hipMemcpyDeviceToHost);
  if (d) (void)hipFree(d);
  return (int)e;
}
