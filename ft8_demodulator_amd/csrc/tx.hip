// tx.hip -- FT8 transmit chain on gfx950: message encoding and GFSK waveform synthesis.
//
// k_encode  one thread per message: payload -> a91 (CRC-14) -> codeword (LDPC generator) -> tones
//           (ft8_generator/crc.py:25-47, ldpc.py:104-131, encoder.py:15-73).
// k_synth   one workgroup per (slot, tile of kSynTile samples): every signal of the slot that
//           overlaps the tile is evaluated sample-parallel with the closed-form GFSK phase of
//           tx_device.h and accumulated in registers, then added to the output once, so the sum
//           over overlapping signals has a fixed order (deterministic) and the output is touched
//           once per tile (modulator.py:27-90 gfsk_modulation_waveform_generator,
//           ft8_modulation_waveform_generator, ft8_generator).
#include "tx_device.h"

namespace ft8 {
namespace {

constexpr int kSynThreads = 256;
constexpr int kSynPer = 8;
constexpr int kSynTile = kSynThreads * kSynPer;

__global__ void k_encode(const uint8_t* msg, int msg_bytes, int n, uint8_t* a91, uint8_t* cw, uint8_t* tones) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  tx::encode(msg + (int64_t)i * msg_bytes, msg_bytes, a91 ? a91 + (int64_t)i * 12 : nullptr, cw ? cw + (int64_t)i * 22 : nullptr,
             tones ? tones + (int64_t)i * tx::kSymbols : nullptr);
}

// first index in [0, n) whose slot is >= s (signals sorted by slot)
__device__ int lower_slot(const ft8_tx_signal* sig, int n, int s) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (sig[mid].slot < s) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <bool CPLX, typename OT, typename AT>
__global__ __launch_bounds__(kSynThreads) void k_synth(SynthLaunch a) {
  FT8_RACE_PROLOGUE();
  __shared__ int s_E[tx::kExt];
  __shared__ int s_PS[tx::kExt + 1];
  __shared__ int s_range[2];
  const int slot = blockIdx.y;
  const int64_t t0 = (int64_t)blockIdx.x * kSynTile;
  if (threadIdx.x == 0) {
    s_range[0] = lower_slot(a.sig, a.n_sig, slot);
    s_range[1] = lower_slot(a.sig, a.n_sig, slot + 1);
  }
  __syncthreads();
  const int lo = s_range[0], hi = s_range[1];
  const int nsps = a.nsps, L = tx::kSymbols * nsps;
  const int off = a.style == 1 ? 0 : nsps;
  AT re[kSynPer], im[kSynPer];
#pragma unroll
  for (int k = 0; k < kSynPer; ++k) re[k] = im[k] = (AT)0;
  for (int i = lo; i < hi; ++i) {
    const ft8_tx_signal sg = a.sig[i];
    if (sg.start >= t0 + kSynTile || sg.start + L <= t0) continue;  // uniform
    __syncthreads();
    const uint8_t* tn = a.tones + (int64_t)i * tx::kSymbols;
    if (threadIdx.x < tx::kExt) {
      const int j = (int)threadIdx.x - 1;  // e_j
      s_E[threadIdx.x] = tn[j < 0 ? 0 : (j > tx::kSymbols - 1 ? tx::kSymbols - 1 : j)];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = 0;
      for (int k = 0; k <= tx::kExt; ++k) {
        s_PS[k] = acc;
        if (k < tx::kExt) acc += s_E[k];
      }
    }
    __syncthreads();
    const double G0 = tx::gfsk_G<double, double>(s_E, s_PS, a.P, nsps, off);
    const double inv_fs = 1.0 / a.fs;
#pragma unroll
    for (int k = 0; k < kSynPer; ++k) {
      const int64_t nabs = t0 + threadIdx.x + (int64_t)k * kSynThreads;
      const int64_t n64 = nabs - sg.start;
      if (n64 < 0 || n64 >= L || nabs >= a.n_samples) continue;
      const int n = (int)n64;
      const double G = tx::gfsk_G<double, double>(s_E, s_PS, a.P, nsps, n + off);
      const double cyc = (sg.f0 * (double)n + 6.25 * (G - G0)) * inv_fs;
      const double fr = cyc - floor(cyc);
      const AT r = tx::gfsk_ramp<AT>(n, L, nsps, a.style) * (AT)sg.amplitude;
      const AT psi = (AT)(2.0 * M_PI) * (AT)fr + (AT)sg.phase;
      AT sn, cs;
      if constexpr (sizeof(AT) == 8) sincos(psi, &sn, &cs);
      else sincosf(psi, &sn, &cs);
      // baseband sin(phi) - j cos(phi) (modulator.py:65), real part = ft8_generator's output
      re[k] += r * sn;
      if constexpr (CPLX) im[k] -= r * cs;
    }
  }
  OT* out = (OT*)a.out;
#pragma unroll
  for (int k = 0; k < kSynPer; ++k) {
    const int64_t nabs = t0 + threadIdx.x + (int64_t)k * kSynThreads;
    if (nabs >= a.n_samples) continue;
    const int64_t o = (int64_t)slot * a.slot_stride + nabs;
    if constexpr (CPLX) {
      out[2 * o] = (OT)((AT)out[2 * o] + re[k]);
      out[2 * o + 1] = (OT)((AT)out[2 * o + 1] + im[k]);
    } else {
      out[o] = (OT)((AT)out[o] + re[k]);
    }
  }
}

}  // namespace

hipError_t launch_encode(const uint8_t* msg, int msg_bytes, int n, uint8_t* a91, uint8_t* cw, uint8_t* tones,
                         hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_encode, dim3((n + 127) / 128), dim3(128), 0, s, msg, msg_bytes, n, a91, cw, tones);
  return hipGetLastError();
}

hipError_t launch_synth(const SynthLaunch& a, hipStream_t s) {
  if (a.n_slots <= 0 || a.n_samples <= 0) return hipSuccess;
  dim3 grid((unsigned)((a.n_samples + kSynTile - 1) / kSynTile), (unsigned)a.n_slots);
  switch (a.dtype) {
    case FT8_F32: hipLaunchKernelGGL((k_synth<false, float, float>), grid, dim3(kSynThreads), 0, s, a); break;
    case FT8_F64: hipLaunchKernelGGL((k_synth<false, double, double>), grid, dim3(kSynThreads), 0, s, a); break;
    case FT8_C64: hipLaunchKernelGGL((k_synth<true, float, float>), grid, dim3(kSynThreads), 0, s, a); break;
    case FT8_C128: hipLaunchKernelGGL((k_synth<true, double, double>), grid, dim3(kSynThreads), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace ft8
