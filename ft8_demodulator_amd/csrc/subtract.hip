// subtract.hip -- subtract-and-redecode support (FT8_FLAG_SUBTRACT, gfx950).
//
// Build-defined: the reference decodes one pass (ft8_decode.py:288-394) and has no subtraction;
// SURVEY.md section 8(f) item 1 asks for it as the next step after the reference path.  The
// re-modulation uses the transmit chain of tx_device.h (the reference generator's encoder and GFSK
// modulator, ft8_generator/encoder.py:15-73, modulator.py:27-90) with the protocol timing.
//
// k_sub_est  one workgroup per decoded record (records of one slot on one XCD, so the slot's
//            samples stay in one L2), skipped for failed records and repeated payloads:
//   1. tones = encode(payload);
//   2. baseband: the samples around the candidate are mixed down to the centre of the 8-tone band
//      and box-car decimated to Q samples per symbol (D = nsps / Q input samples each);
//   3. fine sync: over start offsets of +-hop/2 (in steps of D samples) and tone-0 offsets of
//      +-bin/2 (5 points) the known tone sequence is correlated symbol by symbol
//      (coherent within a symbol, power summed over the 79 symbols); the best point is refined by
//      a parabola through its neighbours in each direction;
//   4. the complex amplitude of every symbol is fitted against the refined GFSK waveform
//      (A_k = 2 sum x conj(c) r / sum r^2, r the ramp) and smoothed [1 2 1] / 4 over symbols.
// k_sub_apply one workgroup per (slot, tile): residual = x - sum over the slot's fitted signals of
//            r(n) Re(A(n) exp(i psi(n))), A linearly interpolated between symbol centres; signals
//            summed in record order (deterministic).
// k_merge    one wave per slot: pass-2 records with a payload not decoded in pass 1 are appended.
#include <algorithm>
#include <mutex>
#include <type_traits>

#include "tx_device.h"

namespace ft8 {
namespace {

constexpr int kSubThreads = 256;
constexpr int kSubRecStride = 32;               // k_sub_est workgroups per slot (a crowded slot: ~21 fits)
constexpr int kSubRestStride = 8;               // ... and per slot in the rest launch (fits >= 32)
constexpr int kSubWaves = kSubThreads / kWave;
constexpr int kMaxQ = 32;
constexpr int kMaxHyp = 1024;
constexpr int kMaxT = kMaxQ + 3;                // start offsets searched: 2 ceil(Q / (2 sps)) + 1
constexpr int kMf = 2;                         // tone-0 search: 2 kMf + 1 points over +-bin/2
// float2 words of k_sub_est's padded baseband rows (-1 .. 81 of Q + 1), rounded up to a 16-B multiple;
// the decimation's twiddle table [D] follows them
__host__ __device__ inline int z_words(int Q) { return ((tx::kSymbols + 4) * (Q + 1) + 1) & ~1; }

// the fitted signal of one record: the public ft8_sub_fit (include/ft8hip.h, ft8_subtract_fits)
using SubEst = ft8_sub_fit;
static_assert(sizeof(((SubEst*)nullptr)->amp) / sizeof(float[2]) == tx::kSymbols, "one amplitude per symbol");

template <typename InT>
__device__ __forceinline__ float ld_sample(const InT* x, int64_t i);
template <>
__device__ __forceinline__ float ld_sample<float>(const float* x, int64_t i) { return x[i]; }
template <>
__device__ __forceinline__ float ld_sample<int16_t>(const int16_t* x, int64_t i) {
  return (float)x[i] / 32767.0f;  // read_wave_file scaling, as the STFT applies it
}

__device__ __forceinline__ float ramp_f(int n, int L, int nsps) { return tx::gfsk_ramp<float>(n, L, nsps, 0); }
// k_sub_list: one wave per slot lists the records worth a fit -- ok, and the first record of the
// slot carrying its payload (a crowded top-k slot decodes ~40 records for ~21 distinct messages) --
// in record order, and marks every record inactive (k_sub_est then activates the ones it fits), so
// k_sub_est's workgroups index fits directly instead of one workgroup per record testing itself
__global__ __launch_bounds__(kWave) void k_sub_list(SubLaunch a) {
  const int slot = blockIdx.x, lane = threadIdx.x;
  const int cnt = min(a.counts[slot], a.cap);
  const ft8_result* rs = a.res + (int64_t)slot * a.cap;
  SubEst* est = reinterpret_cast<SubEst*>(a.est) + (int64_t)slot * a.cap;
  int32_t* list = a.list + (int64_t)slot * (a.cap + 1);
  int n = 0;
  for (int j0 = 0; j0 < cnt; j0 += kWave) {
    const int j = j0 + lane;
    bool keep = false;
    if (j < cnt) {
      const ft8_result r = rs[j];
      keep = r.ok != 0;
      for (int q = 0; q < j && keep; ++q) {
        if (!rs[q].ok) continue;
        bool eq = true;
        for (int b = 0; b < 10; ++b) eq = eq && rs[q].payload[b] == r.payload[b];
        keep = !eq;
      }
      est[j].active = 0;
    }
    const uint64_t m = __ballot(keep);
    if (keep) list[n + __popcll(m & ((1ull << lane) - 1ull))] = j;
    n += __popcll(m);
  }
  if (lane == 0) list[a.cap] = n;
}

// REST = false: workgroup rec0 of a slot fits record rec0 (no loop: 108 VGPRs, four waves per
// SIMD); REST = true: the records past kSubRecStride, kSubRecStride + rec0 + j kSubRestStride (a
// loop over records lets the compiler keep loop-invariant values live: ~170 VGPRs), a second
// launch whose workgroups exit at once unless a slot decoded more than kSubRecStride messages
template <typename InT, bool REST>
__global__ __launch_bounds__(kSubThreads) void k_sub_est(SubLaunch a) {
  FT8_RACE_PROLOGUE();
  // dynamic LDS: the decimated baseband z (phases 2-3), then the float pulse table (phase 4).  z is
  // stored in rows of Q + 1 (one pad): row r + 1 holds z[1 + r Q .. 1 + (r + 1) Q), r = -1 .. 81,
  // so symbol k's window starts a row (z_at below) and the lanes' reads (one symbol per lane) are
  // 2 (Q + 1) dwords apart -- distinct banks for even Q.  Unpadded, the lanes of a ds_read_b64
  // were 2 Q dwords apart: at Q = 32 one bank for all 32 lanes of a group (32-way conflicts; 169 M
  // conflict cycles per 334-slot launch, r4_v30_sub_pmc.json)
  extern __shared__ float4 s_dyn[];
  float2* s_z = reinterpret_cast<float2*>(s_dyn);
  float4* s_D = s_dyn;  // phase 4: the pulse table's symbol-relative differences (see k_sub_apply)
  __shared__ float s_metric[kMaxHyp];
  __shared__ int s_E[tx::kExt];
  __shared__ int s_PS[tx::kExt + 1];
  __shared__ uint8_t s_tones[80];
  __shared__ float s_ph0[tx::kSymbols + 1];
  __shared__ float2 s_A[tx::kSymbols];
  __shared__ int s_flag;

  // records of one slot on one XCD (workgroup id % 8); kSubRecStride workgroups per slot, each
  // taking records rec0, rec0 + kSubRecStride, ... (a slot decodes ~20: one record per workgroup,
  // instead of round 3's one workgroup per record slot of the capacity, ~93 % of them empty)
  const int w = blockIdx.x;
  const int j8 = w / 8;
  constexpr int kStride = REST ? kSubRestStride : kSubRecStride;
  const int slot = (w % 8) + 8 * (j8 / kStride);
  const int rec0 = j8 % kStride;
  if (slot >= a.n_slots) return;
  const int32_t* list = a.list + (int64_t)slot * (a.cap + 1);
  const int nfit = list[a.cap];
  for (int i = rec0 + (REST ? kSubRecStride : 0); i < nfit; i += kStride) {
  __syncthreads();  // the previous record's LDS reads are done
  const int rec = list[i];
  SubEst* est = reinterpret_cast<SubEst*>(a.est) + (int64_t)slot * a.cap + rec;
  const ft8_result* rs = a.res + (int64_t)slot * a.cap;
  const ft8_result r = rs[rec];  // ok, and its payload's first record in the slot (k_sub_list)
  if (threadIdx.x < kWave) tx::encode_tones_wave(r.payload, threadIdx.x, s_tones);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int k = 0; k < tx::kExt; ++k) {
      const int j = k - 1;
      const int e = s_tones[j < 0 ? 0 : (j > tx::kSymbols - 1 ? tx::kSymbols - 1 : j)];
      s_E[k] = e;
      s_PS[k] = acc;
      acc += e;
    }
    s_PS[tx::kExt] = acc;
  }
  __syncthreads();

  const InT* x = reinterpret_cast<const InT*>(a.x) + (int64_t)slot * a.slot_stride;
  const int nsps = a.nsps, Q = a.Q, D = nsps / Q, L = tx::kSymbols * nsps;
  const int Mt = (Q + 2 * (nsps / a.hop) - 1) / (2 * (nsps / a.hop));  // ceil((hop / 2) / D)
  const int Mg = Mt + 1;
  const int Mz = tx::kSymbols * Q + 2 * Mg;
  // z[m] -> its padded position (m >= 0; Mg - Mt = 1 is the first window's start)
  auto z_at = [Q](int m) { const int u = m - 1 + Q; return u + (int)((unsigned)u / (unsigned)Q); };
  const double fs = (double)a.fs;
  const int64_t s0 = (int64_t)(a.t_lo + r.abs_time) * a.hop;
  const double ftone = (double)(a.f_lo + r.abs_freq) * fs / (double)a.nfft;
  const double fmix = ftone + 3.5 * 6.25;

  // ---- 2. mixed-down, box-car decimated baseband z[m], samples [nb + m D, nb + (m + 1) D):
  // z[m] = w_m sum_i x[nb + m D + i] t_i with t_i = exp(-2 pi i fmix i / fs) (a table of D twiddles
  // in LDS, each from the exact phase) and w_m = exp(-2 pi i fmix (nb + m D) / fs).  A thread owns
  // z[tid + 256 j]: two fmas per sample.  (Round 4 rotated a per-z phasor by one complex multiply
  // per sample, ~20 VALU per sample with its per-sample range tests.)  Records whose window lies
  // inside the slot (all but the slot's edges) read float32 samples four at a time, unchecked.
  {
    constexpr int kZ = (tx::kSymbols * kMaxQ + 2 * (kMaxQ / 2 + 2) + kSubThreads - 1) / kSubThreads;
    const int64_t nb = s0 - (int64_t)Mg * D;
    float2* s_tw = s_z + z_words(Q);
    for (int i = threadIdx.x; i < D; i += kSubThreads) {
      const double cyc = fmix * (double)i / fs;
      float sn, cs;
      sincospif((float)(-2.0 * (cyc - floor(cyc))), &sn, &cs);
      s_tw[i] = make_float2(cs, sn);
    }
    __syncthreads();
    const bool inside = nb >= 0 && nb + (int64_t)Mz * D <= a.n_samples;  // workgroup-uniform
#pragma unroll 1
    for (int j = 0; j < kZ; ++j) {
      const int m = threadIdx.x + j * kSubThreads;
      if (m >= Mz) break;
      const int64_t n0 = nb + (int64_t)m * D;
      const InT* xp = x + n0;
      float ax = 0.f, ay = 0.f;
      if (std::is_same<InT, float>::value && inside && (D & 3) == 0) {
        for (int i = 0; i < D; i += 4) {
          float4 v;
          __builtin_memcpy(&v, xp + i, sizeof(v));  // 4-byte aligned
          const float4 t01 = *reinterpret_cast<const float4*>(s_tw + i);
          const float4 t23 = *reinterpret_cast<const float4*>(s_tw + i + 2);
          ax = fmaf(v.x, t01.x, ax);
          ay = fmaf(v.x, t01.y, ay);
          ax = fmaf(v.y, t01.z, ax);
          ay = fmaf(v.y, t01.w, ay);
          ax = fmaf(v.z, t23.x, ax);
          ay = fmaf(v.z, t23.y, ay);
          ax = fmaf(v.w, t23.z, ax);
          ay = fmaf(v.w, t23.w, ay);
        }
      } else {
        for (int i = 0; i < D; ++i) {
          const int64_t n = n0 + i;
          if (n >= 0 && n < a.n_samples) {
            const float v = ld_sample<InT>(xp, i);
            const float2 t = s_tw[i];
            ax = fmaf(v, t.x, ax);
            ay = fmaf(v, t.y, ay);
          }
        }
      }
      const double cyc = fmix * (double)n0 / fs;
      float ws, wc;
      sincospif((float)(-2.0 * (cyc - floor(cyc))), &ws, &wc);
      s_z[z_at(m)] = make_float2(ax * wc - ay * ws, ax * ws + ay * wc);
    }
  }
  __syncthreads();

  // ---- 3. fine sync over (start, tone-0) hypotheses
  const double bin = fs / (double)a.nfft;
  const int Mf = kMf;
  const double fstep = 0.5 * bin / kMf;
  const int nT = 2 * Mt + 1, nF = 2 * Mf + 1;
  const int H = min(nT * nF, kMaxHyp);
  // per-(tone-0 offset, tone) rotation of one decimated sample and its powers w^q, q <= Q, each from
  // its exact phase (one LDS read and four fmas per sample of a coherent window; round 4 advanced
  // w^q by a complex multiply per sample)
  float2* s_W = s_z + z_words(Q) + ((D + 1) & ~1);  // after the twiddles of phase 2: [nF * 8][Q + 1]
  for (int e = threadIdx.x; e < nF * 8 * (Q + 1); e += kSubThreads) {
    const int ft = e / (Q + 1), q = e - ft * (Q + 1);
    const int t = ft & 7, dfi = ft / 8 - Mf;
    const double nu = (double)t * 6.25 + dfi * fstep - 3.5 * 6.25;  // Hz relative to fmix
    const double cyc = nu * (double)D * (double)q / fs;
    float s_, c_;
    sincospif((float)(-2.0 * (cyc - floor(cyc))), &s_, &c_);
    s_W[e] = make_float2(c_, s_);
  }
  __syncthreads();
  // sliding windows: a wave owns one tone-0 offset at a time and a lane one symbol (k, k + 64);
  // the lane's coherent window C(dt) = sum_q z[.. + dt + q] w^q slides over every start offset with
  // one complex update per step, C(dt + 1) = conj(w) (C(dt) - z[dt] + z[dt + Q] w^Q), and the wave
  // sums |C|^2 over the symbols with a fixed shuffle tree (deterministic)
  {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int f = wv; f < nF; f += kSubWaves) {
      float msum[kMaxT];
#pragma unroll
      for (int d = 0; d < kMaxT; ++d) msum[d] = 0.f;
      for (int k = lane; k < tx::kSymbols; k += kWave) {
        const float2* Wp = s_W + (f * 8 + s_tones[k]) * (Q + 1);
        const float2 w = Wp[1], wq = Wp[Q];
        const float2* zp = s_z + (k + 1) * (Q + 1);  // = z_at(Mg - Mt + k Q): z[.. + j] at zp[j + j / Q]
        float2 acc = make_float2(0.f, 0.f);
        for (int q = 0; q < Q; ++q) {
          const float2 z = zp[q], W = Wp[q];
          acc.x = fmaf(z.x, W.x, fmaf(-z.y, W.y, acc.x));
          acc.y = fmaf(z.x, W.y, fmaf(z.y, W.x, acc.y));
        }
#pragma unroll
        for (int d = 0; d < kMaxT; ++d) {
          if (d < nT) {
            msum[d] += acc.x * acc.x + acc.y * acc.y;
            if (d + 1 < nT) {
              const int dq = d + (d >= Q ? 1 : 0);  // d < 2 Q
              const float2 zo = zp[dq], zn = zp[dq + Q + 1];
              const float tx_ = acc.x - zo.x + (zn.x * wq.x - zn.y * wq.y);
              const float ty_ = acc.y - zo.y + (zn.x * wq.y + zn.y * wq.x);
              acc = make_float2(tx_ * w.x + ty_ * w.y, ty_ * w.x - tx_ * w.y);
            }
          }
        }
      }
#pragma unroll
      for (int d = 0; d < kMaxT; ++d) {
        if (d < nT) {
          float v = msum[d];
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
          if (lane == 0) s_metric[d * nF + f] = v;
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int b = 0;
    for (int h = 1; h < H; ++h)
      if (s_metric[h] > s_metric[b]) b = h;
    s_flag = b;
  }
  __syncthreads();
  const int hb = s_flag;
  const int dtb = hb / nF - Mt, dfb = hb % nF - Mf;
  auto parab = [](float m_, float m0, float mp) {
    const float den = m_ - 2.f * m0 + mp;
    if (!(den < 0.f)) return 0.f;
    return fminf(0.5f, fmaxf(-0.5f, 0.5f * (m_ - mp) / den));
  };
  const float ddt = (dtb > -Mt && dtb < Mt) ? parab(s_metric[hb - nF], s_metric[hb], s_metric[hb + nF]) : 0.f;
  const float ddf = (dfb > -Mf && dfb < Mf) ? parab(s_metric[hb - 1], s_metric[hb], s_metric[hb + 1]) : 0.f;
  const int64_t start = s0 + (int64_t)llrintf(((float)dtb + ddt) * (float)D);
  const double f0 = ftone + ((double)dfb + (double)ddf) * fstep;

  // ---- phase at every symbol start, exact (double), protocol timing (off = nsps); the float
  // pulse table replaces z in LDS
  __syncthreads();
  if (threadIdx.x <= tx::kSymbols) {
    const int k = threadIdx.x;
    const double G0 = tx::gfsk_G<double, double>(s_E, s_PS, a.P, nsps, nsps);
    const double G = tx::gfsk_G<double, double>(s_E, s_PS, a.P, nsps, (k + 1) * nsps);
    const double cyc = (f0 * (double)k * nsps + 6.25 * (G - G0)) / fs;
    s_ph0[k] = (float)(cyc - floor(cyc));
  }
  for (int i = threadIdx.x; i < nsps; i += kSubThreads) {
    const float* P = a.Pf;
    s_D[i] = make_float4(P[i + 2 * nsps] - P[2 * nsps], P[i + nsps] - P[nsps], P[i] - P[0], 0.0f);
  }
  __syncthreads();

  // ---- 4. complex amplitude per symbol (one wave per symbol at a time; a lane's samples of the
  // symbol are loaded kPf at a time before they are used: two round trips per symbol for nsps <=
  // 2048; 32 at a time took 211 VGPRs once the ramp left the loop)
  {
    constexpr int kPf = 16;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float f0r = (float)(f0 / fs), sr = (float)(6.25 / fs);
    for (int k = wv; k < tx::kSymbols; k += kSubWaves) {
      float ax = 0.f, ay = 0.f, rr = 0.f;
      const float ph = s_ph0[k];
      const int64_t nsym = start + (int64_t)k * nsps;
      const bool inside = nsym >= 0 && nsym + nsps <= a.n_samples;
      const float E0 = (float)s_E[k], E1 = (float)s_E[k + 1], E2 = (float)s_E[k + 2];
      // the amplitude ramp is 1 except in the first and last symbols (wave-uniform): those take
      // a plain loop with the ramp, every other symbol the batched loads with rp = 1
      if (k == 0 || k == tx::kSymbols - 1) {
#pragma unroll 1
        for (int i = lane; i < nsps; i += kWave) {
          const int64_t n = nsym + i;
          if (!(n >= 0 && n < a.n_samples)) continue;
          const float rp = ramp_f(k * nsps + i, L, nsps);
          const float4 dd = s_D[i];
          const float cyc = ph + (float)i * f0r + sr * (E0 * dd.x + E1 * dd.y + E2 * dd.z);
          const float fr = __builtin_amdgcn_fractf(cyc);
          const float sn = __builtin_amdgcn_sinf(fr), cs = __builtin_amdgcn_cosf(fr);
          const float vr = ld_sample<InT>(x, n) * rp;
          ax += vr * cs;
          ay -= vr * sn;
          rr += rp * rp;
        }
      } else {
        // rp = 1: vr = v * 1, and sum rp^2 is the number of samples the symbol has in the slot (a sum
        // of 1.0s is exact in any order, so it is that count, not a per-sample add); inside the
        // slot (wave-uniform, all but the slot's edges) the samples are read without range tests
        const int64_t lo_n = max<int64_t>(nsym, 0), hi_n = min<int64_t>(nsym + nsps, a.n_samples);
        rr = (lane == 0 && hi_n > lo_n) ? (float)(hi_n - lo_n) : 0.f;
        for (int i0 = lane; i0 < nsps; i0 += kPf * kWave) {
          float v[kPf];
          const InT* xp = x + nsym + i0;
#pragma unroll
          for (int u = 0; u < kPf; ++u) {
            const int i = i0 + u * kWave;
            const int64_t n = nsym + i;
            v[u] = 0.f;
            if (i < nsps && (inside || (n >= 0 && n < a.n_samples))) v[u] = ld_sample<InT>(xp, u * kWave);
          }
#pragma unroll
          for (int u = 0; u < kPf; ++u) {
            const int i = i0 + u * kWave;
            if (i >= nsps) continue;
            const float4 dd = s_D[i];  // the change of G over the symbol's first i samples
            const float cyc = ph + (float)i * f0r + sr * (E0 * dd.x + E1 * dd.y + E2 * dd.z);
            const float fr = __builtin_amdgcn_fractf(cyc);  // v_sin / v_cos take revolutions
            const float sn = __builtin_amdgcn_sinf(fr), cs = __builtin_amdgcn_cosf(fr);
            const float vr = v[u];  // 0 outside the slot: adds +-0, as the skipped sample did
            ax += vr * cs;
            ay -= vr * sn;
          }
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        ax += __shfl_xor(ax, o);
        ay += __shfl_xor(ay, o);
        rr += __shfl_xor(rr, o);
      }
      if (lane == 0) s_A[k] = rr > 0.f ? make_float2(2.f * ax / rr, 2.f * ay / rr) : make_float2(0.f, 0.f);
    }
  }
  __syncthreads();
  // ---- smoothing over symbols, write the record
  if (threadIdx.x < tx::kSymbols) {
    const int k = threadIdx.x;
    float2 v;
    if (k == 0) v = make_float2((2.f * s_A[0].x + s_A[1].x) / 3.f, (2.f * s_A[0].y + s_A[1].y) / 3.f);
    else if (k == tx::kSymbols - 1)
      v = make_float2((s_A[k - 1].x + 2.f * s_A[k].x) / 3.f, (s_A[k - 1].y + 2.f * s_A[k].y) / 3.f);
    else
      v = make_float2(0.25f * (s_A[k - 1].x + 2.f * s_A[k].x + s_A[k + 1].x),
                      0.25f * (s_A[k - 1].y + 2.f * s_A[k].y + s_A[k + 1].y));
    est->amp[k][0] = v.x;
    est->amp[k][1] = v.y;
  }
  if (threadIdx.x <= tx::kSymbols) est->phase0[threadIdx.x] = s_ph0[threadIdx.x];
  if (threadIdx.x < 80) est->tones[threadIdx.x] = threadIdx.x < tx::kSymbols ? s_tones[threadIdx.x] : 0;
  if (threadIdx.x == 0) {
    est->start = start;
    est->f0 = f0;
    est->active = 1;
  }
  if (!REST) break;
  }  // records
}

constexpr int kApThreads = 512;
constexpr int kApPer = 16;
constexpr int kApTile = kApThreads * kApPer;   // samples per workgroup
constexpr int kApFits = 4;                     // fits staged in LDS per batch
constexpr int kApList = 1024;                  // overlapping fits listed per pass over the records

// One workgroup per (slot, tile of 8192 samples).  Wave 0 lists the fits that overlap the tile, in
// record order; per batch of kApFits fits, everything one SYMBOL of a fit needs is staged once:
// s_S1 = (E[k], E[k+1], E[k+2], phase0[k]) -- the extended tones whose pulses reach symbol k and
// its start phase -- s_S2 = (A[k], A[k] - A[k-1]) and s_S3 = A[k+1] - A[k], the amplitude and its
// slopes before and after the symbol centre (A clamped at the ends, as in the interpolation).  A
// thread's 16 samples are 512 apart; per fit it finds its first sample's symbol k and offset i once
// (one floor division), keeps symbol k's state in registers, and reloads it only when i wraps past
// nsps (every ~4 samples at 12 kHz).  Per sample and fit that leaves the pulse-table read, the phase,
// fract / sin / cos, the interpolated amplitude and one add -- round 4's form re-derived the symbol
// state (6 LDS reads, clamps, selects and their addresses) for every sample.  The amplitude ramp
// (first and last symbol only) is a table of nsps / 8 floats in LDS, the values tx_device.h's
// gfsk_ramp computes (both ramps of the protocol timing are 0.5 (1 - cos(8 pi j / nsps))).
// Every arithmetic step is the round-4 form's, in its order: the residual is bit-identical.
template <typename InT>
__global__ __launch_bounds__(kApThreads) void k_sub_apply(SubLaunch a) {
  FT8_RACE_PROLOGUE();
  __shared__ float4 s_S1[kApFits][tx::kSymbols];
  __shared__ float4 s_S2[kApFits][tx::kSymbols];
  __shared__ float2 s_S3[kApFits][tx::kSymbols];
  __shared__ long long s_start[kApFits];
  __shared__ float s_f0r[kApFits];
  __shared__ short s_list[kApList];
  __shared__ int s_nlist;
  // the pulse table's three symbol-relative differences per in-symbol offset i, one float4 each:
  // (P[i + 2 nsps] - P[2 nsps], P[i + nsps] - P[nsps], P[i] - P[0], t(i)) -- one ds_read_b128 and
  // no subtractions per sample; then the ramp table [nsps / 8]
  extern __shared__ float4 s_D[];
  const int slot = blockIdx.y;
  const int64_t t0 = (int64_t)blockIdx.x * kApTile;
  const int nsps = a.nsps, L = tx::kSymbols * nsps, nramp = nsps / 8;
  float* s_R = reinterpret_cast<float*>(s_D + nsps);
  const float fsf = (float)a.fs, inv_nsps = 1.0f / (float)nsps, sr = 6.25f / fsf;
  const int cnt = min(a.counts[slot], a.cap);
  const SubEst* est = reinterpret_cast<const SubEst*>(a.est) + (int64_t)slot * a.cap;
  // samples t0 + tid + 512 kk with kk < nv exist (16 except in a slot's last tile)
  const int64_t rem = a.n_samples - (t0 + (int64_t)threadIdx.x);
  const int nv = rem <= 0 ? 0 : (int)min<int64_t>(kApPer, (rem + kApThreads - 1) / kApThreads);
  float acc[kApPer];
#pragma unroll
  for (int k = 0; k < kApPer; ++k) acc[k] = 0.f;
  for (int i = threadIdx.x; i < nsps; i += kApThreads) {
    const float* P = a.Pf;
    // .w: the sample's position from the symbol centre in symbols, t(i) (the amplitude interpolation)
    s_D[i] = make_float4(P[i + 2 * nsps] - P[2 * nsps], P[i + nsps] - P[nsps], P[i] - P[0],
                         ((float)i + 0.5f) * inv_nsps - 0.5f);
  }
  for (int i = threadIdx.x; i < nramp; i += kApThreads) s_R[i] = ramp_f(i, L, nsps);
  for (int j0 = 0; j0 < cnt; j0 += kApList) {
    __syncthreads();  // the previous list is consumed
    if (threadIdx.x < kWave) {
      // the fits of records [j0, j0 + kApList) that overlap this tile, in record order
      const int lane = threadIdx.x;
      int n = 0;
      for (int jb = j0; jb < min(cnt, j0 + kApList); jb += kWave) {
        const int j = jb + lane;
        bool hit = false;
        if (j < cnt && est[j].active) {
          const int64_t st = est[j].start;
          hit = st < t0 + kApTile && st + L > t0;
        }
        const uint64_t m = __ballot(hit);
        if (hit) s_list[n + __popcll(m & ((1ull << lane) - 1ull))] = (short)(j - j0);
        n += __popcll(m);
      }
      if (lane == 0) s_nlist = n;
    }
    __syncthreads();
    const int nl = s_nlist;
    for (int b0 = 0; b0 < nl; b0 += kApFits) {
      const int nb = min(kApFits, nl - b0);
      __syncthreads();  // the previous batch is consumed
      for (int q = threadIdx.x; q < nb * tx::kSymbols; q += kApThreads) {
        const int f = q / tx::kSymbols, k = q - f * tx::kSymbols;
        const SubEst* e = est + j0 + s_list[b0 + f];
        const int km = k > 0 ? k - 1 : 0, kp = k < tx::kSymbols - 1 ? k + 1 : k;
        s_S1[f][k] = make_float4((float)e->tones[km], (float)e->tones[k], (float)e->tones[kp], e->phase0[k]);
        const float cx = e->amp[k][0], cy = e->amp[k][1];
        s_S2[f][k] = make_float4(cx, cy, cx - e->amp[km][0], cy - e->amp[km][1]);
        s_S3[f][k] = make_float2(e->amp[kp][0] - cx, e->amp[kp][1] - cy);
      }
      if (threadIdx.x < nb) {
        const SubEst* e = est + j0 + s_list[b0 + threadIdx.x];
        s_start[threadIdx.x] = e->start;
        s_f0r[threadIdx.x] = (float)(e->f0 / (double)a.fs);
      }
      __syncthreads();
      for (int f = 0; f < nb; ++f) {
        const int64_t start = s_start[f];
        const float f0r = s_f0r[f];
        const int nr0 = (int)(t0 + threadIdx.x - start);  // |nr0| < 2^31: slots hold < 2^31 samples
        int k = nr0 >= 0 ? nr0 / nsps : -((-nr0 + nsps - 1) / nsps);  // floor
        int i = nr0 - k * nsps;
        // symbol k's state (zeros outside the waveform: those samples are skipped)
        float4 e4 = make_float4(0.f, 0.f, 0.f, 0.f), a4 = e4;
        float2 r2 = make_float2(0.f, 0.f);
        bool edge = false;  // symbol 0 or 78: the amplitude ramps
        if ((unsigned)k < (unsigned)tx::kSymbols) {
          e4 = s_S1[f][k];
          a4 = s_S2[f][k];
          r2 = s_S3[f][k];
          edge = k == 0 || k == tx::kSymbols - 1;
        }
#pragma unroll
        for (int kk = 0; kk < kApPer; ++kk) {
          if ((unsigned)k < (unsigned)tx::kSymbols && kk < nv) {
            // the change of G over the symbol's first i samples (tx_device.h's pulse table)
            const float4 dd = s_D[i];
            const float g = e4.x * dd.x + e4.y * dd.y + e4.z * dd.z;
            const float fi = (float)i;
            const float cyc = e4.w + fi * f0r + sr * g;
            const float fr = __builtin_amdgcn_fractf(cyc);  // v_sin / v_cos take revolutions
            const float sn = __builtin_amdgcn_sinf(fr), cs = __builtin_amdgcn_cosf(fr);
            const float t = dd.w;  // position from the symbol centre
            const float dx = t < 0.f ? a4.z : r2.x, dy = t < 0.f ? a4.w : r2.y;
            const float Ax = a4.x + t * dx, Ay = a4.y + t * dy;
            float v = Ax * cs - Ay * sn;
            // the amplitude ramp: 1 except in the first nsps / 8 samples of symbol 0 and the last
            // nsps / 8 of symbol 78 (the same float as 1 * v elsewhere)
            if (edge) {
              const int j = k == 0 ? i : nsps - 1 - i;
              if (j < nramp) v = s_R[j] * v;
            }
            acc[kk] += v;
          }
          i += kApThreads;
          if (i >= nsps) {
            do {
              i -= nsps;
              ++k;
            } while (i >= nsps);
            if ((unsigned)k < (unsigned)tx::kSymbols) {
              e4 = s_S1[f][k];
              a4 = s_S2[f][k];
              r2 = s_S3[f][k];
              edge = k == 0 || k == tx::kSymbols - 1;
            }
          }
        }
      }
    }
  }
  const InT* x = reinterpret_cast<const InT*>(a.x) + (int64_t)slot * a.slot_stride;
  float* out = a.residual + (int64_t)slot * a.slot_stride;
#pragma unroll
  for (int kk = 0; kk < kApPer; ++kk) {
    const int64_t nabs = t0 + threadIdx.x + (int64_t)kk * kApThreads;
    if (nabs < a.n_samples) out[nabs] = ld_sample<InT>(x, nabs) - acc[kk];
  }
}

__device__ __forceinline__ bool same_payload(const ft8_result& p, const ft8_result& q) {
  bool eq = true;
#pragma unroll
  for (int b = 0; b < 10; ++b) eq = eq && p.payload[b] == q.payload[b];
  return eq;
}

__global__ __launch_bounds__(kWave) void k_merge(ft8_result* out, int32_t* counts, int cap, const ft8_result* out1,
                                                 const int32_t* counts1, int cap1, const ft8_result* out2,
                                                 const int32_t* counts2, int cap2) {
  const int slot = blockIdx.x, lane = threadIdx.x;
  const int c1 = counts1[slot], c1v = min(c1, cap1);
  const int c2 = min(counts2[slot], cap2);
  const ft8_result* p1 = out1 + (int64_t)slot * cap1;
  const ft8_result* p2 = out2 + (int64_t)slot * cap2;
  for (int c = lane; c < min(c1v, cap); c += kWave) out[(int64_t)slot * cap + c] = p1[c];
  int base = c1;
  for (int c0 = 0; c0 < c2; c0 += kWave) {
    const int c = c0 + lane;
    bool keep = false;
    ft8_result r{};
    if (c < c2) {
      r = p2[c];
      keep = r.ok != 0;
      for (int j = 0; j < c1v && keep; ++j) keep = !same_payload(p1[j], r);
    }
    const unsigned long long m = __ballot(keep);
    const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
    if (keep && pos < cap) {
      r.pass_index = 1;
      out[(int64_t)slot * cap + pos] = r;
    }
    base += __popcll(m);
  }
  if (lane == 0) counts[slot] = base;
}

}  // namespace

size_t sub_est_bytes() { return sizeof(SubEst); }

// dynamic LDS above the default 64 KB needs the kernel's attribute raised first (the pulse table is
// nsps float4s: 61.4 KB at 24 kHz, more above)
// The attribute is set once per kernel instantiation and device, and again only when a launch needs
// more than any before it (it was a host-side call per launch); static + dynamic LDS is
// compared against the 64 KB default, the kernel's static size queried once.
template <typename K>
static hipError_t allow_lds(K kern, size_t dyn) {
  constexpr int kMaxDev = 64;
  static std::mutex mu;
  static size_t static_lds[kMaxDev];
  static size_t granted[kMaxDev];
  static bool queried[kMaxDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) dev = 0;
  std::lock_guard<std::mutex> lk(mu);
  if (!queried[dev]) {
    hipFuncAttributes fa{};
    static_lds[dev] = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kern)) == hipSuccess ? fa.sharedSizeBytes : 0;
    queried[dev] = true;
  }
  if (static_lds[dev] + dyn <= 64 * 1024 || dyn <= granted[dev]) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
  if (e == hipSuccess) granted[dev] = dyn;
  return e;
}

hipError_t launch_sub_est(const SubLaunch& a, hipStream_t s) {
  if (a.n_slots <= 0 || a.n_samples <= 0) return hipSuccess;
  if (a.Q <= 0 || a.Q > kMaxQ || a.nsps % a.Q != 0 || a.hop <= 0 || a.nsps % a.hop != 0) return hipErrorInvalidValue;
  if (a.cap > 0) {
    hipLaunchKernelGGL(k_sub_list, dim3(a.n_slots), dim3(kWave), 0, s, a);
    const unsigned grid = (unsigned)(((a.n_slots + 7) / 8) * 8 * (int64_t)kSubRecStride);
    // the rest launch: 8 workgroups per slot that exit at once unless the slot holds more than
    // kSubRecStride fits
    const unsigned grid_rest = (unsigned)(((a.n_slots + 7) / 8) * 8 * (int64_t)kSubRestStride);
    // padded z rows -1 .. 81, the decimation's twiddles and the fine sync's rotation powers (phases
    // 2-3), then the pulse table (phase 4)
    const int D = a.nsps / a.Q;
    const size_t mz = (size_t)z_words(a.Q) + (size_t)((D + 1) & ~1) + (size_t)(2 * kMf + 1) * 8 * (a.Q + 1);
    const size_t lds = std::max(mz * sizeof(float2), (size_t)a.nsps * sizeof(float4));
    hipError_t e = hipSuccess;
    if (a.dtype == FT8_I16) {
      if ((e = allow_lds(k_sub_est<int16_t, false>, lds)) != hipSuccess) return e;
      hipLaunchKernelGGL((k_sub_est<int16_t, false>), dim3(grid), dim3(kSubThreads), lds, s, a);
      if (a.cap > kSubRecStride) {
        if ((e = allow_lds(k_sub_est<int16_t, true>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k_sub_est<int16_t, true>), dim3(grid_rest), dim3(kSubThreads), lds, s, a);
      }
    } else {
      if ((e = allow_lds(k_sub_est<float, false>, lds)) != hipSuccess) return e;
      hipLaunchKernelGGL((k_sub_est<float, false>), dim3(grid), dim3(kSubThreads), lds, s, a);
      if (a.cap > kSubRecStride) {
        if ((e = allow_lds(k_sub_est<float, true>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k_sub_est<float, true>), dim3(grid_rest), dim3(kSubThreads), lds, s, a);
      }
    }
    return hipGetLastError();
  }
  return hipSuccess;
}

hipError_t launch_sub_apply(const SubLaunch& a, hipStream_t s) {
  if (a.n_slots <= 0 || a.n_samples <= 0) return hipSuccess;
  dim3 g2((unsigned)((a.n_samples + kApTile - 1) / kApTile), (unsigned)a.n_slots);
  const size_t lds2 = (size_t)a.nsps * sizeof(float4) + (size_t)(a.nsps / 8) * sizeof(float);
  hipError_t e = hipSuccess;
  if (a.dtype == FT8_I16) {
    if ((e = allow_lds(k_sub_apply<int16_t>, lds2)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_sub_apply<int16_t>, g2, dim3(kApThreads), lds2, s, a);
  } else {
    if ((e = allow_lds(k_sub_apply<float>, lds2)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_sub_apply<float>, g2, dim3(kApThreads), lds2, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_merge_pass(ft8_result* out, int32_t* counts, int cap, const ft8_result* out1,
                             const int32_t* counts1, int cap1, const ft8_result* out2, const int32_t* counts2,
                             int cap2, int n_slots, hipStream_t s) {
  if (n_slots <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_merge, dim3(n_slots), dim3(kWave), 0, s, out, counts, cap, out1, counts1, cap1, out2, counts2,
                     cap2);
  return hipGetLastError();
}

}  // namespace ft8
