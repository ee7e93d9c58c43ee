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
//      +-bin/2 (in steps of 6.25/16 Hz) the known tone sequence is correlated symbol by symbol
//      (coherent within a symbol, power summed over the 79 symbols); the best point is refined by
//      a parabola through its neighbours in each direction;
//   4. the complex amplitude of every symbol is fitted against the refined GFSK waveform
//      (A_k = 2 sum x conj(c) r / sum r^2, r the ramp) and smoothed [1 2 1] / 4 over symbols.
// k_sub_apply one workgroup per (slot, tile): residual = x - sum over the slot's fitted signals of
//            r(n) Re(A(n) exp(i psi(n))), A linearly interpolated between symbol centres; signals
//            summed in record order (deterministic).
// k_merge    one wave per slot: pass-2 records with a payload not decoded in pass 1 are appended.
#include "tx_device.h"

namespace ft8 {
namespace {

constexpr int kSubThreads = 256;
constexpr int kSubWaves = kSubThreads / kWave;
constexpr int kMaxQ = 32;
constexpr int kMaxMg = 2 * kMaxQ + 1;          // margin in decimated samples (sps >= 1)
constexpr int kMaxZ = tx::kSymbols * kMaxQ + 2 * kMaxMg;
constexpr int kMaxHyp = 1024;
constexpr double kFStep = 6.25 / 16.0;         // Hz, tone-0 search step

struct SubEst {
  int32_t active, pad;
  int64_t start;           // refined first sample of the waveform in the slot
  double f0;               // refined tone-0 frequency, Hz
  float A[tx::kSymbols][2];
  float ph0[tx::kSymbols + 1];   // phase (cycles, fractional part) at the start of every symbol
  uint8_t tones[80];
};

template <typename InT>
__device__ __forceinline__ float ld_sample(const InT* x, int64_t i);
template <>
__device__ __forceinline__ float ld_sample<float>(const float* x, int64_t i) { return x[i]; }
template <>
__device__ __forceinline__ float ld_sample<int16_t>(const int16_t* x, int64_t i) {
  return (float)x[i] / 32767.0f;  // read_wave_file scaling, as the STFT applies it
}

// change of G over the first i samples of symbol k (protocol timing: u = (k + 1) nsps + i),
// relative to the symbol start; float is plenty inside one symbol
__device__ __forceinline__ float dG(const int* E, const float* Pf, int nsps, int k, int i) {
  return (float)E[k] * (Pf[i + 2 * nsps] - Pf[2 * nsps]) + (float)E[k + 1] * (Pf[i + nsps] - Pf[nsps]) +
         (float)E[k + 2] * (Pf[i] - Pf[0]);
}

__device__ __forceinline__ float ramp_f(int n, int L, int nsps) { return tx::gfsk_ramp<float>(n, L, nsps, 0); }

template <typename InT>
__global__ __launch_bounds__(kSubThreads) void k_sub_est(SubLaunch a) {
  __shared__ float2 s_z[kMaxZ];
  __shared__ float s_metric[kMaxHyp];
  __shared__ int s_E[tx::kExt];
  __shared__ int s_PS[tx::kExt + 1];
  __shared__ uint8_t s_tones[80];
  __shared__ float s_ph0[tx::kSymbols + 1];
  __shared__ float2 s_A[tx::kSymbols];
  __shared__ float s_bv[kSubWaves];
  __shared__ int s_bi[kSubWaves];
  __shared__ int s_flag;

  // records of one slot on one XCD (workgroup id % 8)
  const int w = blockIdx.x;
  const int j8 = w / 8;
  const int slot = (w % 8) + 8 * (j8 / a.cap);
  const int rec = j8 % a.cap;
  if (slot >= a.n_slots) return;
  const int cnt = min(a.counts[slot], a.cap);
  if (rec >= cnt) return;
  SubEst* est = reinterpret_cast<SubEst*>(a.est) + (int64_t)slot * a.cap + rec;
  const ft8_result* rs = a.res + (int64_t)slot * a.cap;
  const ft8_result r = rs[rec];
  // a failed record, or a payload an earlier record of the slot already carries: nothing to fit
  bool dup = false;
  for (int j = threadIdx.x; j < rec; j += kSubThreads) {
    if (!rs[j].ok) continue;
    bool eq = true;
    for (int b = 0; b < 10; ++b) eq = eq && rs[j].payload[b] == r.payload[b];
    dup = dup || eq;
  }
  dup = __syncthreads_or(dup);
  if (!r.ok || dup) {
    if (threadIdx.x == 0) est->active = 0;
    return;
  }
  if (threadIdx.x == 0) {
    tx::encode(r.payload, 10, nullptr, nullptr, s_tones);
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
  const double fs = (double)a.fs;
  const int64_t s0 = (int64_t)(a.t_lo + r.abs_time) * a.hop;
  const double ftone = (double)(a.f_lo + r.abs_freq) * fs / (double)a.nfft;
  const double fmix = ftone + 3.5 * 6.25;

  // ---- 2. mixed-down, box-car decimated baseband z[m], samples [nb + m D, nb + (m + 1) D)
  {
    const int64_t nb = s0 - (int64_t)Mg * D;
    float ss, sc;
    sincospif((float)(-2.0 * fmix / fs), &ss, &sc);
    const float2 step = make_float2(sc, ss);
    for (int m = threadIdx.x; m < Mz; m += kSubThreads) {
      const int64_t n0 = nb + (int64_t)m * D;
      const double cyc = fmix * (double)n0 / fs;
      float ws, wc;
      sincospif((float)(-2.0 * (cyc - floor(cyc))), &ws, &wc);
      float2 wv = make_float2(wc, ws), acc = make_float2(0.f, 0.f);
      for (int i = 0; i < D; ++i) {
        const int64_t n = n0 + i;
        if (n >= 0 && n < a.n_samples) {
          const float v = ld_sample<InT>(x, n);
          acc.x += v * wv.x;
          acc.y += v * wv.y;
        }
        wv = make_float2(wv.x * step.x - wv.y * step.y, wv.x * step.y + wv.y * step.x);
      }
      s_z[m] = acc;
    }
  }
  __syncthreads();

  // ---- 3. fine sync over (start, tone-0) hypotheses
  const double bin = fs / (double)a.nfft;
  const int Mf = max(1, (int)floor(0.5 * bin / kFStep + 0.5));
  const int nT = 2 * Mt + 1, nF = 2 * Mf + 1;
  const int H = min(nT * nF, kMaxHyp);
  float bv = -1.f;
  int bi = 0;
  for (int h = threadIdx.x; h < H; h += kSubThreads) {
    const int dt = h / nF - Mt, dfi = h % nF - Mf;
    float2 st[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const double nu = (double)t * 6.25 + dfi * kFStep - 3.5 * 6.25;  // Hz relative to fmix
      float s_, c_;
      sincospif((float)(-2.0 * nu * D / fs), &s_, &c_);
      st[t] = make_float2(c_, s_);
    }
    float metric = 0.f;
    for (int k = 0; k < tx::kSymbols; ++k) {
      const float2 stp = st[s_tones[k]];
      const float2* zp = s_z + Mg + dt + k * Q;
      float2 wv = make_float2(1.f, 0.f), acc = make_float2(0.f, 0.f);
      for (int q = 0; q < Q; ++q) {
        const float2 z = zp[q];
        acc.x += z.x * wv.x - z.y * wv.y;
        acc.y += z.x * wv.y + z.y * wv.x;
        wv = make_float2(wv.x * stp.x - wv.y * stp.y, wv.x * stp.y + wv.y * stp.x);
      }
      metric += acc.x * acc.x + acc.y * acc.y;
    }
    s_metric[h] = metric;
    if (metric > bv) { bv = metric; bi = h; }
  }
  {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o);
      const int oi = __shfl_xor(bi, o);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { s_bv[wv] = bv; s_bi[wv] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
      int b = 0;
      for (int i = 1; i < kSubWaves; ++i)
        if (s_bv[i] > s_bv[b] || (s_bv[i] == s_bv[b] && s_bi[i] < s_bi[b])) b = i;
      s_flag = s_bi[b];
    }
    __syncthreads();
  }
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
  const double f0 = ftone + ((double)dfb + (double)ddf) * kFStep;

  // ---- phase at every symbol start, exact (double), protocol timing (off = nsps)
  if (threadIdx.x <= tx::kSymbols) {
    const int k = threadIdx.x;
    const double G0 = tx::gfsk_G<double, double>(s_E, s_PS, a.P, nsps, nsps);
    const double G = tx::gfsk_G<double, double>(s_E, s_PS, a.P, nsps, (k + 1) * nsps);
    const double cyc = (f0 * (double)k * nsps + 6.25 * (G - G0)) / fs;
    s_ph0[k] = (float)(cyc - floor(cyc));
  }
  __syncthreads();

  // ---- 4. complex amplitude per symbol (one wave per symbol at a time)
  {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float f0r = (float)(f0 / fs), sr = (float)(6.25 / fs);
    for (int k = wv; k < tx::kSymbols; k += kSubWaves) {
      float ax = 0.f, ay = 0.f, rr = 0.f;
      const float ph = s_ph0[k];
      for (int i = lane; i < nsps; i += kWave) {
        const int nr = k * nsps + i;
        const int64_t n = start + nr;
        if (n < 0 || n >= a.n_samples) continue;
        const float rp = ramp_f(nr, L, nsps);
        const float cyc = ph + (float)i * f0r + sr * dG(s_E, a.Pf, nsps, k, i);
        float sn, cs;
        sincospif(2.f * (cyc - floorf(cyc)), &sn, &cs);
        const float v = ld_sample<InT>(x, n) * rp;
        ax += v * cs;
        ay -= v * sn;
        rr += rp * rp;
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
    est->A[k][0] = v.x;
    est->A[k][1] = v.y;
  }
  if (threadIdx.x <= tx::kSymbols) est->ph0[threadIdx.x] = s_ph0[threadIdx.x];
  if (threadIdx.x < 80) est->tones[threadIdx.x] = threadIdx.x < tx::kSymbols ? s_tones[threadIdx.x] : 0;
  if (threadIdx.x == 0) {
    est->start = start;
    est->f0 = f0;
    est->active = 1;
  }
}

constexpr int kApPer = 8;
constexpr int kApTile = kSubThreads * kApPer;

template <typename InT>
__global__ __launch_bounds__(kSubThreads) void k_sub_apply(SubLaunch a) {
  __shared__ int s_E[tx::kExt];
  __shared__ float2 s_A[tx::kSymbols];
  __shared__ float s_ph0[tx::kSymbols + 1];
  const int slot = blockIdx.y;
  const int64_t t0 = (int64_t)blockIdx.x * kApTile;
  const int nsps = a.nsps, L = tx::kSymbols * nsps;
  const float fsf = (float)a.fs;
  const int cnt = min(a.counts[slot], a.cap);
  const SubEst* est = reinterpret_cast<const SubEst*>(a.est) + (int64_t)slot * a.cap;
  float acc[kApPer];
#pragma unroll
  for (int k = 0; k < kApPer; ++k) acc[k] = 0.f;
  for (int j = 0; j < cnt; ++j) {
    const SubEst* e = est + j;
    if (!e->active) continue;
    const int64_t start = e->start;
    if (start >= t0 + kApTile || start + L <= t0) continue;
    __syncthreads();
    if (threadIdx.x < tx::kExt) {
      const int jj = (int)threadIdx.x - 1;
      s_E[threadIdx.x] = e->tones[jj < 0 ? 0 : (jj > tx::kSymbols - 1 ? tx::kSymbols - 1 : jj)];
    }
    if (threadIdx.x < tx::kSymbols) s_A[threadIdx.x] = make_float2(e->A[threadIdx.x][0], e->A[threadIdx.x][1]);
    if (threadIdx.x <= tx::kSymbols) s_ph0[threadIdx.x] = e->ph0[threadIdx.x];
    __syncthreads();
    const float f0r = (float)(e->f0 / (double)a.fs), sr = 6.25f / fsf;
#pragma unroll
    for (int kk = 0; kk < kApPer; ++kk) {
      const int64_t nabs = t0 + threadIdx.x + (int64_t)kk * kSubThreads;
      const int64_t nr64 = nabs - start;
      if (nr64 < 0 || nr64 >= L || nabs >= a.n_samples) continue;
      const int nr = (int)nr64;
      const int k = nr / nsps, i = nr - k * nsps;
      const float cyc = s_ph0[k] + (float)i * f0r + sr * dG(s_E, a.Pf, nsps, k, i);
      float sn, cs;
      sincospif(2.f * (cyc - floorf(cyc)), &sn, &cs);
      const float t = ((float)i + 0.5f) / (float)nsps - 0.5f;  // position from the symbol centre
      float2 A;
      if (t < 0.f) {
        const float2 p = s_A[k > 0 ? k - 1 : 0], c = s_A[k];
        A = make_float2(c.x + t * (c.x - p.x), c.y + t * (c.y - p.y));
      } else {
        const float2 c = s_A[k], nx = s_A[k < tx::kSymbols - 1 ? k + 1 : k];
        A = make_float2(c.x + t * (nx.x - c.x), c.y + t * (nx.y - c.y));
      }
      acc[kk] += ramp_f(nr, L, nsps) * (A.x * cs - A.y * sn);
    }
  }
  const InT* x = reinterpret_cast<const InT*>(a.x) + (int64_t)slot * a.slot_stride;
  float* out = a.residual + (int64_t)slot * a.slot_stride;
#pragma unroll
  for (int kk = 0; kk < kApPer; ++kk) {
    const int64_t nabs = t0 + threadIdx.x + (int64_t)kk * kSubThreads;
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

hipError_t launch_subtract(const SubLaunch& a, hipStream_t s) {
  if (a.n_slots <= 0 || a.n_samples <= 0) return hipSuccess;
  if (a.Q <= 0 || a.Q > kMaxQ || a.nsps % a.Q != 0 || a.hop <= 0 || a.nsps % a.hop != 0) return hipErrorInvalidValue;
  if (a.cap > 0) {
    const unsigned grid = (unsigned)(((a.n_slots + 7) / 8) * 8 * (int64_t)a.cap);
    if (a.dtype == FT8_I16)
      hipLaunchKernelGGL(k_sub_est<int16_t>, dim3(grid), dim3(kSubThreads), 0, s, a);
    else
      hipLaunchKernelGGL(k_sub_est<float>, dim3(grid), dim3(kSubThreads), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  dim3 g2((unsigned)((a.n_samples + kApTile - 1) / kApTile), (unsigned)a.n_slots);
  if (a.dtype == FT8_I16)
    hipLaunchKernelGGL(k_sub_apply<int16_t>, g2, dim3(kSubThreads), 0, s, a);
  else
    hipLaunchKernelGGL(k_sub_apply<float>, g2, dim3(kSubThreads), 0, s, a);
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
