// drift.hip -- frequency-drift correction of FT8 beacon signals on gfx950 (ft8_drift_correct).
//
// Replaces correct_frequency_drift / detect_signal_continuity of the reference's beacon receiver
// (src/ft8_tools/ft8_beacon_receiver/frequency_correction.py:42-659) for a batch of independent
// signals.  The spectrogram passes are the STFT kernel with its argmax epilogue (stft.hip: the
// per-frame argmax over frequency of :222-224 and :383-384 without writing the waterfall); this
// file holds the estimation and the de-rotation:
//
// k_drift_fit1  one workgroup per signal: the continuity metric of every window (:65-81: residual
//               variance of a least-squares line through window_size argmax indices; evaluated
//               exactly in integer arithmetic, var = (Syy Sxx - Sxy^2) / (n^2 Sxx)), the segment
//               scan (:96-113, ballot masks + bit scan), the longest segment (:239, first on ties),
//               optional middle trimming (:311-330) and the linear fit of frequency against time
//               (:332-348) -> f_shift_rate.
// k_drift_fit2  one workgroup per signal: the masked, mean-removed argmax track of the linearly
//               compensated signal (:419-431), its full cross-correlation with the three-Costas
//               template (:433), the peak (:462-463), the regression points of the three sync
//               blocks (:502-519) and the polynomial fit (:526-541, centred least squares as
//               LinearRegression does, solved by modified Gram-Schmidt), the rate of :650-654.
// k_derotate    one thread per sample: stage 1 the linear carrier of :352, stage 2 the polynomial
//               carrier of :598-611, each phase formed in float64 with NumPy's operation order
//               (complex-by-real division is a multiplication by the reciprocal, as NumPy does).
//
// No sklearn: LinearRegression(fit_intercept=True) is the least-squares solution of the centred
// problem, which these kernels compute directly.
#include <cmath>

#include "ft8_internal.h"

namespace ft8 {
namespace {

constexpr int kFitThreads = 256;
constexpr int kFitWaves = kFitThreads / kWave;
constexpr int kMaxTmpl = 4096;   // three_sync_correlation_seq length held in LDS
constexpr int kMaxPts = 1024;    // regression points of the sync fit
constexpr double kTwoPi = 6.283185307179586;  // fl(2 pi): -2j * np.pi has imaginary part -fl(2 pi)

// block-wide sum (every thread gets the same value; fixed order -> deterministic)
__device__ double block_sum(double v, double* red) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < kFitWaves; ++k) t += red[k];
  return t;
}

// ---- stage 1 ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kFitThreads) void k_drift_fit1(DriftFitLaunch a) {
  FT8_RACE_PROLOGUE();
  __shared__ int s_idx[kDriftMaxT];
  __shared__ unsigned long long s_flag[kDriftMaxT / kWave];
  __shared__ double s_red[kFitWaves];
  __shared__ int s_seg[3];
  const int slot = blockIdx.x;
  const int T = a.T;
  const ft8_drift_params& p = a.p;
  const int32_t* idx = a.idx + (int64_t)slot * T;
  for (int i = threadIdx.x; i < T; i += kFitThreads) s_idx[i] = idx[i];
  __syncthreads();

  const int w = p.window_size_factor * p.steps_per_symbol;
  const int nwin = T - w + 1;
  const double maxvar = p.max_variance_factor * ((double)a.F * (double)a.F);
  ft8_drift_result r{};
  if (w > 0 && nwin > 0) {
    // constant sums of x = 0 .. w-1.  Exact in int64 for window <= 64 and indices < 8192 (host
    // checks): Sxx <= 1.4e6, Syy <= 6.9e10, Syy Sxx and Sxy^2 (<= Syy Sxx) <= 9.6e16.
    const int64_t n = w;
    const int64_t X = n * (n - 1) / 2;
    const int64_t XX = (n - 1) * n * (2 * n - 1) / 6;
    const int64_t Sxx = n * XX - X * X;
    const double den = (double)(n * n * Sxx);
    double* metric = a.metric ? a.metric + (int64_t)slot * nwin : nullptr;
    for (int i0 = 0; i0 < nwin; i0 += kFitThreads) {
      const int i = i0 + threadIdx.x;
      bool flag = false;
      if (i < nwin) {
        int64_t Y = 0, YY = 0, XY = 0;
        for (int j = 0; j < w; ++j) {
          const int64_t y = s_idx[i + j];
          Y += y;
          YY += y * y;
          XY += (int64_t)j * y;
        }
        const int64_t Syy = n * YY - Y * Y;
        const int64_t Sxy = n * XY - X * Y;
        // residual variance of the least-squares line (population variance, residual mean 0)
        const double var = Sxx > 0 ? (double)(Syy * Sxx - Sxy * Sxy) / den : 0.0;
        if (metric) metric[i] = -var;
        flag = -var > -maxvar;  // continuity_metric > -max_variance (:95)
      }
      const unsigned long long m = __ballot(flag);
      if ((threadIdx.x & (kWave - 1)) == 0 && i0 + (int)(threadIdx.x & ~(kWave - 1)) < nwin)
        s_flag[(i0 + (int)(threadIdx.x & ~(kWave - 1))) / kWave] = m;
    }
    __syncthreads();
    // segment scan (:99-113): one thread walks the transitions of the flag bits
    if (threadIdx.x == 0) {
      int nseg = 0, bs = 0, be = 0, st = 0;
      bool in = false;
      int32_t* segs = a.segments ? a.segments + (int64_t)slot * a.max_segments * 2 : nullptr;
      auto record = [&](int s0, int e0) {
        if (segs && nseg < a.max_segments) { segs[2 * nseg] = s0; segs[2 * nseg + 1] = e0; }
        if (nseg == 0 || e0 - s0 > be - bs) { bs = s0; be = e0; }
        ++nseg;
      };
      for (int c = 0; c * kWave < nwin; ++c) {
        const int valid = min(kWave, nwin - c * kWave);
        const unsigned long long vm = valid < kWave ? ((1ull << valid) - 1) : ~0ull;
        const unsigned long long m = s_flag[c] & vm;
        unsigned long long t = (m ^ ((m << 1) | (in ? 1ull : 0ull))) & vm;
        while (t) {
          const int b = __builtin_ctzll(t);
          t &= t - 1;
          if ((m >> b) & 1ull) { in = true; st = c * kWave + b; }
          else { in = false; record(st, c * kWave + b); }
        }
      }
      if (in) record(st, T - 1);  // :111-112: the open segment ends at len(max_freq_indices) - 1
      s_seg[0] = nseg;
      s_seg[1] = bs;
      s_seg[2] = be;
    }
    __syncthreads();
  } else if (threadIdx.x == 0) {
    s_seg[0] = 0;
  }
  __syncthreads();
  const int nseg = s_seg[0];
  if (nseg == 0) {  // :235-236
    if (threadIdx.x == 0) {
      r.status = FT8_DRIFT_NO_SEGMENT;
      a.res[slot] = r;
    }
    return;
  }
  int s0 = s_seg[1], e0 = s_seg[2];
  r.n_segments = nseg;
  r.seg_start = s0;
  r.seg_end = e0;
  // middle trimming (:311-330)
  if (p.fit_middle_percent < 100) {
    const int len = e0 - s0;
    const double tp = ((double)(100 - p.fit_middle_percent) / 2.0) / 100.0;
    const int trim = (int)((double)len * tp);
    if (trim > 0 && 2 * trim < len) { s0 += trim; e0 -= trim; }
  }
  const int m = e0 - s0;
  if (m <= 0) {  // LinearRegression.fit on zero samples raises ValueError
    if (threadIdx.x == 0) {
      r.status = FT8_DRIFT_VALUE_ERROR;
      a.res[slot] = r;
    }
    return;
  }
  // least squares of max_freqs = idx * freq_step against time_axis = i * time_step (:241-348)
  const double fstep = p.sym_bin / (double)p.bins_per_tone;
  const double tstep = p.sym_t / (double)p.steps_per_symbol;
  double st = 0.0, sf = 0.0;
  for (int i = s0 + threadIdx.x; i < e0; i += kFitThreads) {
    st += (double)i * tstep;
    sf += (double)s_idx[i] * fstep;
  }
  const double tm = block_sum(st, s_red) / (double)m;
  const double fm = block_sum(sf, s_red) / (double)m;
  double stt = 0.0, stf = 0.0;
  for (int i = s0 + threadIdx.x; i < e0; i += kFitThreads) {
    const double dt = (double)i * tstep - tm;
    const double df = (double)s_idx[i] * fstep - fm;
    stt += dt * dt;
    stf += dt * df;
  }
  stt = block_sum(stt, s_red);
  stf = block_sum(stf, s_red);
  if (threadIdx.x == 0) {
    const double rate = stt > 0.0 ? stf / stt : 0.0;
    r.rate1 = rate;
    r.rate_per_sample = rate / p.sample_rate;
    r.status = p.precise_sync ? FT8_DRIFT_PENDING : FT8_DRIFT_LINEAR;
    a.res[slot] = r;
  }
}

// ---- stage 2 ---------------------------------------------------------------------------------
// Python slice bound normalisation for a sequence of length T
__device__ __forceinline__ int py_norm(int v, int T) { return v < 0 ? max(v + T, 0) : min(v, T); }

__global__ __launch_bounds__(kFitThreads) void k_drift_fit2(DriftFitLaunch a) {
  FT8_RACE_PROLOGUE();
  __shared__ int s_idx[kDriftMaxT];
  __shared__ double s_tmpl[kMaxTmpl];
  __shared__ double s_px[kMaxPts], s_py[kMaxPts];
  __shared__ double s_red[kFitWaves];
  __shared__ double s_bv[kFitWaves];
  __shared__ int s_bi[kFitWaves];
  const int slot = blockIdx.x;
  ft8_drift_result r = a.res[slot];
  if (r.status != FT8_DRIFT_PENDING) return;  // uniform over the workgroup
  const int T = a.T;
  const ft8_drift_params& p = a.p;
  const int32_t* idx = a.idx + (int64_t)slot * T;
  for (int i = threadIdx.x; i < T; i += kFitThreads) s_idx[i] = idx[i];
  const int L = a.n_tmpl;
  for (int i = threadIdx.x; i < L; i += kFitThreads) s_tmpl[i] = a.tmpl[i];
  __syncthreads();

  const int tosr = p.steps_per_symbol;
  const int w = p.window_size_factor * tosr;
  const double fstep = p.sym_bin / (double)p.bins_per_tone;
  // masked track (:419-431): f2[s:e] - mean(f2[s:e]) inside the slice, 0 elsewhere
  const int ms = py_norm(r.seg_start, T);
  const int me = max(py_norm(r.seg_end + w - 2, T), ms);
  double sm = 0.0;
  for (int i = ms + threadIdx.x; i < me; i += kFitThreads) sm += (double)s_idx[i] * fstep;
  sm = block_sum(sm, s_red);
  const double mean = me > ms ? sm / (double)(me - ms) : 0.0;
  auto masked = [&](int i) -> double { return (double)s_idx[i] * fstep - mean; };

  // full correlation (:433): c[k] = sum_n masked[n + k - (L - 1)] tmpl[n], k in [0, T + L - 1)
  const int K = T + L - 1;
  double bv = -__builtin_huge_val();
  int bi = 0x7fffffff;
  for (int k = threadIdx.x; k < K; k += kFitThreads) {
    const int off = k - (L - 1);
    const int n0 = max(0, ms - off), n1 = min(L, me - off);
    double c = 0.0;
    for (int n = n0; n < n1; ++n) c += masked(n + off) * s_tmpl[n];
    if (c > bv || (c == bv && k < bi)) { bv = c; bi = k; }
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const double ov = __shfl_xor(bv, off);
    const int oi = __shfl_xor(bi, off);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  if ((threadIdx.x & (kWave - 1)) == 0) { s_bv[threadIdx.x / kWave] = bv; s_bi[threadIdx.x / kWave] = bi; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int k = 1; k < kFitWaves; ++k)
    if (s_bv[k] > bv || (s_bv[k] == bv && s_bi[k] < bi)) { bv = s_bv[k]; bi = s_bi[k]; }
  const int sync_idx = bi - (L - 1) + (2 * tosr) / 2;  // :463
  r.sync_idx = sync_idx;

  // regression points of the three sync blocks (:502-519), Python slicing semantics
  const double xs = p.sym_t / (double)tosr;
  int nx = 0, ny = 0;
  for (int i = 0; i < 3; ++i) {
    const int st = i * (p.nsync_sym + p.ndata_sym / 2) * tosr + sync_idx;
    const int en = st + (p.nsync_sym - 1) * tosr;
    if (st < T) {
      const int stop = min(en, T);
      for (int j = st; j < stop && nx < kMaxPts; ++j) s_px[nx++] = (double)j * xs;
      const int y0 = py_norm(st, T), y1 = py_norm(stop, T);
      for (int j = y0; j < y1 && ny < kMaxPts; ++j) {
        const bool in = j >= ms && j < me;
        s_py[ny++] = in ? masked(j) : 0.0;
      }
    }
  }
  r.n_points = nx;
  const int deg = p.poly_degree;
  if (nx < 10) {
    r.status = FT8_DRIFT_FEW_POINTS;  // :521-523
  } else if (!(nx > deg + 1)) {
    r.status = FT8_DRIFT_UNDERDETERMINED;  // :659
  } else if (nx != ny || deg < 0) {
    r.status = FT8_DRIFT_VALUE_ERROR;
  } else if (deg != 1 && deg != 2) {
    r.status = FT8_DRIFT_DEGREE;  // :630-631
  } else {
    // centred least squares on [x, x^2] (the bias column centres to zero: coef[0] = 0)
    const int n = nx;
    double sx = 0.0, sx2 = 0.0, sy = 0.0;
    for (int j = 0; j < n; ++j) {
      const double x = s_px[j];
      sx += x;
      sx2 += x * x;
      sy += s_py[j];
    }
    const double xm = sx / n, x2m = sx2 / n, ym = sy / n;
    double c1 = 0.0, c2 = 0.0;
    if (deg == 1) {
      double aa = 0.0, ab = 0.0;
      for (int j = 0; j < n; ++j) {
        const double a1 = s_px[j] - xm, b = s_py[j] - ym;
        aa += a1 * a1;
        ab += a1 * b;
      }
      c1 = aa > 0.0 ? ab / aa : 0.0;
    } else {
      // modified Gram-Schmidt on the centred columns a1 = x - xm, a2 = x^2 - x2m
      double r11 = 0.0;
      for (int j = 0; j < n; ++j) { const double a1 = s_px[j] - xm; r11 += a1 * a1; }
      r11 = sqrt(r11);
      double r12 = 0.0, z1 = 0.0;
      for (int j = 0; j < n; ++j) {
        const double q1 = (s_px[j] - xm) / r11;
        r12 += q1 * (s_px[j] * s_px[j] - x2m);
        z1 += q1 * (s_py[j] - ym);
      }
      double r22 = 0.0;
      for (int j = 0; j < n; ++j) {
        const double v = (s_px[j] * s_px[j] - x2m) - r12 * ((s_px[j] - xm) / r11);
        r22 += v * v;
      }
      r22 = sqrt(r22);
      double z2 = 0.0;
      for (int j = 0; j < n; ++j) {
        const double v = (s_px[j] * s_px[j] - x2m) - r12 * ((s_px[j] - xm) / r11);
        z2 += (v / r22) * (s_py[j] - ym);
      }
      c2 = r22 > 0.0 ? z2 / r22 : 0.0;
      c1 = r11 > 0.0 ? (z1 - r12 * c2) / r11 : 0.0;
    }
    const double b = ym - (xm * c1 + x2m * c2);
    r.coef[0] = 0.0;
    r.coef[1] = c1;
    r.coef[2] = c2;
    r.intercept = b;
    const double x0 = s_px[0], x1 = s_px[n - 1];
    const double first = (x0 * c1 + (deg == 2 ? (x0 * x0) * c2 : 0.0)) + b;  // predict (:650-653)
    const double last = (x1 * c1 + (deg == 2 ? (x1 * x1) * c2 : 0.0)) + b;
    const double real = (first - last) / (x0 - x1) + r.rate1;  // :650
    r.rate_per_sample = real / p.sample_rate;
    r.status = FT8_DRIFT_FULL;
  }
  a.res[slot] = r;
}

// ---- de-rotation -----------------------------------------------------------------------------
constexpr int kRotThreads = 256;
constexpr int kRotPer = 4;

template <typename InT, bool CPLX>
__global__ __launch_bounds__(kRotThreads) void k_derotate1(DerotateLaunch a) {
  const int slot = blockIdx.y;
  const ft8_drift_result& r = a.res[slot];
  const bool copy = r.status == FT8_DRIFT_NO_SEGMENT || r.status == FT8_DRIFT_VALUE_ERROR;
  const double rate = r.rate1;
  const InT* x = reinterpret_cast<const InT*>(a.x) + (int64_t)slot * a.slot_stride * (CPLX ? 2 : 1);
  double2* out = reinterpret_cast<double2*>(a.out) + (int64_t)slot * a.n_samples;
  const int64_t base = ((int64_t)blockIdx.x * kRotThreads * kRotPer) + threadIdx.x;
#pragma unroll
  for (int u = 0; u < kRotPer; ++u) {
    const int64_t n = base + (int64_t)u * kRotThreads;
    if (n >= a.n_samples) break;
    double xr, xi;
    if constexpr (CPLX) { xr = (double)x[2 * n]; xi = (double)x[2 * n + 1]; }
    else { xr = (double)x[n]; xi = 0.0; }
    if (copy) { out[n] = make_double2(xr, xi); continue; }
    // :352  np.exp(-2j*np.pi*(f_shift_rate*array_range**2/2/fs)/(fs))
    const double v = ((rate * (double)(n * n)) / 2.0) / a.fs;
    const double th = (-kTwoPi * v) * a.inv_fs;
    double s, c;
    sincos(th, &s, &c);
    out[n] = make_double2(xr * c - xi * s, xr * s + xi * c);
  }
}

__global__ __launch_bounds__(kRotThreads) void k_derotate2(DerotateLaunch a, int deg) {
  const int slot = blockIdx.y;
  const ft8_drift_result& r = a.res[slot];
  if (r.status != FT8_DRIFT_FULL) return;
  const double c1 = r.coef[1], c2 = r.coef[2];
  const double k1 = -kTwoPi * c1;  // (-2j*np.pi*f_shift_rate_final).imag
  double2* out = reinterpret_cast<double2*>(a.out) + (int64_t)slot * a.n_samples;
  const int64_t base = ((int64_t)blockIdx.x * kRotThreads * kRotPer) + threadIdx.x;
#pragma unroll
  for (int u = 0; u < kRotPer; ++u) {
    const int64_t n = base + (int64_t)u * kRotThreads;
    if (n >= a.n_samples) break;
    double th;
    if (deg == 1) {
      th = (k1 * (double)(n * n)) * a.inv_2fs2;  // :603
    } else {
      const double t = (double)n / a.fs;        // :609-611
      const double ph = (c1 * (t * t)) / 2.0 + (c2 * pow(t, 3.0)) / 3.0;
      th = -kTwoPi * ph;
    }
    double s, c;
    sincos(th, &s, &c);
    const double2 y = out[n];
    out[n] = make_double2(y.x * c - y.y * s, y.x * s + y.y * c);
  }
}

}  // namespace

hipError_t launch_drift_fit(int stage, const DriftFitLaunch& a, hipStream_t s) {
  if (a.n_slots <= 0) return hipSuccess;
  if (stage == 1) hipLaunchKernelGGL(k_drift_fit1, dim3(a.n_slots), dim3(kFitThreads), 0, s, a);
  else hipLaunchKernelGGL(k_drift_fit2, dim3(a.n_slots), dim3(kFitThreads), 0, s, a);
  return hipGetLastError();
}

int drift_max_template() { return kMaxTmpl; }
int drift_max_points() { return kMaxPts; }

hipError_t launch_derotate1(const DerotateLaunch& a, hipStream_t s) {
  if (a.n_slots <= 0 || a.n_samples <= 0) return hipSuccess;
  const dim3 grid((unsigned)((a.n_samples + kRotThreads * kRotPer - 1) / (kRotThreads * kRotPer)), (unsigned)a.n_slots);
  switch (a.dtype) {
    case FT8_F32: hipLaunchKernelGGL((k_derotate1<float, false>), grid, dim3(kRotThreads), 0, s, a); break;
    case FT8_F64: hipLaunchKernelGGL((k_derotate1<double, false>), grid, dim3(kRotThreads), 0, s, a); break;
    case FT8_C64: hipLaunchKernelGGL((k_derotate1<float, true>), grid, dim3(kRotThreads), 0, s, a); break;
    case FT8_C128: hipLaunchKernelGGL((k_derotate1<double, true>), grid, dim3(kRotThreads), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_derotate2(const DerotateLaunch& a, int deg, hipStream_t s) {
  if (a.n_slots <= 0 || a.n_samples <= 0 || (deg != 1 && deg != 2)) return hipSuccess;
  const dim3 grid((unsigned)((a.n_samples + kRotThreads * kRotPer - 1) / (kRotThreads * kRotPer)), (unsigned)a.n_slots);
  hipLaunchKernelGGL(k_derotate2, grid, dim3(kRotThreads), 0, s, a, deg);
  return hipGetLastError();
}

}  // namespace ft8
