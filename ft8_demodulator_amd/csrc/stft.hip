// stft.hip -- STFT power spectrum in dB for FT8 slots (gfx950).
//
// Replaces calculate_spectrogram (reference spectrogram_analyse.py:19-66: periodic Hann window,
// nperseg = int(0.16 fs), hop = nperseg // steps_per_symbol, nfft = int(fs / 6.25 * bpt),
// two-sided |FFT|^2 / (sum w)^2, 10 log10(1e-12 + P)) and the f >= 0 / band / time masks of
// decode_ft8_message (ft8_decode.py:322-341).
//
// One workgroup (256 threads, 4 waves) per (frame, slot).  Real input uses the half-length
// trick: z[n] = w x[2n] + i w x[2n+1] is transformed with a P = nfft/2 point complex FFT and the
// spectrum of the real frame is recovered as X[k] = (Z[k] + Z*[P-k])/2 - i W_N^k (Z[k] - Z*[P-k])/2,
// halving the FFT work.  Complex (I/Q) input transforms the full nfft points.  The FFT is a
// Stockham autosort mixed-radix (2,3,4,5,7,8) transform held in LDS: every stage loads its
// butterflies into registers, barriers, and writes the permuted outputs back, so one LDS buffer of
// P complex values suffices (15 KB fp32 at 12 kHz).  The first stage reads the frame straight from
// HBM (coalesced across lanes, window applied on the fly), the epilogue writes the kept bins of the
// dB waterfall row-contiguously (waterfall layout [slot][frame][bin], frequency fastest).
//
// Precision: float32 samples (and int16 WAV samples, scaled x/32767 in float32 as read_wave_file
// does) are transformed in float32 and produce a float32 waterfall, as SciPy does for complex64;
// float64 / complex128 input runs in float64 (SciPy complex128).  The FFT is not bit-identical to
// pocketfft; tests bound the difference (tests/test_gpu_stft.py).
#include "ft8_internal.h"

namespace ft8 {
namespace {

constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ cplx<T> cadd(cplx<T> a, cplx<T> b) { return {a.x + b.x, a.y + b.y}; }
template <typename T>
__device__ __forceinline__ cplx<T> csub(cplx<T> a, cplx<T> b) { return {a.x - b.x, a.y - b.y}; }
template <typename T>
__device__ __forceinline__ cplx<T> cmul(cplx<T> a, cplx<T> b) {
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
template <typename T>
__device__ __forceinline__ cplx<T> cscale(cplx<T> a, T s) { return {a.x * s, a.y * s}; }
// multiply by -i
template <typename T>
__device__ __forceinline__ cplx<T> mul_mi(cplx<T> a) { return {a.y, -a.x}; }

// ---- in-register forward DFTs of radix R (W_R = exp(-2 pi i / R)) ---------------------------
template <int R, typename T>
struct Dft;

template <typename T>
struct Dft<2, T> {
  __device__ static void run(cplx<T>* a) {
    cplx<T> t = a[1];
    a[1] = csub(a[0], t);
    a[0] = cadd(a[0], t);
  }
};
template <typename T>
struct Dft<3, T> {
  __device__ static void run(cplx<T>* a) {
    const T s3 = (T)0.86602540378443864676;
    cplx<T> t = cadd(a[1], a[2]);
    cplx<T> d = csub(a[1], a[2]);
    cplx<T> m = {a[0].x - (T)0.5 * t.x, a[0].y - (T)0.5 * t.y};
    cplx<T> e = {s3 * d.y, -s3 * d.x};  // -i s3 (a1 - a2)
    a[0] = cadd(a[0], t);
    a[1] = cadd(m, e);
    a[2] = csub(m, e);
  }
};
template <typename T>
struct Dft<4, T> {
  __device__ static void run(cplx<T>* a) {
    cplx<T> t0 = cadd(a[0], a[2]), t1 = csub(a[0], a[2]);
    cplx<T> t2 = cadd(a[1], a[3]), t3 = mul_mi(csub(a[1], a[3]));
    a[0] = cadd(t0, t2);
    a[2] = csub(t0, t2);
    a[1] = cadd(t1, t3);
    a[3] = csub(t1, t3);
  }
};
template <typename T>
struct Dft<5, T> {
  __device__ static void run(cplx<T>* a) {
    const T c1 = (T)0.30901699437494742410, c2 = (T)-0.80901699437494742410;
    const T s1 = (T)0.95105651629515357212, s2 = (T)0.58778525229247312917;
    cplx<T> t1 = cadd(a[1], a[4]), t2 = cadd(a[2], a[3]);
    cplx<T> t3 = csub(a[1], a[4]), t4 = csub(a[2], a[3]);
    cplx<T> b1 = {a[0].x + c1 * t1.x + c2 * t2.x, a[0].y + c1 * t1.y + c2 * t2.y};
    cplx<T> b2 = {a[0].x + c2 * t1.x + c1 * t2.x, a[0].y + c2 * t1.y + c1 * t2.y};
    cplx<T> e1 = {s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y};
    cplx<T> e2 = {s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y};
    a[0] = cadd(a[0], cadd(t1, t2));
    a[1] = {b1.x + e1.y, b1.y - e1.x};
    a[4] = {b1.x - e1.y, b1.y + e1.x};
    a[2] = {b2.x + e2.y, b2.y - e2.x};
    a[3] = {b2.x - e2.y, b2.y + e2.x};
  }
};
template <typename T>
struct Dft<8, T> {
  __device__ static void run(cplx<T>* a) {
    const T r = (T)0.70710678118654752440;
    cplx<T> e[4] = {a[0], a[2], a[4], a[6]};
    cplx<T> o[4] = {a[1], a[3], a[5], a[7]};
    Dft<4, T>::run(e);
    Dft<4, T>::run(o);
    cplx<T> w1 = {(o[1].x + o[1].y) * r, (o[1].y - o[1].x) * r};
    cplx<T> w2 = mul_mi(o[2]);
    cplx<T> w3 = {(o[3].y - o[3].x) * r, -(o[3].x + o[3].y) * r};
    a[0] = cadd(e[0], o[0]);
    a[4] = csub(e[0], o[0]);
    a[1] = cadd(e[1], w1);
    a[5] = csub(e[1], w1);
    a[2] = cadd(e[2], w2);
    a[6] = csub(e[2], w2);
    a[3] = cadd(e[3], w3);
    a[7] = csub(e[3], w3);
  }
};
template <typename T>
struct Dft<7, T> {
  __device__ static void run(cplx<T>* a) {
    const T c[7] = {(T)1.0, (T)0.62348980185873353053, (T)-0.22252093395631440429,
                    (T)-0.90096886790241912624, (T)-0.90096886790241912624,
                    (T)-0.22252093395631440429, (T)0.62348980185873353053};
    const T s[7] = {(T)0.0, (T)0.78183148246802980871, (T)0.97492791218182360702,
                    (T)0.43388373911755812048, (T)-0.43388373911755812048,
                    (T)-0.97492791218182360702, (T)-0.78183148246802980871};
    cplx<T> y[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      cplx<T> acc = a[0];
#pragma unroll
      for (int r = 1; r < 7; ++r) {
        const int m = (r * k) % 7;
        // a[r] * (c - i s)
        acc.x += a[r].x * c[m] + a[r].y * s[m];
        acc.y += a[r].y * c[m] - a[r].x * s[m];
      }
      y[k] = acc;
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) a[k] = y[k];
  }
};

// ---- frame loader: FFT input z[idx] of frame `frame` of slot `slot` --------------------------
template <typename InT>
__device__ __forceinline__ float load_f32(const InT* p, int64_t i);
template <>
__device__ __forceinline__ float load_f32<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float load_f32<int16_t>(const int16_t* p, int64_t i) {
  return (float)p[i] / 32767.0f;  // read_wave_file: float32(x) / iinfo(int16).max
}

template <typename InT, bool CPLX, typename CT>
struct FrameSrc {
  const InT* x;   // frame start (real: InT samples; complex: InT = CT pairs)
  const CT* w;
  int L;          // nperseg
  __device__ __forceinline__ cplx<CT> operator()(int idx) const {
    if constexpr (CPLX) {
      if (idx >= L) return {(CT)0, (CT)0};
      const CT* xc = reinterpret_cast<const CT*>(x);
      const CT wv = w[idx];
      return {wv * xc[2 * idx], wv * xc[2 * idx + 1]};
    } else {
      const int n0 = 2 * idx;
      CT a = (CT)0, b = (CT)0;
      if constexpr (sizeof(CT) == 4) {
        if (n0 < L) a = w[n0] * load_f32<InT>(x, n0);
        if (n0 + 1 < L) b = w[n0 + 1] * load_f32<InT>(x, n0 + 1);
      } else {
        if (n0 < L) a = w[n0] * (CT)x[n0];
        if (n0 + 1 < L) b = w[n0 + 1] * (CT)x[n0 + 1];
      }
      return {a, b};
    }
  }
};

// One Stockham stage of radix R.  MAXV = max complex values per thread (P <= 256 * MAXV).
template <int R, int MAXV, bool FIRST, typename CT, typename Src>
__device__ __forceinline__ void stockham_stage(cplx<CT>* buf, int P, int Ns, const cplx<CT>* tw,
                                               const Src& src) {
  constexpr int MAXB = (MAXV + R - 1) / R;
  const int nbf = P / R;
  const int tid = threadIdx.x;
  cplx<CT> v[MAXB][R];
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int j = tid + b * kThreads;
    if (j < nbf) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (FIRST) v[b][r] = src(j + r * nbf);
        else v[b][r] = buf[j + r * nbf];
      }
    }
  }
  if constexpr (!FIRST) __syncthreads();
  const int tstep = P / (Ns * R);
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int j = tid + b * kThreads;
    if (j < nbf) {
      const int k = j % Ns;
      if (!FIRST && k != 0) {
#pragma unroll
        for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], tw[r * k * tstep]);
      }
      Dft<R, CT>::run(v[b]);
      const int d0 = (j / Ns) * Ns * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) buf[d0 + r * Ns] = v[b][r];
    }
  }
  __syncthreads();
}

template <int MAXV, bool FIRST, typename CT, typename Src>
__device__ void run_stage(int R, cplx<CT>* buf, int P, int Ns, const cplx<CT>* tw, const Src& src) {
  switch (R) {
    case 2: stockham_stage<2, MAXV, FIRST>(buf, P, Ns, tw, src); break;
    case 3: stockham_stage<3, MAXV, FIRST>(buf, P, Ns, tw, src); break;
    case 4: stockham_stage<4, MAXV, FIRST>(buf, P, Ns, tw, src); break;
    case 5: stockham_stage<5, MAXV, FIRST>(buf, P, Ns, tw, src); break;
    case 7: stockham_stage<7, MAXV, FIRST>(buf, P, Ns, tw, src); break;
    default: stockham_stage<8, MAXV, FIRST>(buf, P, Ns, tw, src); break;
  }
}

struct StftArgs {
  const void* samples;
  int64_t slot_stride;
  int nperseg, hop, nfft;
  int t_lo, f_lo, nf_out, nt_out;
  const void* window;
  double scale;
  void* out;
  int P, nstages;
  int radix[16];
  const void* tw;
  const void* post;
};

template <typename InT, bool CPLX, typename CT, int MAXV>
__global__ __launch_bounds__(kThreads) void k_stft(StftArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cplx<CT>* buf = reinterpret_cast<cplx<CT>*>(smem);
  const int frame = a.t_lo + blockIdx.x;
  const int slot = blockIdx.y;
  const InT* xs = reinterpret_cast<const InT*>(a.samples) +
                  (int64_t)slot * a.slot_stride * (CPLX ? 2 : 1) + (int64_t)frame * a.hop * (CPLX ? 2 : 1);
  FrameSrc<InT, CPLX, CT> src{xs, reinterpret_cast<const CT*>(a.window), a.nperseg};
  const cplx<CT>* tw = reinterpret_cast<const cplx<CT>*>(a.tw);
  const int P = a.P;

  int Ns = 1;
  run_stage<MAXV, true>(a.radix[0], buf, P, Ns, tw, src);
  Ns *= a.radix[0];
  for (int s = 1; s < a.nstages; ++s) {
    run_stage<MAXV, false>(a.radix[s], buf, P, Ns, tw, src);
    Ns *= a.radix[s];
  }

  // epilogue: power spectrum -> dB for bins [f_lo, f_lo + nf_out)
  const CT scale = (CT)a.scale;
  CT* out = reinterpret_cast<CT*>(a.out) + ((int64_t)slot * a.nt_out + blockIdx.x) * a.nf_out;
  const int N = a.nfft;
  const cplx<CT>* post = reinterpret_cast<const cplx<CT>*>(a.post);
  for (int i = threadIdx.x; i < a.nf_out; i += kThreads) {
    const int k = a.f_lo + i;
    cplx<CT> X;
    if constexpr (CPLX) {
      X = buf[k];
    } else {
      const int kk = (k <= P) ? k : N - k;  // real signal: X[N-k] = conj X[k]
      const cplx<CT> A = buf[kk == P ? 0 : kk];
      const cplx<CT> Bc = buf[kk == 0 ? 0 : P - kk];
      const cplx<CT> B = {Bc.x, -Bc.y};
      const cplx<CT> s = cadd(A, B), d = csub(A, B);
      const cplx<CT> wd = cmul(post[kk], d);
      // X = s/2 - i wd/2
      X = {(CT)0.5 * (s.x + wd.y), (CT)0.5 * (s.y - wd.x)};
    }
    const CT pw = (X.x * X.x + X.y * X.y) * scale;
    if constexpr (sizeof(CT) == 4) {
      const float v = 1e-12f + pw;
      out[i] = 10.0f * log10f(v);
    } else {
      out[i] = 10.0 * log10(1e-12 + pw);
    }
  }
}

template <typename InT, bool CPLX, typename CT>
hipError_t launch_t(const StftLaunch& L, const StftArgs& a, hipStream_t s) {
  dim3 grid(L.t_hi - L.t_lo, L.n_slots);
  const size_t lds = (size_t)a.P * sizeof(cplx<CT>);
  auto go = [&](auto kern) {
    if (lds > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, grid, dim3(kThreads), lds, s, a);
    return hipGetLastError();
  };
  if (a.P <= kThreads * 8) return go(k_stft<InT, CPLX, CT, 8>);
  if (a.P <= kThreads * 16) return go(k_stft<InT, CPLX, CT, 16>);
  return go(k_stft<InT, CPLX, CT, 32>);
}

}  // namespace

hipError_t launch_stft(const StftLaunch& L, hipStream_t s) {
  StftArgs a{};
  a.samples = L.samples;
  a.slot_stride = L.slot_stride;
  a.nperseg = L.nperseg;
  a.hop = L.hop;
  a.nfft = L.nfft;
  a.t_lo = L.t_lo;
  a.f_lo = L.f_lo;
  a.nf_out = L.f_hi - L.f_lo;
  a.nt_out = L.t_hi - L.t_lo;
  a.window = L.window;
  a.scale = L.scale;
  a.out = L.out;
  a.P = L.plan.P;
  a.nstages = L.plan.nstages;
  for (int i = 0; i < 16; ++i) a.radix[i] = L.plan.radix[i];
  a.tw = L.plan.tw;
  a.post = L.plan.post;
  if (a.nt_out <= 0 || a.nf_out <= 0 || L.n_slots <= 0) return hipSuccess;
  switch (L.dtype) {
    case FT8_F32: return launch_t<float, false, float>(L, a, s);
    case FT8_I16: return launch_t<int16_t, false, float>(L, a, s);
    case FT8_F64: return launch_t<double, false, double>(L, a, s);
    case FT8_C64: return launch_t<float, true, float>(L, a, s);
    case FT8_C128: return launch_t<double, true, double>(L, a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace ft8
