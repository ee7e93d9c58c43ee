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
// Stockham autosort mixed-radix (16,8,4,2,15,5,3,7; largest first, so a 3840-point
// transform is 16 x 16 x 15: three LDS round trips) transform held in LDS: every stage loads its
// butterflies into registers, barriers, and writes the permuted outputs back, so one LDS buffer of
// P complex values suffices (15 KB fp32 at 12 kHz).  The first stage reads the frame straight from
// HBM (coalesced across lanes, window applied on the fly), the epilogue writes the kept bins of the
// dB waterfall row-contiguously (waterfall layout [slot][frame][bin], frequency fastest).
//
// Precision: (this file is compiled with FMA contraction, see the Makefile) float32 samples (and
// int16 WAV samples, scaled x/32767 in float32 as read_wave_file does) are transformed in float32 and produce a float32 waterfall, as SciPy does for complex64;
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

// 16 = 4 x 4 (Cooley-Tukey, internal twiddles W_16^(n2 k1)), output in natural order
template <typename T>
struct Dft<16, T> {
  __device__ static void run(cplx<T>* a) {
    const T c1 = (T)0.92387953251128675613, s1 = (T)0.38268343236508977173, r = (T)0.70710678118654752440;
    cplx<T> A[4][4];  // [n2][k1]
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
      cplx<T> v[4] = {a[n2], a[4 + n2], a[8 + n2], a[12 + n2]};
      Dft<4, T>::run(v);
#pragma unroll
      for (int k1 = 0; k1 < 4; ++k1) A[n2][k1] = v[k1];
    }
    // W_16^m = exp(-2 pi i m / 16), m = n2 k1 in [0, 9]
    const cplx<T> w[10] = {{(T)1, (T)0}, {c1, -s1}, {r, -r}, {s1, -c1}, {(T)0, (T)-1},
                           {-s1, -c1}, {-r, -r}, {-c1, -s1}, {(T)-1, (T)0}, {-c1, s1}};
#pragma unroll
    for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
      for (int k1 = 1; k1 < 4; ++k1) A[n2][k1] = cmul(A[n2][k1], w[n2 * k1]);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      cplx<T> v[4] = {A[0][k1], A[1][k1], A[2][k1], A[3][k1]};
      Dft<4, T>::run(v);
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) a[k1 + 4 * k2] = v[k2];
    }
  }
};
// 15 = 3 x 5 prime-factor (no internal twiddles): n = (5 n1 + 3 n2) mod 15, k = (10 k1 + 6 k2) mod 15
template <typename T>
struct Dft<15, T> {
  __device__ static void run(cplx<T>* a) {
    cplx<T> Y[3][5];
#pragma unroll
    for (int n1 = 0; n1 < 3; ++n1) {
#pragma unroll
      for (int n2 = 0; n2 < 5; ++n2) Y[n1][n2] = a[(5 * n1 + 3 * n2) % 15];
      Dft<5, T>::run(Y[n1]);
    }
#pragma unroll
    for (int k2 = 0; k2 < 5; ++k2) {
      cplx<T> v[3] = {Y[0][k2], Y[1][k2], Y[2][k2]};
      Dft<3, T>::run(v);
#pragma unroll
      for (int k1 = 0; k1 < 3; ++k1) a[(10 * k1 + 6 * k2) % 15] = v[k1];
    }
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

// LDS index with one pad element per 16: the Stockham writes of the early stages go out with a
// stride of R complex values across lanes (16 x 16 B = 256 B for float64 radix 16, every lane on the
// same banks); padded, the stride is 17 and a 64-lane write needs the minimum number of passes.
__device__ __forceinline__ int pidx(int i) { return i + (i >> 4); }

// One Stockham stage of radix R.  MAXV = max complex values per thread (P <= 256 * MAXV).
// HALF (first stage only): inputs j + r nbf with r >= R / 2 are the frame's zero padding (real
// input, nperseg <= P), set as constants so the butterfly's first layer folds away
template <int R, int MAXV, bool FIRST, typename CT, typename Src, bool HALF = false, int TH = kThreads>
__device__ __forceinline__ void stockham_stage(cplx<CT>* buf, int P, int Ns, const cplx<CT>* tw,
                                               const Src& src) {
  constexpr int MAXB = (MAXV + R - 1) / R;
  const int nbf = P / R;
  const int tid = threadIdx.x;
  cplx<CT> v[MAXB][R];
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int j = tid + b * TH;
    if (j < nbf) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (FIRST && HALF) v[b][r] = r < R / 2 ? src(j + r * nbf) : cplx<CT>{(CT)0, (CT)0};
        else if constexpr (FIRST) v[b][r] = src(j + r * nbf);
        else v[b][r] = buf[pidx(j + r * nbf)];
      }
    }
  }
  if constexpr (!FIRST) __syncthreads();
  const int tstep = P / (Ns * R);
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int j = tid + b * TH;
    if (j < nbf) {
      const int k = j % Ns;
      if (!FIRST && k != 0) {
        if constexpr (sizeof(CT) == 4 && R <= 8) {
          // float32, radix <= 8: the powers of w = W^(k tstep) by recurrence from one table read
          // (relative error <= 7 ulp) instead of R - 1 dependent L1 gathers.  The 14-step chain of a
          // radix-15 stage moved bins 60 dB below a frame's peak by up to 1.4e-3 dB at P = 9 600
          // (the test bound is 1e-3): radices 15 and 16 keep the table
          const cplx<CT> w = tw[k * tstep];
          cplx<CT> wr = w;
#pragma unroll
          for (int r = 1; r < R; ++r) {
            v[b][r] = cmul(v[b][r], wr);
            if (r + 1 < R) wr = cmul(wr, w);
          }
        } else {
#pragma unroll
          for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], tw[r * k * tstep]);
        }
      }
      Dft<R, CT>::run(v[b]);
      const int d0 = (j / Ns) * Ns * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) buf[pidx(d0 + r * Ns)] = v[b][r];
    }
  }
  __syncthreads();
}

template <int MAXV, bool FIRST, int TH = kThreads, typename CT, typename Src>
__device__ void run_stage(int R, cplx<CT>* buf, int P, int Ns, const cplx<CT>* tw, const Src& src) {
  switch (R) {
    case 2: stockham_stage<2, MAXV, FIRST, CT, Src, false, TH>(buf, P, Ns, tw, src); break;
    case 3: stockham_stage<3, MAXV, FIRST, CT, Src, false, TH>(buf, P, Ns, tw, src); break;
    case 4: stockham_stage<4, MAXV, FIRST, CT, Src, false, TH>(buf, P, Ns, tw, src); break;
    case 5: stockham_stage<5, MAXV, FIRST, CT, Src, false, TH>(buf, P, Ns, tw, src); break;
    case 7: stockham_stage<7, MAXV, FIRST, CT, Src, false, TH>(buf, P, Ns, tw, src); break;
    case 15: stockham_stage<15, MAXV, FIRST, CT, Src, false, TH>(buf, P, Ns, tw, src); break;
    case 16: stockham_stage<16, MAXV, FIRST, CT, Src, false, TH>(buf, P, Ns, tw, src); break;
    default: stockham_stage<8, MAXV, FIRST, CT, Src, false, TH>(buf, P, Ns, tw, src); break;
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
  int32_t* argmax;  // non-null: per-frame argmax of the kept dB row instead of the row itself
  int n_slots, per_xcd;
  // k_stftc3840 screening (complex128 argmax): frames whose float32 argmax is not certain are
  // appended to list[0 .. *list_count) as slot * nt_out + frame, and re-done in float64
  int32_t* list;
  int32_t* list_count;
};

// np.argmax order: the first NaN wins, else the largest value, ties to the lower index
template <typename CT>
__device__ __forceinline__ bool argmax_better(CT av, int ai, CT bv, int bi) {
  const bool an = av != av, bn = bv != bv;
  if (an != bn) return an;
  if (!an && av != bv) return av > bv;
  return ai < bi;
}

template <typename CT>
__device__ __forceinline__ CT db_of(CT v) {
  if constexpr (sizeof(CT) == 4) return 10.0f * log10f(v);
  else return 10.0 * log10(v);
}

// np.argmax order of the dB values 10 log10(level) decided on the levels: levels further apart
// than a relative 1e-9 (float64; 1e-4 for float32 -- far above the log's few-ulp error) order their
// dB values the same way; closer ones (and NaN) compare their dB values exactly, first index on
// ties.  Every decision equals the comparison of the (dB, -index) keys, so any reduction tree
// returns np.argmax of the dB row while taking a log only for near ties.
// (Measured and not kept in round 3, profiles/r3_drift_stft_ab.log: the log path as a call
// (__noinline__), 11.5 -> 12.6 ms per float64 drift call; an early first-index return for exactly
// equal levels, 12.9 ms -- each changed the code generation of the inlined comparison sites.)
template <typename CT>
__device__ __forceinline__ bool level_better(CT la, int ia, CT lb, int ib) {
  constexpr CT eps = sizeof(CT) == 4 ? (CT)1e-4 : (CT)1e-9;
  if (la == la && lb == lb) {
    if (la > lb * ((CT)1 + eps)) return true;
    if (lb > la * ((CT)1 + eps)) return false;
  }
  return argmax_better(db_of(la), ia, db_of(lb), ib);
}

template <typename InT, bool CPLX, typename CT, int MAXV>
// two resident waves per SIMD for P <= 4096 (the LDS allows two float64 3840-point workgroups per
// CU; the radix-16/15 stages then fit 256 VGPRs), one for the 8192- and 10240-point variants (a
// 16384-point float32 variant, 64 values per thread, trips a gfx950 code-generation error)
__global__ __launch_bounds__(kThreads, (MAXV <= 16 ? 2 : 1)) void k_stft(StftArgs a) {
  FT8_RACE_PROLOGUE();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cplx<CT>* buf = reinterpret_cast<cplx<CT>*>(smem);
  // XCD-aware order: hardware deals workgroup ids round-robin over the 8 XCDs, so consecutive
  // ids would put neighbouring (overlapping) frames on different L2s.  Each XCD instead takes a
  // contiguous run of (slot, frame) pairs, and overlapping frames share its L2.
  const int nt = a.nt_out;
  const int r = (int)(blockIdx.x & 7) * a.per_xcd + (int)(blockIdx.x >> 3);
  if (r >= nt * a.n_slots) return;
  const int slot = r / nt;
  const int fi = r - slot * nt;
  const int frame = a.t_lo + fi;
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
  const int N = a.nfft;
  const cplx<CT>* post = reinterpret_cast<const cplx<CT>*>(a.post);
  // the argument of the log for kept bin i: 1e-12 + |X|^2 / (sum w)^2
  auto level = [&](int i) -> CT {
    const int k = a.f_lo + i;
    cplx<CT> X;
    if constexpr (CPLX) {
      X = buf[pidx(k)];
    } else {
      const int kk = (k <= P) ? k : N - k;  // real signal: X[N-k] = conj X[k]
      const cplx<CT> A = buf[pidx(kk == P ? 0 : kk)];
      const cplx<CT> Bc = buf[pidx(kk == 0 ? 0 : P - kk)];
      const cplx<CT> B = {Bc.x, -Bc.y};
      const cplx<CT> s = cadd(A, B), d = csub(A, B);
      const cplx<CT> wd = cmul(post[kk], d);
      // X = s/2 - i wd/2
      X = {(CT)0.5 * (s.x + wd.y), (CT)0.5 * (s.y - wd.x)};
    }
    const CT pw = (X.x * X.x + X.y * X.y) * scale;
    return (CT)1e-12 + pw;
  };
  if (a.argmax == nullptr) {
    CT* out = reinterpret_cast<CT*>(a.out) + ((int64_t)slot * a.nt_out + fi) * a.nf_out;
    if constexpr (sizeof(CT) == 4) {
      // 10 log10(v) = (10 log10 2) log2(v): v_log_f32 on a normal argument (v >= 1e-12), as
      // k_stft3840p; log10f's correctly rounded libm sequence took ~25 VALU per bin
      constexpr float kDb = 3.0102999566398119521f;
      for (int i = threadIdx.x; i < a.nf_out; i += kThreads) out[i] = kDb * __builtin_amdgcn_logf(level(i));
    } else {
      for (int i = threadIdx.x; i < a.nf_out; i += kThreads) out[i] = db_of(level(i));
    }
    return;
  }
  // argmax (np.argmax of the dB row) in one pass on the levels (level_better)
  unsigned char* scratch = smem + (size_t)(P + P / 16 + 1) * sizeof(cplx<CT>);
  CT* sv = reinterpret_cast<CT*>(scratch);
  int* si = reinterpret_cast<int*>(scratch + sizeof(CT) * (kThreads / kWave));
  const int w = threadIdx.x / kWave;
  CT vm = -__builtin_huge_val();
  int vi = 0x7fffffff;
  for (int i = threadIdx.x; i < a.nf_out; i += kThreads) {
    const CT v = level(i);
    if (level_better(v, i, vm, vi)) { vm = v; vi = i; }
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const CT ov = __shfl_xor(vm, off);
    const int oi = __shfl_xor(vi, off);
    if (level_better(ov, oi, vm, vi)) { vm = ov; vi = oi; }
  }
  if ((threadIdx.x & (kWave - 1)) == 0) { sv[w] = vm; si[w] = vi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kThreads / kWave; ++k)
      if (level_better(sv[k], si[k], vm, vi)) { vm = sv[k]; vi = si[k]; }
    a.argmax[(int64_t)slot * nt + fi] = vi;
  }
}

// ---- k_stft_sp: the generic transform with a compile-time radix plan (round 4) -------------------
// Real float32 / int16 input with the dB epilogue, for the plans of the reference's other
// geometries: 20 kHz at bpt = sps = 2 (P = 3 200 = 16 x 8 x 5 x 5, the bundled recording's rate), 12 kHz
// at bpt = sps = 10 (P = 9 600 = 16 x 8 x 15 x 5, the decode test's) and 6 kHz (P = 960 = 16 x 4 x 15).
// k_stft's runtime radix switch keeps every case's registers live (206 VGPRs at P = 3 200, two
// waves per SIMD; 439 at P = 9 600); with the stages fixed each holds only its own butterflies, and
// the first stage's zero-padded half (nperseg <= P) is constant-folded.
// the stages after the first with compile-time P and Ns: the stage's index math (j % Ns, j / Ns,
// the twiddle stride P / (Ns R)) folds to shifts and constant multiplies
template <int P, int NS, int MAXV, typename Src, int R, int... Rest>
__device__ __forceinline__ void sp_stages(cplx<float>* buf, const cplx<float>* tw, const Src& src) {
  stockham_stage<R, MAXV, false>(buf, P, NS, tw, src);
  if constexpr (sizeof...(Rest) > 0) sp_stages<P, NS * R, MAXV, Src, Rest...>(buf, tw, src);
}

template <typename InT, int P, int MAXV, int R0, int... Rs>
__global__ __launch_bounds__(kThreads) void k_stft_sp(StftArgs a) {
  FT8_RACE_PROLOGUE();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cplx<float>* buf = reinterpret_cast<cplx<float>*>(smem);
  const int nt = a.nt_out;
  const int r = (int)(blockIdx.x & 7) * a.per_xcd + (int)(blockIdx.x >> 3);  // XCD-aware, as k_stft
  if (r >= nt * a.n_slots) return;
  const int slot = r / nt;
  const int fi = r - slot * nt;
  const int frame = a.t_lo + fi;
  const InT* xs = reinterpret_cast<const InT*>(a.samples) + (int64_t)slot * a.slot_stride + (int64_t)frame * a.hop;
  FrameSrc<InT, false, float> src{xs, reinterpret_cast<const float*>(a.window), a.nperseg};
  const cplx<float>* tw = reinterpret_cast<const cplx<float>*>(a.tw);
  stockham_stage<R0, MAXV, true, float, FrameSrc<InT, false, float>, true>(buf, P, 1, tw, src);
  sp_stages<P, R0, MAXV, FrameSrc<InT, false, float>, Rs...>(buf, tw, src);

  const float scale = (float)a.scale;
  const cplx<float>* post = reinterpret_cast<const cplx<float>*>(a.post);
  constexpr float kDb = 3.0102999566398119521f;  // 10 log10(v) = (10 log10 2) log2(v), v >= 1e-12
  float* out = reinterpret_cast<float*>(a.out) + ((int64_t)slot * a.nt_out + fi) * a.nf_out;
  for (int i = threadIdx.x; i < a.nf_out; i += kThreads) {
    const int k = a.f_lo + i;
    const int kk = (k <= P) ? k : 2 * P - k;  // real signal (nfft = 2 P): X[N-k] = conj X[k]
    const cplx<float> A = buf[pidx(kk == P ? 0 : kk)];
    const cplx<float> Bc = buf[pidx(kk == 0 ? 0 : P - kk)];
    const cplx<float> B = {Bc.x, -Bc.y};
    const cplx<float> sm = cadd(A, B), d = csub(A, B);
    const cplx<float> wd = cmul(post[kk], d);
    const cplx<float> X = {0.5f * (sm.x + wd.y), 0.5f * (sm.y - wd.x)};  // X = s/2 - i wd/2
    out[i] = kDb * __builtin_amdgcn_logf(1e-12f + (X.x * X.x + X.y * X.y) * scale);
  }
}

// the static plans k_stft_sp is built for: {P, radices...}
struct SpPlan {
  int P, n, r[5];
};
constexpr SpPlan kSpPlans[] = {{3200, 4, {16, 8, 5, 5}}, {9600, 4, {16, 8, 15, 5}}, {960, 3, {16, 4, 15}}};

// ---- k_stftc3840: complex input, nfft = 3840, nperseg = 1920, hop = 240 M (M in 1, 2, 4, 8) -----
// The beacon receiver's geometry (12 kHz complex baseband, frequency_correction.py; the reference
// test runs steps_per_symbol = 8, hop 240).  P = 3840 = 16 x 16 x 15: 256 threads, one butterfly per
// thread per stage, one padded LDS buffer.  Thread t < 240 owns the stage-1 inputs z[t + 240 r],
// r < 8 (r >= 8 is the zero padding, so stage 1 is a half-input 16-point DFT); a frame advances by M
// of those positions, so the thread keeps its 8 raw samples in registers and loads only M new ones
// per frame (one at hop 240) -- every sample is read from HBM once -- prefetched while the current
// frame is transformed.  Twiddles are powers of two per-thread seeds (recurrence); the stage-3 outputs
// X[t + 256 r] come out in natural order in registers, so the epilogue (dB row or argmax) reads no
// LDS.  Workgroups walk runs of kC38Chunk frames of one signal, runs of one signal on one XCD.
constexpr int kC38P = 3840;
constexpr int kC38Threads = 256;
constexpr int kC38Chunk = 32;

// 16-point DFT of a[0..7] with a[8..15] = 0 (4 x 4 Cooley-Tukey), in place, natural order
template <typename T>
__device__ __forceinline__ void dft16_half_t(cplx<T>* a) {
  const T c1 = (T)0.92387953251128675613, s1 = (T)0.38268343236508977173, rr = (T)0.70710678118654752440;
  const cplx<T> w[10] = {{(T)1, (T)0}, {c1, -s1}, {rr, -rr}, {s1, -c1}, {(T)0, (T)-1},
                         {-s1, -c1}, {-rr, -rr}, {-c1, -s1}, {(T)-1, (T)0}, {-c1, s1}};
  cplx<T> A[4][4];  // [n2][k1]
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
    const cplx<T> x0 = a[n2], x1 = a[4 + n2];
    A[n2][0] = cadd(x0, x1);
    A[n2][1] = cadd(x0, mul_mi(x1));
    A[n2][2] = csub(x0, x1);
    A[n2][3] = csub(x0, mul_mi(x1));
  }
#pragma unroll
  for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1) A[n2][k1] = cmul(A[n2][k1], w[n2 * k1]);
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    cplx<T> v[4] = {A[0][k1], A[1][k1], A[2][k1], A[3][k1]};
    Dft<4, T>::run(v);
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) a[k1 + 4 * k2] = v[k2];
  }
}

template <typename InT, typename CT>
__device__ __forceinline__ cplx<CT> load_c(const InT* x, int64_t n) {
  if constexpr (sizeof(InT) == 8) {
    const double2 v = *reinterpret_cast<const double2*>(x + 2 * n);
    return {(CT)v.x, (CT)v.y};
  } else {
    const float2 v = *reinterpret_cast<const float2*>(x + 2 * n);
    return {(CT)v.x, (CT)v.y};
  }
}

// AMAX: the argmax epilogue (its own instantiation: a kernel carrying both epilogues is allocated
// for the dB one's fifteen inlined float64 log10)
// MODE: 0 dB rows, 1 argmax (level_better), 2 float32 screening argmax (CT = float; uncertain
// frames listed), 3 the listed frames again in float64 (CT = double), one frame at a time
constexpr int kScreenKappa = 256;  // FFT error bound factor of the screening test (see below)
template <typename InT, typename CT, int M, int MODE>
__global__ __launch_bounds__(kC38Threads, 2) void k_stftc3840(StftArgs a) {
  FT8_RACE_PROLOGUE();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cplx<CT>* buf = reinterpret_cast<cplx<CT>*>(smem);
  CT* sv = reinterpret_cast<CT*>(smem + (size_t)(kC38P + kC38P / 16 + 1) * sizeof(cplx<CT>));
  int* si = reinterpret_cast<int*>(sv + kC38Threads / kWave);
  CT* wl = sv + 16;  // the window, staged once per workgroup (registers are the scarce resource)
  const int t = threadIdx.x;
  const int w_id = t / kWave;
  const int nt = a.nt_out;
  const int chunks = (nt + kC38Chunk - 1) / kC38Chunk;
  const int rr = (int)(blockIdx.x & 7) * a.per_xcd + (int)(blockIdx.x >> 3);
  if (MODE != 3 && rr >= chunks * a.n_slots) return;
  if (MODE == 3 && (int)blockIdx.x >= *a.list_count) return;
  int slot = rr / chunks;
  const int c = rr - slot * chunks;
  int f_begin = c * kC38Chunk, f_end = min(nt, f_begin + kC38Chunk);
  const cplx<CT>* tw = reinterpret_cast<const cplx<CT>*>(a.tw);  // W_3840^m
  const CT* win = reinterpret_cast<const CT*>(a.window);
  const bool s1 = t < 240;
  for (int n = t; n < 1920; n += kC38Threads) wl[n] = win[n];
  __syncthreads();  // stage 1 reads other threads' window entries
  // twiddle seeds: stage 2 W_256^k = W_3840^(15 k) (k = t % 16), stage 3 W_3840^t; their powers are
  // formed by complex recurrence each frame (relative error ~15 ulp, far inside the tolerances)
  cplx<CT> s2 = tw[15 * (t & 15)], s3 = tw[t];
  const CT scale = (CT)a.scale;
  constexpr bool amax = MODE != 0;
  const int k_lo = a.f_lo, k_hi = a.f_lo + a.nf_out;
  // MODE 3: workgroup l takes listed frames l, l + gridDim, ...: one frame at a time, its 8 raw
  // samples per thread loaded afresh
  const int n_list = MODE == 3 ? *a.list_count : 0;
  for (int l = blockIdx.x;; l += gridDim.x) {
  if constexpr (MODE == 3) {
    if (l >= n_list) break;
    const int code = a.list[l];
    slot = code / nt;
    f_begin = code - slot * nt;
    f_end = f_begin + 1;
  }
  const InT* xs = reinterpret_cast<const InT*>(a.samples) + (int64_t)slot * a.slot_stride * 2;
  cplx<CT> raw[8];
  {
    const int64_t base = (int64_t)(a.t_lo + f_begin) * a.hop;
#pragma unroll
    for (int r = 0; r < 8; ++r) raw[r] = s1 ? load_c<InT, CT>(xs, base + t + 240 * r) : cplx<CT>{(CT)0, (CT)0};
  }
  for (int f = f_begin; f < f_end; ++f) {
    // re-opaque the seeds so the per-frame twiddle powers are not hoisted into ~60 live registers
    if constexpr (sizeof(CT) == 8) {
      asm volatile("" : "+v"(s2.x), "+v"(s2.y), "+v"(s3.x), "+v"(s3.y));
    } else {
      asm volatile("" : "+v"(s2.x), "+v"(s2.y), "+v"(s3.x), "+v"(s3.y));
    }
    cplx<CT> nx[M];
    const bool more = f + 1 < f_end;
    if (s1 && more) {
      const int64_t base = (int64_t)(a.t_lo + f + 1) * a.hop;
#pragma unroll
      for (int q = 0; q < M; ++q) nx[q] = load_c<InT, CT>(xs, base + t + 240 * (8 - M + q));
    }
    cplx<CT> v[16];
    // stage 1: radix 16, Ns = 1 -> buf[16 t + k].  The window comes from LDS each frame.
    if (s1) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const CT wv = wl[t + 240 * r];
        v[r] = {wv * raw[r].x, wv * raw[r].y};
      }
      dft16_half_t<CT>(v);
#pragma unroll
      for (int k = 0; k < 16; ++k) buf[17 * t + k] = v[k];  // pidx(16 t + k)
    }
    __syncthreads();
    // stage 2: radix 16, Ns = 16: buf[t + 240 r] -> twiddle W_256^(r k), k = t % 16 -> buf[(t/16) 256 + k + 16 r]
    if (s1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = buf[pidx(t) + 255 * r];  // pidx(t + 240 r)
    }
    __syncthreads();
    if (s1) {
      const int k = t & 15;
      cplx<CT> wr = s2;
#pragma unroll
      for (int r = 1; r < 16; ++r) {
        v[r] = cmul(v[r], wr);
        wr = cmul(wr, s2);
      }
      Dft<16, CT>::run(v);
      const int d0 = (t >> 4) * 256 + k;
#pragma unroll
      for (int r = 0; r < 16; ++r) buf[pidx(d0) + 17 * r] = v[r];  // pidx(d0 + 16 r)
    }
    __syncthreads();
    // stage 3: radix 15, Ns = 256: buf[t + 256 r] -> twiddle W_3840^(r t) -> X[t + 256 r]
#pragma unroll
    for (int r = 0; r < 15; ++r) v[r] = buf[pidx(t) + 272 * r];  // pidx(t + 256 r)
    __syncthreads();  // the next frame's stage 1 may overwrite buf
    {
      cplx<CT> wr = s3;
#pragma unroll
      for (int r = 1; r < 15; ++r) {
        v[r] = cmul(v[r], wr);
        wr = cmul(wr, s3);
      }
    }
    Dft<15, CT>::run(v);
    // epilogue on the registers: level = 1e-12 + |X|^2 / (sum w)^2 of kept bins
    CT lv[15];
#pragma unroll
    for (int r = 0; r < 15; ++r) lv[r] = (CT)1e-12 + (v[r].x * v[r].x + v[r].y * v[r].y) * scale;
    if constexpr (!amax) {
      CT* out = reinterpret_cast<CT*>(a.out) + ((int64_t)slot * nt + f) * a.nf_out;
#pragma unroll
      for (int r = 0; r < 15; ++r) {
        const int k = t + 256 * r;
        if (k >= k_lo && k < k_hi) {
          if constexpr (sizeof(CT) == 4) out[k - k_lo] = 10.0f * log10f(lv[r]);
          else out[k - k_lo] = 10.0 * log10(lv[r]);
        }
      }
    } else if constexpr (MODE == 2) {
      // float32 screening: the two largest kept levels (first index on equal ones) and the total
      // energy of the frame's spectrum.  An FFT's rounding error in any one bin is bounded by a
      // small multiple of u log2(N) times the spectrum's L2 norm (u = 2^-24), so with
      // delta = kappa u sqrt(E) (kappa = 256, over ten times the analytic constant with the
      // twiddle recurrences' ~15 ulp) the float64 transform orders bins i1 and i2 the same way
      // whenever L1 - L2 > 2 (2 sqrt(L1) delta + delta^2) + 8 u L1; the float64 argmax then is i1.
      // Every other frame is listed and transformed again in float64 (MODE 3).
      float l1 = -INFINITY, l2 = -INFINITY, es = 0.0f;
      int i1 = 0x7fffffff;
#pragma unroll
      for (int r = 0; r < 15; ++r) {
        const int k = t + 256 * r;
        es += lv[r] - 1e-12f;
        if (k >= k_lo && k < k_hi) {
          if (lv[r] > l1 || (lv[r] == l1 && k < i1)) {
            l2 = l1;
            l1 = lv[r];
            i1 = k;
          } else if (lv[r] > l2) {
            l2 = lv[r];
          }
        }
      }
#pragma unroll
      for (int off = kWave / 2; off > 0; off >>= 1) {
        const float o1 = __shfl_xor(l1, off), o2 = __shfl_xor(l2, off);
        const int oi = __shfl_xor(i1, off);
        es += __shfl_xor(es, off);
        if (o1 > l1 || (o1 == l1 && oi < i1)) {
          l2 = fmaxf(l1, o2);
          l1 = o1;
          i1 = oi;
        } else {
          l2 = fmaxf(l2, o1);
        }
      }
      // the 16 words before the window: l1 [0, 4), si's indices [4, 8), l2 [8, 12), es [12, 16)
      float* s_l = reinterpret_cast<float*>(sv);
      if ((t & (kWave - 1)) == 0) {
        s_l[w_id] = l1;
        si[w_id] = i1;
        s_l[8 + w_id] = l2;
        s_l[12 + w_id] = es;
      }
      __syncthreads();
      if (t == 0) {
        double e_tot = s_l[12];
        for (int q = 1; q < kC38Threads / kWave; ++q) {
          const float o1 = s_l[q], o2 = s_l[8 + q];
          const int oi = si[q];
          e_tot += s_l[12 + q];
          if (o1 > l1 || (o1 == l1 && oi < i1)) {
            l2 = fmaxf(l1, o2);
            l1 = o1;
            i1 = oi;
          } else {
            l2 = fmaxf(l2, o1);
          }
        }
        const double u = 0x1p-24;
        const double delta = kScreenKappa * u * sqrt(fmax(e_tot, 0.0) * 1.0001);
        const double need = 2.0 * (2.0 * sqrt((double)l1) * delta + delta * delta) + 8.0 * u * (double)l1;
        const int64_t fi = (int64_t)slot * nt + f;
        if ((double)l1 - (double)l2 > need && l1 == l1) {
          a.argmax[fi] = i1 - k_lo;
        } else {
          const int pos = atomicAdd(a.list_count, 1);
          a.list[pos] = (int)fi;
        }
      }
    } else {
      // one-pass argmax of the dB row on the levels (level_better)
      CT vm = -__builtin_huge_val();
      int vi = 0x7fffffff;
#pragma unroll
      for (int r = 0; r < 15; ++r) {
        const int k = t + 256 * r;
        if (k >= k_lo && k < k_hi && level_better(lv[r], k, vm, vi)) { vm = lv[r]; vi = k; }
      }
#pragma unroll
      for (int off = kWave / 2; off > 0; off >>= 1) {
        const CT ov = __shfl_xor(vm, off);
        const int oi = __shfl_xor(vi, off);
        if (level_better(ov, oi, vm, vi)) { vm = ov; vi = oi; }
      }
      if ((t & (kWave - 1)) == 0) { sv[w_id] = vm; si[w_id] = vi; }
      __syncthreads();
      if (t == 0) {
        for (int k = 1; k < kC38Threads / kWave; ++k)
          if (level_better(sv[k], si[k], vm, vi)) { vm = sv[k]; vi = si[k]; }
        a.argmax[(int64_t)slot * nt + f] = vi - k_lo;
      }
    }
    // slide the raw samples by M positions
    if (more) {
#pragma unroll
      for (int r = 0; r < 8 - M; ++r) raw[r] = raw[r + M];
#pragma unroll
      for (int q = 0; q < M; ++q) raw[8 - M + q] = nx[q];
    }
  }
  if constexpr (MODE != 3) break;  // a run of frames: one pass of the outer loop
  }
}

template <typename InT, typename CT>
hipError_t launch_c3840(const StftLaunch& L, StftArgs a, hipStream_t s) {
  const int chunks = (a.nt_out + kC38Chunk - 1) / kC38Chunk;
  a.per_xcd = (int)(((int64_t)chunks * L.n_slots + 7) / 8);
  const dim3 grid((unsigned)(8 * a.per_xcd));
  const size_t lds = (size_t)(kC38P + kC38P / 16 + 1) * sizeof(cplx<CT>) + 16 * sizeof(CT) + 1920 * sizeof(CT);
  auto go = [&](auto kern) {
    if (lds > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, grid, dim3(kC38Threads), lds, s, a);
    return hipGetLastError();
  };
  auto go_m = [&](auto am) {
    constexpr int AM = decltype(am)::value;
    switch (L.hop) {
      case 240: return go(k_stftc3840<InT, CT, 1, AM>);
      case 480: return go(k_stftc3840<InT, CT, 2, AM>);
      case 960: return go(k_stftc3840<InT, CT, 4, AM>);
      default: return go(k_stftc3840<InT, CT, 8, AM>);
    }
  };
  if (a.argmax == nullptr) return go_m(std::integral_constant<int, 0>{});
  return go_m(std::integral_constant<int, 1>{});
}

// complex128 argmax in two steps: the float32 transform decides every frame whose argmax the
// float32 error bound settles (MODE 2), the float64 transform redoes the others (MODE 3, a
// persistent grid over the device-side list; typically a few percent of the frames)
hipError_t launch_c3840_screened(const StftLaunch& L, StftArgs a, hipStream_t s) {
  a.list = L.screen_list;
  a.list_count = L.screen_count;
  hipError_t e = hipMemsetAsync(L.screen_count, 0, sizeof(int32_t), s);
  if (e != hipSuccess) return e;
  const int chunks = (a.nt_out + kC38Chunk - 1) / kC38Chunk;
  a.per_xcd = (int)(((int64_t)chunks * L.n_slots + 7) / 8);
  const size_t lds32 = (size_t)(kC38P + kC38P / 16 + 1) * sizeof(cplx<float>) + 16 * sizeof(float) + 1920 * sizeof(float);
  const size_t lds64 = (size_t)(kC38P + kC38P / 16 + 1) * sizeof(cplx<double>) + 16 * sizeof(double) + 1920 * sizeof(double);
  auto go = [&](auto kern, dim3 grid, size_t lds, const StftArgs& args) {
    if (lds > 64 * 1024) {
      hipError_t e2 = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)lds);
      if (e2 != hipSuccess) return e2;
    }
    hipLaunchKernelGGL(kern, grid, dim3(kC38Threads), lds, s, args);
    return hipGetLastError();
  };
  const dim3 g1((unsigned)(8 * a.per_xcd));
  const int64_t frames = (int64_t)a.nt_out * L.n_slots;
  // the screen transforms in float32 (the plan's tables are float64 for complex128 input)
  StftArgs a32 = a;
  a32.tw = L.screen_tw;
  a32.window = L.screen_window;
  const dim3 g2((unsigned)std::min<int64_t>(frames, 512));  // two float64 workgroups per CU
  switch (L.hop) {
    case 240:
      if ((e = go(k_stftc3840<double, float, 1, 2>, g1, lds32, a32)) != hipSuccess) return e;
      return go(k_stftc3840<double, double, 1, 3>, g2, lds64, a);
    case 480:
      if ((e = go(k_stftc3840<double, float, 2, 2>, g1, lds32, a32)) != hipSuccess) return e;
      return go(k_stftc3840<double, double, 2, 3>, g2, lds64, a);
    case 960:
      if ((e = go(k_stftc3840<double, float, 4, 2>, g1, lds32, a32)) != hipSuccess) return e;
      return go(k_stftc3840<double, double, 4, 3>, g2, lds64, a);
    default:
      if ((e = go(k_stftc3840<double, float, 8, 2>, g1, lds32, a32)) != hipSuccess) return e;
      return go(k_stftc3840<double, double, 8, 3>, g2, lds64, a);
  }
}

// ---- k_stft_dft: direct DFT for lengths the FFT plans cannot take ---------------------------
// (a prime factor above 7, e.g. 32 768 Hz: nfft = 10 485 = 3 x 5 x 3 x 233; odd real nfft; nfft
// above the LDS FFT limit).  One workgroup per (bin block of 256, frame, slot): the windowed frame
// is staged in LDS, each thread sums its bin X[k] = sum_n z[n] W^(k n) sequentially in n, the twiddle
// advanced by complex recurrence and re-seeded from the exact table entry W^((k n) mod nfft) every
// 32 samples.  A fallback for correctness on any geometry, O(nperseg) work per bin.
constexpr int kDftThreads = 256;
constexpr int kDftReseed = 32;

template <typename InT, bool CPLX, typename CT>
__global__ __launch_bounds__(kDftThreads) void k_stft_dft(StftArgs a) {
  FT8_RACE_PROLOGUE();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cplx<CT>* z = reinterpret_cast<cplx<CT>*>(smem);
  const int nbb = (a.nf_out + kDftThreads - 1) / kDftThreads;
  const int fi = blockIdx.x / nbb, bb = blockIdx.x - fi * nbb;
  const int slot = blockIdx.y;
  const int frame = a.t_lo + fi;
  const InT* xs = reinterpret_cast<const InT*>(a.samples) +
                  (int64_t)slot * a.slot_stride * (CPLX ? 2 : 1) + (int64_t)frame * a.hop * (CPLX ? 2 : 1);
  const CT* win = reinterpret_cast<const CT*>(a.window);
  const int L = a.nperseg, N = a.nfft;
  for (int n = threadIdx.x; n < L; n += kDftThreads) {
    CT re, im = (CT)0;
    if constexpr (CPLX) {
      re = (CT)xs[2 * n];
      im = (CT)xs[2 * n + 1];
    } else if constexpr (sizeof(CT) == 4) {
      re = load_f32<InT>(xs, n);
    } else {
      re = (CT)xs[n];
    }
    z[n] = {win[n] * re, win[n] * im};
  }
  __syncthreads();
  const int i = bb * kDftThreads + threadIdx.x;
  if (i >= a.nf_out) return;
  const int k = a.f_lo + i;
  const cplx<CT>* tw = reinterpret_cast<const cplx<CT>*>(a.tw);  // W_N^m, m in [0, N)
  const cplx<CT> step = tw[k % N];
  cplx<CT> acc = {(CT)0, (CT)0};
  for (int n0 = 0; n0 < L; n0 += kDftReseed) {
    cplx<CT> w = tw[(int)(((int64_t)k * n0) % N)];
    const int n1 = min(L, n0 + kDftReseed);
    for (int n = n0; n < n1; ++n) {
      const cplx<CT> v = cmul(z[n], w);
      acc = cadd(acc, v);
      w = cmul(w, step);
    }
  }
  const CT pw = (acc.x * acc.x + acc.y * acc.y) * (CT)a.scale;
  CT* out = reinterpret_cast<CT*>(a.out) + ((int64_t)slot * a.nt_out + fi) * a.nf_out;
  if constexpr (sizeof(CT) == 4) out[i] = 10.0f * log10f(1e-12f + pw);
  else out[i] = 10.0 * log10(1e-12 + pw);
}

// ---- k_stft_blue: chirp-z (Bluestein) transform for lengths the Stockham plans cannot take ---------
// (an nfft with a prime factor above 7, e.g. the reference drift test's 32 768 Hz: nfft 10 485 =
// 3^2 x 5 x 233; an odd nfft with real input).  With c(k) = exp(-i pi k^2 / N), the frame's DFT is
//   X[k] = c(k) sum_{n < L} a[n] conj(c(k - n)),   a[n] = c(n) w[n] x[n],
// a linear convolution of the L windowed samples with a chirp filter.  Output bins are taken in
// blocks of B = P - L + 1 (overlap-save): block b's bins k0 + t (k0 = b B, t < B) are samples
// t + L - 1 of the length-P circular convolution of a with h_b[m] = conj(c(k0 + m - (L - 1))),
// m < B + L - 1, which no wrap-around reaches.  One workgroup per (slot, frame, block): a -> FFT_P
// (LDS Stockham, P a power of two) -> times FFT_P(h_b) (precomputed per plan) -> inverse FFT_P (the
// forward stages on the conjugate) -> c(k) y / P.  O(P log P) per block instead of the direct DFT's
// O(L) per bin: for the 32 768 Hz complex128 geometry (P 8192, L 5242, two blocks cover the kept
// f >= 0 half) ~2 MFLOP per frame against ~220.
template <typename InT, bool CPLX, typename CT>
struct BlueSrc {
  const InT* x;       // frame start (complex: InT = CT pairs)
  const CT* w;        // window
  const cplx<CT>* c;  // chirp
  int L;
  __device__ __forceinline__ cplx<CT> operator()(int n) const {
    if (n >= L) return {(CT)0, (CT)0};
    CT re, im = (CT)0;
    if constexpr (CPLX) {
      const CT* xc = reinterpret_cast<const CT*>(x);
      re = xc[2 * n];
      im = xc[2 * n + 1];
    } else if constexpr (sizeof(CT) == 4) {
      re = load_f32<InT>(x, n);
    } else {
      re = (CT)x[n];
    }
    const cplx<CT> z = {w[n] * re, w[n] * im};
    return cmul(z, c[n]);
  }
};

struct BlueArgs {
  StftArgs s;
  int L, B, blk0, nblk_run;  // blocks blk0 .. blk0 + nblk_run - 1 cover the kept bins
  const void* chirp;
  const void* hspec;
};

// TH threads: 512 for P > 4096 (the float64 8192-point image is 139 KB: one workgroup per CU, so
// 256 threads left 4 waves per CU through every stage's barriers)
template <typename InT, bool CPLX, typename CT, int MAXV, int TH>
__global__ __launch_bounds__(TH, 1) void k_stft_blue(BlueArgs b) {
  FT8_RACE_PROLOGUE();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cplx<CT>* buf = reinterpret_cast<cplx<CT>*>(smem);
  const StftArgs& a = b.s;
  // XCD-aware order as k_stft: each XCD takes a contiguous run of (slot, frame, block) triples, so a
  // frame's blocks and its neighbours (overlapping samples) share one L2
  const int nt = a.nt_out;
  const int r = (int)(blockIdx.x & 7) * a.per_xcd + (int)(blockIdx.x >> 3);
  if (r >= nt * a.n_slots * b.nblk_run) return;
  const int blk = b.blk0 + r % b.nblk_run;
  const int sf = r / b.nblk_run;
  const int slot = sf / nt, fi = sf - slot * nt;
  const int frame = a.t_lo + fi;
  const InT* xs = reinterpret_cast<const InT*>(a.samples) +
                  (int64_t)slot * a.slot_stride * (CPLX ? 2 : 1) + (int64_t)frame * a.hop * (CPLX ? 2 : 1);
  const cplx<CT>* chirp = reinterpret_cast<const cplx<CT>*>(b.chirp);
  BlueSrc<InT, CPLX, CT> src{xs, reinterpret_cast<const CT*>(a.window), chirp, b.L};
  const cplx<CT>* tw = reinterpret_cast<const cplx<CT>*>(a.tw);
  const int P = a.P;
  // forward FFT of a
  int Ns = 1;
  run_stage<MAXV, true, TH>(a.radix[0], buf, P, Ns, tw, src);
  Ns *= a.radix[0];
  for (int st = 1; st < a.nstages; ++st) {
    run_stage<MAXV, false, TH>(a.radix[st], buf, P, Ns, tw, src);
    Ns *= a.radix[st];
  }
  // times the block's filter spectrum, conjugated: the forward stages then give P conj(y)
  const cplx<CT>* H = reinterpret_cast<const cplx<CT>*>(b.hspec) + (int64_t)blk * P;
  for (int k = threadIdx.x; k < P; k += TH) {
    const cplx<CT> y = cmul(buf[pidx(k)], H[k]);
    buf[pidx(k)] = {y.x, -y.y};
  }
  __syncthreads();
  Ns = 1;
  for (int st = 0; st < a.nstages; ++st) {
    run_stage<MAXV, false, TH>(a.radix[st], buf, P, Ns, tw, src);
    Ns *= a.radix[st];
  }
  // bins of this block inside the kept range -> dB row (argmax requests reduce the rows afterwards)
  const int k0 = blk * b.B;
  const int lo = max(k0, a.f_lo), hi = min(k0 + b.B, a.f_lo + a.nf_out);
  const CT inv = (CT)1 / (CT)P, scale = (CT)a.scale;
  CT* out = reinterpret_cast<CT*>(a.out) + ((int64_t)slot * a.nt_out + fi) * a.nf_out;
  for (int k = lo + (int)threadIdx.x; k < hi; k += TH) {
    const cplx<CT> v = buf[pidx(k - k0 + b.L - 1)];
    const cplx<CT> X = cmul(chirp[k], cplx<CT>{v.x * inv, -v.y * inv});
    const CT pw = (X.x * X.x + X.y * X.y) * scale;
    out[k - a.f_lo] = db_of((CT)1e-12 + pw);
  }
}

// np.argmax of each dB row [slot][frame][nf] (the direct-DFT path's argmax): one wave per row
template <typename CT>
__global__ __launch_bounds__(kWave) void k_row_argmax(const CT* rows, int nf, int64_t n_rows, int32_t* idx) {
  const int64_t r = blockIdx.x;
  if (r >= n_rows) return;
  const CT* row = rows + r * nf;
  CT bv = -__builtin_huge_val();
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < nf; i += kWave)
    if (argmax_better(row[i], i, bv, bi)) { bv = row[i]; bi = i; }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const CT ov = __shfl_xor(bv, off);
    const int oi = __shfl_xor(bi, off);
    if (argmax_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
  }
  if (threadIdx.x == 0) idx[r] = bi;
}

template <typename InT, bool CPLX, typename CT>
hipError_t launch_dft(const StftLaunch& L, const StftArgs& a, hipStream_t s) {
  const size_t lds = (size_t)L.nperseg * sizeof(cplx<CT>);
  if (lds > (size_t)kMaxDftLds) return hipErrorInvalidValue;
  auto kern = k_stft_dft<InT, CPLX, CT>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  const int nbb = (a.nf_out + kDftThreads - 1) / kDftThreads;
  hipLaunchKernelGGL(kern, dim3((unsigned)(nbb * a.nt_out), (unsigned)L.n_slots), dim3(kDftThreads), lds, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !L.argmax) return e;
  const int64_t rows = (int64_t)a.nt_out * L.n_slots;
  hipLaunchKernelGGL(k_row_argmax<CT>, dim3((unsigned)rows), dim3(kWave), 0, s, reinterpret_cast<const CT*>(a.out),
                     a.nf_out, rows, L.argmax);
  return hipGetLastError();
}

template <typename InT, bool CPLX, typename CT>
hipError_t launch_blue(const StftLaunch& L, const StftArgs& a, hipStream_t s) {
  BlueArgs b{};
  b.s = a;
  b.s.argmax = nullptr;  // the rows are written; an argmax request reduces them below
  b.L = L.plan.L;
  b.B = L.plan.B;
  b.blk0 = a.f_lo / b.B;
  b.nblk_run = (a.f_lo + a.nf_out - 1) / b.B - b.blk0 + 1;
  b.chirp = L.plan.chirp;
  b.hspec = L.plan.hspec;
  const int64_t units = (int64_t)a.nt_out * L.n_slots * b.nblk_run;
  b.s.per_xcd = (int)((units + 7) / 8);
  const size_t lds = (size_t)(a.P + a.P / 16 + 1) * sizeof(cplx<CT>);
  if (a.P > 512 * 16 || L.plan.L > a.P) return hipErrorInvalidValue;
  const bool wide = a.P > kThreads * 16;
  auto kern = !wide ? k_stft_blue<InT, CPLX, CT, 16, kThreads> : k_stft_blue<InT, CPLX, CT, 16, 512>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(8 * b.s.per_xcd)), dim3(wide ? 512 : kThreads), lds, s, b);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !L.argmax) return e;
  const int64_t rows = (int64_t)a.nt_out * L.n_slots;
  hipLaunchKernelGGL(k_row_argmax<CT>, dim3((unsigned)rows), dim3(kWave), 0, s, reinterpret_cast<const CT*>(a.out),
                     a.nf_out, rows, L.argmax);
  return hipGetLastError();
}

template <typename InT, bool CPLX, typename CT>
hipError_t launch_t(const StftLaunch& L, const StftArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)(8 * a.per_xcd));  // see k_stft: a.per_xcd (slot, frame) pairs per XCD
  // pidx padding + the argmax epilogue's cross-wave scratch
  const size_t lds = (size_t)(a.P + a.P / 16 + 1) * sizeof(cplx<CT>) + 64;
  auto go = [&](auto kern) {
    if (lds > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, grid, dim3(kThreads), lds, s, a);
    return hipGetLastError();
  };
  if constexpr (!CPLX && sizeof(CT) == 4) {
    // a static plan for the reference's other real-input geometries (dB rows, nperseg <= P)
    auto plan_is = [&](const SpPlan& q) {
      if (a.P != q.P || a.nstages != q.n || a.argmax != nullptr || a.nperseg > a.P) return false;
      for (int i = 0; i < q.n; ++i)
        if (a.radix[i] != q.r[i]) return false;
      return true;
    };
    if (plan_is(kSpPlans[0])) return go(k_stft_sp<InT, 3200, 13, 16, 8, 5, 5>);
    if (plan_is(kSpPlans[1])) return go(k_stft_sp<InT, 9600, 38, 16, 8, 15, 5>);
    if (plan_is(kSpPlans[2])) return go(k_stft_sp<InT, 960, 4, 16, 4, 15>);
  }
  if (a.P <= kThreads * 8) return go(k_stft<InT, CPLX, CT, 8>);
  // P <= 3840 (3840 = 16 x 16 x 15: one butterfly per thread per stage) keeps half the registers
  // of the P <= 4096 variant, whose radix-15 stage would hold two butterflies per thread
  if (a.P <= kThreads * 15) return go(k_stft<InT, CPLX, CT, 15>);
  if (a.P <= kThreads * 16) return go(k_stft<InT, CPLX, CT, 16>);
  if constexpr (sizeof(CT) == 8) {
    return go(k_stft<InT, CPLX, CT, 32>);  // float64: P <= 8192 (kMaxFftP64)
  } else {
    if (a.P <= kThreads * 32) return go(k_stft<InT, CPLX, CT, 32>);
    return go(k_stft<InT, CPLX, CT, 40>);  // float32 P <= 10240, e.g. nfft 19200 (12 kHz, bpt 10)
  }
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
  a.argmax = L.argmax;
  a.n_slots = L.n_slots;
  a.per_xcd = (int)(((int64_t)a.nt_out * L.n_slots + 7) / 8);
  if (a.nt_out <= 0 || a.nf_out <= 0 || L.n_slots <= 0) return hipSuccess;
  if (L.plan.blue) {
    switch (L.dtype) {
      case FT8_F32: return launch_blue<float, false, float>(L, a, s);
      case FT8_I16: return launch_blue<int16_t, false, float>(L, a, s);
      case FT8_F64: return launch_blue<double, false, double>(L, a, s);
      case FT8_C64: return launch_blue<float, true, float>(L, a, s);
      case FT8_C128: return launch_blue<double, true, double>(L, a, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (L.plan.dft) {
    a.argmax = nullptr;  // the DFT kernel writes dB rows; launch_dft reduces them to the argmax
    switch (L.dtype) {
      case FT8_F32: return launch_dft<float, false, float>(L, a, s);
      case FT8_I16: return launch_dft<int16_t, false, float>(L, a, s);
      case FT8_F64: return launch_dft<double, false, double>(L, a, s);
      case FT8_C64: return launch_dft<float, true, float>(L, a, s);
      case FT8_C128: return launch_dft<double, true, double>(L, a, s);
      default: return hipErrorInvalidValue;
    }
  }
  // production geometry (12 kHz, bins_per_tone = steps_per_symbol = 2): stft3840.hip's packed kernel
  if (stft3840_eligible(L)) return launch_stft3840(L, s);
  // the reference's other real-input geometries (20 kHz, 12 kHz at bpt 10, 6 kHz): packed plans
  if (stftpk_eligible(L)) return launch_stftpk(L, s);
  // complex input in the beacon receiver's geometry (12 kHz: nfft 3840, nperseg 1920, hop 240 M)
  if ((L.dtype == FT8_C64 || L.dtype == FT8_C128) && L.nfft == kC38P && L.nperseg == 1920 && a.P == kC38P &&
      (L.hop == 240 || L.hop == 480 || L.hop == 960 || L.hop == 1920)) {
    if (L.dtype == FT8_C128 && L.argmax && L.screen_list && L.screen_tw && L.screen_window)
      return launch_c3840_screened(L, a, s);
    if (L.dtype == FT8_C128) return launch_c3840<double, double>(L, a, s);
    return launch_c3840<float, float>(L, a, s);
  }
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
