// capi.hip -- host side of libft8hip.so: context, STFT plans, scratch, launches, C-ABI.
//
// See include/ft8hip.h for the contract.  Everything below runs on the host; all numerical work is
// in the kernels of stft.hip / sync.hip / bp.hip.  No path here computes a decode on the CPU.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ft8_internal.h"

#ifndef FT8_BUILD_ID
#define FT8_BUILD_ID "unversioned"
#endif
#ifndef FT8_BUILD_FLAGS
#define FT8_BUILD_FLAGS ""
#endif

using namespace ft8;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

struct PlanEntry {
  int nfft;
  bool cplx;   // complex-input path (P = nfft) vs real-input half-length path (P = nfft/2)
  bool f64;
  int L = 0;   // nperseg (chirp-z plans are built for one)
  FftPlan plan;
  void* tw = nullptr;
  void* post = nullptr;
  void* chirp = nullptr;
  void* hspec = nullptr;
};

struct WinEntry {
  int L;
  bool f64;
  void* w = nullptr;
  double scale;
};

struct TimedLaunch {
  int stage;
  hipEvent_t a, b;
};

}  // namespace

struct ft8_ctx {
  int device = 0;
  std::string err;
  std::vector<PlanEntry> plans;
  std::vector<WinEntry> wins;
  DevBuf wf, scores, smask, cand, cand_score, cand_count, warn, rowsum, res_all, work, stats, llr, tie;
  // first ticket of the next k_bp launch per claim counter in `work` (8 B each: [0] ft8_bp's, [1 + k]
  // decode chunk k's); reset with the buffer, which is zeroed whenever it is (re)allocated
  std::vector<unsigned long long> work_base;
  // FT8_FLAG_SUBTRACT: residual samples, per-record fits, pass-1 / pass-2 records
  DevBuf residual, sub_est, sub_list, out1, counts1, out2, counts2;
  DevBuf screen;  // complex128 argmax STFT: [count][frames] uncertain-frame list (stft.hip)
  int64_t screen_frames = 0;  // frames of the last screened call (0: the last call was not screened)
  int sub_slots = 0, sub_cap = 0;  // shape of the fits in sub_est (ft8_subtract_fits)
  // cumulative GFSK pulse of the transmit chain for one nsps (double and float)
  int gfsk_nsps = 0;
  DevBuf gfsk_P, gfsk_Pf;
  // frequency-drift correction: per-frame argmax, three-Costas correlation template (cached per
  // steps_per_symbol / nsync / ndata)
  DevBuf drift_idx, drift_tmpl;
  int tmpl_key[3] = {0, 0, 0};
  int tmpl_len = 0;
  bool timing = false;
  uint32_t stage_mask = 0xFFFFFFFFu;  // stages that record events while timing is on
  std::vector<TimedLaunch> pending;
  std::vector<hipEvent_t> pool;
  double ms[FT8_N_STAGES] = {0};
  int64_t launches[FT8_N_STAGES] = {0};
  // decode_batch pipeline: slot chunks spread over internal streams (0 = one chain on the caller's
  // stream); BP grid residency in waves per SIMD
  int chunk_slots = 0, n_streams = 0, bp_waves = 4;
  std::vector<hipStream_t> streams;
  hipEvent_t fork = nullptr;
  std::vector<hipEvent_t> joins;
  // the kernels of the last single-chain ft8_decode_batch, for ft8_replay_stage (benchmarking):
  // valid until the next entry point that may reallocate the context's scratch
  bool replay_ok = false;
  // the stream of the last entry point that enqueued work, and an event recorded on it after that
  // work (StreamOrder): a call on another stream first waits for it
  hipStream_t last_stream = nullptr;
  hipEvent_t last_done = nullptr;
  bool have_last = false;
  StftLaunch last_stft{};
  SyncLaunch last_sync{};
  BpLaunch last_bp{};
  CompactLaunch last_compact{};
};

namespace {

int fail(ft8_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hipfail(ft8_ctx* c, hipError_t e, const char* where) {
  return fail(c, FT8_E_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int ensure(ft8_ctx* c, DevBuf& b, size_t bytes);

// ensure() for a buffer that must read as zeros when (re)allocated: the k_bp work counters, which
// every k_bp launch leaves at 0 again (bp.hip), so they are cleared only here
// *reallocated (optional) reports whether the buffer was (re)allocated and zeroed; a grown buffer
// can come back at the old address, so the test is the capacity as well as the pointer
int ensure_zeroed(ft8_ctx* c, DevBuf& b, size_t bytes, hipStream_t s, bool* reallocated = nullptr) {
  void* old = b.p;
  const size_t old_cap = b.cap;
  if (reallocated) *reallocated = false;
  int rc = ensure(c, b, bytes);
  if (rc || (b.p == old && b.cap == old_cap)) return rc;
  if (reallocated) *reallocated = true;
  hipError_t e = hipMemsetAsync(b.p, 0, b.cap, s);
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "memset");
}

// the k_bp claim counters (8 B each) and their host-side ticket bases: whenever the counters are
// (re)allocated they read 0, so every base restarts at 0 and the vector covers the new capacity
int ensure_work(ft8_ctx* c, int n_counters, hipStream_t s) {
  bool fresh = false;
  int rc = ensure_zeroed(c, c->work, sizeof(unsigned long long) * (size_t)n_counters, s, &fresh);
  if (rc) return rc;
  if (fresh) c->work_base.assign(c->work.cap / sizeof(unsigned long long), 0ull);
  return FT8_OK;
}

int ensure(ft8_ctx* c, DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return FT8_OK;
  if (b.p) {
    (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
  }
  size_t want = bytes + bytes / 4;
  hipError_t e = hipMalloc(&b.p, want);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(c, FT8_E_NOMEM, std::string("hipMalloc failed for ") + std::to_string(want) + " bytes");
  }
  b.cap = want;
  return FT8_OK;
}

hipEvent_t get_event(ft8_ctx* c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}

struct StageTimer {
  ft8_ctx* c;
  int stage;
  hipStream_t s;
  hipEvent_t a = nullptr;
  StageTimer(ft8_ctx* c_, int st, hipStream_t s_) : c(c_), stage(st), s(s_) {
    if (c->timing && ((c->stage_mask >> st) & 1u)) {
      a = get_event(c);
      (void)hipEventRecord(a, s);
    }
  }
  void done() {
    if (c->timing && a) {
      hipEvent_t b = get_event(c);
      (void)hipEventRecord(b, s);
      c->pending.push_back({stage, a, b});
      a = nullptr;
    }
  }
};

// Stream order of a context's work.  The scratch buffers, the k_bp claim counters and their
// host-side ticket bases assume that a context's launches run one after another; an entry point
// that uses them, called on a stream other than the previous such call's, first waits (device side,
// no host sync) for an event recorded after that call's work.  (Entry points that touch no context
// state -- ft8_sync_score, ft8_llr, ft8_normalize, ft8_encode, ft8_pack_decodes, ft8_crc14,
// ft8_ldpc_check -- take no part, so they never serialise two contexts' streams.)  Without it, two streams sharing one context (e.g. one
// host thread alternating torch streams) would run two calls' kernels concurrently on the same
// scratch and interleave the tickets of two k_bp launches.
struct StreamOrder {
  ft8_ctx* c;
  hipStream_t s;
  StreamOrder(ft8_ctx* c_, hipStream_t s_) : c(c_), s(s_) {
    if (!c) return;
    if (c->have_last && c->last_stream != s) (void)hipStreamWaitEvent(s, c->last_done, 0);
  }
  ~StreamOrder() {
    if (!c) return;
    DeviceGuard dg(c->device);  // the event lives on the context's device
    if (!c->last_done && hipEventCreateWithFlags(&c->last_done, hipEventDisableTiming) != hipSuccess) {
      c->last_done = nullptr;
      return;
    }
    if (hipEventRecord(c->last_done, s) == hipSuccess) {
      c->last_stream = s;
      c->have_last = true;
    }
  }
};

// NumPy pairwise summation of a complex64 array with zero imaginary parts (real part returned),
// CFLOAT_pairwise_sum with n counted in floats (loops_utils.h.src)
float cfloat_pairwise_re(const float* re, long n_floats) {
  if (n_floats < 8) {
    float rr = -0.0f;
    for (long i = 0; i < n_floats; i += 2) rr += re[i / 2];
    return rr;
  } else if (n_floats <= 128) {
    float r[4];
    for (int j = 0; j < 4; ++j) r[j] = re[j];
    long i;
    for (i = 8; i < n_floats - (n_floats % 8); i += 8)
      for (int j = 0; j < 4; ++j) r[j] += re[i / 2 + j];
    float rr = (r[0] + r[1]) + (r[2] + r[3]);
    for (; i < n_floats; i += 2) rr += re[i / 2];
    return rr;
  } else {
    long n2 = n_floats / 2;
    n2 -= n2 % 8;
    return cfloat_pairwise_re(re, n2) + cfloat_pairwise_re(re + n2 / 2, n_floats - n2);
  }
}

double double_pairwise(const double* a, long n) {
  if (n < 8) {
    double r = -0.0;
    for (long i = 0; i < n; ++i) r += a[i];
    return r;
  } else if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    long i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  } else {
    long n2 = n / 2;
    n2 -= n2 % 8;
    return double_pairwise(a, n2) + double_pairwise(a + n2, n - n2);
  }
}

// periodic Hann window exactly as scipy.signal.get_window('hann', L) builds it:
// general_cosine(L + 1, [0.5, 0.5]) truncated, fac = linspace(-pi, pi, L + 1)
std::vector<double> hann(int L) {
  std::vector<double> w(L);
  const double start = -M_PI, stop = M_PI;
  const double step = (stop - start) / (double)L;
  for (int i = 0; i < L; ++i) {
    const double fac = (double)i * step + start;
    w[i] = (0.0 + 0.5 * 1.0) + 0.5 * std::cos(fac);
  }
  if (L == 1) w[0] = 1.0;
  return w;
}

int get_window(ft8_ctx* c, int L, bool f64, WinEntry** out) {
  for (auto& w : c->wins)
    if (w.L == L && w.f64 == f64) { *out = &w; return FT8_OK; }
  std::vector<double> w = hann(L);
  WinEntry e;
  e.L = L;
  e.f64 = f64;
  hipError_t he;
  if (f64) {
    double s = 0.0 + double_pairwise(w.data(), L);
    e.scale = 1.0 / (s * s);
    he = hipMalloc(&e.w, sizeof(double) * L);
    if (he == hipSuccess) he = hipMemcpy(e.w, w.data(), sizeof(double) * L, hipMemcpyHostToDevice);
  } else {
    std::vector<float> w32(L);
    for (int i = 0; i < L; ++i) w32[i] = (float)w[i];
    float s = 0.0f + cfloat_pairwise_re(w32.data(), 2L * L);
    float sq = s * s;
    e.scale = (double)(1.0f / sq);
    he = hipMalloc(&e.w, sizeof(float) * L);
    if (he == hipSuccess) he = hipMemcpy(e.w, w32.data(), sizeof(float) * L, hipMemcpyHostToDevice);
  }
  if (he != hipSuccess) return hipfail(c, he, "window upload");
  c->wins.push_back(e);
  *out = &c->wins.back();
  return FT8_OK;
}

bool factor(int P, FftPlan& pl) {
  pl.nstages = 0;
  int r = P;
  auto take = [&](int f) {
    while (r % f == 0 && pl.nstages < 16) {
      pl.radix[pl.nstages++] = f;
      r /= f;
    }
  };
  // few, large register-resident stages: every stage is one LDS round trip
  take(16);
  take(8);
  take(4);
  take(2);
  take(15);
  take(5);
  take(3);
  take(7);
  return r == 1 && pl.nstages > 0;
}

// in-place radix-2 FFT (long double, host) of a power-of-two length: the chirp-z filter spectra
void host_fft_pow2(std::vector<long double>& re, std::vector<long double>& im) {
  const size_t n = re.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) {
      std::swap(re[i], re[j]);
      std::swap(im[i], im[j]);
    }
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    for (size_t k = 0; k < len / 2; ++k) {
      const long double ang = -2.0L * M_PIl * (long double)k / (long double)len;
      const long double wr = cosl(ang), wi = sinl(ang);
      for (size_t i = k; i < n; i += len) {
        const size_t j = i + len / 2;
        const long double xr = re[j] * wr - im[j] * wi, xi = re[j] * wi + im[j] * wr;
        re[j] = re[i] - xr;
        im[j] = im[i] - xi;
        re[i] += xr;
        im[i] += xi;
      }
    }
  }
}

// exp(-i pi j^2 / N) from the exact residue j^2 mod 2N
void chirp_of(int64_t j, int N, long double* cr, long double* ci) {
  const int64_t r = (j * j) % (2 * (int64_t)N);
  const long double ang = -M_PIl * (long double)r / (long double)N;
  *cr = cosl(ang);
  *ci = sinl(ang);
}

// the chirp-z tables of a plan (P = the convolution length, a power of two): chirp c(k), k < nfft,
// and the spectra of the nblk block filters h_b[m] = conj(c(b B + m - (L - 1))), m < P
int blue_tables(ft8_ctx* c, PlanEntry& e, int nfft, int L, int P, bool f64) {
  const int B = P - L + 1;
  const int nblk = (nfft + B - 1) / B;
  const size_t esz = f64 ? 16 : 8;
  std::vector<unsigned char> ch(esz * nfft), hs(esz * (size_t)nblk * P);
  auto put = [&](std::vector<unsigned char>& v, size_t i, long double xr, long double xi) {
    if (f64) { double t[2] = {(double)xr, (double)xi}; memcpy(&v[esz * i], t, 16); }
    else { float t[2] = {(float)xr, (float)xi}; memcpy(&v[esz * i], t, 8); }
  };
  for (int k = 0; k < nfft; ++k) {
    long double cr, ci;
    chirp_of(k, nfft, &cr, &ci);
    put(ch, k, cr, ci);
  }
  std::vector<long double> re(P), im(P);
  for (int b = 0; b < nblk; ++b) {
    for (int m = 0; m < P; ++m) {
      long double cr, ci;
      chirp_of((int64_t)b * B + m - (L - 1), nfft, &cr, &ci);
      re[m] = cr;
      im[m] = -ci;
    }
    host_fft_pow2(re, im);
    for (int m = 0; m < P; ++m) put(hs, (size_t)b * P + m, re[m], im[m]);
  }
  hipError_t he = hipMalloc(&e.chirp, ch.size());
  if (he == hipSuccess) he = hipMalloc(&e.hspec, hs.size());
  if (he == hipSuccess) he = hipMemcpy(e.chirp, ch.data(), ch.size(), hipMemcpyHostToDevice);
  if (he == hipSuccess) he = hipMemcpy(e.hspec, hs.data(), hs.size(), hipMemcpyHostToDevice);
  if (he != hipSuccess) return hipfail(c, he, "chirp-z plan upload");
  e.plan.L = L;
  e.plan.B = B;
  e.plan.nblk = nblk;
  e.plan.chirp = e.chirp;
  e.plan.hspec = e.hspec;
  return FT8_OK;
}

int get_plan(ft8_ctx* c, int nfft, bool cplx, bool f64, int nperseg, FftPlan* out) {
  for (auto& p : c->plans)
    // a fallback plan (chirp-z or direct DFT) was chosen for one nperseg: the choice between the
    // two depends on it, so such a plan is reused only for that nperseg
    if (p.nfft == nfft && p.cplx == cplx && p.f64 == f64 && (!(p.plan.blue || p.plan.dft) || p.L == nperseg)) {
      *out = p.plan;
      return FT8_OK;
    }
  PlanEntry e;
  e.nfft = nfft;
  e.cplx = cplx;
  e.f64 = f64;
  int P = cplx ? nfft : nfft / 2;
  e.plan.dft = 0;
  e.plan.blue = 0;
  // lengths the LDS Stockham FFT cannot take (a prime factor above 7, odd real nfft, above the
  // compiled limit) take the chirp-z transform when its convolution fits the LDS FFT and is the
  // cheaper one, else the direct DFT kernel (P = nfft, tw = W_nfft^m)
  const int max_p = f64 ? kMaxFftP64 : (cplx ? kMaxFftComplex : kMaxFftReal / 2);
  if ((!cplx && (nfft % 2)) || P > max_p || !factor(P, e.plan)) {
    if (nfft > kMaxDft) return fail(c, FT8_E_RANGE, "nfft " + std::to_string(nfft) + " exceeds the compiled DFT limit");
    // chirp-z: P a power of two >= L + (bins needed) - 1, capped at the LDS FFT limit; cost per frame
    // ~ blocks x 2 x 5 P log2 P against the direct DFT's 8 L per kept bin
    const int need = cplx ? nfft : (nfft + 1) / 2;
    const int pmax = f64 ? kMaxBlueP64 : kMaxBlueP32;
    int M = 1;
    while (M < nperseg + need - 1 && M < pmax) M <<= 1;
    int lg = 0;
    while ((1 << lg) < M) ++lg;
    const double blocks = M > nperseg ? std::ceil((double)need / (double)(M - nperseg + 1)) : 0.0;
    const bool blue = M > nperseg && blocks * 10.0 * M * lg < 8.0 * nperseg * need;
    if (blue && factor(M, e.plan)) {
      P = M;
      e.plan.blue = 1;
      e.L = nperseg;
      int rc = blue_tables(c, e, nfft, nperseg, M, f64);
      if (rc) return rc;
    } else {
      P = nfft;
      e.plan.dft = 1;
      e.plan.nstages = 0;
      e.L = nperseg;
    }
  }
  e.plan.P = P;
  // twiddles W_P^m and post-processing W_N^k (N = 2P), from long double angles
  const size_t esz = f64 ? 16 : 8;
  std::vector<unsigned char> tw(esz * P), post(esz * (P + 1));
  for (int m = 0; m < P; ++m) {
    const long double ang = -2.0L * M_PIl * (long double)m / (long double)P;
    const double cr = (double)cosl(ang), ci = (double)sinl(ang);
    if (f64) { double v[2] = {cr, ci}; memcpy(&tw[esz * m], v, 16); }
    else { float v[2] = {(float)cr, (float)ci}; memcpy(&tw[esz * m], v, 8); }
  }
  for (int k = 0; k <= P; ++k) {
    const long double ang = -2.0L * M_PIl * (long double)k / (long double)(2 * P);
    const double cr = (double)cosl(ang), ci = (double)sinl(ang);
    if (f64) { double v[2] = {cr, ci}; memcpy(&post[esz * k], v, 16); }
    else { float v[2] = {(float)cr, (float)ci}; memcpy(&post[esz * k], v, 8); }
  }
  hipError_t he = hipMalloc(&e.tw, tw.size());
  if (he == hipSuccess) he = hipMalloc(&e.post, post.size());
  if (he == hipSuccess) he = hipMemcpy(e.tw, tw.data(), tw.size(), hipMemcpyHostToDevice);
  if (he == hipSuccess) he = hipMemcpy(e.post, post.data(), post.size(), hipMemcpyHostToDevice);
  if (he != hipSuccess) return hipfail(c, he, "fft plan upload");
  e.plan.tw = e.tw;
  e.plan.post = e.post;
  c->plans.push_back(e);
  *out = e.plan;
  return FT8_OK;
}

struct Geo {
  int nperseg, hop, noverlap, nfft, frames;
};

// the sample rate a parameter block names: the exact Hz when given (ABI 2), else the integral field
double rate_of(const ft8_params* p) { return p->sample_rate_hz > 0.0 ? p->sample_rate_hz : (double)p->sample_rate; }

// fs in double: the reference computes both lengths on the float it was given (a float fs such as
// 10e3 or 12006.3 is legal there), so int(0.16 * 12006.3) = 1921, not int(0.16 * 12006) = 1920
int geometry(double fs, int bpt, int sps, int64_t n, Geo* g, std::string* why) {
  if (!(fs > 0.0) || !(fs < 2e9) || bpt <= 0 || sps <= 0) { *why = "sample_rate, bins_per_tone and steps_per_symbol must be positive"; return FT8_E_ARG; }
  g->nperseg = (int)(0.16 * fs);                         // spectrogram_analyse.py:32
  g->noverlap = g->nperseg - g->nperseg / sps;           // :33
  g->nfft = (int)(fs / 6.25 * (double)bpt);              // :34
  if (g->noverlap >= g->nperseg) g->noverlap = g->nperseg - 1;  // :42-43
  g->hop = g->nperseg - g->noverlap;
  if (g->nperseg < 1) { *why = "nperseg must be a positive integer"; return FT8_E_ARG; }
  if (g->nfft < g->nperseg) { *why = "nfft must be greater than or equal to nperseg."; return FT8_E_ARG; }
  g->frames = (n < g->nperseg) ? 0 : (int)((n - g->noverlap) / g->hop);
  return FT8_OK;
}

bool is_f64_dtype(int dt) { return dt == FT8_F64 || dt == FT8_C128; }
bool is_cplx_dtype(int dt) { return dt == FT8_C64 || dt == FT8_C128; }

int do_stft(ft8_ctx* c, const void* samples, int dtype, int64_t n_samples, int n_slots, int64_t slot_stride,
            const ft8_params* p, void* d_wf, hipStream_t s) {
  Geo g;
  std::string why;
  int rc = geometry(rate_of(p), p->bins_per_tone, p->steps_per_symbol, n_samples, &g, &why);
  if (rc) return fail(c, rc, why);
  if (dtype < FT8_F32 || dtype > FT8_I16) return fail(c, FT8_E_ARG, "unknown sample dtype");
  if (p->t_lo < 0 || p->t_hi > g.frames || p->t_lo > p->t_hi)
    return fail(c, FT8_E_ARG, "frame range [t_lo, t_hi) outside [0, " + std::to_string(g.frames) + ")");
  if (p->f_lo < 0 || p->f_hi > g.nfft || p->f_lo > p->f_hi)
    return fail(c, FT8_E_ARG, "bin range [f_lo, f_hi) outside [0, nfft)");
  if (p->t_hi == p->t_lo || p->f_hi == p->f_lo || n_slots == 0) return FT8_OK;
  const bool f64 = is_f64_dtype(dtype), cplx = is_cplx_dtype(dtype);
  StftLaunch L{};
  rc = get_plan(c, g.nfft, cplx, f64, g.nperseg, &L.plan);
  if (rc) return rc;
  if (L.plan.dft && (size_t)g.nperseg * (f64 ? 16 : 8) > (size_t)kMaxDftLds)
    return fail(c, FT8_E_RANGE, "nperseg " + std::to_string(g.nperseg) + " exceeds the direct-DFT limit");
  WinEntry* w = nullptr;
  rc = get_window(c, g.nperseg, f64, &w);
  if (rc) return rc;
  L.samples = samples;
  L.dtype = dtype;
  L.n_samples = n_samples;
  L.slot_stride = slot_stride;
  L.n_slots = n_slots;
  L.nperseg = g.nperseg;
  L.hop = g.hop;
  L.nfft = g.nfft;
  L.t_lo = p->t_lo;
  L.t_hi = p->t_hi;
  L.f_lo = p->f_lo;
  L.f_hi = p->f_hi;
  L.window = w->w;
  L.scale = w->scale;
  L.out = d_wf;
  c->last_stft = L;
  StageTimer tm(c, 0, s);
  hipError_t e = launch_stft(L, s);
  tm.done();
  if (e != hipSuccess) return hipfail(c, e, "stft launch");
  return FT8_OK;
}

struct Grid {
  int t0, NT, NF;
};
Grid grid_of(int T, int F, int sps, int bpt) {
  // ft8_find_candidates ranges (ft8_decode.py:108-109)
  Grid g;
  const int nb = T / sps;
  g.t0 = -10 * sps;
  const int t_end = nb * sps - sps * 59;
  g.NT = t_end > g.t0 ? t_end - g.t0 : 0;
  g.NF = F - 7 * bpt > 0 ? F - 7 * bpt : 0;
  return g;
}
// score scratch per slot: elements (the full grid NT x NF, or the compact layout NT x nseg x 128)
// and segment-mask words
size_t score_elems(const Grid& g) { return (size_t)g.NT * n_segments(g.NF) * kSegCols; }
size_t smask_words(const Grid& g) { return (size_t)g.NT * n_segments(g.NF) * 2; }

int decode_pass(ft8_ctx* c, const void* d_samples, int dtype, int64_t n_samples, int32_t n_slots,
                int64_t slot_stride, const ft8_params* p, ft8_result* d_out, int32_t* d_counts, int32_t cap,
                hipStream_t s);
int subtract_core(ft8_ctx* c, const void* x, int dtype, float* resid, int64_t n_samples, int n_slots,
                  int64_t x_stride, int64_t r_stride, const ft8_params* p, const ft8_result* res,
                  const int32_t* counts, int cap, hipStream_t s);
int gfsk_tables(ft8_ctx* c, int nsps);
int sync_select_core(ft8_ctx* c, const void* d_wf, int wf_f64, int n_slots, int T, int F, const ft8_params* p,
                     int32_t* cand, double* cand_score, int32_t* cand_count, void* scores, uint64_t* smask,
                     int compact, int32_t* warn, RowSummary* rowsum, hipStream_t s, int32_t* tie = nullptr);

int do_sync_select(ft8_ctx* c, const void* d_wf, int wf_f64, int n_slots, int T, int F, const ft8_params* p,
                   int32_t* cand, double* cand_score, int32_t* cand_count, void* d_scores, hipStream_t s) {
  if (p->steps_per_symbol <= 0 || p->bins_per_tone <= 0) return fail(c, FT8_E_ARG, "bad oversampling factors");
  if (p->flags & ~(FT8_FLAG_TOPK | FT8_FLAG_SUBTRACT)) return fail(c, FT8_E_ARG, "unknown bits in ft8_params.flags");
  const int N = p->max_candidates;
  if (N > kMaxCandidates)
    return fail(c, FT8_E_RANGE, "max_candidates > " + std::to_string(kMaxCandidates) + " is not supported");
  Grid g = grid_of(T, F, p->steps_per_symbol, p->bins_per_tone);
  if (N <= 0 || g.NT == 0 || g.NF == 0 || n_slots == 0) {
    hipError_t e = hipMemsetAsync(cand_count, 0, sizeof(int32_t) * (size_t)(n_slots > 0 ? n_slots : 0), s);
    return e == hipSuccess ? FT8_OK : hipfail(c, e, "memset");
  }
  const size_t esz = wf_f64 ? 8 : 4;
  int rc;
  // without a caller grid the scores stay in the compact layout (only passing scores written)
  void* scores = d_scores;
  if (!scores) {
    if ((rc = ensure(c, c->scores, esz * (size_t)n_slots * score_elems(g)))) return rc;
    scores = c->scores.p;
  }
  if ((rc = ensure(c, c->smask, sizeof(uint64_t) * (size_t)n_slots * smask_words(g)))) return rc;
  if ((rc = ensure(c, c->warn, sizeof(int32_t) * (size_t)n_slots))) return rc;
  if ((rc = ensure(c, c->rowsum, sizeof(RowSummary) * (size_t)n_slots * g.NT * n_segments(g.NF)))) return rc;
  // float32 scores: k_select leaves equal scores in scan order and k_tie_apply replays the
  // reference heap for the slots that have them (the same code k_llr runs inside decode_batch)
  int32_t* tie = nullptr;
  if (!wf_f64) {
    if ((rc = ensure(c, c->tie, sizeof(int32_t) * (size_t)n_slots * tie_stride(N)))) return rc;
    tie = (int32_t*)c->tie.p;
  }
  int32_t* warn = (int32_t*)c->warn.p;
  if ((rc = sync_select_core(c, d_wf, wf_f64, n_slots, T, F, p, cand, cand_score, cand_count, scores,
                             (uint64_t*)c->smask.p, d_scores == nullptr, warn, (RowSummary*)c->rowsum.p, s, tie)))
    return rc;
  if (tie) {
    const TieArgs ta{n_slots, N, cand_count, warn, tie, cand_score};
    hipError_t e = launch_tie_apply(ta, cand, cand_score, s);
    if (e != hipSuccess) return hipfail(c, e, "tie launch");
  }
  return FT8_OK;
}

// score + select on caller-provided scratch (scores [n_slots][score_elems], smask
// [n_slots][smask_words], warn [n_slots], rowsum [n_slots][NT][nseg]); compact: the score kernel may
// write only the passing scores (k_score2 path, reference selection), else the full grid
int sync_select_core(ft8_ctx* c, const void* d_wf, int wf_f64, int n_slots, int T, int F, const ft8_params* p,
                     int32_t* cand, double* cand_score, int32_t* cand_count, void* scores, uint64_t* smask,
                     int compact, int32_t* warn, RowSummary* rowsum, hipStream_t s, int32_t* tie) {
  const int N = p->max_candidates;
  Grid g = grid_of(T, F, p->steps_per_symbol, p->bins_per_tone);
  SyncLaunch L{};
  L.wf = d_wf;
  L.wf_f64 = wf_f64;
  L.n_slots = n_slots;
  L.T = T;
  L.F = F;
  L.sps = p->steps_per_symbol;
  L.bpt = p->bins_per_tone;
  L.t0 = g.t0;
  L.NT = g.NT;
  L.NF = g.NF;
  L.scores = scores;
  L.smask = smask;
  L.compact = compact;
  L.N = N;
  L.min_score = p->min_score;
  L.min_score_f64 = p->min_score_f64;
  L.cand = cand;
  L.cand_score = cand_score;
  L.cand_count = cand_count;
  L.warn = warn;
  L.rowsum = rowsum;
  L.tie = tie;
  L.topk = (p->flags & FT8_FLAG_TOPK) ? 1 : 0;
  c->last_sync = L;
  StageTimer t1(c, 1, s);
  hipError_t e = launch_score(L, s);
  t1.done();
  if (e != hipSuccess) return hipfail(c, e, "score launch");
  StageTimer t2(c, 2, s);
  e = launch_select(L, s);
  t2.done();
  if (e != hipSuccess) return hipfail(c, e, "select launch");
  return FT8_OK;
}

int decode_pass(ft8_ctx* c, const void* d_samples, int dtype, int64_t n_samples, int32_t n_slots,
                int64_t slot_stride, const ft8_params* p, ft8_result* d_out, int32_t* d_counts, int32_t cap,
                hipStream_t s) {
  const int T = p->t_hi - p->t_lo, F = p->f_hi - p->f_lo;
  const bool f64 = is_f64_dtype(dtype);
  const size_t esz = f64 ? 8 : 4;
  const int N = p->max_candidates;
  Grid gr = grid_of(T, F, p->steps_per_symbol, p->bins_per_tone);
  int rc;

  // slot chunks, each an independent STFT -> score/select -> LLR -> BP -> compact chain; chunks
  // alternate over the internal streams so one chunk's BP (FP64 VALU) overlaps the next chunk's
  // STFT / score (LDS, HBM)
  const int csz = (c->n_streams > 0 && c->chunk_slots > 0) ? c->chunk_slots : n_slots;
  const int n_chunks = (n_slots + csz - 1) / csz;
  const int n_str = (c->n_streams > 0 && n_chunks > 1) ? std::min(c->n_streams, n_chunks) : 0;
  // k_bp claim counters: [0] belongs to ft8_bp (a caller stream), [1 + k] to chunk k
  if ((rc = ensure_work(c, n_chunks + 1, s))) return rc;
  hipError_t e = hipSuccess;
  if (n_str > 0) {
    while ((int)c->streams.size() < n_str) {
      hipStream_t st;
      if ((e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) != hipSuccess) return hipfail(c, e, "stream");
      c->streams.push_back(st);
      hipEvent_t ev;
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return hipfail(c, e, "event");
      c->joins.push_back(ev);
    }
    if (!c->fork && (e = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming)) != hipSuccess)
      return hipfail(c, e, "event");
    if ((e = hipEventRecord(c->fork, s)) != hipSuccess) return hipfail(c, e, "fork");
    for (int i = 0; i < n_str; ++i)
      if ((e = hipStreamWaitEvent(c->streams[i], c->fork, 0)) != hipSuccess) return hipfail(c, e, "fork wait");
  }
  const size_t in_esz = dtype == FT8_I16 ? 2 : dtype == FT8_F32 ? 4 : (dtype == FT8_F64 || dtype == FT8_C64) ? 8 : 16;
  for (int k = 0; k < n_chunks; ++k) {
    const int c0 = k * csz, ns = std::min(csz, n_slots - c0);
    hipStream_t cs = n_str > 0 ? c->streams[k % n_str] : s;
    char* wf = (char*)c->wf.p + esz * (size_t)c0 * T * F;
    const char* xs = (const char*)d_samples + in_esz * (size_t)c0 * slot_stride;
    if ((rc = do_stft(c, xs, dtype, n_samples, ns, slot_stride, p, wf, cs))) return rc;
    int32_t* cand = (int32_t*)c->cand.p + 2 * (size_t)c0 * N;
    double* cand_score = (double*)c->cand_score.p + (size_t)c0 * N;
    int32_t* cand_count = (int32_t*)c->cand_count.p + c0;
    // float32 scores: equal scores keep the select order through LLR/BP and are reordered by
    // k_compact after k_llr's first workgroups replayed the reference heap
    int32_t* tie = f64 ? nullptr : (int32_t*)c->tie.p + (size_t)c0 * tie_stride(N);
    int32_t* warn = (int32_t*)c->warn.p + c0;
    if ((rc = sync_select_core(c, wf, f64, ns, T, F, p, cand, cand_score, cand_count,
                               (char*)c->scores.p + esz * (size_t)c0 * score_elems(gr),
                               (uint64_t*)c->smask.p + (size_t)c0 * smask_words(gr), 1, (int32_t*)c->warn.p + c0,
                               (RowSummary*)c->rowsum.p + (size_t)c0 * gr.NT * n_segments(gr.NF), cs, tie)))
      return rc;
    BpLaunch B{};
    B.wf = wf;
    B.wf_f64 = f64;
    B.T = T;
    B.F = F;
    B.sps = p->steps_per_symbol;
    B.bpt = p->bins_per_tone;
    B.cand = cand;
    B.cand_score = cand_score;
    B.cand_count = cand_count;
    B.N = N;
    B.n_slots = ns;
    B.slot0 = c0;
    B.n_items = ns * N;
    B.mode = 0;
    B.normalize = 1;
    B.max_iterations = p->max_iterations;
    B.llr_out = (double*)c->llr.p + (size_t)FT8_LDPC_N * c0 * N;
    B.llr_in = B.llr_out;
    B.res = (ft8_result*)c->res_all.p + (size_t)c0 * N;
    B.work = (unsigned long long*)c->work.p + 1 + k;
    B.work_base = &c->work_base[1 + k];
    B.stats = (unsigned long long*)c->stats.p;
    B.clock = c->timing && c->stats.p ? (unsigned long long*)c->stats.p + 4 : nullptr;
    B.grid_waves = c->bp_waves;  // resident waves per SIMD of the persistent grid (kernel maximum 4)
    B.tie = tie;
    B.warn = warn;
    StageTimer t6(c, 6, cs);
    e = launch_llr(B, cs);
    t6.done();
    if (e != hipSuccess) return hipfail(c, e, "llr launch");
    StageTimer t3(c, 3, cs);
    e = launch_bp(B, cs);
    t3.done();
    if (e != hipSuccess) return hipfail(c, e, "bp launch");
    CompactLaunch C{};
    C.res = B.res;
    C.cand_count = cand_count;
    C.n_slots = ns;
    C.N = N;
    C.out = d_out ? d_out + (size_t)c0 * cap : nullptr;
    C.counts = d_counts + c0;
    C.cap = cap;
    C.warn = warn;
    C.tie = tie;
    c->last_bp = B;
    c->last_compact = C;
    StageTimer t4(c, 4, cs);
    e = launch_compact(C, cs);
    t4.done();
    if (e != hipSuccess) return hipfail(c, e, "compact launch");
  }
  for (int i = 0; i < n_str; ++i) {
    if ((e = hipEventRecord(c->joins[i], c->streams[i])) != hipSuccess) return hipfail(c, e, "join");
    if ((e = hipStreamWaitEvent(s, c->joins[i], 0)) != hipSuccess) return hipfail(c, e, "join wait");
  }
  c->replay_ok = n_chunks == 1;
  return FT8_OK;
}

// cumulative GFSK frequency pulse P[0 .. 3 nsps] of the transmit chain (tx_device.h), double and
// float, built once per nsps: p(i) = gauss_window_generator(2.0, (i - 1.5 nsps) / nsps)
// (modulator.py:20-25, 33-34), P[i + 1] = P[i] + p(i)
int gfsk_tables(ft8_ctx* c, int nsps) {
  if (c->gfsk_nsps == nsps && c->gfsk_P.p) return FT8_OK;
  const int n = 3 * nsps + 1;
  int rc;
  if ((rc = ensure(c, c->gfsk_P, sizeof(double) * n))) return rc;
  if ((rc = ensure(c, c->gfsk_Pf, sizeof(float) * n))) return rc;
  std::vector<double> P(n);
  std::vector<float> Pf(n);
  const double k = M_PI * std::sqrt(2.0 / std::log(2.0)), bt = 2.0;
  P[0] = 0.0;
  for (int i = 0; i < 3 * nsps; ++i) {
    const double t = ((double)i - 1.5 * (double)nsps) / (double)nsps;
    const double w = 0.5 * (std::erf(k * bt * (t + 0.5)) - std::erf(k * bt * (t - 0.5)));
    P[i + 1] = P[i] + w;
  }
  for (int i = 0; i < n; ++i) Pf[i] = (float)P[i];
  hipError_t e = hipMemcpy(c->gfsk_P.p, P.data(), sizeof(double) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->gfsk_Pf.p, Pf.data(), sizeof(float) * n, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hipfail(c, e, "gfsk table upload");
  c->gfsk_nsps = nsps;
  return FT8_OK;
}

// decimated samples per symbol of the subtraction's fine sync: 32 when nsps allows, else the
// largest divisor of nsps in [8, 32]
int sub_q(int nsps) {
  for (int q = 32; q >= 8; --q)
    if (nsps % q == 0) return q;
  return 0;
}

int subtract_core(ft8_ctx* c, const void* x, int dtype, float* resid, int64_t n_samples, int n_slots,
                  int64_t x_stride, int64_t r_stride, const ft8_params* p, const ft8_result* res,
                  const int32_t* counts, int cap, hipStream_t s) {
  Geo g;
  std::string why;
  int rc = geometry(rate_of(p), p->bins_per_tone, p->steps_per_symbol, n_samples, &g, &why);
  if (rc) return fail(c, rc, why);
  if (dtype != FT8_F32 && dtype != FT8_I16) return fail(c, FT8_E_UNSUPPORTED, "subtraction needs float32 or int16 samples");
  if (x_stride != r_stride) return fail(c, FT8_E_ARG, "residual and sample strides differ");
  c->sub_slots = c->sub_cap = -1;  // no valid fits until this subtraction has been launched
  const int Q = sub_q(g.nperseg);
  if (Q == 0 || g.nperseg % g.hop != 0)
    return fail(c, FT8_E_UNSUPPORTED, "subtraction needs nsps with a divisor in [8, 32] and hop | nsps");
  if ((rc = gfsk_tables(c, g.nperseg))) return rc;
  if ((rc = ensure(c, c->sub_est, sub_est_bytes() * (size_t)n_slots * (size_t)(cap > 0 ? cap : 1)))) return rc;
  if ((rc = ensure(c, c->sub_list, sizeof(int32_t) * (size_t)n_slots * (size_t)(cap + 1)))) return rc;
  SubLaunch L{};
  L.x = x;
  L.dtype = dtype;
  L.residual = resid;
  L.n_samples = n_samples;
  L.slot_stride = x_stride;
  L.n_slots = n_slots;
  L.fs = rate_of(p);
  L.nsps = g.nperseg;
  L.hop = g.hop;
  L.nfft = g.nfft;
  L.t_lo = p->t_lo;
  L.f_lo = p->f_lo;
  L.res = res;
  L.counts = counts;
  L.cap = cap;
  L.P = (const double*)c->gfsk_P.p;
  L.Pf = (const float*)c->gfsk_Pf.p;
  L.est = c->sub_est.p;
  L.list = (int32_t*)c->sub_list.p;
  L.Q = Q;
  StageTimer tm(c, 7, s);
  hipError_t e = launch_sub_est(L, s);
  tm.done();
  if (e != hipSuccess) return hipfail(c, e, "subtract launch");
  StageTimer tm2(c, 11, s);
  e = launch_sub_apply(L, s);
  tm2.done();
  if (e != hipSuccess) return hipfail(c, e, "subtract launch");
  c->sub_slots = n_slots;
  c->sub_cap = cap;
  return FT8_OK;
}

// ---- frequency-drift correction ----------------------------------------------------------------
// kept f >= 0 bins of a two-sided spectrum after fftshift (frequency_correction.py:198-200)
int drift_bins(int nfft) { return (nfft + 1) / 2; }

int stft_argmax_core(ft8_ctx* c, const void* x, int dtype, int64_t n_samples, int n_slots, int64_t stride,
                     const ft8_params* p, int32_t* idx, hipStream_t s) {
  Geo g;
  std::string why;
  int rc = geometry(rate_of(p), p->bins_per_tone, p->steps_per_symbol, n_samples, &g, &why);
  if (rc) return fail(c, rc, why);
  if (dtype < FT8_F32 || dtype > FT8_I16) return fail(c, FT8_E_ARG, "unknown sample dtype");
  if (p->t_lo < 0 || p->t_hi > g.frames || p->t_lo > p->t_hi)
    return fail(c, FT8_E_ARG, "frame range [t_lo, t_hi) outside [0, " + std::to_string(g.frames) + ")");
  if (p->f_lo < 0 || p->f_hi > g.nfft || p->f_lo >= p->f_hi) return fail(c, FT8_E_ARG, "bin range [f_lo, f_hi) empty or outside [0, nfft)");
  if (p->t_hi == p->t_lo || n_slots == 0) return FT8_OK;
  const bool f64 = is_f64_dtype(dtype), cplx = is_cplx_dtype(dtype);
  StftLaunch L{};
  if ((rc = get_plan(c, g.nfft, cplx, f64, g.nperseg, &L.plan))) return rc;
  if (L.plan.dft || L.plan.blue) {
    // the direct DFT and the chirp-z path write the dB rows, then reduce each to its argmax: stage
    // them in wf
    if (L.plan.dft && (size_t)g.nperseg * (f64 ? 16 : 8) > (size_t)kMaxDftLds)
      return fail(c, FT8_E_RANGE, "nperseg " + std::to_string(g.nperseg) + " exceeds the direct-DFT limit");
    const size_t bytes = (size_t)n_slots * (p->t_hi - p->t_lo) * (p->f_hi - p->f_lo) * (f64 ? 8 : 4);
    if ((rc = ensure(c, c->wf, bytes))) return rc;
    L.out = c->wf.p;
  }
  WinEntry* w = nullptr;
  if ((rc = get_window(c, g.nperseg, f64, &w))) return rc;
  L.samples = x;
  L.dtype = dtype;
  L.n_samples = n_samples;
  L.slot_stride = stride;
  L.n_slots = n_slots;
  L.nperseg = g.nperseg;
  L.hop = g.hop;
  L.nfft = g.nfft;
  L.t_lo = p->t_lo;
  L.t_hi = p->t_hi;
  L.f_lo = p->f_lo;
  L.f_hi = p->f_hi;
  L.window = w->w;
  L.scale = w->scale;
  L.argmax = idx;
  // the geometries launch_stft sends to k_stftc3840 (stft.hip)
  if (dtype == FT8_C128 && !L.plan.dft && !L.plan.blue && g.nfft == 3840 && g.nperseg == 1920 &&
      (g.hop == 240 || g.hop == 480 || g.hop == 960 || g.hop == 1920)) {
    const size_t frames = (size_t)n_slots * (size_t)(p->t_hi - p->t_lo);
    if ((rc = ensure(c, c->screen, sizeof(int32_t) * (frames + 1)))) return rc;
    L.screen_count = (int32_t*)c->screen.p;
    L.screen_list = L.screen_count + 1;
    // the screening pass transforms in float32: its own twiddles and window
    FftPlan fp;
    if ((rc = get_plan(c, g.nfft, true, false, g.nperseg, &fp))) return rc;
    WinEntry* wf32 = nullptr;
    if ((rc = get_window(c, g.nperseg, false, &wf32))) return rc;
    if (fp.P != 3840 || fp.dft || fp.blue) return fail(c, FT8_E_UNSUPPORTED, "float32 screening plan");
    L.screen_tw = fp.tw;
    L.screen_window = wf32->w;
    c->screen_frames = (int64_t)frames;
  } else {
    c->screen_frames = 0;
  }
  StageTimer tm(c, 8, s);
  hipError_t e = launch_stft(L, s);
  tm.done();
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "stft argmax launch");
}

int check_drift_params(ft8_ctx* c, const ft8_drift_params* p) {
  if (p->bins_per_tone <= 0 || p->steps_per_symbol <= 0) return fail(c, FT8_E_ARG, "bins_per_tone and steps_per_symbol must be positive");
  if (p->sample_rate <= 0 || p->sample_rate != std::floor(p->sample_rate) || p->sample_rate > 2e9)
    return fail(c, FT8_E_UNSUPPORTED, "sample_rate must be a positive integral number of Hz");
  const int w = p->window_size_factor * p->steps_per_symbol;
  if (w < 1) return fail(c, FT8_E_ARG, "window_size_factor * steps_per_symbol must be >= 1");
  if (w > kDriftMaxWindow) return fail(c, FT8_E_RANGE, "continuity window exceeds " + std::to_string(kDriftMaxWindow));
  if (p->nsync_sym < 1 || p->nsync_sym > 7) return fail(c, FT8_E_ARG, "nsync_sym must be in [1, 7] (the Costas array has 7 tones)");
  if (p->ndata_sym < 0) return fail(c, FT8_E_ARG, "ndata_sym must be >= 0");
  if (3 * (p->nsync_sym - 1) * p->steps_per_symbol > drift_max_points())
    return fail(c, FT8_E_RANGE, "sync regression points exceed the compiled limit");
  return FT8_OK;
}

// three_sync_correlation_seq (frequency_correction.py:386-407), NumPy's operation order
int drift_template(ft8_ctx* c, const ft8_drift_params* p) {
  const int tosr = p->steps_per_symbol, ns = p->nsync_sym, nd = p->ndata_sym;
  if (c->tmpl_len > 0 && c->tmpl_key[0] == tosr && c->tmpl_key[1] == ns && c->tmpl_key[2] == nd) return FT8_OK;
  const int sps2 = 2 * tosr;
  static const int costas[7] = {3, 1, 4, 0, 6, 5, 2};
  double seq[7];
  for (int k = 0; k < 7; ++k) seq[k] = (double)(costas[k] + 1) - 4.0;  // - np.mean(...) = 4.0 exactly
  // t = np.linspace(-1, 1, sps2 + 1); gfsk_shape = gfsk_pulse(2.0, t)  (:27-40)
  const double step = 2.0 / (double)sps2;
  const double kk = M_PI * std::sqrt(2.0 / std::log(2.0));
  const double kb = kk * 2.0;
  std::vector<double> shape(sps2 + 1);
  for (int j = 0; j <= sps2; ++j) {
    const double t = j == sps2 ? 1.0 : (double)j * step + -1.0;
    shape[j] = 0.5 * (std::erf(kb * (t + 0.5)) - std::erf(kb * (t - 0.5)));
  }
  const int L1 = (ns - 1) * tosr + sps2 + 1;
  std::vector<double> one(L1, 0.0);
  for (int k = 0; k < ns; ++k)
    for (int j = 0; j <= sps2; ++j) one[k * tosr + j] += shape[j] * seq[k];
  const int L3 = (3 * ns + nd - 1) * tosr + 1 + sps2;
  if (L3 > drift_max_template()) return fail(c, FT8_E_RANGE, "sync template exceeds the compiled limit");
  std::vector<double> three(L3, 0.0);
  for (int i = 0; i < 3; ++i) {
    const int s0 = i * (ns + nd / 2) * tosr;
    if (s0 + L1 > L3) return fail(c, FT8_E_ARG, "sync blocks do not fit the template (the reference raises ValueError)");
    for (int j = 0; j < L1; ++j) three[s0 + j] = one[j];
  }
  int rc = ensure(c, c->drift_tmpl, sizeof(double) * L3);
  if (rc) return rc;
  hipError_t e = hipMemcpy(c->drift_tmpl.p, three.data(), sizeof(double) * L3, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hipfail(c, e, "template upload");
  c->tmpl_key[0] = tosr;
  c->tmpl_key[1] = ns;
  c->tmpl_key[2] = nd;
  c->tmpl_len = L3;
  return FT8_OK;
}

int drift_fit_core(ft8_ctx* c, int stage, const int32_t* idx, int n_slots, int T, int F, const ft8_drift_params* p,
                   ft8_drift_result* res, double* metric, int32_t* segments, int max_segments, hipStream_t s) {
  int rc = check_drift_params(c, p);
  if (rc) return rc;
  if (T > kDriftMaxT) return fail(c, FT8_E_RANGE, "more than " + std::to_string(kDriftMaxT) + " frames per signal");
  if (F < 1 || F > 8192) return fail(c, FT8_E_RANGE, "freq_bins must be in [1, 8192]");
  DriftFitLaunch L{};
  L.idx = idx;
  L.n_slots = n_slots;
  L.T = T;
  L.F = F;
  L.p = *p;
  L.res = res;
  L.metric = metric;
  L.segments = segments;
  L.max_segments = segments ? max_segments : 0;
  if (stage == 2) {
    if ((rc = drift_template(c, p))) return rc;
    L.tmpl = (const double*)c->drift_tmpl.p;
    L.n_tmpl = c->tmpl_len;
  }
  StageTimer tm(c, 9, s);
  hipError_t e = launch_drift_fit(stage, L, s);
  tm.done();
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "drift fit launch");
}

}  // namespace

// ============================================================================================
extern "C" {

int ft8_abi_version(void) { return FT8HIP_ABI_VERSION; }

int ft8_limits(int32_t* max_candidates, int32_t* max_fft_real, int32_t* max_fft_complex) {
  if (max_candidates) *max_candidates = kMaxCandidates;
  if (max_fft_real) *max_fft_real = kMaxFftReal;
  if (max_fft_complex) *max_fft_complex = kMaxFftComplex;
  return FT8_OK;
}

int ft8_create(int device, ft8_ctx** out) {
  if (!out) return FT8_E_ARG;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return FT8_E_HIP;
  if (device < 0 || device >= n) return FT8_E_ARG;
  ft8_ctx* c = new (std::nothrow) ft8_ctx();
  if (!c) return FT8_E_NOMEM;
  c->device = device;
  *out = c;
  return FT8_OK;
}

int ft8_destroy(ft8_ctx* c) {
  if (!c) return FT8_OK;
  {
    DeviceGuard dg(c->device);
    for (auto* b : {&c->wf, &c->scores, &c->smask, &c->cand, &c->cand_score, &c->cand_count, &c->warn, &c->rowsum,
                    &c->res_all, &c->work, &c->stats, &c->llr, &c->tie, &c->residual, &c->sub_est, &c->sub_list, &c->screen, &c->out1,
                    &c->counts1, &c->out2, &c->counts2, &c->gfsk_P, &c->gfsk_Pf, &c->drift_idx, &c->drift_tmpl})
      if (b->p) (void)hipFree(b->p);
    for (auto& p : c->plans) {
      if (p.tw) (void)hipFree(p.tw);
      if (p.post) (void)hipFree(p.post);
      if (p.chirp) (void)hipFree(p.chirp);
      if (p.hspec) (void)hipFree(p.hspec);
    }
    for (auto& w : c->wins)
      if (w.w) (void)hipFree(w.w);
    for (auto& t : c->pending) {
      (void)hipEventDestroy(t.a);
      (void)hipEventDestroy(t.b);
    }
    for (auto ev : c->pool) (void)hipEventDestroy(ev);
    for (auto st : c->streams) (void)hipStreamDestroy(st);
    for (auto ev : c->joins) (void)hipEventDestroy(ev);
    if (c->fork) (void)hipEventDestroy(c->fork);
    if (c->last_done) (void)hipEventDestroy(c->last_done);
  }
  delete c;
  return FT8_OK;
}

const char* ft8_last_error(const ft8_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ft8_geometry(int32_t fs, int32_t bpt, int32_t sps, int64_t n, int32_t* nperseg, int32_t* hop, int32_t* nfft,
                 int32_t* frames) {
  return ft8_geometry_hz((double)fs, bpt, sps, n, nperseg, hop, nfft, frames);
}

int ft8_geometry_hz(double fs, int32_t bpt, int32_t sps, int64_t n, int32_t* nperseg, int32_t* hop, int32_t* nfft,
                    int32_t* frames) {
  Geo g;
  std::string why;
  int rc = geometry(fs, bpt, sps, n, &g, &why);
  if (rc) return rc;
  if (nperseg) *nperseg = g.nperseg;
  if (hop) *hop = g.hop;
  if (nfft) *nfft = g.nfft;
  if (frames) *frames = g.frames;
  return FT8_OK;
}

int ft8_stft(ft8_ctx* c, const void* d_samples, int dtype, int64_t n_samples, int32_t n_slots, int64_t slot_stride,
             const ft8_params* p, void* d_wf, void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (c) c->replay_ok = false;
  if (!c || !p || (!d_samples && n_slots > 0) || (!d_wf && n_slots > 0)) return fail(c, FT8_E_ARG, "null argument");
  DeviceGuard dg(c->device);
  return do_stft(c, d_samples, dtype, n_samples, n_slots, slot_stride, p, d_wf, (hipStream_t)stream);
}

int ft8_stft_screen_stats(ft8_ctx* c, int64_t* frames_redone, int64_t* frames) {
  if (!c || !frames_redone || !frames) return fail(c, FT8_E_ARG, "null argument");
  *frames_redone = 0;
  *frames = c->screen_frames;
  if (c->screen_frames == 0) return FT8_OK;
  DeviceGuard dg(c->device);
  int32_t n = 0;
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(&n, c->screen.p, sizeof(int32_t), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hipfail(c, e, "screen count");
  *frames_redone = n;
  return FT8_OK;
}

int ft8_stft_method(ft8_ctx* c, int32_t fs, int32_t bpt, int32_t sps, int64_t n, int dtype) {
  if (!c) return FT8_E_ARG;
  if (dtype < FT8_F32 || dtype > FT8_I16) return fail(c, FT8_E_ARG, "unknown sample dtype");
  Geo g;
  std::string why;
  int rc = geometry(fs, bpt, sps, n, &g, &why);
  if (rc) return fail(c, rc, why);
  DeviceGuard dg(c->device);
  StftLaunch L{};
  if ((rc = get_plan(c, g.nfft, is_cplx_dtype(dtype), is_f64_dtype(dtype), g.nperseg, &L.plan))) return rc;
  if (L.plan.blue) return FT8_STFT_CHIRPZ;
  if (L.plan.dft) return FT8_STFT_DFT;
  L.dtype = dtype;
  L.nfft = g.nfft;
  L.nperseg = g.nperseg;
  L.hop = g.hop;
  L.slot_stride = 2;  // the packed kernel's only stride condition (even) is the caller's
  return stft3840_eligible(L) ? FT8_STFT_PACKED3840 : FT8_STFT_STOCKHAM;
}

int ft8_sync_select(ft8_ctx* c, const void* d_wf, int wf_f64, int32_t n_slots, int32_t T, int32_t F,
                    const ft8_params* p, int32_t* d_cand, double* d_cand_score, int32_t* d_cand_count,
                    void* d_scores, void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (c) c->replay_ok = false;
  if (!c || !p || !d_cand_count) return fail(c, FT8_E_ARG, "null argument");
  if (T < 0 || F < 0 || n_slots < 0) return fail(c, FT8_E_ARG, "negative size");
  DeviceGuard dg(c->device);
  return do_sync_select(c, d_wf, wf_f64, n_slots, T, F, p, d_cand, d_cand_score, d_cand_count, d_scores,
                        (hipStream_t)stream);
}

int ft8_sync_score(ft8_ctx* c, const void* d_wf, int wf_f64, int32_t T, int32_t F, int32_t sps, int32_t bpt,
                   const int32_t* d_cand, int32_t n, void* d_out, int32_t* d_err, void* stream) {
  if (c) c->replay_ok = false;
  if (!c || n < 0 || (n > 0 && (!d_wf || !d_cand || !d_out || !d_err))) return fail(c, FT8_E_ARG, "bad argument");
  if (T <= 0 || F <= 0 || sps <= 0 || bpt <= 0) return fail(c, FT8_E_ARG, "empty waterfall or bad oversampling");
  DeviceGuard dg(c->device);
  hipError_t e = launch_score_list(d_wf, wf_f64, T, F, sps, bpt, d_cand, n, d_out, d_err, (hipStream_t)stream);
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "score launch");
}

int ft8_llr(ft8_ctx* c, const void* d_wf, int wf_f64, int32_t T, int32_t F, int32_t sps, int32_t bpt,
            const int32_t* d_cand, int32_t n, int normalize, double* d_llr, void* stream) {
  if (c) c->replay_ok = false;
  if (!c || !d_llr || (!d_cand && n > 0) || sps <= 0 || bpt <= 0) return fail(c, FT8_E_ARG, "bad argument");
  if (n <= 0) return FT8_OK;
  DeviceGuard dg(c->device);
  BpLaunch L{};
  L.wf = d_wf;
  L.wf_f64 = wf_f64;
  L.T = T;
  L.F = F;
  L.sps = sps;
  L.bpt = bpt;
  L.cand = d_cand;
  L.n_items = n;
  L.mode = 1;
  L.normalize = normalize;
  L.llr_out = d_llr;
  StageTimer tm(c, 6, (hipStream_t)stream);
  hipError_t e = launch_llr(L, (hipStream_t)stream);
  tm.done();
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "llr launch");
}

int ft8_normalize(ft8_ctx* c, const double* d_in, int32_t n, double* d_out, void* stream) {
  if (c) c->replay_ok = false;
  if (!c || (n > 0 && (!d_in || !d_out))) return fail(c, FT8_E_ARG, "bad argument");
  if (n <= 0) return FT8_OK;
  DeviceGuard dg(c->device);
  BpLaunch L{};
  L.mode = 2;
  L.llr_in = d_in;
  L.n_items = n;
  L.normalize = 1;
  L.llr_out = d_out;
  StageTimer tm(c, 6, (hipStream_t)stream);
  hipError_t e = launch_llr(L, (hipStream_t)stream);
  tm.done();
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "normalize launch");
}

int ft8_bp(ft8_ctx* c, const double* d_llr, int32_t n, int32_t max_iterations, uint8_t* d_plain, ft8_result* d_res,
           void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (c) c->replay_ok = false;
  if (!c || (!d_llr && n > 0)) return fail(c, FT8_E_ARG, "bad argument");
  if (n <= 0) return FT8_OK;
  DeviceGuard dg(c->device);
  int rc;
  if ((rc = ensure_work(c, 1, (hipStream_t)stream))) return rc;  // counter [0]: ft8_bp's own
  BpLaunch L{};
  L.mode = 2;
  L.llr_in = d_llr;
  L.n_items = n;
  L.normalize = 0;
  L.max_iterations = max_iterations;
  L.plain_out = d_plain;
  L.res = d_res;
  L.work = (unsigned long long*)c->work.p;
  L.work_base = &c->work_base[0];
  L.stats = (unsigned long long*)c->stats.p;
  L.clock = c->timing && c->stats.p ? (unsigned long long*)c->stats.p + 4 : nullptr;
  StageTimer tm(c, 3, (hipStream_t)stream);
  hipError_t e = launch_bp(L, (hipStream_t)stream);
  tm.done();
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "bp launch");
}

int ft8_decode_batch(ft8_ctx* c, const void* d_samples, int dtype, int64_t n_samples, int32_t n_slots,
                     int64_t slot_stride, const ft8_params* p, ft8_result* d_out, int32_t* d_counts,
                     int32_t cap, void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (c) c->replay_ok = false;
  if (!c || !p || !d_counts || (n_slots > 0 && !d_samples) || n_slots < 0 || cap < 0)
    return fail(c, FT8_E_ARG, "bad argument");
  if (cap > 0 && !d_out) return fail(c, FT8_E_ARG, "null output with positive capacity");
  DeviceGuard dg(c->device);
  hipStream_t s = (hipStream_t)stream;
  if (n_slots == 0) return FT8_OK;
  StageTimer whole(c, 5, s);
  Geo g;
  std::string why;
  int rc = geometry(rate_of(p), p->bins_per_tone, p->steps_per_symbol, n_samples, &g, &why);
  if (rc) return fail(c, rc, why);
  const int T = p->t_hi - p->t_lo, F = p->f_hi - p->f_lo;
  const bool f64 = is_f64_dtype(dtype);
  const size_t esz = f64 ? 8 : 4;
  const int N = p->max_candidates;
  Grid gr = grid_of(T > 0 ? T : 0, F > 0 ? F : 0, p->steps_per_symbol, p->bins_per_tone);
  if (T <= 0 || F <= 0 || N <= 0 || gr.NT == 0 || gr.NF == 0) {
    // nothing to search: validate the ranges, report zero decodes
    if (p->t_lo < 0 || p->t_hi > g.frames || p->f_lo < 0 || p->f_hi > g.nfft)
      return fail(c, FT8_E_ARG, "frame/bin range outside the spectrogram");
    hipError_t e = hipMemsetAsync(d_counts, 0, sizeof(int32_t) * n_slots, s);
    whole.done();
    return e == hipSuccess ? FT8_OK : hipfail(c, e, "memset");
  }
  if (N > kMaxCandidates)
    return fail(c, FT8_E_RANGE, "max_candidates > " + std::to_string(kMaxCandidates) + " is not supported");
  if ((rc = ensure(c, c->wf, esz * (size_t)n_slots * T * F))) return rc;
  if ((rc = ensure(c, c->cand, sizeof(int32_t) * 2 * (size_t)n_slots * N))) return rc;
  if ((rc = ensure(c, c->cand_score, sizeof(double) * (size_t)n_slots * N))) return rc;
  if ((rc = ensure(c, c->cand_count, sizeof(int32_t) * (size_t)n_slots))) return rc;
  if ((rc = ensure(c, c->res_all, sizeof(ft8_result) * (size_t)n_slots * N))) return rc;
  if ((rc = ensure(c, c->llr, sizeof(double) * FT8_LDPC_N * (size_t)n_slots * N))) return rc;
  if ((rc = ensure(c, c->scores, esz * (size_t)n_slots * score_elems(gr)))) return rc;
  if ((rc = ensure(c, c->smask, sizeof(uint64_t) * (size_t)n_slots * smask_words(gr)))) return rc;
  if ((rc = ensure(c, c->warn, sizeof(int32_t) * (size_t)n_slots))) return rc;
  if ((rc = ensure(c, c->rowsum, sizeof(RowSummary) * (size_t)n_slots * gr.NT * n_segments(gr.NF)))) return rc;
  if (!f64 && (rc = ensure(c, c->tie, sizeof(int32_t) * (size_t)n_slots * tie_stride(N)))) return rc;
  if (p->steps_per_symbol <= 0 || p->bins_per_tone <= 0) return fail(c, FT8_E_ARG, "bad oversampling factors");
  if (p->flags & ~(FT8_FLAG_TOPK | FT8_FLAG_SUBTRACT)) return fail(c, FT8_E_ARG, "unknown bits in ft8_params.flags");
  if (!(p->flags & FT8_FLAG_SUBTRACT)) {
    if ((rc = decode_pass(c, d_samples, dtype, n_samples, n_slots, slot_stride, p, d_out, d_counts, cap, s))) return rc;
    whole.done();
    return FT8_OK;
  }
  // ---- FT8_FLAG_SUBTRACT: pass 1 (complete record lists), subtract, pass 2 on the residual, merge
  if (dtype != FT8_F32 && dtype != FT8_I16)
    return fail(c, FT8_E_UNSUPPORTED, "FT8_FLAG_SUBTRACT needs float32 or int16 samples");
  if ((rc = ensure(c, c->out1, sizeof(ft8_result) * (size_t)n_slots * N))) return rc;
  if ((rc = ensure(c, c->out2, sizeof(ft8_result) * (size_t)n_slots * N))) return rc;
  if ((rc = ensure(c, c->counts1, sizeof(int32_t) * (size_t)n_slots))) return rc;
  if ((rc = ensure(c, c->counts2, sizeof(int32_t) * (size_t)n_slots))) return rc;
  if ((rc = ensure(c, c->residual, sizeof(float) * (size_t)n_slots * n_samples))) return rc;
  ft8_result* out1 = (ft8_result*)c->out1.p;
  ft8_result* out2 = (ft8_result*)c->out2.p;
  int32_t* counts1 = (int32_t*)c->counts1.p;
  int32_t* counts2 = (int32_t*)c->counts2.p;
  float* resid = (float*)c->residual.p;
  if ((rc = decode_pass(c, d_samples, dtype, n_samples, n_slots, slot_stride, p, out1, counts1, N, s))) return rc;
  if ((rc = subtract_core(c, d_samples, dtype, resid, n_samples, n_slots, slot_stride, n_samples, p, out1, counts1,
                          N, s)))
    return rc;
  if ((rc = decode_pass(c, resid, FT8_F32, n_samples, n_slots, n_samples, p, out2, counts2, N, s))) return rc;
  hipError_t e = launch_merge_pass(d_out, d_counts, cap, out1, counts1, N, out2, counts2, N, n_slots, s);
  if (e != hipSuccess) return hipfail(c, e, "merge launch");
  c->replay_ok = false;
  whole.done();
  return FT8_OK;
}

int ft8_encode(ft8_ctx* c, const uint8_t* d_msg, int32_t msg_bytes, int32_t n, uint8_t* d_a91, uint8_t* d_codeword,
               uint8_t* d_tones, void* stream) {
  if (c) c->replay_ok = false;
  if (!c || n < 0 || (n > 0 && !d_msg)) return fail(c, FT8_E_ARG, "bad argument");
  if (msg_bytes != 10 && msg_bytes != 12) return fail(c, FT8_E_ARG, "msg_bytes must be 10 (payload) or 12 (a91)");
  if (n == 0) return FT8_OK;
  DeviceGuard dg(c->device);
  hipError_t e = launch_encode(d_msg, msg_bytes, n, d_a91, d_codeword, d_tones, (hipStream_t)stream);
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "encode launch");
}

int ft8_synthesize(ft8_ctx* c, const uint8_t* d_tones, const ft8_tx_signal* d_signals, int32_t n_signals,
                   int32_t sample_rate, int32_t style, void* d_out, int out_dtype, int64_t n_samples, int32_t n_slots,
                   int64_t slot_stride, void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (c) c->replay_ok = false;
  if (!c || n_signals < 0 || n_slots < 0 || n_samples < 0 || sample_rate <= 0) return fail(c, FT8_E_ARG, "bad argument");
  if (style != FT8_TX_PROTOCOL && style != FT8_TX_REFERENCE) return fail(c, FT8_E_ARG, "unknown ft8_tx_style");
  if (out_dtype != FT8_F32 && out_dtype != FT8_F64 && out_dtype != FT8_C64 && out_dtype != FT8_C128)
    return fail(c, FT8_E_ARG, "out_dtype must be FT8_F32, FT8_F64, FT8_C64 or FT8_C128");
  if (n_signals == 0 || n_slots == 0 || n_samples == 0) return FT8_OK;
  if (!d_tones || !d_signals || !d_out) return fail(c, FT8_E_ARG, "null argument");
  if (slot_stride < n_samples && n_slots > 1) return fail(c, FT8_E_ARG, "slot_stride < n_samples");
  const int nsps = (int)(0.16 * (double)sample_rate);  // modulator.py:31 int(FT8_SYMBOL_TIME_S * fs)
  if (nsps < 8) return fail(c, FT8_E_ARG, "sample_rate too low (nsps < 8)");
  DeviceGuard dg(c->device);
  int rc = gfsk_tables(c, nsps);
  if (rc) return rc;
  SynthLaunch L{};
  L.tones = d_tones;
  L.sig = d_signals;
  L.n_sig = n_signals;
  L.nsps = nsps;
  L.style = style;
  L.fs = (double)sample_rate;
  L.P = (const double*)c->gfsk_P.p;
  L.out = d_out;
  L.dtype = out_dtype;
  L.n_samples = n_samples;
  L.slot_stride = slot_stride;
  L.n_slots = n_slots;
  hipError_t e = launch_synth(L, (hipStream_t)stream);
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "synthesize launch");
}

int ft8_subtract(ft8_ctx* c, const void* d_samples, int dtype, float* d_residual, int64_t n_samples, int32_t n_slots,
                 int64_t slot_stride, const ft8_params* p, const ft8_result* d_res, const int32_t* d_counts, int32_t cap,
                 void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (c) c->replay_ok = false;
  if (!c || !p || n_slots < 0 || cap < 0 || n_samples < 0) return fail(c, FT8_E_ARG, "bad argument");
  if (n_slots == 0 || n_samples == 0) {
    // nothing to fit: an empty subtraction's (zero) fits are valid, a zero-length one's never written
    c->sub_slots = n_slots == 0 ? 0 : -1;
    c->sub_cap = n_slots == 0 ? cap : -1;
    return FT8_OK;
  }
  if (!d_samples || !d_residual || !d_counts || (cap > 0 && !d_res)) return fail(c, FT8_E_ARG, "null argument");
  if (slot_stride < n_samples && n_slots > 1) return fail(c, FT8_E_ARG, "slot_stride < n_samples");
  DeviceGuard dg(c->device);
  return subtract_core(c, d_samples, dtype, d_residual, n_samples, n_slots, slot_stride, slot_stride, p, d_res,
                       d_counts, cap, (hipStream_t)stream);
}

int ft8_subtract_fits(ft8_ctx* c, ft8_sub_fit* d_out, int32_t n_slots, int32_t cap, void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (!c || (!d_out && n_slots > 0 && cap > 0)) return fail(c, FT8_E_ARG, "bad argument");
  if (n_slots != c->sub_slots || cap != c->sub_cap)
    return fail(c, FT8_E_ARG, "n_slots / cap differ from the last subtraction's (" + std::to_string(c->sub_slots) +
                                  " / " + std::to_string(c->sub_cap) + ")");
  if (n_slots == 0 || cap == 0) return FT8_OK;
  DeviceGuard dg(c->device);
  static_assert(sizeof(ft8_sub_fit) == 1056, "ft8_sub_fit layout");
  hipError_t e = hipMemcpyAsync(d_out, c->sub_est.p, sizeof(ft8_sub_fit) * (size_t)n_slots * cap,
                                hipMemcpyDeviceToDevice, (hipStream_t)stream);
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "fits copy");
}

int ft8_stft_argmax(ft8_ctx* c, const void* d_samples, int dtype, int64_t n_samples, int32_t n_slots,
                    int64_t slot_stride, const ft8_params* p, int32_t* d_idx, void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (c) c->replay_ok = false;
  if (!c || !p || (n_slots > 0 && (!d_samples || !d_idx))) return fail(c, FT8_E_ARG, "null argument");
  if (n_slots < 0 || n_samples < 0) return fail(c, FT8_E_ARG, "negative size");
  if (n_slots > 1 && slot_stride < n_samples) return fail(c, FT8_E_ARG, "slot_stride < n_samples");
  DeviceGuard dg(c->device);
  return stft_argmax_core(c, d_samples, dtype, n_samples, n_slots, slot_stride, p, d_idx, (hipStream_t)stream);
}

int ft8_drift_fit(ft8_ctx* c, int32_t stage, const int32_t* d_idx, int32_t n_slots, int32_t T, int32_t F,
                  const ft8_drift_params* p, ft8_drift_result* d_res, double* d_metric, int32_t* d_segments,
                  int32_t max_segments, void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (c) c->replay_ok = false;
  if (!c || !p) return fail(c, FT8_E_ARG, "null argument");
  if (stage != 1 && stage != 2) return fail(c, FT8_E_ARG, "stage must be 1 or 2");
  if (n_slots < 0 || T < 0 || max_segments < 0) return fail(c, FT8_E_ARG, "negative size");
  if (n_slots == 0) return FT8_OK;
  if (!d_res || (T > 0 && !d_idx)) return fail(c, FT8_E_ARG, "null argument");
  DeviceGuard dg(c->device);
  return drift_fit_core(c, stage, d_idx, n_slots, T, F, p, d_res, d_metric, d_segments, max_segments,
                        (hipStream_t)stream);
}

int ft8_drift_correct(ft8_ctx* c, const void* d_samples, int dtype, int64_t n_samples, int32_t n_slots,
                      int64_t slot_stride, const ft8_drift_params* p, void* d_out, ft8_drift_result* d_res,
                      void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (c) c->replay_ok = false;
  if (!c || !p) return fail(c, FT8_E_ARG, "null argument");
  if (n_slots < 0 || n_samples < 0) return fail(c, FT8_E_ARG, "negative size");
  if (n_slots == 0) return FT8_OK;
  if (!d_samples || !d_out || !d_res) return fail(c, FT8_E_ARG, "null argument");
  if (n_slots > 1 && slot_stride < n_samples) return fail(c, FT8_E_ARG, "slot_stride < n_samples");
  if (dtype != FT8_F32 && dtype != FT8_F64 && dtype != FT8_C64 && dtype != FT8_C128)
    return fail(c, FT8_E_UNSUPPORTED, "drift correction takes float32/float64/complex64/complex128 samples");
  int rc = check_drift_params(c, p);
  if (rc) return rc;
  DeviceGuard dg(c->device);
  hipStream_t s = (hipStream_t)stream;
  Geo g;
  std::string why;
  const int fs = (int)p->sample_rate;
  if ((rc = geometry(fs, p->bins_per_tone, p->steps_per_symbol, n_samples, &g, &why))) return fail(c, rc, why);
  if (g.frames == 0) return fail(c, FT8_E_ARG, "input shorter than one symbol (the reference's argmax of an empty spectrogram raises)");
  if (g.frames > kDriftMaxT) return fail(c, FT8_E_RANGE, "more than " + std::to_string(kDriftMaxT) + " frames per signal");
  const int T = g.frames, F = drift_bins(g.nfft);
  if ((rc = ensure(c, c->drift_idx, sizeof(int32_t) * (size_t)n_slots * T))) return rc;
  int32_t* idx = (int32_t*)c->drift_idx.p;
  ft8_params sp{};
  sp.sample_rate = fs;
  sp.bins_per_tone = p->bins_per_tone;
  sp.steps_per_symbol = p->steps_per_symbol;
  sp.f_lo = 0;
  sp.f_hi = F;
  sp.t_lo = 0;
  sp.t_hi = T;
  if ((rc = stft_argmax_core(c, d_samples, dtype, n_samples, n_slots, slot_stride, &sp, idx, s))) return rc;
  if ((rc = drift_fit_core(c, 1, idx, n_slots, T, F, p, d_res, nullptr, nullptr, 0, s))) return rc;
  DerotateLaunch D{};
  D.x = d_samples;
  D.dtype = dtype;
  D.slot_stride = slot_stride;
  D.out = (double*)d_out;
  D.n_samples = n_samples;
  D.n_slots = n_slots;
  D.res = d_res;
  D.fs = p->sample_rate;
  D.inv_fs = 1.0 / p->sample_rate;
  D.inv_2fs2 = 1.0 / (2.0 * p->sample_rate * p->sample_rate);
  {
    StageTimer tm(c, 10, s);
    hipError_t e = launch_derotate1(D, s);
    tm.done();
    if (e != hipSuccess) return hipfail(c, e, "derotate launch");
  }
  if (!p->precise_sync) return FT8_OK;
  if ((rc = stft_argmax_core(c, d_out, FT8_C128, n_samples, n_slots, n_samples, &sp, idx, s))) return rc;
  if ((rc = drift_fit_core(c, 2, idx, n_slots, T, F, p, d_res, nullptr, nullptr, 0, s))) return rc;
  StageTimer tm(c, 10, s);
  hipError_t e = launch_derotate2(D, p->poly_degree, s);
  tm.done();
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "derotate launch");
}

const char* ft8_build_id(void) { return FT8_BUILD_ID; }
const char* ft8_build_flags(void) { return FT8_BUILD_FLAGS; }

int ft8_replay_stage(ft8_ctx* c, int32_t stage, int32_t reps, void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (!c || reps < 0) return fail(c, FT8_E_ARG, "bad argument");
  if (!c->replay_ok) return fail(c, FT8_E_ARG, "no single-chain ft8_decode_batch to replay");
  DeviceGuard dg(c->device);
  hipStream_t s = (hipStream_t)stream;
  for (int r = 0; r < reps; ++r) {
    hipError_t e;
    switch (stage) {
      case 0: e = launch_stft(c->last_stft, s); break;
      case 1: e = launch_score(c->last_sync, s); break;
      case 2: e = launch_select(c->last_sync, s); break;
      case 3: e = launch_bp(c->last_bp, s); break;
      case 4: e = launch_compact(c->last_compact, s); break;
      case 6: e = launch_llr(c->last_bp, s); break;
      default: return fail(c, FT8_E_ARG, "stage " + std::to_string(stage) + " cannot be replayed");
    }
    if (e != hipSuccess) return hipfail(c, e, "replay launch");
  }
  return FT8_OK;
}

int ft8_set_pipeline(ft8_ctx* c, int32_t chunk_slots, int32_t n_streams, int32_t bp_waves_per_simd) {
  if (!c || chunk_slots < 0 || n_streams < 0 || n_streams > 8 || bp_waves_per_simd < 1 || bp_waves_per_simd > 4)
    return fail(c, FT8_E_ARG, "bad pipeline setting");
  c->chunk_slots = chunk_slots;
  c->n_streams = n_streams;
  c->bp_waves = bp_waves_per_simd;
  return FT8_OK;
}

int64_t ft8_pack_bytes(int32_t n_slots, int32_t capacity) {
  if (n_slots < 0 || capacity < 0) return -1;
  return pack_header_bytes(n_slots) + (int64_t)capacity * (int64_t)sizeof(ft8_result);
}

int ft8_pack_decodes(ft8_ctx* c, const ft8_result* d_records, const int32_t* d_counts, int32_t n_slots, int32_t cap,
                     int32_t capacity, int32_t slot_offset, void* d_send, ft8_result* d_overflow, void* stream) {
  if (!c || !d_send || n_slots < 0 || cap < 0 || capacity < 0) return fail(c, FT8_E_ARG, "bad argument");
  if (n_slots > 0 && (!d_counts || (cap > 0 && !d_records))) return fail(c, FT8_E_ARG, "null records or counts");
  if ((int64_t)n_slots * cap > INT32_MAX) return fail(c, FT8_E_RANGE, "n_slots * cap exceeds 2^31 rows");
  if (((uintptr_t)d_send & 7) || ((uintptr_t)d_overflow & 7)) return fail(c, FT8_E_ARG, "buffers must be 8-byte aligned");
  DeviceGuard dg(c->device);
  hipError_t e = launch_pack(d_records, d_counts, n_slots, cap, capacity, slot_offset, (uint8_t*)d_send, d_overflow,
                             (hipStream_t)stream);
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "pack launch");
}

int ft8_select_warnings(ft8_ctx* c, int32_t* d_out, int32_t n_slots, void* stream) {
  StreamOrder order_(c, (hipStream_t)stream);
  if (!c || !d_out || n_slots < 0) return fail(c, FT8_E_ARG, "bad argument");
  if (n_slots == 0) return FT8_OK;
  if (!c->warn.p || c->warn.cap < sizeof(int32_t) * n_slots) return fail(c, FT8_E_ARG, "no selection has run");
  DeviceGuard dg(c->device);
  hipError_t e = hipMemcpyAsync(d_out, c->warn.p, sizeof(int32_t) * n_slots, hipMemcpyDeviceToDevice,
                                (hipStream_t)stream);
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "copy warnings");
}

int ft8_crc14(ft8_ctx* c, const uint8_t* d_msg, const int32_t* d_nbits, int32_t n, uint16_t* d_crc, void* stream) {
  if (c) c->replay_ok = false;
  if (!c || (n > 0 && (!d_msg || !d_nbits || !d_crc))) return fail(c, FT8_E_ARG, "bad argument");
  DeviceGuard dg(c->device);
  hipError_t e = launch_crc14(d_msg, d_nbits, n, d_crc, (hipStream_t)stream);
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "crc14 launch");
}

int ft8_ldpc_check(ft8_ctx* c, const uint8_t* d_bits, int32_t n, int32_t* d_errors, void* stream) {
  if (c) c->replay_ok = false;
  if (!c || (n > 0 && (!d_bits || !d_errors))) return fail(c, FT8_E_ARG, "bad argument");
  DeviceGuard dg(c->device);
  hipError_t e = launch_ldpc_check(d_bits, n, d_errors, (hipStream_t)stream);
  return e == hipSuccess ? FT8_OK : hipfail(c, e, "ldpc_check launch");
}

int ft8_set_timing(ft8_ctx* c, int enable) {
  if (!c) return FT8_E_ARG;
  c->timing = enable != 0;
  if (c->timing && !c->stats.p) {
    DeviceGuard dg(c->device);
    const size_t bytes = (size_t)kStatRows * kStatStride * sizeof(unsigned long long);
    int rc = ensure(c, c->stats, bytes);
    if (rc) return rc;
    hipError_t e = hipMemset(c->stats.p, 0, bytes);
    if (e != hipSuccess) return hipfail(c, e, "stats reset");
  }
  return FT8_OK;
}

int ft8_set_timing_stages(ft8_ctx* c, uint32_t mask) {
  if (!c) return FT8_E_ARG;
  c->stage_mask = mask;
  return FT8_OK;
}

// the k_bp counter rows (kStatRows x kStatStride) summed per column (column 6, the longest wave,
// by maximum); reset zeroes columns [c0, c0 + 4) of every row
static int read_stat_rows(ft8_ctx* c, int c0, int reset, unsigned long long* out4) {
  std::vector<unsigned long long> v((size_t)kStatRows * kStatStride);
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(v.data(), c->stats.p, v.size() * sizeof(v[0]), hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset)
    e = hipMemset2D((char*)c->stats.p + c0 * sizeof(v[0]), kStatStride * sizeof(v[0]), 0, 4 * sizeof(v[0]), kStatRows);
  if (e != hipSuccess) return hipfail(c, e, "counters");
  for (int i = 0; i < 4; ++i) out4[i] = 0;
  for (int r = 0; r < kStatRows; ++r)
    for (int i = 0; i < 4; ++i) {
      const unsigned long long x = v[(size_t)r * kStatStride + c0 + i];
      out4[i] = (c0 + i == 6) ? std::max(out4[i], x) : out4[i] + x;
    }
  return FT8_OK;
}

int ft8_get_counters(ft8_ctx* c, int64_t* out4, int reset) {
  if (!c || !out4) return FT8_E_ARG;
  for (int i = 0; i < 4; ++i) out4[i] = 0;
  if (!c->stats.p) return FT8_OK;
  DeviceGuard dg(c->device);
  unsigned long long v[4];
  int rc = read_stat_rows(c, 0, reset, v);
  if (rc) return rc;
  for (int i = 0; i < 4; ++i) out4[i] = (int64_t)v[i];
  return FT8_OK;
}

int ft8_get_bp_clock(ft8_ctx* c, int64_t* out5, int reset) {
  if (!c || !out5) return FT8_E_ARG;
  for (int i = 0; i < 5; ++i) out5[i] = 0;
  DeviceGuard dg(c->device);
  int khz = 0;
  hipError_t e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device);
  if (e != hipSuccess) return hipfail(c, e, "wall clock rate");
  out5[4] = khz;
  if (!c->stats.p) return FT8_OK;
  unsigned long long v[4];
  int rc = read_stat_rows(c, 4, reset, v);
  if (rc) return rc;
  for (int i = 0; i < 4; ++i) out5[i] = (int64_t)v[i];
  return FT8_OK;
}

int ft8_get_timing(ft8_ctx* c, double* ms, int64_t* launches, int reset) {
  if (!c) return FT8_E_ARG;
  DeviceGuard dg(c->device);
  for (auto& t : c->pending) {
    hipError_t e = hipEventSynchronize(t.b);
    if (e != hipSuccess) return hipfail(c, e, "event sync");
    float v = 0.f;
    (void)hipEventElapsedTime(&v, t.a, t.b);
    c->ms[t.stage] += v;
    c->launches[t.stage] += 1;
    c->pool.push_back(t.a);
    c->pool.push_back(t.b);
  }
  c->pending.clear();
  for (int i = 0; i < FT8_N_STAGES; ++i) {
    if (ms) ms[i] = c->ms[i];
    if (launches) launches[i] = c->launches[i];
    if (reset) {
      c->ms[i] = 0;
      c->launches[i] = 0;
    }
  }
  return FT8_OK;
}

}  // extern "C"
