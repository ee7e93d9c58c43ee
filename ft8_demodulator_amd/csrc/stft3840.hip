// stft3840.hip -- the production STFT geometry (12 kHz, bins_per_tone = steps_per_symbol = 2: real
// input, nfft = 3840, nperseg = 1920, hop = 960) with packed float32 complex arithmetic (gfx950).
//
// Same transform as stft.hip's generic path (calculate_spectrogram, reference
// spectrogram_analyse.py:19-66, and the f >= 0 / band / time masks of ft8_decode.py:322-341): the
// 3840-point real FFT of each Hann-windowed frame is a P = 1920-point complex FFT of
// z[n] = w x[2n] + i w x[2n+1] plus a post-twiddle pass, P = 16 x 8 x 15 in three Stockham stages
// with compile-time radices, then |X|^2 / (sum w)^2 -> 10 log10(1e-12 + .) written once.
//
// A complex value lives in one aligned register pair (re, im) and every complex operation is a
// VOP3P packed float32 instruction: an addition or subtraction is one v_pk_add_f32; a product is
// v_pk_mul_f32 + v_pk_fma_f32 with operand selection (op_sel) and per-half negation (neg_lo/hi)
// doing the swap and the sign; multiplications by -i and conjugations fold into the neighbouring
// addition.  The compiler does not form these selections itself (it builds the swapped operand
// with extra moves), so the few instructions that need them are written as inline assembly.
// This file is built with packed math enabled and FMA contraction (Makefile); the FFT is not
// pocketfft in either case, and tests bound the dB error (tests/test_gpu_stft.py).
//
// Work decomposition: 256 threads (four waves) transform TWO frames per pass: stages 1 and 3 run
// frame A on threads 0..127 and frame B on 128..255 (120 / 128 of each half busy), stage 2 both
// frames' radix-8 butterfly j = t on 240 threads, the epilogue both frames' bins; one LDS image per
// frame with every stage in place, twiddles formed in registers by recurrence from per-thread
// seeds; a workgroup walks a run of consecutive frames of one slot, each thread loading its next
// frame's raw samples as soon as stage 1 has consumed the current ones.  With the full band kept
// (the decoder's waterfall; round 4) the epilogue runs on stage 3's registers: stage 3's threads
// are permuted so every bin pair (k, P - k) lies in one wave, 32 lanes apart, and the partner
// values cross by ds_bpermute -- stage 3 writes nothing back, one barrier per pass less.
#include "ft8_internal.h"

namespace ft8 {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

// ---- packed complex helpers -------------------------------------------------------------------
// (a.x b.x - a.y b.y, a.x b.y + a.y b.x)
__device__ __forceinline__ f2 cmul(f2 a, f2 b) {
  f2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
// a + (-i) b = (a.x + b.y, a.y - b.x)
__device__ __forceinline__ f2 add_mi(f2 a, f2 b) {
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a - (-i) b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ f2 sub_mi(f2 a, f2 b) {
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a + conj(b) = (a.x + b.x, a.y - b.y)
__device__ __forceinline__ f2 add_cj(f2 a, f2 b) {
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a - conj(b) = (a.x - b.x, a.y + b.y)
__device__ __forceinline__ f2 sub_cj(f2 a, f2 b) {
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// (a.x + b.y, a.x - b.y) and (a.y - b.x, a.y + b.x): the real and imaginary parts of a + (-i) b
// and a - (-i) b side by side
__device__ __forceinline__ f2 re_pm(f2 a, f2 b) {
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 im_mp(f2 a, f2 b) {
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 splat(float s) { return f2{s, s}; }

// ---- in-register DFTs (W_R = exp(-2 pi i / R)) --------------------------------------------------
__device__ __forceinline__ void dft4(f2* a) {
  const f2 t0 = a[0] + a[2], t1 = a[0] - a[2], t2 = a[1] + a[3], d = a[1] - a[3];
  a[0] = t0 + t2;
  a[2] = t0 - t2;
  a[1] = add_mi(t1, d);
  a[3] = sub_mi(t1, d);
}
__device__ __forceinline__ void dft8(f2* a) {
  const f2 r = splat(0.70710678118654752440f);
  f2 e[4] = {a[0], a[2], a[4], a[6]};
  f2 o[4] = {a[1], a[3], a[5], a[7]};
  dft4(e);
  dft4(o);
  const f2 w1 = add_mi(o[1], o[1]) * r;  // o1 W_8 = r (o1.x + o1.y, o1.y - o1.x)
  const f2 v3 = add_mi(o[3], o[3]) * r;  // o3 W_8^3 = -i (o3 W_8)
  a[0] = e[0] + o[0];
  a[4] = e[0] - o[0];
  a[1] = e[1] + w1;
  a[5] = e[1] - w1;
  a[2] = add_mi(e[2], o[2]);
  a[6] = sub_mi(e[2], o[2]);
  a[3] = add_mi(e[3], v3);
  a[7] = sub_mi(e[3], v3);
}
__device__ __forceinline__ void dft3(f2* a) {
  const f2 t = a[1] + a[2], d = (a[1] - a[2]) * splat(0.86602540378443864676f);
  const f2 m = a[0] - splat(0.5f) * t;
  a[0] = a[0] + t;
  a[1] = add_mi(m, d);
  a[2] = sub_mi(m, d);
}
__device__ __forceinline__ void dft5(f2* a) {
  const f2 c1 = splat(0.30901699437494742410f), c2 = splat(-0.80901699437494742410f);
  const f2 s1 = splat(0.95105651629515357212f), s2 = splat(0.58778525229247312917f);
  const f2 t1 = a[1] + a[4], t2 = a[2] + a[3], t3 = a[1] - a[4], t4 = a[2] - a[3];
  const f2 b1 = a[0] + c1 * t1 + c2 * t2;
  const f2 b2 = a[0] + c2 * t1 + c1 * t2;
  const f2 e1 = s1 * t3 + s2 * t4;
  const f2 e2 = s2 * t3 - s1 * t4;
  a[0] = a[0] + (t1 + t2);
  a[1] = add_mi(b1, e1);
  a[4] = sub_mi(b1, e1);
  a[2] = add_mi(b2, e2);
  a[3] = sub_mi(b2, e2);
}
// 15 = 3 x 5 prime-factor (no internal twiddles): n = (5 n1 + 3 n2) mod 15, k = (10 k1 + 6 k2) mod 15
__device__ __forceinline__ void dft15(const f2* x, f2* y) {
  f2 Y[3][5];
#pragma unroll
  for (int n1 = 0; n1 < 3; ++n1) {
#pragma unroll
    for (int n2 = 0; n2 < 5; ++n2) Y[n1][n2] = x[(5 * n1 + 3 * n2) % 15];
    dft5(Y[n1]);
  }
#pragma unroll
  for (int k2 = 0; k2 < 5; ++k2) {
    f2 v[3] = {Y[0][k2], Y[1][k2], Y[2][k2]};
    dft3(v);
#pragma unroll
    for (int k1 = 0; k1 < 3; ++k1) y[(10 * k1 + 6 * k2) % 15] = v[k1];
  }
}
__device__ __forceinline__ f2 w16(int m) {  // exp(-2 pi i m / 16), m in [0, 9]
  constexpr float c[10] = {1.0f, 0.92387953251128675613f, 0.70710678118654752440f, 0.38268343236508977173f,
                           0.0f, -0.38268343236508977173f, -0.70710678118654752440f, -0.92387953251128675613f,
                           -1.0f, -0.92387953251128675613f};
  constexpr float sn[10] = {0.0f, -0.38268343236508977173f, -0.70710678118654752440f, -0.92387953251128675613f,
                            -1.0f, -0.92387953251128675613f, -0.70710678118654752440f, -0.38268343236508977173f,
                            0.0f, 0.38268343236508977173f};
  return f2{c[m], sn[m]};
}
// 16-point DFT of x[0..7] with x[8..15] = 0 (4 x 4 Cooley-Tukey), y in natural order
__device__ __forceinline__ void dft16_half(const f2* x, f2* y) {
  f2 A[4][4];  // [n2][k1]
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
    const f2 a = x[n2], b = x[4 + n2];
    A[n2][0] = a + b;
    A[n2][1] = add_mi(a, b);
    A[n2][2] = a - b;
    A[n2][3] = sub_mi(a, b);
  }
#pragma unroll
  for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1)
      if (n2 * k1 != 4) A[n2][k1] = cmul(A[n2][k1], w16(n2 * k1));
  // k1 = 2: A[2][2] carries W_16^4 = -i, folded into its butterflies
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    if (k1 == 2) {
      const f2 t0 = add_mi(A[0][2], A[2][2]), t1 = sub_mi(A[0][2], A[2][2]);
      const f2 t2 = A[1][2] + A[3][2], d = A[1][2] - A[3][2];
      y[2] = t0 + t2;
      y[10] = t0 - t2;
      y[6] = add_mi(t1, d);
      y[14] = sub_mi(t1, d);
    } else {
      f2 v[4] = {A[0][k1], A[1][k1], A[2][k1], A[3][k1]};
      dft4(v);
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) y[k1 + 4 * k2] = v[k2];
    }
  }
}

// 16-point DFT of x[0], x[1] with x[2..15] = 0: y[k] = x0 + W_16^k x1, y[k + 8] = x0 - W_16^k x1
// (k < 8), y in natural order -- the first stage of a frame whose window covers at most 2 of the 16
// inputs per butterfly (k_stft_pk's 9 600-point plan at 12 kHz: 1 920 samples of the 9 600-pair
// half)
__device__ __forceinline__ void dft16_two(f2 x0, f2 x1, f2* y) {
  const f2 r = splat(0.70710678118654752440f);
  const f2 t1 = cmul(x1, w16(1)), t3 = cmul(x1, w16(3)), t5 = cmul(x1, w16(5)), t7 = cmul(x1, w16(7));
  const f2 t2 = add_mi(x1, x1) * r;  // x1 W_8 = r (x1.x + x1.y, x1.y - x1.x)
  y[0] = x0 + x1;
  y[8] = x0 - x1;
  y[4] = add_mi(x0, x1);             // W_16^4 = -i
  y[12] = sub_mi(x0, x1);
  y[2] = x0 + t2;
  y[10] = x0 - t2;
  y[6] = add_mi(x0, t2);             // W_16^6 = -i W_16^2
  y[14] = sub_mi(x0, t2);
  y[1] = x0 + t1;
  y[9] = x0 - t1;
  y[3] = x0 + t3;
  y[11] = x0 - t3;
  y[5] = x0 + t5;
  y[13] = x0 - t5;
  y[7] = x0 + t7;
  y[15] = x0 - t7;
}

template <typename InT>
__device__ __forceinline__ f2 load_pair(const InT* x, int64_t n0) {
  if constexpr (sizeof(InT) == 4) {
    const float2 v = *reinterpret_cast<const float2*>(x + n0);
    return f2{v.x, v.y};
  } else {
    const short2 v = *reinterpret_cast<const short2*>(x + n0);
    return f2{(float)v.x / 32767.0f, (float)v.y / 32767.0f};  // read_wave_file: float32(x) / iinfo(int16).max
  }
}

constexpr int kP = 1920;
// four waves, TWO frames per pass (round 3): stage 1 and stage 3 run frame A on threads 0..127 and
// frame B on 128..255, stage 2 does both frames' radix-8 butterfly j = t (sharing its twiddles), the
// epilogue both frames' bins k = t + 256 i (sharing the post-twiddle recurrence).  One frame per
// pass left stages 1 and 3 on 120 / 128 of the 256 threads -- two of the four waves waited at the
// barrier through the two heaviest stages.
constexpr int kThreads38 = 256;
// frames per workgroup (six passes), 16 workgroups per 186-frame slot.  Round 3 measured 6 best
// (0.171 ms against 0.173-0.176 for 12); with the full-band epilogue in registers (one barrier per
// pass fewer) 12 is: 0.150 / 0.150 ms against 0.153 / 0.156 for 6, 0.154 for 8, 0.159-0.160 for 4
// (interleaved, profiles/r4_v29_chunk_ab.log)
constexpr int kChunk = 12;
static_assert(kThreads38 == 256 && kChunk % 2 == 0, "two frames per pass on 2 x 128 threads");
// one LDS image per frame, every stage in place, with pidx padding (stage 1 writes with a
// 16-complex stride across lanes: 128 B, 32-way bank conflicts unpadded)
constexpr int kBuf = kP + (kP - 1) / 16;

struct Args {
  const void* samples;
  int64_t slot_stride;
  int t_lo, f_lo, nf_out, nt_out;
  const float* window;
  float scale;
  float* out;
  const f2* tw;    // W_1920^m
  const f2* post;  // W_3840^k, k in [0, 1920]
};

__device__ __forceinline__ int pidx(int i) { return i + (i >> 4); }
// LDS accesses one ds_read_b64 / ds_write_b64 each (volatile): merged ds_read2_b64 / ds_write2_b64
// move half the bytes per LDS cycle, and their 8-bit offsets made the compiler keep a base
// register per pair of positions (~20 VGPRs of addresses live through the frame loop)
typedef __attribute__((address_space(3))) f2 lds_f2;
__device__ __forceinline__ f2 lds_ld(const f2* p) { return *(const volatile lds_f2*)p; }
__device__ __forceinline__ void lds_st(f2* p, f2 v) { *(volatile lds_f2*)p = v; }

// FULL: every f >= 0 bin kept (no band mask; the decoder's waterfall), its epilogue fused into stage 3
template <typename InT, bool FULL>
__global__ __launch_bounds__(kThreads38, 4) void k_stft3840p(Args a) {
  FT8_RACE_PROLOGUE();
  __shared__ f2 buf[2][kBuf];  // frame A, frame B
  // the window as pairs (w[2n], w[2n+1]) (round 5: read from L1 every pass instead -- 32.6 KB of
  // LDS -- measured 0.160 vs 0.149 ms per 256-slot launch, profiles/r5_d_ab.log; not kept)
  __shared__ f2 wl[kP / 2];
  const int t = threadIdx.x;
  // stages 1 and 3: the frame this thread works on (A = 0, B = 1); wave-uniform, so in an SGPR
  const int role = __builtin_amdgcn_readfirstlane(t >> 7);
  const int u = t & 127;    // ... and its index there
  const int chunks = (a.nt_out + kChunk - 1) / kChunk;
  const int slot = blockIdx.x / chunks;
  const int c = blockIdx.x - slot * chunks;
  const int f_begin = c * kChunk, f_end = min(a.nt_out, f_begin + kChunk);
  // twiddle seeds: stage 2 W_128^k (k = t % 16), stage 3 W_1920^u, epilogue W_3840^(f_lo + t) and
  // its 256-bin step; their powers are formed by complex recurrence each pass (relative error
  // ~15 ulp, far inside the dB tolerance)
  // stage 3's index: u, or (FULL) a permutation of u that puts bin k's partner P - k in the same
  // wave, 32 lanes over (see the epilogue below): lanes 0..31 of the frame's first wave take u =
  // 0..31, lane 32 u = 64, lanes 33..63 u = 127..97; the second wave's lanes 0..31 u = 32..63 and
  // lanes 32..63 u = 96..65
  const int lane = t & 63, half = __builtin_amdgcn_readfirstlane((t >> 6) & 1);
  const int u3 = !FULL ? u : half == 0 ? (lane < 32 ? lane : lane == 32 ? 64 : 160 - lane) : (lane < 32 ? 32 + lane : 128 - lane);
  f2 s2 = a.tw[15 * (t & 15)], s3 = a.tw[u3];
  const bool rec_post = a.f_lo + a.nf_out <= kP;
  constexpr bool full = FULL;
  // 10 log10(v) = (10 log10 2) log2(v): v_log_f32 on a normal argument (v >= 1e-12)
  constexpr float kDb = 3.0102999566398119521f;
  // post-twiddle seeds: the full band walks k = u + 128 r (stage 3's own bins), a band k = f_lo + t
  // + 256 i
  f2 p0 = full ? a.post[u3] : a.post[min(a.f_lo + t, kP)];
  const f2 pstep = a.post[full ? 128 : kThreads38];
  const f2 qscale = splat(0.25f * a.scale);  // |2 X|^2 / 4 / (sum w)^2 (powers of two: exact)

  for (int n = t; n < kP / 2; n += kThreads38) wl[n] = *reinterpret_cast<const f2*>(a.window + 2 * n);
  const bool s1 = u < 120;
  const InT* xs = reinterpret_cast<const InT*>(a.samples) + (int64_t)slot * a.slot_stride;
  // raw pairs (x[2n], x[2n+1]), n = u + 120 r, of this thread's frame of the pass; loaded for the
  // next pass as soon as stage 1 has consumed them
  f2 raw[8];
  auto load_raw = [&](int fr) {
    const int64_t base = (int64_t)(a.t_lo + fr) * 960;
#pragma unroll
    for (int r = 0; r < 8; ++r) raw[r] = load_pair<InT>(xs, base + 2 * (u + 120 * r));
  };
  if (s1 && f_begin + role < f_end) load_raw(f_begin + role);
  for (int f = f_begin; f < f_end; f += 2) {
    // re-opaque the seeds so the per-pass twiddle powers are not hoisted into ~50 live registers
    asm volatile("" : "+v"(s2), "+v"(s3), "+v"(p0));
    const bool haveB = f + 1 < f_end;        // workgroup-uniform
    const bool mine = role == 0 || haveB;    // wave-uniform
    f2* const img = buf[role];
    // stage 1: radix 16, Ns = 1: inputs z[u + 120 r] (r >= 8 is zero padding) -> img[16 u + k]
    __syncthreads();  // the previous pass's epilogue has finished reading both images
    if (s1 && mine) {
      f2 z[8], y[16];
#pragma unroll
      for (int r = 0; r < 8; ++r) z[r] = lds_ld(&wl[u + 120 * r]) * raw[r];
      dft16_half(z, y);
#pragma unroll
      for (int k = 0; k < 16; ++k) lds_st(&img[17 * u + k], y[k]);  // pidx(16 u + k)
      if (f + 2 + role < f_end) load_raw(f + 2 + role);  // in flight through stages 2, 3 and the epilogue
    }
    __syncthreads();
    // stage 2: radix 8, Ns = 16: butterfly j = t (j < 240) of both frames
    {
      const int j = t;
      f2 va[8], vb[8];
      if (j < 240) {
        auto bfly = [&](const f2* img_, f2* v) {
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = lds_ld(&img_[pidx(j) + 255 * r]);  // pidx(j + 240 r)
          if ((j & 15) != 0) {
            f2 w = s2;  // W_128^(r k)
#pragma unroll
            for (int r = 1; r < 8; ++r) {
              v[r] = cmul(v[r], w);
              if (r < 7) w = cmul(w, s2);
            }
          }
          dft8(v);
        };
        bfly(buf[0], va);
        // frame B's reads after frame A's butterfly: interleaving the two needs ~100 more VGPRs
        asm volatile("" : "+v"(s2) : : "memory");  // and its twiddle powers recomputed, not kept
        if (haveB) bfly(buf[1], vb);
      }
      __syncthreads();  // every stage-2 read of the images is done: write in place
      if (j < 240) {
        const int d0 = (j >> 4) * 128 + (j & 15);
#pragma unroll
        for (int r = 0; r < 8; ++r) lds_st(&buf[0][pidx(d0) + 17 * r], va[r]);  // pidx(d0 + 16 r)
        if (haveB) {
#pragma unroll
          for (int r = 0; r < 8; ++r) lds_st(&buf[1][pidx(d0) + 17 * r], vb[r]);
        }
      }
    }
    __syncthreads();
    // stage 3: radix 15, Ns = 128: j = u3, natural order, in place (a thread writes the 15 positions
    // it read)
    if (mine) {
      f2 v[15], y[15];
#pragma unroll
      for (int r = 0; r < 15; ++r) v[r] = lds_ld(&img[pidx(u3) + 136 * r]);  // pidx(u3 + 128 r)
      if (u3 != 0) {
        f2 w = s3;  // W_1920^(r u3)
#pragma unroll
        for (int r = 1; r < 15; ++r) {
          v[r] = cmul(v[r], w);
          if (r < 14) w = cmul(w, s3);
        }
      }
      dft15(v, y);
      if constexpr (!FULL) {
#pragma unroll
        for (int r = 0; r < 15; ++r) lds_st(&img[pidx(u3) + 136 * r], y[r]);
      } else {
        // the epilogue from stage 3's registers (round 4).  The thread holds Z[u3 + 128 r]; bin k's
        // partner P - k = (128 - u3) + 128 (14 - r) is element 14 - r of u = 128 - u3, 32 lanes
        // over in this wave (u3 = 0 and 64: the thread itself, at 15 - r and 14 - r).  The thread
        // takes the pairs of its r = 0..7 (r = 7 only for u3 <= 64: past it k > P / 2), so it needs
        // its partner's 7..14: eight ds_bpermute pairs instead of the image written back and read
        // again (the LDS store path was the kernel's busiest), and one barrier less per pass.
        const bool self = half == 0 && (lane & 31) == 0;
        const int src = (self ? lane : lane ^ 32) << 2;
        if (half == 0) {
          // u3 = 0 pairs r with its own 15 - r (r >= 1) and bin 0 with itself, where u3 = 64 pairs
          // r with 14 - r: lane 0 offers itself its 8..14 and Z[0] in the slots of 7..14 (a
          // wave-uniform branch, first waves only); its own y[7] (A of the pair (7, 8)) is kept
          const bool z0 = lane == 0;
          v[7] = y[7];
#pragma unroll
          for (int r = 7; r < 14; ++r) y[r] = z0 ? y[r + 1] : y[r];
          y[14] = z0 ? y[0] : y[14];
        } else {
          v[7] = y[7];
        }
        f2 pr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pr[j].x = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(y[7 + j].x)));
          pr[j].y = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(y[7 + j].y)));
        }
        f2 pw_k = p0;  // W_3840^k, k = u3 + 128 r
        float* out = a.out + ((int64_t)slot * a.nt_out + f + role) * a.nf_out;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const f2 wk = pw_k;
          if (r < 7) pw_k = cmul(pw_k, pstep);
          if (r == 7 && u3 > 64) break;
          const f2 A = r == 7 ? v[7] : y[r];
          const f2 B = pr[7 - r];  // partner element 14 - r
          const f2 sm = add_cj(A, B), df = sub_cj(A, B);
          const f2 wd = cmul(wk, df);
          const f2 re = re_pm(sm, wd), im = im_mp(sm, wd);  // (X1.x, X2.x), (X1.y, -X2.y)
          const f2 pp = (re * re + im * im) * qscale + splat(1e-12f);
          const f2 d = f2{__builtin_amdgcn_logf(pp.x), __builtin_amdgcn_logf(pp.y)} * splat(kDb);
          const int k = u3 + 128 * r;
          out[k] = d.x;
          if (k != 0 && k != kP / 2) out[kP - k] = d.y;
        }
      }
    }
    if constexpr (FULL) continue;  // the next pass's first barrier orders stage 3's reads before stage 1
    __syncthreads();
    // epilogue: real-signal spectrum X[k] = (s - i W_N^k d) / 2 with s = Z[k] + conj Z[P-k],
    // d = Z[k] - conj Z[P-k]; power, dB, kept bins -- frame A then frame B per bin block
    const int nfr = haveB ? 2 : 1;
    {
      f2 pw_k = p0;  // W_3840^k for k = f_lo + i (recurrence over i += 256)
      for (int i = t; i < a.nf_out; i += kThreads38) {
        const int k = a.f_lo + i;
        const int kk = (k <= kP) ? k : 2 * kP - k;
        const f2 wk = rec_post ? pw_k : a.post[kk];
        pw_k = cmul(pw_k, pstep);
        for (int q = 0; q < nfr; ++q) {
          const f2 A = lds_ld(&buf[q][pidx(kk == kP ? 0 : kk)]);
          const f2 B = lds_ld(&buf[q][pidx(kk == 0 ? 0 : kP - kk)]);
          const f2 sm = add_cj(A, B), df = sub_cj(A, B);
          const f2 wd = cmul(wk, df);
          const f2 X = add_mi(sm, wd);
          const f2 qq = X * X;
          const float pw = (qq.x + qq.y) * qscale.x + 1e-12f;
          a.out[((int64_t)slot * a.nt_out + f + q) * a.nf_out + i] = kDb * __builtin_amdgcn_logf(pw);
        }
      }
    }
  }
}

// ---- k_stft_pk: the reference's other real-input geometries with packed float32 (round 4) ------
// The same transform as k_stft_sp (stft.hip) for its compile-time plans -- 20 kHz at bpt = sps = 2
// (P = 3 200 = 16 x 8 x 5 x 5, the bundled recording's rate), 12 kHz at bpt = sps = 10 (P = 9 600 =
// 16 x 8 x 15 x 5, the decode test's), 6 kHz (P = 960 = 16 x 4 x 15) -- written with this file's
// packed complex helpers: one frame per 256-thread workgroup, Stockham stages in place in one padded
// LDS image (every stage reads its inputs, a barrier, then writes), the first stage a radix-16 DFT
// of the frame's nonzero half (dft16_half), twiddles W_(Ns R)^(k r) as powers of one table read
// (radix <= 8; the radix-15 stage reads its 14 from the table: that chain's rounding moved bins 60 dB
// below a frame's peak past the 1e-3 dB test bound at P = 9 600), the real-input post-twiddle and dB
// in the epilogue.  k_stft_sp's scalar complex code issued ~7x the VALU instructions per frame of
// k_stft3840p's packed form for 1.7x the points.
template <int R>
__device__ __forceinline__ void dft_r(f2* v) {
  if constexpr (R == 4) {
    dft4(v);
  } else if constexpr (R == 5) {
    dft5(v);
  } else if constexpr (R == 8) {
    dft8(v);
  } else {
    static_assert(R == 15, "radix 4, 5, 8 or 15");
    f2 y[15];
    dft15(v, y);
#pragma unroll
    for (int r = 0; r < 15; ++r) v[r] = y[r];
  }
}

struct PkArgs {
  const void* samples;
  int64_t slot_stride;
  int t_lo, f_lo, nf_out, nt_out, hop, nperseg, n_slots, per_xcd;
  const float* window;
  float scale;
  float* out;
  const f2* tw;    // W_P^m, m in [0, P)
  const f2* post;  // W_2P^k, k in [0, P]
};

// one Stockham stage (not the first): butterfly j = t + TH b of nbf = P / R, Ns = NS
template <int TH, int P, int NS, int R>
__device__ __forceinline__ void pk_stage(f2* buf, const f2* tw, const int t) {
  constexpr int NBF = P / R, NB = (NBF + TH - 1) / TH, TSTEP = P / (NS * R);
  // every index step is a multiple of 16, so pidx(x + 16 m) = pidx(x) + 17 m: one address per
  // butterfly and immediates (as k_stft3840p)
  static_assert(NBF % 16 == 0 && NS % 16 == 0, "linear padded index steps");
  constexpr int RSTEP = NBF + NBF / 16, WSTEP = NS + NS / 16;
  f2 v[NB][R];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = t + TH * b;
    if (j < NBF) {
      const int base = pidx(j);
#pragma unroll
      for (int r = 0; r < R; ++r) v[b][r] = lds_ld(&buf[base + r * RSTEP]);
    }
  }
  __syncthreads();  // every read of the image is done: write in place
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = t + TH * b;
    if (j < NBF) {
      const int k = j % NS;
      if (k != 0) {
        if constexpr (R <= 8) {
          const f2 w = tw[k * TSTEP];
          f2 wr = w;
#pragma unroll
          for (int r = 1; r < R; ++r) {
            v[b][r] = cmul(v[b][r], wr);
            if (r + 1 < R) wr = cmul(wr, w);
          }
        } else {
#pragma unroll
          for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], tw[r * k * TSTEP]);
        }
      }
      dft_r<R>(v[b]);
      const int wbase = pidx((j / NS) * NS * R + k);
#pragma unroll
      for (int r = 0; r < R; ++r) lds_st(&buf[wbase + r * WSTEP], v[b][r]);
    }
  }
  __syncthreads();
}

template <int TH, int P, int NS, int R, int... Rest>
__device__ __forceinline__ void pk_stages(f2* buf, const f2* tw, const int t) {
  pk_stage<TH, P, NS, R>(buf, tw, t);
  if constexpr (sizeof...(Rest) > 0) pk_stages<TH, P, NS * R, Rest...>(buf, tw, t);
}

// TH threads per frame: 256, or 640 for the 9 600-point plan, whose 82 KB image allows only two
// workgroups per CU (8 resident waves at 256 threads: the barriers between stages left the SIMDs
// idle); its stages' 600 / 1 200 / 640 / 1 920 butterflies fill 640 lanes to 94-100 %.
// A workgroup transforms FR consecutive frames of one slot in turn (round 5; the 3 200- and
// 960-point plans two, the 9 600-point one one): the window pairs its stage-1 inputs take are the
// same in every frame and stay in registers, and the frame's loads carry no per-lane branch.  One
// frame per workgroup had the 20 kHz plan's waves 73 % of their time in waits (its loads, each in
// its own branch, at the head of every frame).  Measured (profiles/r5_{j,k,m,p}_geo_*): 20 kHz STFT
// 0.54-0.56 ms -> 0.455-0.475 at FR 2 (FR 3 / 4 / 6 / 8: 0.45 / 0.46 / 0.46 / 0.48-0.51; the next
// frame prefetched into registers: 0.51); the 9 600-point plan keeps one frame (0.85-1.20 ms at any
// FR > 1, where the loop-invariant stage addresses stay live: up to 144 VGPRs).
constexpr int kPkFrames = 2;
template <typename InT, int TH, int FR, int P, int... Rs>
__global__ __launch_bounds__(TH) void k_stft_pk(PkArgs a) {
  FT8_RACE_PROLOGUE();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_pk[];
  f2* buf = reinterpret_cast<f2*>(smem_pk);
  const int t = threadIdx.x;
  const int nt = a.nt_out;
  const int chunks = (nt + FR - 1) / FR;
  const int rr = (int)(blockIdx.x & 7) * a.per_xcd + (int)(blockIdx.x >> 3);  // XCD-aware, as k_stft
  if (rr >= chunks * a.n_slots) return;
  const int slot = rr / chunks;
  const int f_begin = (rr - slot * chunks) * FR, f_end = min(nt, f_begin + FR);
  // stage 1: radix 16, Ns = 1, over the frame's nonzero half: inputs z[j + r P / 16], r < 8, with
  // z[n] = (w[2n] x[2n], w[2n+1] x[2n+1]) (zero past nperseg) -> buf[16 j + k]
  constexpr int NBF = P / 16, NB = (NBF + TH - 1) / TH;
  // FR > 1: a stage-1 operand is the pair at min(n0, nperseg - 2) (in bounds for every lane), then a
  // select: the pair itself, (x[n0], 0) at n0 = nperseg - 1, or zero
  auto pick = [&](int n0, f2 p) {
    return n0 + 1 < a.nperseg ? p : f2{n0 < a.nperseg ? p.y : 0.0f, 0.0f};
  };
  auto window_pair = [&](int n0) {
    return pick(n0, *reinterpret_cast<const f2*>(a.window + min(n0, a.nperseg - 2)));
  };
  f2 wz[NB][8];
  if constexpr (FR > 1) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int r = 0; r < 8; ++r) wz[b][r] = t + TH * b < NBF ? window_pair(2 * (t + TH * b + r * NBF)) : f2{0.0f, 0.0f};
    }
  }
  const InT* xslot = reinterpret_cast<const InT*>(a.samples) + (int64_t)slot * a.slot_stride;
  constexpr float kDb = 3.0102999566398119521f;  // 10 log10(v) = (10 log10 2) log2(v), v >= 1e-12
  const float qscale = 0.25f * a.scale;          // |2 X|^2 / 4 / (sum w)^2
  // at most two nonzero inputs per stage-1 butterfly (n0 = 2 (j + r P / 16) >= nperseg for r >= 2):
  // the pruned 16-point DFT (workgroup-uniform)
  const bool two = a.nperseg <= 4 * NBF;
#pragma unroll 1
  for (int fi = f_begin; fi < f_end; ++fi) {
    if (fi > f_begin) __syncthreads();  // the previous frame's epilogue has read the image
    const InT* xs = xslot + (int64_t)(a.t_lo + fi) * a.hop;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int j = t + TH * b;
      if (j < NBF) {
        f2 z[8], y[16];
        if constexpr (FR > 1) {
          // every lane loads (the pair at min(n0, nperseg - 2), in bounds) and selects, so a frame's
          // loads issue together: a load inside a per-lane branch waited for each in turn
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int n0 = 2 * (j + r * NBF);
            z[r] = wz[b][r] * pick(n0, load_pair<InT>(xs, min(n0, a.nperseg - 2)));
          }
        } else {
          // one frame per workgroup (the 9 600-point plan: its 1 920-sample window covers a fifth of
          // the transformed half): per-lane branches, so the zero part's loads are skipped
          const int rn = two ? 2 : 8;
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int n0 = 2 * (j + r * NBF);
            if (r >= rn) {
              z[r] = f2{0.0f, 0.0f};
            } else if (n0 + 1 < a.nperseg) {
              z[r] = *reinterpret_cast<const f2*>(a.window + n0) * load_pair<InT>(xs, n0);
            } else {
              z[r] = f2{n0 < a.nperseg ? a.window[n0] * load_pair<InT>(xs, n0).x : 0.0f, 0.0f};
            }
          }
        }
        if (FR == 1 && two) dft16_two(z[0], z[1], y);
        else dft16_half(z, y);
#pragma unroll
        for (int k = 0; k < 16; ++k) lds_st(&buf[17 * j + k], y[k]);  // pidx(16 j + k)
      }
    }
    __syncthreads();
    // re-opaque the thread index and the tables' addresses each frame, so the stages' LDS
    // addresses and twiddle loads (the same in every frame) are recomputed, not hoisted out of the
    // loop into ~90 live registers
    const f2* tw = a.tw;
    const f2* post = a.post;
    int tf = t;
    if constexpr (FR > 1) asm volatile("" : "+s"(tw), "+s"(post), "+v"(tf));
    pk_stages<TH, P, 16, Rs...>(buf, tw, tf);
    // epilogue: X[k] = (s - i W_2P^k d) / 2, s = Z[k] + conj Z[P-k], d = Z[k] - conj Z[P-k]
    float* out = a.out + ((int64_t)slot * nt + fi) * a.nf_out;
    if (a.f_lo == 0 && a.nf_out == P) {
      // every f >= 0 bin kept: bins k and P - k share s and d (k_stft3840p's full-band epilogue):
      // one pair of LDS reads, one post-twiddle and one packed power for both
      for (int k = t; k <= P / 2; k += TH) {
        const f2 A = lds_ld(&buf[pidx(k)]);
        const f2 B = lds_ld(&buf[pidx(k == 0 ? 0 : P - k)]);
        const f2 sm = add_cj(A, B), df = sub_cj(A, B);
        const f2 wd = cmul(post[k], df);
        const f2 re = re_pm(sm, wd), im = im_mp(sm, wd);  // (X1.x, X2.x), (X1.y, -X2.y)
        const f2 pp = (re * re + im * im) * splat(qscale) + splat(1e-12f);
        out[k] = kDb * __builtin_amdgcn_logf(pp.x);
        if (k != 0 && k != P / 2) out[P - k] = kDb * __builtin_amdgcn_logf(pp.y);
      }
      continue;
    }
    for (int i = t; i < a.nf_out; i += TH) {
      const int k = a.f_lo + i;
      const int kk = (k <= P) ? k : 2 * P - k;  // real signal: X[N-k] = conj X[k]
      const f2 A = lds_ld(&buf[pidx(kk == P ? 0 : kk)]);
      const f2 B = lds_ld(&buf[pidx(kk == 0 ? 0 : P - kk)]);
      const f2 sm = add_cj(A, B), df = sub_cj(A, B);
      const f2 wd = cmul(post[kk], df);
      const f2 X = add_mi(sm, wd);
      const f2 qq = X * X;
      out[i] = kDb * __builtin_amdgcn_logf((qq.x + qq.y) * qscale + 1e-12f);
    }
  }
}

}  // namespace

bool stft3840_eligible(const StftLaunch& L) {
  return !L.argmax && !L.plan.dft && !L.plan.blue && (L.dtype == FT8_F32 || L.dtype == FT8_I16) && L.nfft == 2 * kP &&
         L.nperseg == kP && L.hop == 960 && L.plan.P == kP && (L.slot_stride % 2) == 0;
}

hipError_t launch_stft3840(const StftLaunch& L, hipStream_t s) {
  Args a{};
  a.samples = L.samples;
  a.slot_stride = L.slot_stride;
  a.t_lo = L.t_lo;
  a.f_lo = L.f_lo;
  a.nf_out = L.f_hi - L.f_lo;
  a.nt_out = L.t_hi - L.t_lo;
  a.window = reinterpret_cast<const float*>(L.window);
  a.scale = (float)L.scale;
  a.out = reinterpret_cast<float*>(L.out);
  a.tw = reinterpret_cast<const f2*>(L.plan.tw);
  a.post = reinterpret_cast<const f2*>(L.plan.post);
  if (a.nt_out <= 0 || a.nf_out <= 0 || L.n_slots <= 0) return hipSuccess;
  const int chunks = (a.nt_out + kChunk - 1) / kChunk;
  const dim3 grid((unsigned)(chunks * L.n_slots));
  const bool full = a.f_lo == 0 && a.nf_out == kP;
  if (L.dtype == FT8_F32) {
    if (full) hipLaunchKernelGGL((k_stft3840p<float, true>), grid, dim3(kThreads38), 0, s, a);
    else hipLaunchKernelGGL((k_stft3840p<float, false>), grid, dim3(kThreads38), 0, s, a);
  } else {
    if (full) hipLaunchKernelGGL((k_stft3840p<int16_t, true>), grid, dim3(kThreads38), 0, s, a);
    else hipLaunchKernelGGL((k_stft3840p<int16_t, false>), grid, dim3(kThreads38), 0, s, a);
  }
  return hipGetLastError();
}

// the plans k_stft_pk is built for
struct PkPlan {
  int P, n, r[4];
};
constexpr int kPk9600Threads = 640;
constexpr PkPlan kPkPlans[] = {{3200, 4, {16, 8, 5, 5}}, {9600, 4, {16, 8, 15, 5}}, {960, 3, {16, 4, 15}}};

static int pk_plan_of(const StftLaunch& L) {
  if (L.argmax || L.plan.dft || L.plan.blue || !(L.dtype == FT8_F32 || L.dtype == FT8_I16)) return -1;
  if (L.nfft != 2 * L.plan.P || L.nperseg > L.plan.P || (L.hop % 2) || (L.slot_stride % 2)) return -1;
  for (int q = 0; q < 3; ++q) {
    const PkPlan& p = kPkPlans[q];
    bool ok = L.plan.P == p.P && L.plan.nstages == p.n;
    for (int i = 0; ok && i < p.n; ++i) ok = L.plan.radix[i] == p.r[i];
    if (ok) return q;
  }
  return -1;
}

bool stftpk_eligible(const StftLaunch& L) { return pk_plan_of(L) >= 0; }

hipError_t launch_stftpk(const StftLaunch& L, hipStream_t s) {
  PkArgs a{};
  a.samples = L.samples;
  a.slot_stride = L.slot_stride;
  a.t_lo = L.t_lo;
  a.f_lo = L.f_lo;
  a.nf_out = L.f_hi - L.f_lo;
  a.nt_out = L.t_hi - L.t_lo;
  a.hop = L.hop;
  a.nperseg = L.nperseg;
  a.n_slots = L.n_slots;
  a.window = reinterpret_cast<const float*>(L.window);
  a.scale = (float)L.scale;
  a.out = reinterpret_cast<float*>(L.out);
  a.tw = reinterpret_cast<const f2*>(L.plan.tw);
  a.post = reinterpret_cast<const f2*>(L.plan.post);
  if (a.nt_out <= 0 || a.nf_out <= 0 || L.n_slots <= 0) return hipSuccess;
  const int q = pk_plan_of(L);
  if (q < 0) return hipErrorInvalidValue;
  // frames per workgroup (FR of the instantiation below)
  const int fr = q == 1 ? 1 : kPkFrames;
  a.per_xcd = (int)(((int64_t)((a.nt_out + fr - 1) / fr) * L.n_slots + 7) / 8);
  const dim3 grid((unsigned)(8 * a.per_xcd));
  const size_t lds = (size_t)(kPkPlans[q].P + kPkPlans[q].P / 16 + 1) * sizeof(f2);
  auto go = [&](auto kern) {
    if (lds > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, grid, dim3(q == 1 ? kPk9600Threads : kThreads38), lds, s, a);
    return hipGetLastError();
  };
  const bool i16 = L.dtype == FT8_I16;
  switch (q) {
    case 0:
      return i16 ? go(k_stft_pk<int16_t, kThreads38, kPkFrames, 3200, 8, 5, 5>)
                 : go(k_stft_pk<float, kThreads38, kPkFrames, 3200, 8, 5, 5>);
    case 1:
      return i16 ? go(k_stft_pk<int16_t, kPk9600Threads, 1, 9600, 8, 15, 5>)
                 : go(k_stft_pk<float, kPk9600Threads, 1, 9600, 8, 15, 5>);
    default:
      return i16 ? go(k_stft_pk<int16_t, kThreads38, kPkFrames, 960, 4, 15>)
                 : go(k_stft_pk<float, kThreads38, kPkFrames, 960, 4, 15>);
  }
}

}  // namespace ft8
