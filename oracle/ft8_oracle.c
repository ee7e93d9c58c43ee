/*
 * oracle/ft8_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference FT8 receive path (Rintazero/ft8_demodulator,
 * src/ft8_tools/ft8_demodulator/ sources) used as the parity checker for the HIP kernels and as the
 * timed "port" CPU baseline in bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path (ft8_demodulator_amd) never does.
 *
 * Every function states the reference lines it follows.  Pinned against golden vectors captured
 * from the reference itself (tests/golden/, generator tools/make_golden.py): candidate lists,
 * scores, LLRs, BP outputs and CRCs are compared bit-for-bit in tests/test_oracle_golden.py.
 *
 * Numerics that matter for bit-exactness (see DESIGN.md "Parity"):
 *   - float32 waterfalls (every WAV) keep the Costas score in float32, accumulated in reference
 *     order (NumPy-2 scalar promotion, ft8_decode.py:57,80-100); float64 waterfalls use double.
 *   - LLRs and BP are double; the LLR normalisation reproduces NumPy's pairwise summation
 *     (np.mean, ft8_decode.py:193-194).
 *   - build with -ffp-contract=off: NumPy evaluates every polynomial without FMA.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../ft8_demodulator_amd/csrc/ft8_ldpc_tables.h"

static const int kCostas[7] = {3, 1, 4, 0, 6, 5, 2};  /* ft8_decode.py:42 */
static const int kGray[8] = {0, 1, 3, 2, 5, 6, 4, 7};  /* ft8_decode.py:39 */
static const uint16_t kChkStart[FT8_LDPC_M + 1] = FT8_CHK_START_INIT;
static const uint8_t kEdgeVar[FT8_LDPC_E] = FT8_EDGE_VAR_INIT;
static const uint16_t kVarEdge[FT8_LDPC_N * 3] = FT8_VAR_EDGE_INIT;

/* Python floor division (ft8_decode.py:59,168 use `//`). */
static inline int floordiv(int a, int b) {
  int q = a / b;
  if ((a % b) != 0 && ((a < 0) != (b < 0))) q--;
  return q;
}

/* ------------------------------------------------------------------------------------------ */
/* Costas sync score: ft8_decode.py:47-100, FT8Candidate.get_log_power ftx_types.py:45-47.     */
/* mag element (freq fi, time ti) lives at mag[fi*sf + ti*st].                                 */
/* ------------------------------------------------------------------------------------------ */
#define DEFINE_SCORE(NAME, T)                                                                  \
  T NAME(const T* mag, long sf, long st, int num_blocks, int sps, int bpt, int at, int af) {  \
    T score = (T)0;                                                                            \
    int n = 0;                                                                                 \
    const int base = floordiv(at, sps);                                                        \
    for (int m = 0; m < 3; ++m) {                                                              \
      for (int k = 0; k < 7; ++k) {                                                            \
        const int block = 36 * m + k;                                                          \
        const int ba = base + block;                                                           \
        if (ba < 0 || ba >= num_blocks) continue;                                              \
        const int tone = kCostas[k];                                                           \
        const long t0 = (long)at + (long)block * sps;                                          \
        const long f0 = (long)af + (long)tone * bpt;                                           \
        const T p = mag[f0 * sf + t0 * st];                                                    \
        if (tone > 0) { score += (T)(p - mag[(f0 - bpt) * sf + t0 * st]); n++; }              \
        if (tone < 7) { score += (T)(p - mag[(f0 + bpt) * sf + t0 * st]); n++; }              \
        if (k > 0 && ba > 0) { score += (T)(p - mag[f0 * sf + (t0 - sps) * st]); n++; }      \
        if (k < 6 && ba + 1 < num_blocks) { score += (T)(p - mag[f0 * sf + (t0 + sps) * st]); n++; } \
      }                                                                                        \
    }                                                                                          \
    if (n == 0 || isnan(score) || isinf(score)) return (T)-INFINITY;                          \
    return score / (T)n;                                                                       \
  }

DEFINE_SCORE(orc_sync_score_f32, float)
DEFINE_SCORE(orc_sync_score_f64, double)

/* Full candidate grid, ft8_decode.py:108-109 (time outer, freq inner).  out[NT*NF] scan order. */
#define DEFINE_GRID(NAME, SCORE, T)                                                            \
  void NAME(const T* mag, long sf, long st, int F, int Tn, int sps, int bpt, T* out) {         \
    const int num_blocks = Tn / sps;                                                           \
    const int t_lo = -10 * sps, t_hi = num_blocks * sps - sps * (58 + 1);                      \
    const int f_hi = F - 7 * bpt;                                                              \
    long i = 0;                                                                                \
    for (int at = t_lo; at < t_hi; ++at)                                                       \
      for (int af = 0; af < f_hi; ++af) out[i++] = SCORE(mag, sf, st, num_blocks, sps, bpt, at, af); \
  }

DEFINE_GRID(orc_score_grid_f32, orc_sync_score_f32, float)
DEFINE_GRID(orc_score_grid_f64, orc_sync_score_f64, double)

/* ------------------------------------------------------------------------------------------ */
/* Candidate selection with the reference's heap semantics, ft8_decode.py:113-140.             */
/* The heap holds (-score, cand); CPython heapq siftdown/siftup.  Exact ties reaching a heap    */
/* comparison raise TypeError in the reference (FT8Candidate has no ordering); here they are    */
/* broken by scan index and reported through *tie_flag.                                        */
/* ------------------------------------------------------------------------------------------ */
typedef struct { double neg; long idx; } hitem;

static int h_less(hitem a, hitem b, int* tie) {
  if (a.neg < b.neg) return 1;
  if (a.neg > b.neg) return 0;
  *tie = 1;
  return a.idx < b.idx;
}
static void h_siftdown(hitem* h, long start, long pos, int* tie) {
  hitem nw = h[pos];
  while (pos > start) {
    long pp = (pos - 1) >> 1;
    if (h_less(nw, h[pp], tie)) { h[pos] = h[pp]; pos = pp; continue; }
    break;
  }
  h[pos] = nw;
}
static void h_siftup(hitem* h, long len, long pos, int* tie) {
  long start = pos;
  hitem nw = h[pos];
  long c = 2 * pos + 1;
  while (c < len) {
    long r = c + 1;
    if (r < len && !h_less(h[c], h[r], tie)) c = r;
    h[pos] = h[c];
    pos = c;
    c = 2 * pos + 1;
  }
  h[pos] = nw;
  h_siftdown(h, start, pos, tie);
}

/* scores[NT*NF] in scan order (float or double given by is_f64).  min_score compared in the
 * score's dtype unless cmp_f64 (NumPy: a Python scalar adopts the array dtype).
 * Writes up to N selected scan indices in final order; returns count.  */
long orc_select(const void* scores, int is_f64, long total, long N, double min_score, int cmp_f64,
                long* out_idx, double* out_score, int* tie_flag) {
  hitem* h = (hitem*)malloc(sizeof(hitem) * (size_t)(N > 0 ? N : 1));
  long len = 0;
  int tie = 0;
  const float ms32 = (float)min_score;
  for (long i = 0; i < total; ++i) {
    double s;
    int skip;
    if (is_f64) {
      s = ((const double*)scores)[i];
      skip = (s == -INFINITY) || (s < min_score);
    } else {
      float s32 = ((const float*)scores)[i];
      s = s32;
      skip = (s32 == -INFINITY) || (cmp_f64 ? ((double)s32 < min_score) : (s32 < ms32));
    }
    if (skip) continue;
    hitem it = {-s, i};
    if (len < N) {
      h[len] = it;
      len++;
      h_siftdown(h, 0, len - 1, &tie);
    } else if (len > 0 && -s < h[0].neg) {
      h[0] = it;
      h_siftup(h, len, 0, &tie);
    }
  }
  /* sorted(candidates, key=lambda x: x[0]): stable on heap-array order */
  for (long a = 1; a < len; ++a) {
    hitem v = h[a];
    long b = a - 1;
    while (b >= 0 && h[b].neg > v.neg) { h[b + 1] = h[b]; b--; }
    h[b + 1] = v;
  }
  for (long a = 0; a < len; ++a) { out_idx[a] = h[a].idx; out_score[a] = -h[a].neg; }
  free(h);
  *tie_flag = tie;
  return len;
}

/* ------------------------------------------------------------------------------------------ */
/* LLR extraction, ft8_decode.py:151-188; normalisation ft8_decode.py:190-198.                 */
/* ------------------------------------------------------------------------------------------ */
static double pymax4(double a, double b, double c, double d) {  /* builtin max: first maximum */
  double m = a;
  if (b > m) m = b;
  if (c > m) m = c;
  if (d > m) m = d;
  return m;
}

#define DEFINE_LLR(NAME, T)                                                                    \
  void NAME(const T* mag, long sf, long st, int num_blocks, int sps, int bpt, int at, int af,  \
            double* log174) {                                                                  \
    const int base = floordiv(at, sps);                                                        \
    for (int k = 0; k < 58; ++k) {                                                             \
      const int sym = k + (k < 29 ? 7 : 14);                                                   \
      const int bi = 3 * k;                                                                    \
      const int block = base + sym;                                                            \
      if (block < 0 || block >= num_blocks) {                                                  \
        log174[bi] = 0; log174[bi + 1] = 0; log174[bi + 2] = 0;                                \
        continue;                                                                              \
      }                                                                                        \
      double s[8], s2[8];                                                                      \
      for (int i = 0; i < 8; ++i)                                                              \
        s[i] = (double)mag[((long)af + (long)i * bpt) * sf + ((long)at + (long)sym * sps) * st]; \
      for (int j = 0; j < 8; ++j) s2[j] = s[kGray[j]];                                         \
      log174[bi + 0] = pymax4(s2[4], s2[5], s2[6], s2[7]) - pymax4(s2[0], s2[1], s2[2], s2[3]); \
      log174[bi + 1] = pymax4(s2[2], s2[3], s2[6], s2[7]) - pymax4(s2[0], s2[1], s2[4], s2[5]); \
      log174[bi + 2] = pymax4(s2[1], s2[3], s2[5], s2[7]) - pymax4(s2[0], s2[2], s2[4], s2[6]); \
    }                                                                                          \
  }

DEFINE_LLR(orc_llr_f32, float)
DEFINE_LLR(orc_llr_f64, double)

/* NumPy's pairwise summation for contiguous float64 (loops_utils.h.src, PW_BLOCKSIZE 128). */
double orc_pairwise_sum(const double* a, long n) {
  if (n < 8) {
    double res = -0.0;
    for (long i = 0; i < n; ++i) res += a[i];
    return res;
  } else if (n <= 128) {
    double r[8], res;
    long i;
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  } else {
    long n2 = n / 2;
    n2 -= n2 % 8;
    return orc_pairwise_sum(a, n2) + orc_pairwise_sum(a + n2, n - n2);
  }
}

/* ftx_normalize_logl, ft8_decode.py:190-198 (np.mean = add.reduce(identity 0) / count). */
void orc_normalize(double* x) {
  double mean = (0.0 + orc_pairwise_sum(x, 174)) / 174.0;
  double d[174];
  for (int i = 0; i < 174; ++i) { double t = x[i] - mean; d[i] = t * t; }
  double var = (0.0 + orc_pairwise_sum(d, 174)) / 174.0;
  double nf = sqrt(24.0 / var);
  for (int i = 0; i < 174; ++i) x[i] *= nf;
}

/* ------------------------------------------------------------------------------------------ */
/* LDPC BP, ldpc_decoder.py:11-113.                                                            */
/* ------------------------------------------------------------------------------------------ */
static double fast_tanh(double x) {  /* ldpc_decoder.py:11-21 */
  if (x < -4.97) x = -4.97;
  if (x > 4.97) x = 4.97;
  double x2 = x * x;
  double a = x * (945.0 + x2 * (105.0 + x2));
  double b = 945.0 + x2 * (420.0 + x2 * 15.0);
  return a / b;
}
static double fast_atanh(double x) {  /* ldpc_decoder.py:23-31 */
  double x2 = x * x;
  double a = x * (945.0 + x2 * (-735.0 + x2 * 64.0));
  double b = (945.0 + x2 * (-1050.0 + x2 * 225.0));
  return a / b;
}

int orc_ldpc_check(const uint8_t* cw) {  /* ldpc_decoder.py:33-52 */
  int errors = 0;
  for (int m = 0; m < FT8_LDPC_M; ++m) {
    int x = 0;
    for (int e = kChkStart[m]; e < kChkStart[m + 1]; ++e) x ^= cw[kEdgeVar[e]];
    if (x) errors++;
  }
  return errors;
}

/* tov[n][j] is the message on edge kVarEdge[3n+j]; toc per check row position. */
int orc_bp_decode(const double* cw, int max_iter, uint8_t* plain) {  /* ldpc_decoder.py:54-113 */
  double tov[FT8_LDPC_N][3];
  double toc[FT8_LDPC_E];
  memset(tov, 0, sizeof(tov));
  memset(toc, 0, sizeof(toc));
  memset(plain, 0, FT8_LDPC_N);
  int min_errors = FT8_LDPC_M;
  for (int it = 0; it < max_iter; ++it) {
    int ones = 0;
    for (int n = 0; n < FT8_LDPC_N; ++n) {
      double msg = cw[n] + ((tov[n][0] + tov[n][1]) + tov[n][2]);
      plain[n] = msg > 0;
      ones += plain[n];
    }
    if (ones == 0) break;
    int errors = orc_ldpc_check(plain);
    if (errors < min_errors) {
      min_errors = errors;
      if (errors == 0) break;
    }
    /* variable -> check (ldpc_decoder.py:89-97) */
    for (int m = 0; m < FT8_LDPC_M; ++m) {
      for (int e = kChkStart[m]; e < kChkStart[m + 1]; ++e) {
        int n = kEdgeVar[e];
        double Tnm = cw[n];
        for (int j = 0; j < 3; ++j)
          if (kVarEdge[3 * n + j] != e) Tnm += tov[n][j];
        toc[e] = fast_tanh(-Tnm / 2);
      }
    }
    /* check -> variable (ldpc_decoder.py:100-108) */
    for (int n = 0; n < FT8_LDPC_N; ++n) {
      for (int j = 0; j < 3; ++j) {
        int e = kVarEdge[3 * n + j];
        int m = 0;
        while (!(e >= kChkStart[m] && e < kChkStart[m + 1])) m++;
        double Tmn = 1.0;
        for (int e2 = kChkStart[m]; e2 < kChkStart[m + 1]; ++e2)
          if (kEdgeVar[e2] != n) Tmn *= toc[e2];
        tov[n][j] = -2 * fast_atanh(Tmn);
      }
    }
  }
  return min_errors;
}

/* ------------------------------------------------------------------------------------------ */
/* CRC-14 and the decode epilogue, crc.py:11-54, ft8_decode.py:200-273.                        */
/* ------------------------------------------------------------------------------------------ */
int orc_crc14(const uint8_t* msg, int num_bits) {  /* crc.py:11-39 */
  int rem = 0, ib = 0;
  for (int i = 0; i < num_bits; ++i) {
    if (i % 8 == 0) { rem ^= msg[ib] << 6; ib++; }
    rem = (rem & 0x2000) ? ((rem << 1) ^ 0x2757) : (rem << 1);
  }
  return rem & 0x3FFF;
}

void orc_pack_bits(const uint8_t* bits, int nbits, uint8_t* out) {  /* ft8_decode.py:200-215 */
  int nb = (nbits + 7) / 8;
  memset(out, 0, (size_t)nb);
  for (int i = 0; i < nbits; ++i)
    if (bits[i]) out[i / 8] |= (uint8_t)(0x80 >> (i % 8));
}

/* ft8_decode_candidate tail (ft8_decode.py:236-273).  Returns 1 on success. */
int orc_decode_tail(const uint8_t* plain, int ldpc_errors, uint8_t* payload, int* crc_ext,
                    int* crc_calc) {
  *crc_ext = 0;
  *crc_calc = 0;
  memset(payload, 0, 10);
  if (ldpc_errors > 0) return 0;
  uint8_t a91[12], buf[12];
  orc_pack_bits(plain, 91, a91);
  *crc_ext = ((a91[9] & 7) << 11) | (a91[10] << 3) | (a91[11] >> 5);  /* crc.py:41-54 */
  memcpy(buf, a91, 10);
  buf[9] &= 0xF8;
  buf[10] = 0;
  buf[11] = 0;
  *crc_calc = orc_crc14(buf, 82);
  if (*crc_ext != *crc_calc) return 0;
  memcpy(payload, a91, 10);
  payload[9] &= 0xF8;
  return 1;
}

/* LDPC encode of a 91-bit message (ft8_generator/ldpc.py:104-131) for test synthesis. */
static const uint8_t kGen[FT8_LDPC_M * 12] = FT8_GEN_ROWS_INIT;
void orc_ldpc_encode(const uint8_t* a91, uint8_t* cw22) {
  memset(cw22, 0, 22);
  memcpy(cw22, a91, 12);
  for (int i = 0; i < FT8_LDPC_M; ++i) {
    int nsum = 0;
    for (int j = 0; j < 12; ++j) nsum ^= __builtin_popcount(kGen[i * 12 + j] & a91[j]) & 1;
    int bit = 91 + i;
    if (nsum) cw22[bit / 8] |= (uint8_t)(0x80 >> (bit % 8));
  }
}

/* ------------------------------------------------------------------------------------------ */
/* Whole waterfall -> decoded records (ft8_decode.py:357-391 minus plotting).                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  double score;
  int32_t abs_time, abs_freq;
  int32_t ldpc_errors, crc_extracted, crc_calculated, ok;
  uint8_t payload[10];
  uint8_t _pad[6];
} orc_record;

#define DEFINE_DECODE(NAME, T, GRID, LLR, ISF64)                                              \
  long NAME(const T* mag, long sf, long st, int F, int Tn, int sps, int bpt, long N,           \
            double min_score, int cmp_f64, int max_iter, orc_record* rec, int* tie_flag) {     \
    const int num_blocks = Tn / sps;                                                           \
    const int t_lo = -10 * sps, t_hi = num_blocks * sps - sps * 59;                            \
    const int f_hi = F - 7 * bpt;                                                              \
    if (t_hi <= t_lo || f_hi <= 0 || N <= 0) { *tie_flag = 0; return 0; }                      \
    const long NT = t_hi - t_lo, NF = f_hi;                                                    \
    T* sc = (T*)malloc(sizeof(T) * (size_t)(NT * NF));                                         \
    GRID(mag, sf, st, F, Tn, sps, bpt, sc);                                                    \
    long* idx = (long*)malloc(sizeof(long) * (size_t)N);                                       \
    double* scs = (double*)malloc(sizeof(double) * (size_t)N);                                 \
    long nc = orc_select(sc, ISF64, NT * NF, N, min_score, cmp_f64, idx, scs, tie_flag);       \
    for (long c = 0; c < nc; ++c) {                                                            \
      const int at = (int)(idx[c] / NF) + t_lo, af = (int)(idx[c] % NF);                       \
      double llr[174];                                                                         \
      uint8_t plain[174];                                                                      \
      LLR(mag, sf, st, num_blocks, sps, bpt, at, af, llr);                                     \
      orc_normalize(llr);                                                                      \
      int err = orc_bp_decode(llr, max_iter, plain);                                           \
      orc_record* r = &rec[c];                                                                 \
      memset(r, 0, sizeof(*r));                                                                \
      r->score = scs[c];                                                                       \
      r->abs_time = at;                                                                        \
      r->abs_freq = af;                                                                        \
      r->ldpc_errors = err;                                                                    \
      r->ok = orc_decode_tail(plain, err, r->payload, &r->crc_extracted, &r->crc_calculated);  \
    }                                                                                          \
    free(sc); free(idx); free(scs);                                                            \
    return nc;                                                                                 \
  }

DEFINE_DECODE(orc_decode_waterfall_f32, float, orc_score_grid_f32, orc_llr_f32, 0)
DEFINE_DECODE(orc_decode_waterfall_f64, double, orc_score_grid_f64, orc_llr_f64, 1)
