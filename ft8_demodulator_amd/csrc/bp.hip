// bp.hip -- soft LLRs, LDPC(174,91) belief propagation and the CRC-14 epilogue (gfx950).
//
// One 64-lane wavefront decodes one candidate; workgroups are single waves (so __syncthreads is a
// wave-local barrier) and persistent: each pulls candidates from a device-scope work counter until
// the batch is drained, so early-exiting candidates (converged or all-zero) free their wave at
// once and the LDPC tables are loaded into registers once per wave, not per candidate.
//
// Per candidate (reference line numbers in src/ft8_tools/ft8_demodulator/):
//   LLR          ft8_extract_likelihood / ft8_extract_symbol (ft8_decode.py:151-188): lanes 0..57
//                own one data symbol each, gather its 8 tone powers, Gray map, max-log LLRs.
//   normalise    ftx_normalize_logl (ft8_decode.py:190-198): mean and variance reproduce NumPy's
//                pairwise summation order exactly (8 accumulators, blocks of 80 + 94) and
//                sqrt(24/var) is correctly rounded, so LLRs are bit-identical to the reference.
//   BP           bp_decode (ldpc_decoder.py:54-113) in float64, edge-parallel: the 522 Tanner-graph
//                edges are dealt to lanes (9 per lane); variable->check and check->variable
//                messages live in LDS (tov, toc: 2 x 4.2 KB) and every sum/product is evaluated in
//                the reference's order, without FMA contraction (-ffp-contract=off), so hard
//                decisions match bit for bit.
//   CRC          pack_bits + extract_crc + compute_crc (ft8_decode.py:200-273, crc.py:11-54).
//
// Roofline: the kernel touches < 2 KB of HBM per candidate; it is bound by float64 VALU issue
// (two IEEE divisions per edge per iteration, ~30 float64 ops per edge per iteration).
#include "ft8_internal.h"

namespace ft8 {
namespace {

__constant__ uint16_t kChkStartD[FT8_LDPC_M + 1] = FT8_CHK_START_INIT;
__constant__ uint8_t kEdgeVarD[FT8_LDPC_E] = FT8_EDGE_VAR_INIT;
__constant__ uint16_t kVarEdgeD[FT8_LDPC_N * 3] = FT8_VAR_EDGE_INIT;
__constant__ uint8_t kEdgeChkD[FT8_LDPC_E] = FT8_EDGE_CHK_INIT;
__constant__ int kGrayD[8] = {0, 1, 3, 2, 5, 6, 4, 7};  // ft8_decode.py:39

constexpr int kEdgeSlots = (FT8_LDPC_E + kWave - 1) / kWave;  // 9
constexpr int kVarSlots = (FT8_LDPC_N + kWave - 1) / kWave;   // 3
constexpr int kChkSlots = (FT8_LDPC_M + kWave - 1) / kWave;   // 2

__device__ __forceinline__ double fast_tanh(double x) {  // ldpc_decoder.py:11-21
  x = x < -4.97 ? -4.97 : x;
  x = x > 4.97 ? 4.97 : x;
  const double x2 = x * x;
  const double a = x * (945.0 + x2 * (105.0 + x2));
  const double b = 945.0 + x2 * (420.0 + x2 * 15.0);
  return a / b;
}
__device__ __forceinline__ double fast_atanh(double x) {  // ldpc_decoder.py:23-31
  const double x2 = x * x;
  const double a = x * (945.0 + x2 * (-735.0 + x2 * 64.0));
  const double b = (945.0 + x2 * (-1050.0 + x2 * 225.0));
  return a / b;
}

// correctly rounded sqrt (math.sqrt): hardware estimate + Tuckerman's test with exact fma residuals
__device__ double sqrt_rn(double x) {
  double y = __builtin_sqrt(x);
  if (!(x > 0.0) || __builtin_isinf(x)) return y;
  for (int it = 0; it < 4; ++it) {
    const double lo = __longlong_as_double(__double_as_longlong(y) - 1);
    const double hi = __longlong_as_double(__double_as_longlong(y) + 1);
    if (__builtin_fma(y, lo, -x) >= 0.0) { y = lo; continue; }   // y*y^- >= x: too large
    if (__builtin_fma(y, hi, -x) < 0.0) { y = hi; continue; }    // y*y^+ <  x: too small
    break;
  }
  return y;
}

__device__ __forceinline__ double pymax4(double a, double b, double c, double d) {
  double m = a;          // builtin max(): first maximum under '>'
  m = b > m ? b : m;
  m = c > m ? c : m;
  m = d > m ? d : m;
  return m;
}

struct WaveTables {
  uint32_t vc[kEdgeSlots];   // var n | other edge a << 8 | other edge b << 18
  uint32_t cv[kEdgeSlots];   // check start | degree << 10 | position << 13
  uint32_t hd[kVarSlots];    // e0 | e1 << 10 | e2 << 20
  uint32_t pc[kChkSlots][2]; // variables of the check (8 bits each), up to 7
  uint32_t pd[kChkSlots];    // degree (0 if slot unused)
};

__device__ void load_tables(WaveTables& t, int lane) {
#pragma unroll
  for (int i = 0; i < kEdgeSlots; ++i) {
    const int e = lane + kWave * i;
    t.vc[i] = 0;
    t.cv[i] = 0;
    if (e < FT8_LDPC_E) {
      const int n = kEdgeVarD[e];
      int o[2], k = 0;
      for (int j = 0; j < 3; ++j) {
        const int ej = kVarEdgeD[3 * n + j];
        if (ej != e) o[k++] = ej;
      }
      t.vc[i] = (uint32_t)n | ((uint32_t)o[0] << 8) | ((uint32_t)o[1] << 18);
      const int m = kEdgeChkD[e];
      const int s = kChkStartD[m], d = kChkStartD[m + 1] - s;
      t.cv[i] = (uint32_t)s | ((uint32_t)d << 10) | ((uint32_t)(e - s) << 13);
    }
  }
#pragma unroll
  for (int i = 0; i < kVarSlots; ++i) {
    const int n = lane + kWave * i;
    t.hd[i] = 0;
    if (n < FT8_LDPC_N)
      t.hd[i] = (uint32_t)kVarEdgeD[3 * n] | ((uint32_t)kVarEdgeD[3 * n + 1] << 10) |
                ((uint32_t)kVarEdgeD[3 * n + 2] << 20);
  }
#pragma unroll
  for (int i = 0; i < kChkSlots; ++i) {
    const int m = lane + kWave * i;
    t.pc[i][0] = t.pc[i][1] = 0;
    t.pd[i] = 0;
    if (m < FT8_LDPC_M) {
      const int s = kChkStartD[m], d = kChkStartD[m + 1] - s;
      t.pd[i] = d;
      for (int j = 0; j < d; ++j) t.pc[i][j >> 2] |= (uint32_t)kEdgeVarD[s + j] << (8 * (j & 3));
    }
  }
}

struct BpArgs {
  const void* wf;
  int wf_f64, T, F, sps, bpt, num_blocks;
  const int32_t* cand;
  const double* cand_score;
  const int32_t* cand_count;
  int N, n_items, mode;
  const double* llr_in;
  int normalize, max_iterations, llr_only;
  double* llr_out;
  uint8_t* plain_out;
  ft8_result* res;
  unsigned* work;
  unsigned long long* stats;  // nullable: [candidates, iterations entered, message passes, converged]
};

struct WaveLds {
  double c[FT8_LDPC_N];
  double tov[FT8_LDPC_E];
  double toc[FT8_LDPC_E];
  double part[16];
  uint8_t bits[FT8_LDPC_N + 2];
  uint8_t a91[12];
  int flag[2];
};

// numpy pairwise sum (loops_utils.h.src) of x[0..174): pw(0,80) + pw(80,94), result in lane 0
__device__ double pairwise174(const double* x, double* part, int lane) {
  if (lane < 8) {
    double r = x[lane];
    for (int i = 8; i < 80; i += 8) r += x[i + lane];
    part[lane] = r;
  } else if (lane < 16) {
    const int j = lane - 8;
    double r = x[80 + j];
    for (int i = 8; i < 88; i += 8) r += x[80 + i + j];
    part[lane] = r;
  }
  __syncthreads();
  double tot = 0.0;
  if (lane == 0) {
    const double s1 = ((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]));
    double s2 = ((part[8] + part[9]) + (part[10] + part[11])) + ((part[12] + part[13]) + (part[14] + part[15]));
    for (int i = 168; i < 174; ++i) s2 += x[i];
    tot = 0.0 + (s1 + s2);  // add.reduce starts from the identity
  }
  __syncthreads();
  return __shfl(tot, 0);
}

template <typename T>
__device__ void extract_llr(const BpArgs& a, const T* wf, int at, int af, double* c, int lane) {
  // ft8_extract_likelihood (ft8_decode.py:164-188)
  if (lane < 58) {
    const int k = lane;
    const int sym = k + (k < 29 ? 7 : 14);
    const int block = floordiv(at, a.sps) + sym;
    double l0 = 0.0, l1 = 0.0, l2 = 0.0;
    if (!(block < 0 || block >= a.num_blocks)) {
      const T* row = wf + (int64_t)(at + sym * a.sps) * a.F + af;
      double s[8], s2[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = (double)row[i * a.bpt];
#pragma unroll
      for (int j = 0; j < 8; ++j) s2[j] = s[kGrayD[j]];
      l0 = pymax4(s2[4], s2[5], s2[6], s2[7]) - pymax4(s2[0], s2[1], s2[2], s2[3]);
      l1 = pymax4(s2[2], s2[3], s2[6], s2[7]) - pymax4(s2[0], s2[1], s2[4], s2[5]);
      l2 = pymax4(s2[1], s2[3], s2[5], s2[7]) - pymax4(s2[0], s2[2], s2[4], s2[6]);
    }
    c[3 * k] = l0;
    c[3 * k + 1] = l1;
    c[3 * k + 2] = l2;
  }
}

__global__ __launch_bounds__(kWave) void k_bp(BpArgs a) {
  __shared__ WaveLds L;
  const int lane = threadIdx.x;
  WaveTables tb;
  load_tables(tb, lane);

  for (;;) {
    unsigned item = 0;
    if (lane == 0) item = atomicAdd(a.work, 1u);
    item = __shfl(item, 0);
    if ((int)item >= a.n_items) break;

    // ---- candidate --------------------------------------------------------------------------
    int slot = 0, at = 0, af = 0, cidx = 0;
    double score = 0.0;
    if (a.mode == 0) {
      slot = item / a.N;
      cidx = item % a.N;
      if (cidx >= a.cand_count[slot]) continue;
      at = a.cand[((int64_t)slot * a.N + cidx) * 2];
      af = a.cand[((int64_t)slot * a.N + cidx) * 2 + 1];
      score = a.cand_score[(int64_t)slot * a.N + cidx];
    } else if (a.mode == 1) {
      slot = a.cand[(int64_t)item * 3];
      at = a.cand[(int64_t)item * 3 + 1];
      af = a.cand[(int64_t)item * 3 + 2];
    }

    // ---- LLRs -------------------------------------------------------------------------------
    if (a.mode == 2) {
      for (int n = lane; n < FT8_LDPC_N; n += kWave) L.c[n] = a.llr_in[(int64_t)item * FT8_LDPC_N + n];
    } else if (a.wf_f64) {
      extract_llr<double>(a, reinterpret_cast<const double*>(a.wf) + (int64_t)slot * a.T * a.F, at, af, L.c, lane);
    } else {
      extract_llr<float>(a, reinterpret_cast<const float*>(a.wf) + (int64_t)slot * a.T * a.F, at, af, L.c, lane);
    }
    __syncthreads();
    if (a.normalize) {  // ftx_normalize_logl (ft8_decode.py:190-198)
      const double mean = pairwise174(L.c, L.part, lane) / 174.0;
      for (int n = lane; n < FT8_LDPC_N; n += kWave) {
        const double d = L.c[n] - mean;
        L.toc[n] = d * d;
      }
      __syncthreads();
      const double var = pairwise174(L.toc, L.part, lane) / 174.0;
      const double nf = sqrt_rn(24.0 / var);
      for (int n = lane; n < FT8_LDPC_N; n += kWave) L.c[n] = L.c[n] * nf;
      __syncthreads();
    }
    if (a.llr_out)
      for (int n = lane; n < FT8_LDPC_N; n += kWave) a.llr_out[(int64_t)item * FT8_LDPC_N + n] = L.c[n];
    if (a.llr_only) continue;

    // ---- belief propagation (ldpc_decoder.py:54-113) ----------------------------------------
    for (int e = lane; e < FT8_LDPC_E; e += kWave) L.tov[e] = 0.0;
    for (int n = lane; n < FT8_LDPC_N + 2; n += kWave) L.bits[n] = 0;
    __syncthreads();
    int min_errors = FT8_LDPC_M;
    int entered = 0, passes = 0;
    for (int iter = 0; iter < a.max_iterations; ++iter) {
      entered++;
      // hard decision: messages = codeword + sum(tov, axis=1) -> c + ((t0 + t1) + t2)
      int ones = 0;
#pragma unroll
      for (int i = 0; i < kVarSlots; ++i) {
        const int n = lane + kWave * i;
        if (n < FT8_LDPC_N) {
          const uint32_t h = tb.hd[i];
          const double sum = (L.tov[h & 1023] + L.tov[(h >> 10) & 1023]) + L.tov[h >> 20];
          const int b = (L.c[n] + sum) > 0.0;
          L.bits[n] = (uint8_t)b;
          ones += b;
        }
      }
      if (!__any(ones != 0)) break;  // np.sum(plain) == 0
      __syncthreads();
      // parity check (ldpc_check, ldpc_decoder.py:33-52)
      int errs = 0;
#pragma unroll
      for (int i = 0; i < kChkSlots; ++i) {
        const int d = tb.pd[i];
        int x = 0;
        for (int j = 0; j < d; ++j) x ^= L.bits[(tb.pc[i][j >> 2] >> (8 * (j & 3))) & 255];
        errs += __popcll(__ballot(x != 0));
      }
      if (errs < min_errors) {
        min_errors = errs;
        if (errs == 0) break;
      }
      // variable -> check: toc = tanh(-(c[n] + others) / 2), others in the variable's check order
#pragma unroll
      for (int i = 0; i < kEdgeSlots; ++i) {
        const int e = lane + kWave * i;
        if (e < FT8_LDPC_E) {
          const uint32_t v = tb.vc[i];
          double t = L.c[v & 255];
          t += L.tov[(v >> 8) & 1023];
          t += L.tov[v >> 18];
          L.toc[e] = fast_tanh(-t / 2);
        }
      }
      __syncthreads();
      // check -> variable: tov = -2 atanh(prod of the other toc of the check, in row order)
#pragma unroll
      for (int i = 0; i < kEdgeSlots; ++i) {
        const int e = lane + kWave * i;
        if (e < FT8_LDPC_E) {
          const uint32_t v = tb.cv[i];
          const int s = v & 1023, d = (v >> 10) & 7, k = v >> 13;
          double p = 1.0;
          for (int j = 0; j < d; ++j)
            if (j != k) p *= L.toc[s + j];
          L.tov[e] = -2 * fast_atanh(p);
        }
      }
      passes++;
      __syncthreads();
    }
    __syncthreads();
    if (a.stats && lane == 0) {
      atomicAdd(&a.stats[0], 1ull);
      atomicAdd(&a.stats[1], (unsigned long long)entered);
      atomicAdd(&a.stats[2], (unsigned long long)passes);
      if (min_errors == 0) atomicAdd(&a.stats[3], 1ull);
    }

    // ---- outputs ------------------------------------------------------------------------------
    if (a.plain_out)
      for (int n = lane; n < FT8_LDPC_N; n += kWave) a.plain_out[(int64_t)item * FT8_LDPC_N + n] = L.bits[n];
    if (a.res) {
      // pack 91 bits MSB first (ft8_decode.py:200-215)
      if (lane < 12) {
        unsigned byte = 0;
        for (int j = 0; j < 8; ++j) {
          const int bi = lane * 8 + j;
          if (bi < 91 && L.bits[bi]) byte |= 0x80u >> j;
        }
        L.a91[lane] = (uint8_t)byte;
      }
      __syncthreads();
      if (lane == 0) {
        ft8_result r;
        r.score = score;
        r.slot = slot;
        r.abs_time = at;
        r.abs_freq = af;
        r.ldpc_errors = (int16_t)min_errors;
        r.cand_index = (uint16_t)cidx;
        r.crc_extracted = 0;
        r.crc_calculated = 0;
        r.ok = 0;
        r.pad = 0;
        for (int i = 0; i < 10; ++i) r.payload[i] = 0;
        if (min_errors == 0) {
          const uint8_t* a91 = L.a91;
          const unsigned ce = ((a91[9] & 7u) << 11) | ((unsigned)a91[10] << 3) | (a91[11] >> 5);
          uint8_t buf[12];
          for (int i = 0; i < 10; ++i) buf[i] = a91[i];
          buf[9] &= 0xF8;
          buf[10] = 0;
          buf[11] = 0;
          unsigned rem = 0;  // crc.py:11-39
          for (int ib = 0; ib < 82; ++ib) {
            if ((ib & 7) == 0) rem ^= (unsigned)buf[ib >> 3] << 6;
            rem = (rem & 0x2000u) ? ((rem << 1) ^ 0x2757u) : (rem << 1);
          }
          const unsigned cc = rem & 0x3FFFu;
          r.crc_extracted = (uint16_t)ce;
          r.crc_calculated = (uint16_t)cc;
          if (ce == cc) {
            r.ok = 1;
            for (int i = 0; i < 10; ++i) r.payload[i] = a91[i];
            r.payload[9] &= 0xF8;
          }
        }
        a.res[item] = r;
      }
    }
    __syncthreads();
  }
}

// one wave per slot: successes in candidate order -> out[slot][0..cap), counts[slot]
__global__ __launch_bounds__(kWave) void k_compact(const ft8_result* res, const int32_t* cand_count,
                                                   int N, ft8_result* out, int32_t* counts, int cap) {
  const int slot = blockIdx.x, lane = threadIdx.x;
  const int nc = cand_count[slot];
  int base = 0;
  for (int c0 = 0; c0 < nc; c0 += kWave) {
    const int c = c0 + lane;
    const bool ok = c < nc && res[(int64_t)slot * N + c].ok;
    const unsigned long long m = __ballot(ok);
    const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
    if (ok && pos < cap) out[(int64_t)slot * cap + pos] = res[(int64_t)slot * N + c];
    base += __popcll(m);
  }
  if (lane == 0) counts[slot] = base;
}

__global__ void k_crc14(const uint8_t* msg, const int32_t* nbits, int n, uint16_t* crc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* m = msg + (int64_t)i * 12;
  const int nb = nbits[i];
  unsigned rem = 0;
  for (int b = 0; b < nb; ++b) {
    if ((b & 7) == 0) rem ^= (unsigned)m[b >> 3] << 6;
    rem = (rem & 0x2000u) ? ((rem << 1) ^ 0x2757u) : (rem << 1);
  }
  crc[i] = (uint16_t)(rem & 0x3FFFu);
}

__global__ void k_ldpc_check(const uint8_t* bits, int n, int32_t* err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* b = bits + (int64_t)i * FT8_LDPC_N;
  int e = 0;
  for (int m = 0; m < FT8_LDPC_M; ++m) {
    int x = 0;
    for (int j = kChkStartD[m]; j < kChkStartD[m + 1]; ++j) x ^= b[kEdgeVarD[j]];
    e += x != 0;
  }
  err[i] = e;
}

}  // namespace

hipError_t launch_bp(const BpLaunch& L, hipStream_t s) {
  if (L.n_items <= 0) return hipSuccess;
  BpArgs a{};
  a.wf = L.wf;
  a.wf_f64 = L.wf_f64;
  a.T = L.T;
  a.F = L.F;
  a.sps = L.sps;
  a.bpt = L.bpt;
  a.num_blocks = L.sps > 0 ? L.T / L.sps : 0;
  a.cand = L.cand;
  a.cand_score = L.cand_score;
  a.cand_count = L.cand_count;
  a.N = L.N;
  a.n_items = L.n_items;
  a.mode = L.mode;
  a.llr_in = L.llr_in;
  a.normalize = L.normalize;
  a.max_iterations = L.max_iterations;
  a.llr_only = L.llr_only;
  a.llr_out = L.llr_out;
  a.plain_out = L.plain_out;
  a.res = L.res;
  a.work = L.work;
  a.stats = L.stats;
  hipError_t e = hipMemsetAsync(L.work, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  const int waves = min(L.n_items, 256 * 24);  // 24 single-wave workgroups per CU
  hipLaunchKernelGGL(k_bp, dim3(waves), dim3(kWave), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_compact(const CompactLaunch& L, hipStream_t s) {
  if (L.n_slots <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_compact, dim3(L.n_slots), dim3(kWave), 0, s, L.res, L.cand_count, L.N, L.out,
                     L.counts, L.cap);
  return hipGetLastError();
}

hipError_t launch_crc14(const uint8_t* msg, const int32_t* nbits, int n, uint16_t* crc, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_crc14, dim3((n + 255) / 256), dim3(256), 0, s, msg, nbits, n, crc);
  return hipGetLastError();
}

hipError_t launch_ldpc_check(const uint8_t* bits, int n, int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ldpc_check, dim3((n + 255) / 256), dim3(256), 0, s, bits, n, err);
  return hipGetLastError();
}

}  // namespace ft8
