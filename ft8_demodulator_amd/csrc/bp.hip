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
//                messages live in LDS (one 4.6 KB array, see WaveLds) and every sum/product is evaluated in
//                the reference's order, without FMA contraction (-ffp-contract=off), so hard
//                decisions match bit for bit.
//   CRC          pack_bits + extract_crc + compute_crc (ft8_decode.py:200-273, crc.py:11-54).
//
// Roofline: the kernel touches < 2 KB of HBM per candidate; it is bound by float64 VALU issue
// (two IEEE divisions per edge per iteration, ~30 float64 ops per edge per iteration).
#include "ft8_internal.h"
#include "heap_replay.h"

namespace ft8 {
namespace {

__constant__ uint16_t kChkStartD[FT8_LDPC_M + 1] = FT8_CHK_START_INIT;
__constant__ uint8_t kEdgeVarD[FT8_LDPC_E] = FT8_EDGE_VAR_INIT;
__constant__ uint16_t kVarEdgeD[FT8_LDPC_N * 3] = FT8_VAR_EDGE_INIT;
__constant__ uint8_t kEdgeChkD[FT8_LDPC_E] = FT8_EDGE_CHK_INIT;
constexpr int kGrayD[8] = {0, 1, 3, 2, 5, 6, 4, 7};  // ft8_decode.py:39

constexpr int kEdgeSlots = (FT8_LDPC_E + kWave - 1) / kWave;  // 9
constexpr int kVarSlots = (FT8_LDPC_N + kWave - 1) / kWave;   // 3
constexpr int kChkSlots = (FT8_LDPC_M + kWave - 1) / kWave;   // 2
// Every lane owns kEdgeSlots edges, kVarSlots bits and kChkSlots checks; the tails are padded with
// dummy edges/bits/checks that read and write only padding slots of the LDS arrays, so the three
// phases are branch-free and the per-lane chains (18 IEEE divisions per sweep) interleave.

// Fixed kernel shape (round 3: the build-time experiment switches of round 2 are gone; DESIGN.md
// section 3 lists what each alternative measured, and the fault one of them caused).  Divisions are
// interleaved three at a time: a variable's three edges, and the nine edge slots of the edge-major
// phase in three groups.  A group size that does not divide kEdgeSlots indexes past the lane's
// register arrays -- undefined behaviour, which the compiler answers by deleting the divisions -- so
// it is pinned and asserted here.
constexpr int kDivGroup = 3;
static_assert(kEdgeSlots % kDivGroup == 0 && kVarSlots == kDivGroup, "division groups tile the slots exactly");
constexpr int kProdGroup = 3;  // check products between scheduling fences (register pressure)
static_assert(kEdgeSlots % kProdGroup == 0, "product groups tile the edge slots");
// Resident waves per SIMD the persistent grid is sized for.  The compiler is given a 3-wave register
// budget: under a 4-wave budget (128 VGPRs) the allocator spills ~50 VGPRs of the fused sweep to
// scratch, while under the 3-wave budget it needs only 123 -- which still leaves 4 waves resident
// per SIMD (512 / 128).
constexpr int kBpWavesPerSimd = 4;
constexpr int kBpLbWaves = 3;
constexpr int kBpGridCus = 256;        // MI355X: 256 CUs
constexpr double kClip2 = 2.0 * 4.97;  // exact: twice fast_tanh's clip bound

// LDS address-space view of a byte address (the product-factor reads compute raw LDS addresses)
typedef __attribute__((address_space(3))) const double lds_f64;
typedef __attribute__((address_space(3))) const uint64_t lds_u64;

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

// IEEE-754 double division, the exact instruction sequence hipcc emits for `x / y` on gfx950
// (div_scale x2, rcp, two Newton steps, mul, fma, div_fmas, div_fixup), written with builtins so
// that N independent divisions can be interleaved stage by stage (ILP N) with bit-identical results.
//
// Fast path: v_div_scale_f64 returns its operand unchanged (VCC = 0) unless the denominator is
// zero / denormal / has a denormal reciprocal, the quotient is denormal, the exponents differ by
// >= 768, or the numerator's biased exponent is <= 53 (|x| < 2^-969); v_div_fixup_f64 returns the
// quotient unchanged for finite normal operands and quotient.  Every denominator here lies in
// [67, 2.1e4] (fast_tanh: 945 + x^2 (420 + 15 x^2) with |x| <= 4.97; fast_atanh: 945 + x^2 (-1050 +
// 225 x^2) with |x| <= 1.0072^6) and every numerator below 2.1e4, so when every numerator of the
// wave satisfies |x| >= 2^-960 the scale/fmas/fixup steps are identities and the short sequence
// below produces the same bits (measured: ~59 vs ~78 SIMD-cycles per wave division).  Otherwise
// the full sequence runs.
//
// NEG2: y holds -b/2 for the reference's denominator b and the result is -2 RN(x/b) (fast_atanh's
// caller scales by -2, ldpc_decoder.py:108).  On the fast path every quotient is normal, so
// RN(x / (-b/2)) == -2 RN(x/b) exactly and the scaling costs nothing; the full path divides by
// b = -2 y (exact) and scales the quotient.
// the short sequence alone, for callers that established its preconditions themselves
template <int N>
__device__ __forceinline__ void div_fast(double* q, const double* x, const double* y) {
  double r[N], e[N], m[N];
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = __builtin_amdgcn_rcp(y[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = __builtin_fma(-y[i], r[i], 1.0);
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = __builtin_fma(r[i], e[i], r[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = __builtin_fma(-y[i], r[i], 1.0);
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = __builtin_fma(r[i], e[i], r[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) m[i] = x[i] * r[i];
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = __builtin_fma(-y[i], m[i], x[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) q[i] = __builtin_fma(e[i], r[i], m[i]);
}

template <int N, bool NEG2 = false>
__device__ __forceinline__ void div_rn(double* q, const double* x, const double* y_in, int fast = 0) {
  // |x| < 2^900 always holds here (clamped / bounded inputs).  A NaN numerator yields NaN on either
  // path (only its payload could differ, which no later comparison or clip can observe), so the
  // test is on the smallest |x| alone: two v_min + one compare per group, and one ballot -- unless
  // the caller established the short path for the whole wave (fast)
  int ok = fast;
  if (!ok) {
    double mn = __builtin_fabs(x[0]);
#pragma unroll
    for (int i = 1; i < N; ++i) mn = __builtin_fmin(mn, __builtin_fabs(x[i]));
    ok = __ballot(mn >= 0x1p-960) == __builtin_amdgcn_read_exec() ? 1 : 0;
  }
  double r[N], e[N], m[N];
  if (ok) {
#pragma unroll
    for (int i = 0; i < N; ++i) r[i] = __builtin_amdgcn_rcp(y_in[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = __builtin_fma(-y_in[i], r[i], 1.0);
#pragma unroll
    for (int i = 0; i < N; ++i) r[i] = __builtin_fma(r[i], e[i], r[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = __builtin_fma(-y_in[i], r[i], 1.0);
#pragma unroll
    for (int i = 0; i < N; ++i) r[i] = __builtin_fma(r[i], e[i], r[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) m[i] = x[i] * r[i];
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = __builtin_fma(-y_in[i], m[i], x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) q[i] = __builtin_fma(e[i], r[i], m[i]);
    return;
  }
  double den[N], num[N], y[N];
  bool f0[N], f1[N];
#pragma unroll
  for (int i = 0; i < N; ++i) y[i] = NEG2 ? -2.0 * y_in[i] : y_in[i];
#pragma unroll
  for (int i = 0; i < N; ++i) den[i] = __builtin_amdgcn_div_scale(x[i], y[i], false, &f0[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = __builtin_amdgcn_rcp(den[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) num[i] = __builtin_amdgcn_div_scale(x[i], y[i], true, &f1[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = __builtin_fma(-den[i], r[i], 1.0);
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = __builtin_fma(r[i], e[i], r[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = __builtin_fma(-den[i], r[i], 1.0);
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = __builtin_fma(r[i], e[i], r[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) m[i] = num[i] * r[i];
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = __builtin_fma(-den[i], m[i], num[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) q[i] = __builtin_amdgcn_div_fmas(e[i], r[i], m[i], f1[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) q[i] = __builtin_amdgcn_div_fixup(q[i], y[i], x[i]);
  if constexpr (NEG2) {
#pragma unroll
    for (int i = 0; i < N; ++i) q[i] = -2.0 * q[i];
  }
  (void)f0;
}

// ---- k_bp message layout ---------------------------------------------------------------------
// One LDS array holds both message sets: a sweep phase loads everything it needs before it stores
// (the workgroup is one lockstep wave), so toc overwrites tov in place and vice versa.
//
// Row-position-major layout.  Checks are renumbered degree-7 first (m' = 0..23 the degree-7 rows,
// 24..82 the degree-6 rows, each group in check order).  The message of edge (m', q), q being the
// edge's position in its check's row (the reference's n_idx, ldpc_decoder.py:85-87, 103-105), lives
// at index q * 83 + m' (q < 6) or 498 + m' (q = 6, m' < 24); indices 522..583 hold the constant
// 1.0 that stands in for a degree-6 row's missing seventh factor (1.0 * t == t exactly).  Hence:
//   * factor f of row m' sits at byte 8 m' + 664 f from the array: a row base plus a compile-time
//     immediate, so the check products need no per-factor address arithmetic;
//   * edge-major phases (fast_tanh, products, fast_atanh) own index lane + 64 i: the lane address
//     plus an immediate;
//   * edge slot i (indices 64 i .. 64 i + 63) holds one row position q, or two adjacent ones qa and
//     qa + 1 (83 > 64).  The product of "every factor but q" in row order then has, at chain
//     position qa, t[qa + 1] for the q = qa lanes and t[qa] for the q = qa + 1 lanes -- one
//     per-lane address; every other factor is common to both groups.
// The per-variable (174 x 3 edge) addresses of the variable-major phase are per-lane tables.
constexpr int kM7 = 24;                              // degree-7 checks (FT8 LDPC(174,91))
constexpr int kQS = FT8_LDPC_M;                      // index stride of one row position (83)
constexpr int kQ6 = 6 * kQS;                         // first index of row position 6 (498)
constexpr int kMsgN = 584;                           // 498 + 83 = 581 used, rounded to 8
constexpr int kOne = kMsgN - 1;                      // a constant 1.0 (padding variables read it)
constexpr int kHdr = 1024;                           // LDS bytes before msg (lane addr - 664 > 0)
static_assert(kEdgeSlots * kWave <= kMsgN && kQ6 + kM7 == FT8_LDPC_E, "row-major message layout");

__host__ __device__ constexpr int q_of(int idx) { return idx < kQ6 ? idx / kQS : 6; }
__host__ __device__ constexpr int qa_of(int i) { return q_of(kWave * i); }
__host__ __device__ constexpr bool mixed_slot(int i) { return q_of(kWave * i + kWave - 1) != q_of(kWave * i); }
// first lane of slot i whose row position is qa + 1 (mixed slots)
__host__ __device__ constexpr int hi_lane(int i) { return kQS * (qa_of(i) + 1) - kWave * i; }
// byte offset, from a lane's row base register, of the row base itself for slot i's lanes
// (index of factor 0 of the lane's row = lane + 64 i - 83 q)
__host__ __device__ constexpr int row_off(int i) { return 8 * (kWave * i - kQS * qa_of(i)); }

struct WaveLds {
  uint8_t bits[256];               // hard decision of every variable (written once per candidate)
  uint8_t a91[16];
  uint8_t rank[FT8_LDPC_M];        // prologue scratch: check m -> m'
  uint8_t chk_of[FT8_LDPC_M];      // prologue scratch: m' -> m
  uint8_t pad_[kHdr - 256 - 16 - 2 * FT8_LDPC_M];
  double msg[kMsgN];               // tov between sweeps; V->C arguments, then toc, within a sweep
};
static_assert(offsetof(WaveLds, msg) == kHdr, "msg follows the header");

// Per-lane tables (registers, built once per wave).
//   va[j], vb[j]: variable n = lane + 64 j (variable-major phase): LDS byte addresses of its three
//                 edge messages in the reference's kFTX_LDPC_Mn order (va, va1, vb)
//   h[k][j]:      check m' = lane + 64 k (parity): its variables as a 174-bit mask, 64-bit word j
//                 (lo, hi) -- the parity is popcount(h & hard decisions) from wave ballots
struct WaveTables {
  uint32_t va[kVarSlots], va1[kVarSlots];
  uint32_t vb[kVarSlots];
  uint32_t h[kChkSlots][kVarSlots][2];
};

// one ds_read_b64 with the offset as its immediate (volatile: the compiler would otherwise pair
// factors into ds_read2_b64, whose 8-bit offsets cannot span a row and cost a VALU add per pair)
__device__ __forceinline__ double ldv(uint32_t addr) {
  return *(const volatile __attribute__((address_space(3))) double*)(uintptr_t)addr;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p;
}

__device__ void load_tables(WaveTables& t, WaveLds& L, int lane) {
  if (lane == 0) {  // degree-7 rows first, each group in check order
    int c7 = 0, c6 = kM7;
    for (int m = 0; m < FT8_LDPC_M; ++m) {
      const int r = (kChkStartD[m + 1] - kChkStartD[m]) == 7 ? c7++ : c6++;
      L.rank[m] = (uint8_t)r;
      L.chk_of[r] = (uint8_t)m;
    }
  }
  __syncthreads();
  const uint32_t msg0 = lds_addr(&L.msg[0]);
  auto addr_of = [&](int e) -> uint32_t {  // edge (CSR index) -> LDS byte address of its message
    const int m = kEdgeChkD[e], q = e - kChkStartD[m], r = L.rank[m];
    return msg0 + 8u * (uint32_t)(q < 6 ? q * kQS + r : kQ6 + r);
  };
#pragma unroll
  for (int j = 0; j < kVarSlots; ++j) {
    const int n = lane + kWave * j;
    if (n < FT8_LDPC_N) {
      t.va[j] = addr_of(kVarEdgeD[3 * n]);
      t.va1[j] = addr_of(kVarEdgeD[3 * n + 1]);
      t.vb[j] = addr_of(kVarEdgeD[3 * n + 2]);
    } else {  // padding variable: reads the constant, never stores (see the sweep)
      const uint32_t one = msg0 + 8u * kOne;
      t.va[j] = t.va1[j] = one;
      t.vb[j] = one;
    }
  }
#pragma unroll
  for (int k = 0; k < kChkSlots; ++k) {
    const int mp = lane + kWave * k;
#pragma unroll
    for (int j = 0; j < kVarSlots; ++j) t.h[k][j][0] = t.h[k][j][1] = 0;
    if (mp < FT8_LDPC_M) {
      const int m = L.chk_of[mp];
      for (int e = kChkStartD[m]; e < kChkStartD[m + 1]; ++e) {
        const int v = kEdgeVarD[e];
#pragma unroll
        for (int j = 0; j < kVarSlots; ++j)
#pragma unroll
          for (int w = 0; w < 2; ++w)
            if (v >> 5 == 2 * j + w) t.h[k][j][w] |= 1u << (v & 31);
      }
    }
  }
  for (int x = FT8_LDPC_E + lane; x < kMsgN; x += kWave) L.msg[x] = 1.0;  // the constants, once
  __syncthreads();
  // keep the tables in registers: opaque values cannot be rematerialised from memory in the loop
#pragma unroll
  for (int j = 0; j < kVarSlots; ++j) asm volatile("" : "+v"(t.va[j]), "+v"(t.vb[j]));
#pragma unroll
  for (int j = 0; j < kVarSlots; ++j) asm volatile("" : "+v"(t.va1[j]));
#pragma unroll
  for (int k = 0; k < kChkSlots; ++k)
#pragma unroll
    for (int j = 0; j < kVarSlots; ++j) asm volatile("" : "+v"(t.h[k][j][0]), "+v"(t.h[k][j][1]));
}

struct BpArgs {
  const void* wf;
  int wf_f64, T, F, sps, bpt, num_blocks;
  const int32_t* cand;
  const double* cand_score;
  const int32_t* cand_count;
  int N, n_items, mode, n_slots;
  const double* llr_in;
  int normalize, max_iterations;
  double* llr_out;
  uint8_t* plain_out;
  ft8_result* res;
  unsigned long long* work;   // claim counter (64-bit, never reset)
  unsigned long long work_base;  // this launch's first ticket (BpLaunch.work_base)
  unsigned long long* stats;  // nullable: per row (kStatRows x kStatStride) [candidates, iterations
                              //  entered, message passes, converged]
  unsigned long long* clock;  // nullable (timed launches only), stats + 4: per row [sum of wave
                              //  shader-clock cycles, sum of wave wall-clock ticks, max wave cycles,
                              //  waves] (ft8_get_bp_clock)
  int slot0;
  int tie_blocks;             // k_llr's first tie_blocks workgroups run tie_order
  TieArgs tie;
};

// The reference heap of one slot whose selected set holds equal scores (k_select left them in
// scan order, warn bit 3): replay it (heap_replay.h) and write the final candidate order
// final rank -> select rank, plus the tie flag (warn bit 0).  One wave, beside the LLR workgroups.
__device__ bool tie_order(const TieArgs& a, int slot) {
  if (slot >= a.n_slots) return false;
  const int w = a.warn[slot];
  if (!(w & 8)) return false;
  const int lane = threadIdx.x, N = a.N;
  const int nsel = __builtin_amdgcn_readfirstlane(a.cand_count[slot]);
  int32_t* t = a.tie + (int64_t)slot * tie_stride(N);
  const int32_t* push = t;
  const int32_t* sel = t + N;
  int32_t* perm = t + 2 * N;
  int32_t* mi = t + 3 * N;
  int32_t* mp = t + 4 * N;
  int32_t* mk = t + 5 * N;
  const int rec = t[7 * N];
  const float* psc = reinterpret_cast<const float*>(t + 7 * N + 2);  // scores in push order
  const double* ssc = a.cand_score + (int64_t)slot * N;              // scores in select order
  unsigned hh[kReplayRegs], hl[kReplayRegs];
  heap_load(psc, push, nsel, hh, hl);
  int tie = heap_pushes(nsel, hh, hl);
  if (rec >= 0) tie |= heap_record(nsel, hh, hl, mono_neg(__int_as_float(t[7 * N + 1])), (unsigned)rec);

  // members: select ranks whose score equals a neighbour's; record each one's heap position
  int M = 0;
  for (int i0 = 0; i0 < nsel; i0 += kWave) {
    const int i = i0 + lane;
    unsigned key = 0, idx = 0;
    bool mem = false;
    if (i < nsel) {
      idx = (unsigned)sel[i];
      key = mono_neg((float)ssc[i]);
      mem = (i > 0 && mono_neg((float)ssc[i - 1]) == key) || (i + 1 < nsel && mono_neg((float)ssc[i + 1]) == key);
    }
    unsigned long long b = __ballot(mem);
    while (b) {
      const int l = __ffsll((long long)b) - 1;
      b &= b - 1;
      const unsigned sl = rdl(idx, l), kl = rdl(key, l);
      unsigned P = 0;
#pragma unroll
      for (int k = 0; k < kReplayRegs; ++k) {
        const int pos = 64 * k + lane;
        const unsigned long long m = __ballot(pos >= 1 && pos <= nsel && hl[k] == sl);
        if (m) P = 64u * k + (unsigned)(__ffsll((long long)m) - 1);
      }
      if (lane == 0) {
        mi[M] = i0 + l;
        mp[M] = (int)P;
        mk[M] = (int)kl;
      }
      ++M;
    }
  }
  for (int i = lane; i < nsel; i += kWave) perm[i] = i;
  __syncthreads();
  // sorted(key=-score) is stable on heap-array order: within a run of equal scores the final
  // rank follows the heap position, the select rank the scan index
  for (int m = lane; m < M; m += kWave) {
    const int i = mi[m], P = mp[m], K = mk[m];
    int below_i = 0, below_p = 0;
    for (int j = 0; j < M; ++j) {
      if (mk[j] == K) {
        below_i += mi[j] < i;
        below_p += mp[j] < P;
      }
    }
    perm[i - below_i + below_p] = i;
  }
  if (lane == 0 && tie) a.warn[slot] = w | 1;
  return true;
}

// ft8_sync_select: the deferred order applied to the candidate list itself
__global__ __launch_bounds__(kWave) void k_tie_apply(TieArgs a, int32_t* cand, double* cand_score) {
  const int slot = blockIdx.x, lane = threadIdx.x, N = a.N;
  if (!tie_order(a, slot)) return;
  __syncthreads();
  const int nsel = a.cand_count[slot];
  int32_t* t = a.tie + (int64_t)slot * tie_stride(N);
  const int32_t* perm = t + 2 * N;
  int32_t* stage = t + 3 * N;  // [nsel] x (time, freq, score lo, score hi)
  int32_t* cs = cand + (int64_t)slot * N * 2;
  double* ss = cand_score + (int64_t)slot * N;
  for (int i = lane; i < nsel; i += kWave) {
    const int src = perm[i];
    stage[4 * i] = cs[2 * src];
    stage[4 * i + 1] = cs[2 * src + 1];
    const long long v = __double_as_longlong(ss[src]);
    stage[4 * i + 2] = (int32_t)v;
    stage[4 * i + 3] = (int32_t)(v >> 32);
  }
  __syncthreads();
  for (int i = lane; i < nsel; i += kWave) {
    cs[2 * i] = stage[4 * i];
    cs[2 * i + 1] = stage[4 * i + 1];
    ss[i] = __longlong_as_double(((long long)stage[4 * i + 3] << 32) | (unsigned)stage[4 * i + 2]);
  }
}

constexpr int kLlrCpw = 4;                  // k_llr: candidates per wave
constexpr int kLlrRow = FT8_LDPC_N + 2;     // LDS row of one candidate's 174 doubles (padded)

// numpy pairwise sum (loops_utils.h.src) of x[u][0..174) for the wave's kLlrCpw candidates at once:
// pw(0,80) + pw(80,94).  Lanes 16 u + l hold candidate u's 16 partial sums (l < 8: the 8
// accumulators of [0, 80), l >= 8: those of [80, 168)), lane 16 u combines them with the tail
// [168, 174) in numpy's order; every lane receives its candidate's sum.  (One candidate per wave,
// as in round 4, kept 48 of the 64 lanes idle through both sums of the normalisation.)
__device__ double pairwise174x4(const double (*x)[kLlrRow], double (*part)[16], int lane) {
  const int u = lane >> 4, l = lane & 15;
  const double* xu = x[u];
  double r;
  if (l < 8) {
    r = xu[l];
    for (int i = 8; i < 80; i += 8) r += xu[i + l];
  } else {
    const int j = l - 8;
    r = xu[80 + j];
    for (int i = 8; i < 88; i += 8) r += xu[80 + i + j];
  }
  part[u][l] = r;
  __syncthreads();
  double tot = 0.0;
  if (l == 0) {
    const double* pu = part[u];
    const double s1 = ((pu[0] + pu[1]) + (pu[2] + pu[3])) + ((pu[4] + pu[5]) + (pu[6] + pu[7]));
    double s2 = ((pu[8] + pu[9]) + (pu[10] + pu[11])) + ((pu[12] + pu[13]) + (pu[14] + pu[15]));
    for (int i = 168; i < 174; ++i) s2 += xu[i];
    tot = 0.0 + (s1 + s2);  // add.reduce starts from the identity
  }
  __syncthreads();
  return __shfl(tot, lane & ~15);
}

// ft8_extract_likelihood (ft8_decode.py:164-188) of the wave's candidates with the gathers spread over
// the wave: lane 8 g + i fetches tone i of symbol 8 r + g in round r, so one load instruction covers
// 8 symbols' rows (one or two cache lines each) instead of 58 rows; the loads of all kLlrCpw
// candidates are issued before the first is used (32 in flight per lane), and the tone powers reach
// their symbol's lane through LDS (stage: 64 symbols x 8 tones per candidate).
template <typename T>
__device__ void extract_llr_x4(const BpArgs& a, const int (&slot)[kLlrCpw], const int (&at)[kLlrCpw],
                               const int (&af)[kLlrCpw], int n_on, double (*c)[kLlrRow], T (*stage)[64 * 8],
                               int lane) {
  const int i = lane & 7, g = lane >> 3;
  const T* wf0 = reinterpret_cast<const T*>(a.wf);
  T v[kLlrCpw][8];
#pragma unroll
  for (int u = 0; u < kLlrCpw; ++u) {
    const int base = floordiv(at[u], a.sps);
    const T* wf = wf0 + (int64_t)slot[u] * a.T * a.F;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int k = 8 * r + g;
      const int sym = k + (k < 29 ? 7 : 14);
      const int block = base + sym;
      v[u][r] = (T)0;
      if (u < n_on && k < 58 && !(block < 0 || block >= a.num_blocks))
        v[u][r] = wf[(int64_t)(at[u] + sym * a.sps) * a.F + af[u] + i * a.bpt];
    }
  }
#pragma unroll
  for (int u = 0; u < kLlrCpw; ++u)
#pragma unroll
    for (int r = 0; r < 8; ++r) stage[u][8 * (8 * r + g) + i] = v[u][r];
  __syncthreads();
  if (lane < 58) {
    const int k = lane;
    const int sym = k + (k < 29 ? 7 : 14);
#pragma unroll
    for (int u = 0; u < kLlrCpw; ++u) {
      if (u >= n_on) break;
      const int block = floordiv(at[u], a.sps) + sym;
      double l0 = 0.0, l1 = 0.0, l2 = 0.0;
      if (!(block < 0 || block >= a.num_blocks)) {
        double s[8], s2[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] = (double)stage[u][8 * k + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) s2[j] = s[kGrayD[j]];
        l0 = pymax4(s2[4], s2[5], s2[6], s2[7]) - pymax4(s2[0], s2[1], s2[2], s2[3]);
        l1 = pymax4(s2[2], s2[3], s2[6], s2[7]) - pymax4(s2[0], s2[1], s2[4], s2[5]);
        l2 = pymax4(s2[1], s2[3], s2[5], s2[7]) - pymax4(s2[0], s2[2], s2[4], s2[6]);
      }
      c[u][3 * k] = l0;
      c[u][3 * k + 1] = l1;
      c[u][3 * k + 2] = l2;
    }
  }
}

// ---- k_llr: one wave per kLlrCpw candidates -> normalised LLRs in global memory --------------------
// modes: 0 per-slot candidate lists (4 consecutive ranks of one slot per wave; ranks >= the slot's
// count skipped), 1 explicit (slot, t, f) list, 2 normalise given LLRs.  Items u = 0 .. n_on - 1 of
// the wave are item0 + u (the active ones are always a prefix).
template <typename T>
__global__ __launch_bounds__(kWave) void k_llr(BpArgs a) {
  __shared__ double c[kLlrCpw][kLlrRow];
  __shared__ double part[kLlrCpw][16];
  __shared__ double bc[kLlrCpw];
  // the gather stage (extraction) and the squared deviations (normalisation) share one buffer: a
  // barrier separates the two uses, and the LDS per wave sets how many waves a CU holds
  constexpr size_t kScratch = sizeof(T) * kLlrCpw * 64 * 8 > sizeof(double) * kLlrCpw * kLlrRow
                                  ? sizeof(T) * kLlrCpw * 64 * 8 : sizeof(double) * kLlrCpw * kLlrRow;
  __shared__ __attribute__((aligned(16))) unsigned char scratch[kScratch];
  double (*sq)[kLlrRow] = reinterpret_cast<double (*)[kLlrRow]>(scratch);
  const int lane = threadIdx.x;
  if ((int)blockIdx.x < a.tie_blocks) {
    tie_order(a.tie, blockIdx.x);
    return;
  }
  const int id = blockIdx.x - a.tie_blocks;  // tie_blocks % 8 == 0 keeps id % 8 == XCD
  int item0, n_on;
  int slot[kLlrCpw] = {0, 0, 0, 0}, at[kLlrCpw] = {0, 0, 0, 0}, af[kLlrCpw] = {0, 0, 0, 0};
  static_assert(kLlrCpw == 4, "four candidates per wave");
  if (a.mode == 0) {
    // workgroup id -> (slot, group of 4 ranks) with slot % 8 == id % 8: all candidates of a slot run
    // on one XCD, so its waterfall rows are fetched into one L2
    const int groups = (a.N + kLlrCpw - 1) / kLlrCpw;
    const int q = id >> 3;
    const int s0 = (q / groups) * 8 + (id & 7);
    const int c0 = (q % groups) * kLlrCpw;
    if (s0 >= a.n_slots) return;
    n_on = min(kLlrCpw, min(a.N, a.cand_count[s0]) - c0);
    item0 = s0 * a.N + c0;
#pragma unroll
    for (int u = 0; u < kLlrCpw; ++u) {
      slot[u] = s0;
      if (u < n_on) {
        at[u] = a.cand[((int64_t)item0 + u) * 2];
        af[u] = a.cand[((int64_t)item0 + u) * 2 + 1];
      }
    }
  } else {
    item0 = id * kLlrCpw;
    n_on = min(kLlrCpw, a.n_items - item0);
    if (a.mode == 1) {
#pragma unroll
      for (int u = 0; u < kLlrCpw; ++u) {
        if (u < n_on) {
          slot[u] = a.cand[((int64_t)item0 + u) * 3];
          at[u] = a.cand[((int64_t)item0 + u) * 3 + 1];
          af[u] = a.cand[((int64_t)item0 + u) * 3 + 2];
        }
      }
    }
  }
  if (n_on <= 0) return;  // wave-uniform
  if (a.mode == 2) {
    for (int e = lane; e < n_on * FT8_LDPC_N; e += kWave) {
      const int u = e / FT8_LDPC_N, n = e - u * FT8_LDPC_N;
      c[u][n] = a.llr_in[(int64_t)(item0 + u) * FT8_LDPC_N + n];
    }
  } else {
    extract_llr_x4<T>(a, slot, at, af, n_on, c, reinterpret_cast<T (*)[64 * 8]>(scratch), lane);
  }
  __syncthreads();
  if (a.normalize) {  // ftx_normalize_logl (ft8_decode.py:190-198), the wave's candidates side by side
    const double mean = pairwise174x4(c, part, lane) / 174.0;
    if ((lane & 15) == 0) bc[lane >> 4] = mean;
    __syncthreads();
    for (int e = lane; e < n_on * FT8_LDPC_N; e += kWave) {
      const int u = e / FT8_LDPC_N, n = e - u * FT8_LDPC_N;
      const double d = c[u][n] - bc[u];
      sq[u][n] = d * d;
    }
    __syncthreads();
    const double var = pairwise174x4(sq, part, lane) / 174.0;
    if ((lane & 15) == 0) bc[lane >> 4] = sqrt_rn(24.0 / var);
    __syncthreads();
    for (int e = lane; e < n_on * FT8_LDPC_N; e += kWave) {
      const int u = e / FT8_LDPC_N, n = e - u * FT8_LDPC_N;
      a.llr_out[(int64_t)(item0 + u) * FT8_LDPC_N + n] = c[u][n] * bc[u];
    }
    return;
  }
  for (int e = lane; e < n_on * FT8_LDPC_N; e += kWave) {
    const int u = e / FT8_LDPC_N, n = e - u * FT8_LDPC_N;
    a.llr_out[(int64_t)(item0 + u) * FT8_LDPC_N + n] = c[u][n];
  }
}

// Phase boundary inside a sweep.  The workgroup is one wave and the LDS executes a wave's
// instructions in order, so a later ds_read sees every earlier ds_write of the wave without
// s_waitcnt / s_barrier; only the compiler must not move LDS accesses across the boundary.
__device__ __forceinline__ void sweep_sync() { asm volatile("" ::: "memory"); }

// np.clip(T, -2 c, 2 c) of fast_tanh's argument in the folded form (c = 4.97); NaN stays NaN when
// the candidate has NaN inputs (nan_in, wave-uniform)
__device__ __forceinline__ double clip2(double T, bool nan_in) {
  const double y = __builtin_fmin(__builtin_fmax(T, -kClip2), kClip2);
  return (nan_in && T != T) ? T : y;
}

// fast_tanh (ldpc_decoder.py:11-20) of kDivGroup clipped arguments in place: y = clip(T, +-2 c) in,
// toc out (see the sweep's phase C for the scaling argument)
// fast: the caller established the short division for the whole wave (sweep_fast)
__device__ __forceinline__ void tanh_group(double* v, int fast = 0) {
  double na[kDivGroup], nb[kDivGroup];
#pragma unroll
  for (int i = 0; i < kDivGroup; ++i) {
    const double yv = v[i], z = yv * yv;
    na[i] = yv * (15120.0 + z * (420.0 + z));
    nb[i] = -30240.0 + z * (-3360.0 + z * -30.0);
  }
  int ok = fast;  // an int, not a bool: a bool crossing blocks would be kept as a VALU lane mask
  if (!ok) {
    double mn = INFINITY;
#pragma unroll
    for (int i = 0; i < kDivGroup; ++i) mn = __builtin_fmin(mn, __builtin_fabs(na[i]));
    ok = __ballot(mn >= 0x1p-480) == __builtin_amdgcn_read_exec() ? 1 : 0;
  }
  if (ok) {
    div_fast<kDivGroup>(v, na, nb);
  } else {
#pragma unroll
    for (int i = 0; i < kDivGroup; ++i) {
      const double xv = -0.5 * v[i], x2 = xv * xv;
      na[i] = xv * (945.0 + x2 * (105.0 + x2));
      nb[i] = 945.0 + x2 * (420.0 + x2 * 15.0);
    }
    div_rn<kDivGroup>(v, na, nb);
  }
}

// min(|hi dword|) of three doubles, the hi dwords read as float32 (v_min3_f32 with abs modifiers).
// For a finite double, |x| >= 2^k (k integer) iff the float32 view of its hi dword, sign cleared,
// is >= the view of 2^k's hi dword (the low dword of 2^k is 0, and non-negative float32 bit
// patterns order as integers).  A NaN's hi dword reads as a quiet float32 NaN, which v_min3 skips.
__device__ __forceinline__ float min3_abs_hi(double a, double b, double c) {
  float m;
  asm("v_min3_f32 %0, |%1|, |%2|, |%3|"
      : "=v"(m)
      : "v"(__double2hiint(a)), "v"(__double2hiint(b)), "v"(__double2hiint(c)));
  return m;
}

// Per-sweep short-division test: true when every V->C argument y of the wave
// (3 x 3 per lane, after np.clip) has |y| >= 2^-100 -- or is NaN, which either division path
// turns into the same NaN (see div_rn).  That one test admits both phases' short divisions:
//   * fast_tanh: |A| = |y| (15120 + z (420 + z)) >= 2^-100 * 15120 > 2^-480 (tanh_group's test);
//   * fast_atanh: every toc stored this sweep is RN(A/B) with |A/B| >= |y| / 10 (the ratio
//     (15120 + 420 z + z^2) / (30240 + 3360 z + 30 z^2) is >= 0.1013 for z = y^2 <= 98.8), so
//     |toc| >= 2^-104, and |toc| <= 1.0073; a product of six of them (or of five and the 1.0
//     that pads a degree-6 row) stays >= 2^-625 with no subnormal step, and the numerator
//     x (945 + x^2 (-735 + 64 x^2)) has |.| >= 219 |x| > 2^-960 (div_rn's test); the
//     denominators are the same normal values on either path.
// 4 v_min3_f32 + 1 compare per sweep instead of 3-4 VALU per division group (6 groups per sweep).
__device__ __forceinline__ bool sweep_fast(const double (&y)[kVarSlots][3]) {
  static_assert(kVarSlots == 3, "three variable slots");
  const float m0 = min3_abs_hi(y[0][0], y[0][1], y[0][2]);
  const float m1 = min3_abs_hi(y[1][0], y[1][1], y[1][2]);
  const float m2 = min3_abs_hi(y[2][0], y[2][1], y[2][2]);
  float m;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(m0), "v"(m1), "v"(m2));
  // hi dword of 2^-100: biased exponent 923 << 20
  const float thr = __int_as_float(923 << 20);
  return __ballot(m < thr) == 0;
}

// tov = -2 fast_atanh(Tmn) (ldpc_decoder.py:22-30, 108) of kDivGroup products in place.
// fast: the caller established the short division for the whole wave (sweep_fast).
__device__ __forceinline__ void atanh_group(double* v, int fast = 0) {
  double na[kDivGroup], nb[kDivGroup];
#pragma unroll
  for (int i = 0; i < kDivGroup; ++i) {
    const double xv = v[i], x2 = xv * xv;
    // -735 + x2 * 64 as one fma: the product by 64 is exact (x2 is a finite square <= 1.02, or
    // NaN), so RN(-735 + RN(64 x2)) == RN(-735 + 64 x2) bit for bit -- one VALU per edge less
    na[i] = xv * (945.0 + x2 * __builtin_fma(x2, 64.0, -735.0));
    // -b/2 for b = 945 + x2 (-1050 + x2 225): every step is the reference's step scaled by -1/2,
    // exact (terms too small to scale exactly are absorbed by the constant they meet)
    nb[i] = (-472.5 + x2 * (525.0 + x2 * -112.5));
  }
  div_rn<kDivGroup, true>(v, na, nb, fast);
}

// Phase D's products: for each of the lane's edge slots, the product of the other toc of the edge's
// check in row order, from 1.0 (1.0 * t0 == t0, so the product starts at the first factor).
__device__ __forceinline__ void check_products(double* x, uint32_t la, int lane) {
#pragma unroll
  for (int i = 0; i < kEdgeSlots; ++i) {
    const int qa = qa_of(i);
    const bool mx = mixed_slot(i);
    const bool hi = mx && lane >= hi_lane(i);
    // row base of the lane (factor 0 of its row): la + row_off(i) for q = qa, 664 less for qa + 1
    const uint32_t rb = hi ? la - 664u : la;
    double p = 0.0;
    bool first = true;
#pragma unroll
    for (int f = 0; f < 7; ++f) {
      double t;
      if (mx && f == qa) {        // t[qa + 1] (q = qa lanes) or t[qa] (q = qa + 1 lanes)
        const uint32_t pa = hi ? rb : rb + 664u;
        t = ldv(pa + (uint32_t)(row_off(i) + 664 * qa));
      } else if (mx && f == qa + 1) {
        continue;
      } else if (!mx && f == qa) {
        continue;
      } else {
        t = ldv(rb + (uint32_t)(row_off(i) + 664 * f));
      }
      p = first ? t : p * t;
      first = false;
    }
    x[i] = p;
    // bound how far the scheduler hoists these loads (register pressure)
    if (i % kProdGroup == kProdGroup - 1) asm volatile("" ::: "memory");
  }
}

// ---- k_bp: persistent waves, one candidate at a time ----------------------------------------------
// modes: 0 per-slot candidate lists (records carry slot / abs_time / abs_freq / score), 2 plain LLRs
template <bool NANSAFE>
__global__ __launch_bounds__(kWave, kBpLbWaves) void k_bp(BpArgs a) {
  // the wave's lifetime in shader-clock cycles and constant-rate wall-clock ticks (counter pass
  // only): cycles per launch are clock-independent, cycles / wall time is the clock the kernel ran at
  const unsigned long long clk0 = a.clock ? clock64() : 0ull, wall0 = a.clock ? wall_clock64() : 0ull;
  __shared__ WaveLds L;
  const int lane = threadIdx.x;
  WaveTables tb;
  load_tables(tb, L, lane);
  // padding variables (variable slot 2, lanes >= 46) never store their V->C arguments
  const bool var2 = lane + kWave * (kVarSlots - 1) < FT8_LDPC_N;
  const uint64_t var2_mask = (1ull << (FT8_LDPC_N - kWave * (kVarSlots - 1))) - 1ull;
  // the lane's message address in the edge-major phases (slot i: + 512 i) and the row-base
  // registers of the two lane groups of a mixed slot (q = qa: la, q = qa + 1: la - 664)
  uint32_t la = lds_addr(&L.msg[0]) + 8u * (uint32_t)lane;
  asm volatile("" : "+v"(la));  // one register (the generic->LDS cast carries a null test)

  // work counters, per wave; flushed once when the wave retires (same-address atomics per
  // candidate would serialise in L2)
  unsigned st_cand = 0, st_iter = 0, st_pass = 0, st_conv = 0;
  for (;;) {
    unsigned long long ticket = 0;
    if (lane == 0) ticket = atomicAdd(a.work, 1ull);
    // wave-uniform: candidate metadata then lives in SGPRs (scalar loads), not VGPRs
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)ticket);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(ticket >> 32));
    // tickets of this launch start at work_base (host-advanced, see BpLaunch); a wave retires at
    // its first ticket past the items -- no counter reset and no retire counter: round 3's
    // last-retiring-wave reset put 4096 same-address atomics on the launch's tail
    const unsigned long long rel = (((unsigned long long)hi << 32) | lo) - a.work_base;
    if (rel >= (unsigned long long)a.n_items) break;
    const unsigned item = (unsigned)rel;

    int slot = 0, at = 0, af = 0, cidx = 0;
    double score = 0.0;
    if (a.mode == 0) {
      slot = item / a.N;
      cidx = item % a.N;
      if (cidx >= a.cand_count[slot]) continue;
      at = a.cand[((int64_t)slot * a.N + cidx) * 2];
      af = a.cand[((int64_t)slot * a.N + cidx) * 2 + 1];
      score = a.cand_score[(int64_t)slot * a.N + cidx];
    }
    double cv_[kVarSlots];  // codeword[n] (the LLR) of the lane's variables
#pragma unroll
    for (int j = 0; j < kVarSlots; ++j) {
      const int n = lane + kWave * j;
      // padding variables (slot 2, lanes >= 46): codeword -1.0, and their three tov read the
      // constant 1.0, so every V->C argument is (-1 + 1) + 1 = 1.0 after the first sweep (-1.0 in
      // it): harmless, never tiny (the wave stays on the short division), never stored
      cv_[j] = n < FT8_LDPC_N ? a.llr_in[(int64_t)item * FT8_LDPC_N + n] : -1.0;
    }

    // NaN LLRs must survive np.clip as NaN; the clip's v_min/v_max would turn them into the bound,
    // so such a candidate (wave-uniform flag) takes the NaN-preserving form.  NaN arises from
    // nothing else (every other message is finite), and the decode path's normalised LLRs are
    // either all NaN (ftx_normalize_logl spreads one NaN to all 174, and the all-zero hard decision
    // then ends the first sweep exactly as in the reference) or none: only the plain-LLR entry
    // point (ft8_bp, NANSAFE) needs the test.
    const bool nan_in = NANSAFE && __ballot(cv_[0] != cv_[0] || cv_[1] != cv_[1] || cv_[2] != cv_[2]) != 0;

    // ---- belief propagation (ldpc_decoder.py:54-113) ----------------------------------------
    // One sweep = the reference iteration.  (A) variable-major: each lane reads its variables'
    // three tov, forms the hard decision c + ((t0 + t1) + t2) (a wave ballot per variable slot)
    // and the three clipped variable->check sums (c + t_a) + t_b in registers; (B) parity of every
    // check from the ballots; (C) fast_tanh of those registers, a variable's three edges being one
    // division group, toc stored into each edge's slot; (D) edge-major: check products ->
    // fast_atanh -> tov.  The first sweep (all tov 0) evaluates fast_tanh once per variable; the
    // last one stops after (B), its message update being unread.
    // tov = 0 on every real edge (indices 0..521; the constants above never change)
#pragma unroll
    for (int i = 0; i < kEdgeSlots; ++i)
      if (i < kEdgeSlots - 1 || lane + kWave * i < FT8_LDPC_E)
        *(__attribute__((address_space(3))) double*)(uintptr_t)(la + 512u * i) = 0.0;
    __syncthreads();
    uint64_t hd[kVarSlots] = {0, 0, 0};  // hard decisions of the last evaluated sweep (ballots)
    int min_errors = FT8_LDPC_M;
    int entered = 0, passes = 0;
    for (int iter = 0; iter < a.max_iterations; ++iter) {
      entered++;
      // re-opaque the tables every sweep: otherwise the compiler hoists derived addresses out of
      // the loop (spilling); recomputing them is one integer op each
#pragma unroll
      for (int j = 0; j < kVarSlots; ++j) asm volatile("" : "+v"(tb.va[j]), "+v"(tb.vb[j]));
      // (A) variable-major: the hard decision and the three clipped variable->check arguments of
      // each of the lane's variables, kept in registers (no LDS store, so no phase boundary)
      double y[kVarSlots][3];
      const bool sweep0 = iter == 0;
      if (sweep0) {
        // every tov is 0: messages = codeword + 0.0 (ldpc_decoder.py:72-73), and the argument of
        // each of a variable's edges is (c + 0.0) + 0.0 == c + 0.0
#pragma unroll
        for (int j = 0; j < kVarSlots; ++j) {
          const double T = cv_[j] + 0.0;
          hd[j] = __ballot(T > 0.0);
          y[j][0] = y[j][1] = y[j][2] = clip2(T, nan_in);
        }
      } else {
#pragma unroll
        for (int j = 0; j < kVarSlots; ++j) {
          const double t0 = *(lds_f64*)(uintptr_t)tb.va[j];
          const double t1 = *(lds_f64*)(uintptr_t)tb.va1[j];
          const double t2 = *(lds_f64*)(uintptr_t)tb.vb[j];
          const double c = cv_[j];
          // messages = codeword + sum(tov, axis=1) (ldpc_decoder.py:72-73)
          hd[j] = __ballot((c + ((t0 + t1) + t2)) > 0.0);
          // Tnm = codeword[n] + the other two tov in check order (ldpc_decoder.py:90-96); fast_tanh's
          // np.clip with the -1/2 folded into the polynomials: y = clip(T, -2 c, 2 c), below
          const double c0 = c + t0;
          y[j][0] = (c + t1) + t2;
          y[j][1] = c0 + t2;
          y[j][2] = c0 + t1;
        }
        // np.clip, NaN-preserving only for a candidate with NaN inputs (a wave-uniform branch)
        if (nan_in) {
#pragma unroll
          for (int j = 0; j < kVarSlots; ++j)
#pragma unroll
            for (int e = 0; e < 3; ++e) y[j][e] = clip2(y[j][e], true);
        } else {
#pragma unroll
          for (int j = 0; j < kVarSlots; ++j)
#pragma unroll
            for (int e = 0; e < 3; ++e) y[j][e] = clip2(y[j][e], false);
        }
      }
      hd[kVarSlots - 1] &= var2_mask;
      // all-zero hard decision -> stop (ldpc_decoder.py:76-78)
      if ((hd[0] | hd[1] | hd[2]) == 0) break;
      // (B) parity check (ldpc_check, ldpc_decoder.py:33-52): popcount of (row mask & decisions)
      int errs = 0;
#pragma unroll
      for (int k = 0; k < kChkSlots; ++k) {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < kVarSlots; ++j) {
          x = __builtin_amdgcn_bitop3_b32(tb.h[k][j][0], (uint32_t)hd[j], x, 0x6a);          // (h & d) ^ x
          x = __builtin_amdgcn_bitop3_b32(tb.h[k][j][1], (uint32_t)(hd[j] >> 32), x, 0x6a);
        }
        errs += __popcll(__ballot(__builtin_popcount(x) & 1));
      }
      if (errs < min_errors) {
        min_errors = errs;
        if (errs == 0) break;
      }
      // the last iteration's message update (ldpc_decoder.py:88-108) is never read: the loop ends
      // after it and the result is the plain / min_errors formed above
      if (iter + 1 == a.max_iterations) break;
      // (C) variable -> check messages: toc = fast_tanh(-Tnm / 2), three interleaved divisions at a
      // time.  From y = -2 x (x the reference's clipped argument): with z = RN(y y) = 4 RN(x x),
      // every step of fast_tanh's polynomials (ldpc_decoder.py:11-20) is the reference's step scaled
      // by a power of two, so na = -A / 32 and nb = B / -32 exactly for
      //   A = y (15120 + z (420 + z)),   B = -30240 + z (-3360 + z (-30)),
      // and toc = RN(na / nb) = RN(A / B): the same real quotient.  The scalings are exact while
      // nothing underflows, which |A| >= 2^-480 (so |y| >= 2^-496) guarantees for the whole wave;
      // the same bound admits the short division.  Otherwise (tiny or zero arguments) the group
      // runs the reference form on x = -y / 2 (tanh_group).
      // variable-major, straight from phase A's registers into each edge's slot
      static_assert(kDivGroup == 3 && kVarSlots == 3, "a division group is one variable's edges");
      // wave-uniform int (a bool crossing blocks would be kept as a VALU lane mask)
      int fast = __builtin_amdgcn_readfirstlane(sweep_fast(y) ? 1 : 0);
      asm volatile("" : "+s"(fast));  // opaque SGPR: branches test it with s_cmp
      if (sweep0) {  // one fast_tanh per variable
        double v[kVarSlots] = {y[0][0], y[1][0], y[2][0]};
        tanh_group(v, fast);
#pragma unroll
        for (int j = 0; j < kVarSlots; ++j) y[j][0] = y[j][1] = y[j][2] = v[j];
      }
#pragma unroll
      for (int j = 0; j < kVarSlots; ++j) {
        if (!sweep0) tanh_group(y[j], fast);
        if (j < kVarSlots - 1 || var2) {
          *(__attribute__((address_space(3))) double*)(uintptr_t)tb.va[j] = y[j][0];
          *(__attribute__((address_space(3))) double*)(uintptr_t)tb.va1[j] = y[j][1];
          *(__attribute__((address_space(3))) double*)(uintptr_t)tb.vb[j] = y[j][2];
        }
        asm volatile("" ::: "memory");  // one group's temporaries at a time (register pressure)
      }
      sweep_sync();
      double x[kEdgeSlots];
      // (D) check -> variable messages: tov = -2 fast_atanh(product of the other toc of the check)
      check_products(x, la, lane);
#pragma unroll
      for (int g = 0; g < kEdgeSlots; g += kDivGroup) atanh_group(&x[g], fast);
#pragma unroll
      for (int i = 0; i < kEdgeSlots; ++i)
        if (i < kEdgeSlots - 1 || lane + kWave * i < FT8_LDPC_E)
          *(__attribute__((address_space(3))) double*)(uintptr_t)(la + 512u * i) = x[i];
      passes++;
      sweep_sync();
    }
    // the hard decision of the last evaluated sweep (all zero if no sweep ran), staged only when
    // something reads it: the plain output, or the payload of a candidate that converged
    // (min_errors is wave-uniform; most candidates never converge and skip the packing)
    const bool pack = a.res && min_errors == 0;
    if (a.plain_out || pack) {
#pragma unroll
      for (int j = 0; j < kVarSlots; ++j) L.bits[lane + kWave * j] = (uint8_t)((hd[j] >> lane) & 1u);
      __syncthreads();
    }
    st_cand++;
    st_iter += entered;
    st_pass += passes;
    st_conv += min_errors == 0;


    // ---- outputs ------------------------------------------------------------------------------
    if (a.plain_out)
      for (int n = lane; n < FT8_LDPC_N; n += kWave) a.plain_out[(int64_t)item * FT8_LDPC_N + n] = L.bits[n];
    if (a.res) {
      // pack 91 bits MSB first (ft8_decode.py:200-215)
      if (pack && lane < 12) {  // lane l packs decision bytes 8l..8l+7 (one 8-byte LDS read)
        const uint64_t w = *reinterpret_cast<const uint64_t*>(&L.bits[8 * lane]);
        const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
        unsigned byte = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) byte |= ((lo >> (8 * j)) & 1u) << (7 - j);
#pragma unroll
        for (int j = 0; j < 4; ++j) byte |= ((hi >> (8 * j)) & 1u) << (3 - j);
        if (lane == 11) byte &= 0xE0u;  // bits 88..90 end the 91-bit message
        L.a91[lane] = (uint8_t)byte;
      }
      __syncthreads();
      if (lane == 0) {
        ft8_result r;
        r.score = score;
        r.slot = a.slot0 + slot;
        r.abs_time = at;
        r.abs_freq = af;
        r.ldpc_errors = (int16_t)min_errors;
        r.cand_index = (uint16_t)cidx;
        r.crc_extracted = 0;
        r.crc_calculated = 0;
        r.ok = 0;
        r.pass_index = 0;
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
  const unsigned row = (blockIdx.x & (unsigned)(kStatRows - 1)) * (unsigned)kStatStride;
  if (a.stats && lane == 0 && st_cand) {
    atomicAdd(&a.stats[row + 0], (unsigned long long)st_cand);
    atomicAdd(&a.stats[row + 1], (unsigned long long)st_iter);
    atomicAdd(&a.stats[row + 2], (unsigned long long)st_pass);
    atomicAdd(&a.stats[row + 3], (unsigned long long)st_conv);
  }
  if (a.clock && lane == 0) {
    const unsigned long long cyc = clock64() - clk0, wall = wall_clock64() - wall0;
    atomicAdd(&a.clock[row + 0], cyc);
    atomicAdd(&a.clock[row + 1], wall);
    atomicMax(&a.clock[row + 2], cyc);
    atomicAdd(&a.clock[row + 3], 1ull);
  }
}

// one wave per slot: successes in candidate order -> out[slot][0..cap), counts[slot]
// (a slot whose order of equal scores was deferred, warn bit 3, is read in its final order)
__global__ __launch_bounds__(kWave) void k_compact(const ft8_result* res, const int32_t* cand_count,
                                                   int N, ft8_result* out, int32_t* counts, int cap,
                                                   const int32_t* warn, const int32_t* tie) {
  const int slot = blockIdx.x, lane = threadIdx.x;
  const int nc = cand_count[slot];
  const int32_t* perm = (tie && (warn[slot] & 8)) ? tie + (int64_t)slot * tie_stride(N) + 2 * N : nullptr;
  const ft8_result* rs = res + (int64_t)slot * N;
  int base = 0;
  for (int c0 = 0; c0 < nc; c0 += kWave) {
    const int c = c0 + lane;
    const int src = c < nc ? (perm ? perm[c] : c) : 0;
    const bool ok = c < nc && rs[src].ok;
    const unsigned long long m = __ballot(ok);
    const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
    if (ok && pos < cap) {
      out[(int64_t)slot * cap + pos] = rs[src];
      if (perm) out[(int64_t)slot * cap + pos].cand_index = (uint16_t)c;
    }
    base += __popcll(m);
  }
  if (lane == 0) counts[slot] = base;
}

// ---- k_pack: a batch's decodes -> one all-gather send buffer (ft8_pack_decodes) -------------------
// One 1024-thread workgroup: the batch's slots in chunks of 1024, each chunk's capped counts turned
// into row offsets by a block scan, then every thread of the block copies rows of the chunk (a row's
// slot found by binary search over the offsets), so a slot with many decodes is not one thread's
// serial copy.  Records are 40 B; a batch holds ~1-30 decodes per slot, so this is a few KB.
constexpr int kPackThreads = 1024;
__global__ __launch_bounds__(kPackThreads) void k_pack(const ft8_result* rec, const int32_t* counts, int n_slots,
                                                       int cap, int capacity, int slot_offset, uint8_t* send,
                                                       ft8_result* overflow) {
  FT8_RACE_PROLOGUE();
  __shared__ int s_off[kPackThreads];
  __shared__ int s_wave[kPackThreads / kWave + 1];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid >> 6;
  int32_t* cnt_out = reinterpret_cast<int32_t*>(send + 8);
  ft8_result* rows = reinterpret_cast<ft8_result*>(send + pack_header_bytes(n_slots));
  int carry = 0;
  for (int base = 0; base < n_slots; base += kPackThreads) {
    const int s = base + tid;
    int c = 0;
    if (s < n_slots) {
      const int raw = counts[s];
      cnt_out[s] = raw;
      c = min(max(raw, 0), cap);
    }
    // exclusive scan of c over the block: wave scans, then the wave totals
    int x = c;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == kWave - 1) s_wave[w] = x;
    __syncthreads();
    if (tid == 0) {
      int acc = 0;
      for (int i = 0; i < kPackThreads / kWave; ++i) {
        const int t = s_wave[i];
        s_wave[i] = acc;
        acc += t;
      }
      s_wave[kPackThreads / kWave] = acc;
    }
    __syncthreads();
    // slots past n_slots get an offset past every row, so the search below never lands on them
    s_off[tid] = s < n_slots ? s_wave[w] + x - c : 0x7fffffff;
    const int ct = s_wave[kPackThreads / kWave];
    __syncthreads();
    for (int r = tid; r < ct; r += kPackThreads) {
      // the last slot whose first row is <= r: zero-count slots share the next slot's offset, so
      // this is the slot holding row r
      int lo = 0, hi = min(kPackThreads, n_slots - base) - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= r) lo = mid;
        else hi = mid - 1;
      }
      ft8_result v = rec[(int64_t)(base + lo) * cap + (r - s_off[lo])];
      v.slot += slot_offset;
      const int dst = carry + r;
      if (dst < capacity) rows[dst] = v;
      else if (overflow) overflow[dst - capacity] = v;
    }
    carry += ct;
    __syncthreads();
  }
  // zero the unused rows (the exchange moves them; keep them deterministic)
  for (int r = carry + tid; r < capacity; r += kPackThreads) {
    uint64_t* p = reinterpret_cast<uint64_t*>(rows + r);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(ft8_result) / 8); ++i) p[i] = 0;
  }
  for (int i = n_slots + tid; i < (int)((pack_header_bytes(n_slots) - 8) / 4); i += kPackThreads) cnt_out[i] = 0;
  if (tid == 0) *reinterpret_cast<int64_t*>(send) = carry;
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

BpArgs make_args(const BpLaunch& L) {
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
  a.n_slots = L.n_slots;
  a.mode = L.mode;
  a.llr_in = L.llr_in;
  a.normalize = L.normalize;
  a.max_iterations = L.max_iterations;
  a.llr_out = L.llr_out;
  a.plain_out = L.plain_out;
  a.res = L.res;
  a.work = L.work;
  a.work_base = L.work_base ? *L.work_base : 0ull;
  a.stats = L.stats;
  a.clock = L.clock;
  a.slot0 = L.slot0;
  a.tie = TieArgs{L.n_slots, L.N, L.cand_count, L.warn, L.tie, L.cand_score};
  a.tie_blocks = (L.tie && L.mode == 0) ? (L.n_slots + 7) / 8 * 8 : 0;
  return a;
}

}  // namespace

hipError_t launch_llr(const BpLaunch& L, hipStream_t s) {
  if (L.n_items <= 0) return hipSuccess;
  BpArgs a = make_args(L);
  const int64_t grid = a.tie_blocks + (L.mode == 0 ? (int64_t)((L.n_slots + 7) / 8) * 8 * ((L.N + kLlrCpw - 1) / kLlrCpw)
                                                    : ((int64_t)L.n_items + kLlrCpw - 1) / kLlrCpw);
  if (L.wf_f64)
    hipLaunchKernelGGL(k_llr<double>, dim3((unsigned)grid), dim3(kWave), 0, s, a);
  else
    hipLaunchKernelGGL(k_llr<float>, dim3((unsigned)grid), dim3(kWave), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_bp(const BpLaunch& L, hipStream_t s) {
  if (L.n_items <= 0) return hipSuccess;
  BpArgs a = make_args(L);
  const int per_simd = max(1, min(L.grid_waves, kBpWavesPerSimd));
  const int waves = min(L.n_items, kBpGridCus * 4 * per_simd);  // resident waves, persistent
  if (L.mode == 0) hipLaunchKernelGGL(k_bp<false>, dim3(waves), dim3(kWave), 0, s, a);
  else hipLaunchKernelGGL(k_bp<true>, dim3(waves), dim3(kWave), 0, s, a);
  const hipError_t e = hipGetLastError();
  // the launch consumes n_items + waves tickets (every item once, then one per wave)
  if (e == hipSuccess && L.work_base) *L.work_base += (unsigned long long)L.n_items + (unsigned long long)waves;
  return e;
}

hipError_t launch_tie_apply(const TieArgs& a, int32_t* cand, double* cand_score, hipStream_t s) {
  if (a.n_slots <= 0 || !a.tie) return hipSuccess;
  hipLaunchKernelGGL(k_tie_apply, dim3(a.n_slots), dim3(kWave), 0, s, a, cand, cand_score);
  return hipGetLastError();
}

hipError_t launch_compact(const CompactLaunch& L, hipStream_t s) {
  if (L.n_slots <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_compact, dim3(L.n_slots), dim3(kWave), 0, s, L.res, L.cand_count, L.N, L.out,
                     L.counts, L.cap, L.warn, L.tie);
  return hipGetLastError();
}

hipError_t launch_pack(const ft8_result* rec, const int32_t* counts, int n_slots, int cap, int capacity,
                       int slot_offset, uint8_t* send, ft8_result* overflow, hipStream_t s) {
  static_assert(sizeof(ft8_result) % 8 == 0, "records are copied as 8-byte words");
  hipLaunchKernelGGL(k_pack, dim3(1), dim3(kPackThreads), 0, s, rec, counts, n_slots, cap, capacity, slot_offset,
                     send, overflow);
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
