// sync.hip -- Costas-7 sync score grid and the reference's candidate selection (gfx950).
//
// k_score2 / k_score replace ft8_sync_score over the ft8_find_candidates grid (reference
// ft8_decode.py:47-100, 108-131; FT8Candidate.get_log_power ftx_types.py:45-47).  Every candidate
// (abs_time, abs_freq) accumulates its up-to-75 dB differences SEQUENTIALLY in the reference order
// (m, k, then tone-1, tone+1, time-1, time+1): on the float32 waterfall of a WAV the reference sums
// in np.float32 (NumPy-2 promotion, ft8_decode.py:57,80-94) and any re-association would change
// the last bit of the score, so the sum is never tree-reduced.
//
// k_score2 (float32 waterfall, bins_per_tone = steps_per_symbol in {1..4, 10}, the production path):
//   * a workgroup owns 128 frequency columns x 22 time rows of the grid of one slot, the rows one
//     residue class mod sps; it stages the three Costas bands of the waterfall those candidates
//     touch one at a time ((22 + 8) rows of stride sps x (128 + 7 bpt) columns, 17 KB at
//     bpt = sps = 2) in LDS;
//   * a wave owns one time row at a time (so every range test of the reference is wave-uniform and
//     compiles to a scalar branch) and each lane two adjacent columns: the pair is accumulated
//     with packed float32 adds (v_pk_add_f32, two independent IEEE sums) from 8-byte LDS reads
//     whose addresses are one per-lane base plus compile-time immediates;
//   * slots map to XCDs (workgroup id % 8), so all tiles of a slot share one L2;
//   * each wave also folds its row into a per-(slot, row) summary -- passing count and largest
//     passing score -- which lets k_select skip the rows it does not need.
// k_score (float64 waterfalls and other oversampling factors) is the plain one-thread-per-
// candidate form of the same sum.
//
// k_select replaces the heap logic of ft8_find_candidates (ft8_decode.py:113-140), one 1024-thread
// workgroup per slot.  The reference heap stores (-score, cand) and admits a candidate into a full
// heap only when it beats heap[0] -- the CURRENT MAXIMUM -- which it then evicts.  The selected set
// is therefore: the first N passing candidates in scan order (time outer, frequency inner), with
// the maximum of those replaced by each later strict new maximum ("record") in turn, i.e. by the
// first occurrence of the global maximum when that lies beyond rank N.  From the row summaries
// the kernel finds the rows holding ranks < N and the row of the global maximum, and scans only
// those; it sorts the set by score, and only when two selected scores are exactly equal (where
// the reference's order depends on heap array positions) replays the reference's N heappushes
// (one wave wide) to rebuild the heap array and reproduce its stable sort.
#include <climits>

#include "ft8_internal.h"
#include "heap_replay.h"

namespace ft8 {
namespace {

__constant__ int kCostasD[7] = {3, 1, 4, 0, 6, 5, 2};  // ft8_decode.py:42
constexpr int kCostasC[7] = {3, 1, 4, 0, 6, 5, 2};

constexpr int kScoreThreads = 256;
constexpr size_t kScoreLdsBudget = 64 * 1024;

struct ScoreArgs {
  const void* wf;
  int T, F, sps, bpt, num_blocks;
  int t0, NT, NF;
  int rlo, nrows;    // staged rows [rlo, rlo + nrows)
  void* scores;
  uint64_t* smask;   // [slot][NT][nseg][2] passing columns per 128-column segment
  int nseg;
  RowSummary* rowsum;
  double min_score;
  int cmp_f64;
  int n_slots, n_bands, n_ctiles;  // k_score2 grid
};

// ft8_find_candidates' admission test (ft8_decode.py:127): not -inf and not below min_score, the
// comparison done in the score's dtype unless min_score is a float64 scalar
template <typename T>
__device__ __forceinline__ bool passes(T s, double ms, int cmp_f64) {
  if (s == (T)-INFINITY) return false;
  if (cmp_f64) return !((double)s < ms);
  return !(s < (T)ms);
}

template <typename T, bool LDS, int TW>
__global__ __launch_bounds__(kScoreThreads) void k_score(ScoreArgs a) {
  FT8_RACE_PROLOGUE();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* tile = reinterpret_cast<T*>(smem);
  const int slot = blockIdx.y;
  const int c0 = blockIdx.x * TW;
  const T* wf = reinterpret_cast<const T*>(a.wf) + (int64_t)slot * a.T * a.F;
  const int ncols = min(TW + 7 * a.bpt, a.F - c0);
  if constexpr (LDS) {
    const int n = a.nrows * ncols;
    for (int i = threadIdx.x; i < n; i += kScoreThreads) {
      const int r = i / ncols, c = i - r * ncols;
      tile[i] = wf[(int64_t)(a.rlo + r) * a.F + c0 + c];
    }
    __syncthreads();
  }
  auto get = [&](int row, int col) -> T {
    if constexpr (LDS) return tile[(row - a.rlo) * ncols + (col - c0)];
    else return wf[(int64_t)row * a.F + col];
  };
  const int lane_col = threadIdx.x % TW;
  const int rgroup = threadIdx.x / TW;
  constexpr int kGroups = kScoreThreads / TW;
  const int af = c0 + lane_col;
  T* out = reinterpret_cast<T*>(a.scores) + (int64_t)slot * a.NT * a.NF;
  RowSummary* rs = a.rowsum + (int64_t)slot * a.NT * a.nseg;
  const int sps = a.sps, bpt = a.bpt, nb = a.num_blocks;
  for (int ti = rgroup; ti < a.NT; ti += kGroups) {
    if (af >= a.NF) continue;
    const int at = a.t0 + ti;
    const int base = floordiv(at, sps);
    T score = (T)0;
    int n = 0;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const int block = 36 * m + k;
        const int ba = base + block;
        if (ba < 0 || ba >= nb) continue;
        const int tone = kCostasD[k];
        const int row = at + block * sps;
        const int col = af + tone * bpt;
        const T p = get(row, col);
        if (tone > 0) { score += (T)(p - get(row, col - bpt)); n++; }
        if (tone < 7) { score += (T)(p - get(row, col + bpt)); n++; }
        if (k > 0 && ba > 0) { score += (T)(p - get(row - sps, col)); n++; }
        if (k < 6 && ba + 1 < nb) { score += (T)(p - get(row + sps, col)); n++; }
      }
    }
    T res;
    if (n == 0 || isnan(score) || isinf(score)) res = (T)-INFINITY;
    else res = score / (T)n;
    out[(int64_t)ti * a.NF + af] = res;
    if (passes(res, a.min_score, a.cmp_f64)) {
      RowSummary* e = rs + (int64_t)ti * a.nseg + af / kSegCols;
      atomicAdd(&e->count, 1u);
      atomicMax(&e->maxkey, order_key((double)res));
      const int c = af % kSegCols;
      atomicOr(reinterpret_cast<unsigned long long*>(
                   &a.smask[(((int64_t)slot * a.NT + ti) * a.nseg + af / kSegCols) * 2 + (c & 1)]),
               1ull << (c >> 1));
    }
  }
}

// ---- k_score_list: ft8_sync_score for arbitrary candidates ------------------------------------------
// One thread per (abs_time, abs_freq), exactly ft8_sync_score (ft8_decode.py:47-100) including what
// the grid kernels never meet: FT8Candidate.get_log_power indexes mag[freq, time] with NumPy's rules
// (ftx_types.py:45-47), so a negative index counts from the end and an index past either end raises
// IndexError -- flagged in err[i] (the score is then meaningless).  Only the time-block test of the
// reference guards the accesses; nothing guards the frequency.
template <typename T>
__global__ void k_score_list(const T* wf, int Tn, int F, int sps, int bpt, const int32_t* cand, int n, T* out,
                             int32_t* err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int at = cand[2 * i], af = cand[2 * i + 1];
  const int nb = Tn / sps;
  bool bad = false;
  auto get = [&](int64_t t, int64_t f) -> T {  // mag[f, t] with NumPy indexing
    if (f < 0) f += F;
    if (t < 0) t += Tn;
    if (f < 0 || f >= F || t < 0 || t >= Tn) { bad = true; return (T)0; }
    return wf[t * F + f];
  };
  const int base = floordiv(at, sps);
  T score = (T)0;
  int cnt = 0;
  for (int m = 0; m < 3; ++m) {
    for (int k = 0; k < 7; ++k) {
      const int block = 36 * m + k;
      const int ba = base + block;
      if (ba < 0 || ba >= nb) continue;
      const int tone = kCostasD[k];
      const int64_t row = (int64_t)at + (int64_t)block * sps, col = (int64_t)af + (int64_t)tone * bpt;
      const T p = get(row, col);
      if (tone > 0) { score += (T)(p - get(row, col - bpt)); cnt++; }
      if (tone < 7) { score += (T)(p - get(row, col + bpt)); cnt++; }
      if (k > 0 && ba > 0) { score += (T)(p - get(row - sps, col)); cnt++; }
      if (k < 6 && ba + 1 < nb) { score += (T)(p - get(row + sps, col)); cnt++; }
    }
  }
  out[i] = (cnt == 0 || isnan(score) || isinf(score)) ? (T)-INFINITY : score / (T)cnt;
  err[i] = bad ? 1 : 0;
}

// ---- k_score2 ----------------------------------------------------------------------------------
constexpr int kS2TW = 128;                 // grid columns per workgroup (64 lanes x 2)
constexpr int kS2R = 22;                   // grid rows per workgroup (88 = 4 x 22 at 12 kHz)
constexpr int kS2Waves = 8;                // row j of the workgroup on wave j % 8
constexpr int kS2Rows = (kS2R + kS2Waves - 1) / kS2Waves;  // rows per wave (3, the last two waves 2)
constexpr int kS2Threads = kS2Waves * kWave;
typedef float f32x2 __attribute__((ext_vector_type(2)));

// A workgroup's 22 grid rows are one residue class mod sps, consecutive in it: abs_time a0 +
// sps j, j < 22.  Every waterfall row those candidates read for Costas band m is a0 + 36 m sps +
// sps (j + k + d) (symbol k, time neighbour d = -1, 0, 1), so the band's tile is 22 + 8 rows of
// stride sps -- one tile row per symbol step, whatever sps is -- instead of 22 + 8 sps consecutive
// rows, most of them unread (at sps = 10, 102 rows for 30 used; sps = 2: 38 for 30).
template <int BPT, int SPS>
struct S2Geom {
  static constexpr int P = (kS2TW + 7 * BPT + 3) & ~3;   // staged columns (multiple of 4: float4 rows)
  static constexpr int H = kS2R + 8;                     // staged rows of one Costas band
  static constexpr int kFloats = H * P;                  // the LDS tile: one band at a time
  static constexpr int Q = P / 4;                        // float4 per staged row
  static constexpr int kIter = (H * Q + kS2Threads - 1) / kS2Threads;  // float4 staged per thread
};

// maximum over the wave (no NaN), on order-preserving integer keys (a float max would re-quiet
// every DPP operand): rotations inside each 16-lane row (DPP row_ror 8, 4, 2, 1), then the four
// row maxima in scalar registers -- instead of six ds_bpermute rounds
__device__ __forceinline__ int fkey(float v) {
  const int i = __float_as_int(v);
  return i ^ ((i >> 31) & 0x7fffffff);
}
template <int CTRL>
__device__ __forceinline__ int dpp_max(int k) {
  return max(k, __builtin_amdgcn_mov_dpp(k, CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_max(float v) {
  int k = fkey(v);
  k = dpp_max<0x128>(k);  // row_ror:8
  k = dpp_max<0x124>(k);  // row_ror:4
  k = dpp_max<0x122>(k);  // row_ror:2
  k = dpp_max<0x121>(k);  // row_ror:1
  const int m = max(max(__builtin_amdgcn_readlane(k, 0), __builtin_amdgcn_readlane(k, 16)),
                    max(__builtin_amdgcn_readlane(k, 32), __builtin_amdgcn_readlane(k, 48)));
  return __int_as_float(m ^ ((m >> 31) & 0x7fffffff));
}

// volatile LDS load: one ds_read_b64 per pair.  The compiler would otherwise merge neighbouring
// pairs into ds_read2_b64, which moves half as many bytes per LDS cycle (measured: k_score2 0.27
// vs 0.30 ms per 256-slot step).
template <int BPT>
__device__ __forceinline__ f32x2 ld2(const float* p) {
  if constexpr (BPT % 2 == 0) return *(const volatile __attribute__((address_space(3))) f32x2*)p;
  else return f32x2{p[0], p[1]};
}

// Costas band m of the tile (staged rows a0 - SPS + 36 m SPS + SPS u, u < H; columns [c0, c0 + P))
// as float4 loads into registers; rows outside the waterfall / columns past F are zero and never
// read by a valid candidate.  Thread t owns float4 t + 512 it.
// The thread's part of that staging, computed once per workgroup: for each of its float4s the
// band-0 row (a sentinel far below 0 when the float4 lies past the tile or past column F) and its
// element offset row * F + col; band m adds 36 m SPS rows to both (round 6: the division by Q,
// the row/column arithmetic and the 64-bit address were re-derived for every band).
template <int BPT, int SPS>
struct S2Stage {
  int row0[S2Geom<BPT, SPS>::kIter];
  int off0[S2Geom<BPT, SPS>::kIter];
};
template <int BPT, int SPS>
__device__ __forceinline__ S2Stage<BPT, SPS> s2_stage(int F, int a0, int c0) {
  using G = S2Geom<BPT, SPS>;
  S2Stage<BPT, SPS> st;
#pragma unroll
  for (int it = 0; it < G::kIter; ++it) {
    const int idx = (int)threadIdx.x + it * kS2Threads;
    const int rw = idx / G::Q, q4 = idx - rw * G::Q;
    const int row = a0 - SPS + SPS * rw, col = c0 + 4 * q4;
    const bool ok = idx < G::H * G::Q && col < F;
    st.row0[it] = ok ? row : INT_MIN / 2;
    st.off0[it] = row * F + col;   // slot waterfalls hold < 2^31 floats
  }
  return st;
}
template <int BPT, int SPS>
__device__ __forceinline__ void s2_load(const float* wf, int T, int F, const S2Stage<BPT, SPS>& st, int m,
                                        float4 (&v)[S2Geom<BPT, SPS>::kIter]) {
  using G = S2Geom<BPT, SPS>;
  const int drow = 36 * m * SPS;                  // wave-uniform
  const float* wb = wf + (int64_t)drow * F;
#pragma unroll
  for (int it = 0; it < G::kIter; ++it) {
    const int row = st.row0[it] + drow;
    v[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)row < (unsigned)T) v[it] = *reinterpret_cast<const float4*>(wb + st.off0[it]);
  }
}

// One workgroup: 128 grid columns x 22 grid rows of one slot (one residue class mod sps, above).
// The three Costas bands of the waterfall the candidates read are staged into LDS ONE AT A TIME
// (17 KB at bpt = sps = 2, 24 KB at bpt = sps = 10), band m + 1's global loads in flight while band m
// is scored;
// each wave keeps its rows' two-column partial sums in registers across the bands, so every score
// still accumulates its 75 terms in the reference's order (band, symbol, tone-1, tone+1, time-1,
// time+1).
template <int BPT, int SPS, bool COMPACT>
__global__ __launch_bounds__(kS2Threads) void k_score2(ScoreArgs a) {
  FT8_RACE_PROLOGUE();
  static_assert(kS2TW == kSegCols, "a workgroup's columns are one score segment");
  using G = S2Geom<BPT, SPS>;
  constexpr int P = G::P;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* tile = reinterpret_cast<float*>(smem);
  // workgroup -> (slot, row tile, column tile); slot % 8 == workgroup id % 8 keeps a slot on one XCD
  const int id = blockIdx.x;
  const int per = a.n_bands * a.n_ctiles;
  const int q = id >> 3;
  const int slot = (q / per) * 8 + (id & 7);
  if (slot >= a.n_slots) return;
  const int r = q % per;
  const int band = r / a.n_ctiles, ct = r - band * a.n_ctiles;
  // band -> (residue class c of the grid rows mod SPS, 22-row tile b of the class)
  const int nbpc = a.n_bands / SPS;
  const int cls = band / nbpc, i0 = (band - cls * nbpc) * kS2R;
  const int cnt = (a.NT - cls + SPS - 1) / SPS;  // grid rows of the class
  if (i0 >= cnt) return;                          // (workgroup-uniform)
  const int a0 = a.t0 + cls + SPS * i0;           // abs_time of the tile's first candidate row
  const int c0 = ct * kS2TW;
  const float* wf = reinterpret_cast<const float*>(a.wf) + (int64_t)slot * a.T * a.F;
  const bool vec = (a.F & 3) == 0;

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int af = c0 + 2 * lane;
  const int nb = a.num_blocks;
  const int rows = min(kS2R, cnt - i0);
  f32x2 score[kS2Rows];
  int n[kS2Rows];
#pragma unroll
  for (int u = 0; u < kS2Rows; ++u) {
    score[u] = f32x2{0.0f, 0.0f};
    n[u] = 0;
  }

  float4 v[G::kIter];
  const S2Stage<BPT, SPS> stg = s2_stage<BPT, SPS>(a.F, a0, c0);
  if (vec) s2_load<BPT, SPS>(wf, a.T, a.F, stg, 0, v);
#pragma unroll 1
  for (int m = 0; m < 3; ++m) {
    if (m > 0) __syncthreads();  // every wave has scored band m - 1
    if (vec) {
#pragma unroll
      for (int it = 0; it < G::kIter; ++it) {
        const int idx = (int)threadIdx.x + it * kS2Threads;
        if (idx < G::H * G::Q) reinterpret_cast<float4*>(tile)[idx] = v[it];
      }
      if (m < 2) s2_load<BPT, SPS>(wf, a.T, a.F, stg, m + 1, v);  // in flight while band m is scored
    } else {
      for (int i = threadIdx.x; i < G::kFloats; i += kS2Threads) {
        const int rr = i / P, cc = i - rr * P;
        const int row = a0 + 36 * m * SPS - SPS + SPS * rr, col = c0 + cc;
        float x = 0.0f;
        if (row >= 0 && row < a.T && col < a.F) x = wf[(int64_t)row * a.F + col];
        tile[i] = x;
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kS2Rows; ++u) {
      const int j = w + u * kS2Waves;        // wave-uniform
      if (j >= rows) continue;
      // block index of the band's first Costas symbol for abs_time a0 + SPS j
      const int lo = floordiv(a0, SPS) + j + 36 * m;
      const float* tb = tile + j * P + 2 * lane;  // tile row j + k + 1: symbol k, +-1: time neighbours
      if (lo >= 0 && lo <= nb - 7) {
        // every symbol of the band and all its neighbours in range: straight-line code
        // (25 differences, in the reference order)
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          const int tone = kCostasC[k];
          const float* rp = tb + (k + 1) * P + tone * BPT;
          const f32x2 pw = ld2<BPT>(rp);
          if (tone > 0) score[u] += pw - ld2<BPT>(rp - BPT);
          if (tone < 7) score[u] += pw - ld2<BPT>(rp + BPT);
          if (k > 0) score[u] += pw - ld2<BPT>(rp - P);
          if (k < 6) score[u] += pw - ld2<BPT>(rp + P);
        }
        n[u] += 25;
      } else if (lo + 6 >= 0 && lo < nb) {
        // a band crossing the waterfall's first or last block: the reference's per-term tests
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          const int ba = lo + k;
          if (ba < 0 || ba >= nb) continue;
          const int tone = kCostasC[k];
          const float* rp = tb + (k + 1) * P + tone * BPT;
          const f32x2 pw = ld2<BPT>(rp);
          if (tone > 0) { score[u] += pw - ld2<BPT>(rp - BPT); n[u]++; }
          if (tone < 7) { score[u] += pw - ld2<BPT>(rp + BPT); n[u]++; }
          if (k > 0 && ba > 0) { score[u] += pw - ld2<BPT>(rp - P); n[u]++; }
          if (k < 6 && ba + 1 < nb) { score[u] += pw - ld2<BPT>(rp + P); n[u]++; }
        }
      }
    }
  }

  float* out = reinterpret_cast<float*>(a.scores) + (COMPACT ? 0 : (int64_t)slot * a.NT * a.NF);
  RowSummary* rs = a.rowsum + (int64_t)slot * a.NT * a.nseg;
#pragma unroll
  for (int u = 0; u < kS2Rows; ++u) {
    const int j = w + u * kS2Waves;
    if (j >= rows) continue;
    float res[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float sc = score[u][c];
      res[c] = (n[u] == 0 || isnan(sc) || isinf(sc)) ? -INFINITY : sc / (float)n[u];
    }
    const int ti = a0 + SPS * j - a.t0;
    const bool v0 = af < a.NF, v1 = af + 1 < a.NF;
    const bool p0 = v0 && passes(res[0], a.min_score, a.cmp_f64);
    const bool p1 = v1 && passes(res[1], a.min_score, a.cmp_f64);
    const uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
    const int64_t seg = ((int64_t)slot * a.NT + ti) * a.nseg + ct;
    if (COMPACT) {
      // the passing scores of the segment, in column order, packed at its start: column 2l has
      // rank popc(b0 below l) + popc(b1 below l), column 2l + 1 one more if column 2l passes
      const uint64_t below = (1ull << lane) - 1ull;
      const int r0 = __popcll(b0 & below) + __popcll(b1 & below);
      float* sv = out + seg * kSegCols;
      if (p0) sv[r0] = res[0];
      if (p1) sv[r0 + (p0 ? 1 : 0)] = res[1];
    } else {
      float* orow = out + (int64_t)ti * a.NF;
      if (v0) orow[af] = res[0];
      if (v1) orow[af + 1] = res[1];
    }
    if (lane == 0) *reinterpret_cast<ulonglong2*>(a.smask + 2 * seg) = make_ulonglong2(b0, b1);
    // the (row, segment) summary: this wave is the segment's only writer, so a plain store (every
    // entry written, none skipped: no memset, no atomics)
    const unsigned cnt = (unsigned)(__popcll(b0) + __popcll(b1));
    unsigned long long key = 0ull;
    if (cnt) {
      float mx = p0 ? res[0] : -INFINITY;
      if (p1) mx = fmaxf(mx, res[1]);
      mx = wave_max(mx);
      key = order_key((double)mx);
    }
    if (lane == 0) {
      RowSummary e;
      e.count = cnt;
      e.pad = 0;
      e.maxkey = key;
      rs[seg - (int64_t)slot * a.NT * a.nseg] = e;
    }
  }
}

template <int BPT, int SPS, bool COMPACT>
hipError_t launch_score2(const SyncLaunch& L, const ScoreArgs& a0, hipStream_t s) {
  using G = S2Geom<BPT, SPS>;
  ScoreArgs a = a0;
  // SPS residue classes of the grid rows, each cut into 22-row tiles (classes hold ceil(NT / SPS)
  // rows at most; a tile past its class's rows exits at once)
  a.n_bands = SPS * ((((L.NT + SPS - 1) / SPS) + kS2R - 1) / kS2R);
  a.n_ctiles = (L.NF + kS2TW - 1) / kS2TW;
  const size_t lds = sizeof(float) * G::kFloats;
  static_assert(sizeof(float) * S2Geom<4, 4>::kFloats <= 64 * 1024, "one band fits the default LDS limit");
  static_assert(sizeof(float) * G::kFloats <= 160 * 1024, "one band fits the CU's LDS");
  if constexpr (sizeof(float) * G::kFloats > 64 * 1024) {
    // (no geometry built today needs it: bpt = sps = 10's band is 30 rows x 200 columns, 24 KB)
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_score2<BPT, SPS, COMPACT>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const int groups = (L.n_slots + 7) / 8;
  const int64_t blocks = (int64_t)groups * 8 * a.n_bands * a.n_ctiles;
  hipLaunchKernelGGL((k_score2<BPT, SPS, COMPACT>), dim3((unsigned)blocks), dim3(kS2Threads), lds, s, a);
  return hipGetLastError();
}

bool score2_path(const SyncLaunch& L) {
  return !L.wf_f64 && L.bpt == L.sps && ((L.bpt >= 1 && L.bpt <= 4) || L.bpt == 10);
}
template <int B>
hipError_t launch_score2_any(const SyncLaunch& L, const ScoreArgs& a, hipStream_t s) {
  return score_compact(L) ? launch_score2<B, B, true>(L, a, s) : launch_score2<B, B, false>(L, a, s);
}

template <typename T, int TW>
hipError_t launch_score_t(const SyncLaunch& L, hipStream_t s) {
  ScoreArgs a{};
  a.wf = L.wf;
  a.T = L.T;
  a.F = L.F;
  a.sps = L.sps;
  a.bpt = L.bpt;
  a.num_blocks = L.T / L.sps;
  a.t0 = L.t0;
  a.NT = L.NT;
  a.NF = L.NF;
  a.scores = L.scores;
  a.smask = L.smask;
  a.nseg = n_segments(L.NF);
  a.rowsum = L.rowsum;
  a.min_score = L.min_score;
  a.cmp_f64 = L.min_score_f64;
  a.n_slots = L.n_slots;
  hipError_t e = hipSuccess;
  if constexpr (sizeof(T) == 4) {
    if (score2_path(L)) {
      switch (L.bpt) {
        case 1: return launch_score2_any<1>(L, a, s);
        case 2: return launch_score2_any<2>(L, a, s);
        case 3: return launch_score2_any<3>(L, a, s);
        case 4: return launch_score2_any<4>(L, a, s);
        case 10: return launch_score2_any<10>(L, a, s);
        default: break;
      }
    }
  }
  // k_score sets the mask bits and the (row, segment) summaries of its passing candidates one by one
  // (k_score2 writes every entry of both: no memset on its path)
  e = hipMemsetAsync(L.smask, 0, sizeof(uint64_t) * 2 * (size_t)L.n_slots * L.NT * a.nseg, s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(L.rowsum, 0, sizeof(RowSummary) * (size_t)L.n_slots * L.NT * a.nseg, s);
  if (e != hipSuccess) return e;
  // rows touched by the grid: [t0 - sps, t0 + NT - 1 + 79 sps], clipped to the waterfall
  a.rlo = max(0, L.t0 - L.sps);
  const int rhi = min(L.T - 1, L.t0 + L.NT - 1 + 79 * L.sps);
  a.nrows = rhi - a.rlo + 1;
  const int ncols = TW + 7 * L.bpt;
  const size_t lds = (size_t)a.nrows * ncols * sizeof(T);
  dim3 grid((L.NF + TW - 1) / TW, L.n_slots);
  if (lds <= kScoreLdsBudget)
    hipLaunchKernelGGL((k_score<T, true, TW>), grid, dim3(kScoreThreads), lds, s, a);
  else
    hipLaunchKernelGGL((k_score<T, false, TW>), grid, dim3(kScoreThreads), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// selection
// ---------------------------------------------------------------------------------------------
constexpr int kSelThreads = 1024;
constexpr int kSelWaves = kSelThreads / kWave;

struct SelectArgs {
  const void* scores;
  int64_t total;
  int NF, t0, N;
  double min_score;
  int cmp_f64;
  int32_t* cand;
  double* cand_score;
  int32_t* cand_count;
  int32_t* warn;
  const RowSummary* rowsum;
  int NT;
  int32_t* tie;  // nullable: defer the order of equal scores (tie_stride(N) ints per slot)
  const uint64_t* smask;  // [slot][NT][nseg][2] passing columns per segment
  int nseg;
  int compact;   // scores hold the compact segment layout (else the full grid)
};

// block-wide exclusive scans over 1024 threads (int sum and double max), via wave shuffles
__device__ int block_excl_sum(int v, int* sh, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < kSelWaves; ++i) { int t = sh[i]; sh[i] = acc; acc += t; }
    sh[kSelWaves] = acc;
  }
  __syncthreads();
  const int r = sh[w] + x - v;
  *total = sh[kSelWaves];
  __syncthreads();
  return r;
}
// bitonic sort of n items by (key asc, sec asc) in LDS (padded to a power of two <= cap)
__device__ void bitonic(double* key, int* sec, int* pay, int n) {
  int m = 1;
  while (m < n) m <<= 1;
  for (int i = n + threadIdx.x; i < m; i += kSelThreads) { key[i] = INFINITY; sec[i] = 0x7fffffff; pay[i] = -1; }
  __syncthreads();
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < m; i += kSelThreads) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const bool gt = key[i] > key[l] || (key[i] == key[l] && sec[i] > sec[l]);
          if (gt == up) {
            double tk = key[i]; key[i] = key[l]; key[l] = tk;
            int ts = sec[i]; sec[i] = sec[l]; sec[l] = ts;
            int tp = pay[i]; pay[i] = pay[l]; pay[l] = tp;
          }
        }
      }
      __syncthreads();
    }
  }
}

// (key asc, sec asc) order of n items in LDS, in place (sec is distinct).  Up to 1024 items: one
// per thread in registers, a bitonic network whose exchanges of partners less than 64 apart are
// wave shuffles and only the six (at 512 items) farther ones go through LDS with barriers -- the
// LDS network (bitonic) takes a barrier for every one of its 45 rounds.  Larger sets take bitonic.
__device__ __forceinline__ bool kv_less(double ka, int sa, double kb, int sb) {
  return ka < kb || (ka == kb && sa < sb);
}
__device__ void sort_kv(double* key, int* sec, int* pay, int n) {
  if (n > kSelThreads) {
    bitonic(key, sec, pay, n);
    return;
  }
  int m = 1;
  while (m < n) m <<= 1;
  const int t = threadIdx.x;
  double k_ = INFINITY;
  int s_ = 0x7fffffff, p_ = -1;
  if (t < n) {
    k_ = key[t];
    s_ = sec[t];
    p_ = pay[t];
  }
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      double ko;
      int so, po;
      if (j >= kWave) {
        __syncthreads();  // every earlier read of the arrays is done
        if (t < m) {
          key[t] = k_;
          sec[t] = s_;
          pay[t] = p_;
        }
        __syncthreads();
        const int q = t ^ j;
        ko = t < m ? key[q] : k_;
        so = t < m ? sec[q] : s_;
        po = t < m ? pay[q] : p_;
      } else {
        ko = __shfl_xor(k_, j);
        so = __shfl_xor(s_, j);
        po = __shfl_xor(p_, j);
      }
      // ascending blocks where (t & k) == 0; the lower index of a pair keeps the smaller there
      const bool up = (t & k) == 0, lower = (t & j) == 0;
      const bool take = (up == lower) ? kv_less(ko, so, k_, s_) : kv_less(k_, s_, ko, so);
      if (take && t < m) {
        k_ = ko;
        s_ = so;
        p_ = po;
      }
    }
  }
  __syncthreads();
  if (t < n) {
    key[t] = k_;
    sec[t] = s_;
    pay[t] = p_;
  }
  __syncthreads();
}

// block-wide maximum of a u64 key
__device__ unsigned long long block_max_u64(unsigned long long v, unsigned long long* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(v, o);
    v = y > v ? y : v;
  }
  if (lane == 0) sh[w] = v;
  __syncthreads();
  unsigned long long m = 0;
  for (int i = 0; i < kSelWaves; ++i) m = sh[i] > m ? sh[i] : m;
  __syncthreads();
  return m;
}

// 32 bits spread to the even bit positions of a 64-bit word
__device__ __forceinline__ uint64_t spread32(uint32_t v) {
  uint64_t x = v;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}
// position of the k-th (0-based) set bit of w (k < popcount(w))
__device__ __forceinline__ int select_bit(uint64_t w, int k) {
  int pos = 0;
#pragma unroll
  for (int width = 32; width > 0; width >>= 1) {
    const int c = __popcll(w & ((1ull << width) - 1ull));
    if (k >= c) {
      k -= c;
      w >>= width;
      pos += width;
    }
  }
  return pos;
}
// rank of column col among the passing columns of a segment (masks: even / odd columns)
__device__ __forceinline__ int seg_rank(uint64_t e, uint64_t o, int col) {
  const int l = col >> 1;
  const uint64_t below = (1ull << l) - 1ull;
  return __popcll(e & ((col & 1) ? (below << 1 | 1ull) : below)) + __popcll(o & below);
}

template <typename T>
__global__ __launch_bounds__(kSelThreads) void k_select(SelectArgs a) {
  FT8_RACE_PROLOGUE();
  __shared__ double s_key[kMaxCandidates + 2];
  __shared__ int s_sec[kMaxCandidates + 2];
  __shared__ int s_pay[kMaxCandidates + 2];
  __shared__ int s_rank[kMaxCandidates];     // scan index of passing candidate #rank (rank < N)
  __shared__ T s_val[kMaxCandidates];        // its score
  __shared__ int s_segoff[kSelThreads];      // a chunk of segments: rank of each one's first entry
  __shared__ uint64_t s_cm[kSelThreads][2];  // its passing columns in column order (0..63, 64..127)
  __shared__ int s_isum[kSelWaves + 1];
  __shared__ unsigned long long s_umax[kSelWaves];
  __shared__ int s_flag[6];
  __shared__ double s_am_v[kSelWaves];
  __shared__ int s_am_i[kSelWaves];

  const int slot = blockIdx.x;
  const int nseg = a.nseg;
  const int64_t seg0 = (int64_t)slot * a.NT * nseg;
  const uint64_t* mk = a.smask + 2 * seg0;
  // a passing score: segment sg (of this slot), its j-th passing column, grid column c
  auto value = [&](int sg, int j, int c) -> T {
    if (a.compact) return reinterpret_cast<const T*>(a.scores)[(seg0 + sg) * kSegCols + j];
    const int row = sg / nseg;
    return reinterpret_cast<const T*>(a.scores)[(int64_t)slot * a.total + (int64_t)row * a.NF + c];
  };
  const RowSummary* rsum = a.rowsum + (int64_t)slot * a.NT * nseg;
  // a row's summary: its segments' passing counts added, their largest keys maxed
  // (16 segments' loads issued back to back: one round trip per row at the 12 kHz geometry's 15)
  auto row_count_key = [&](int r, int* cnt, unsigned long long* key) {
    int c_ = 0;
    unsigned long long k_ = 0ull;
    const RowSummary* rr = rsum + (int64_t)r * nseg;
    for (int s0 = 0; s0 < nseg; s0 += 16) {
      uint4 e[16];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        e[u] = s0 + u < nseg ? *reinterpret_cast<const uint4*>(rr + s0 + u) : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const unsigned long long k2 = ((unsigned long long)e[u].w << 32) | e[u].z;
        c_ += (int)e[u].x;
        k_ = k2 > k_ ? k2 : k_;
      }
    }
    *cnt = c_;
    *key = k_;
  };
  const int N = a.N;

  // ---- row summaries: total passing, rows holding ranks < N, first row of the global maximum
  if (threadIdx.x == 0) { s_flag[4] = a.NT; s_flag[5] = a.NT; }
  int total_pass = 0;
  unsigned long long gkey = 0, key0 = 0;
  for (int r0 = 0; r0 < a.NT; r0 += kSelThreads) {
    const int r = r0 + threadIdx.x;
    int cnt = 0;
    unsigned long long key = 0ull;
    if (r < a.NT) row_count_key(r, &cnt, &key);
    if (r0 == 0) key0 = key;   // this thread's first row: the maximum search below reuses it
    int ctot;
    const int ex = total_pass + block_excl_sum(cnt, s_isum, &ctot);
    if (cnt > 0 && ex < N && ex + cnt >= N) s_flag[4] = r + 1;  // exactly one row holds rank N-1
    const unsigned long long m = block_max_u64(key, s_umax);
    gkey = m > gkey ? m : gkey;
    total_pass += ctot;
  }
  __syncthreads();
  if (gkey != 0)
    for (int r = threadIdx.x; r < a.NT; r += kSelThreads) {
      int c_;
      unsigned long long k_ = key0;
      if (r >= kSelThreads) row_count_key(r, &c_, &k_);
      if (k_ == gkey) atomicMin(&s_flag[5], r);
    }
  __syncthreads();
  const int r_end = s_flag[4];   // rows [0, r_end) hold every rank < N
  const int g_row = s_flag[5];   // first row holding the global maximum (NT if nothing passes)
  const T g_val = (T)key_value(gkey);
  const int nsel = min(total_pass, N);

  // ---- ranks < N in scan order, from the segment masks of rows [0, r_end): chunks of segments,
  // an exclusive count scan gives each segment's first rank, then one thread per rank finds its
  // segment (binary search) and column (select in the column-order mask) and loads its score
  const int seg_end = r_end * nseg;
  int carry = 0;
  for (int g0 = 0; g0 < seg_end && carry < nsel; g0 += kSelThreads) {
    const int sg = g0 + (int)threadIdx.x;
    uint64_t e = 0, o = 0;
    if (sg < seg_end) {
      e = mk[2 * sg];
      o = mk[2 * sg + 1];
    }
    int ctot;
    const int off = carry + block_excl_sum(__popcll(e) + __popcll(o), s_isum, &ctot);
    s_segoff[threadIdx.x] = off;
    s_cm[threadIdx.x][0] = spread32((uint32_t)e) | (spread32((uint32_t)o) << 1);
    s_cm[threadIdx.x][1] = spread32((uint32_t)(e >> 32)) | (spread32((uint32_t)(o >> 32)) << 1);
    __syncthreads();
    const int n_here = min(kSelThreads, seg_end - g0);
    for (int r = carry + (int)threadIdx.x; r < min(carry + ctot, nsel); r += kSelThreads) {
      int lo = 0, hi = n_here - 1;  // the last segment whose first rank is <= r
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_segoff[mid] <= r) lo = mid;
        else hi = mid - 1;
      }
      const int j = r - s_segoff[lo];
      const uint64_t w0 = s_cm[lo][0];
      const int n0 = __popcll(w0);
      const int col = j < n0 ? select_bit(w0, j) : 64 + select_bit(s_cm[lo][1], j - n0);
      const int sgl = g0 + lo;
      const int row = sgl / nseg;
      const int c = (sgl - row * nseg) * kSegCols + col;
      s_rank[r] = row * a.NF + c;
      s_val[r] = value(sgl, j, c);
    }
    carry += ctot;
    __syncthreads();
  }

  // ---- a record exists iff the first occurrence of the global maximum has rank >= N, i.e. iff
  // the maximum exceeds every score of the first N (ft8_decode.py:134-137); it then ends in the heap
  double m1 = -INFINITY;
  for (int i = threadIdx.x; i < nsel; i += kSelThreads) m1 = fmax(m1, (double)s_val[i]);
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m1 = fmax(m1, __shfl_xor(m1, o));
    if (lane == 0) s_am_v[w] = m1;
    __syncthreads();
    m1 = -INFINITY;
    for (int i = 0; i < kSelWaves; ++i) m1 = fmax(m1, s_am_v[i]);
    __syncthreads();
  }
  const bool has_rec = nsel > 0 && total_pass > N && (double)g_val > m1;
  if (threadIdx.x == 0) { s_flag[0] = 0; s_flag[1] = 0; s_flag[3] = 0; s_am_i[0] = 0x7fffffff; }
  __syncthreads();
  if (has_rec) {
    // first column of row g_row holding the maximum (every earlier row's maximum is smaller)
    const int64_t rs0 = (int64_t)g_row * nseg;
    for (int c = threadIdx.x; c < a.NF; c += kSelThreads) {
      const int sg = (int)(rs0 + c / kSegCols), col = c % kSegCols;
      const uint64_t e = mk[2 * sg], o = mk[2 * sg + 1];
      if (!(((col & 1) ? o : e) >> (col >> 1) & 1ull)) continue;
      if ((double)value(sg, seg_rank(e, o, col), c) == (double)g_val) atomicMin(&s_am_i[0], g_row * a.NF + c);
    }
    __syncthreads();
  }
  const int gi = s_am_i[0];

  // the heap keeps the first N; each record evicts the current maximum (the top of the first N,
  // then the previous record): the final set is the first N with its top replaced by the last
  // record (ft8_decode.py:134-137)
  for (int i = threadIdx.x; i < nsel; i += kSelThreads) {
    const int idx = s_rank[i];
    s_key[i] = -(double)s_val[i];
    s_sec[i] = idx;
    s_pay[i] = idx;
  }
  __syncthreads();
  if (has_rec) {
    // the top of the first N (largest score, first in scan order among equals) is evicted; if its
    // score occurs twice among the first N the reference heap may have compared the two (tie)
    int top = 0x7fffffff;
    double tk = INFINITY;
    for (int i = threadIdx.x; i < nsel; i += kSelThreads)
      if (s_key[i] < tk || (s_key[i] == tk && s_sec[i] < s_sec[top])) { tk = s_key[i]; top = i; }
    {
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ok = __shfl_xor(tk, o);
        const int ot = __shfl_xor(top, o);
        const bool better = ot != 0x7fffffff &&
                            (top == 0x7fffffff || ok < tk || (ok == tk && s_sec[ot] < s_sec[top]));
        if (better) { tk = ok; top = ot; }
      }
      if (lane == 0) { s_am_v[w] = tk; s_isum[w] = top; }
      __syncthreads();
      if (threadIdx.x == 0) {
        for (int i = 1; i < kSelWaves; ++i) {
          const int ot = s_isum[i];
          if (ot == 0x7fffffff) continue;
          if (top == 0x7fffffff || s_am_v[i] < tk || (s_am_v[i] == tk && s_sec[ot] < s_sec[top])) {
            tk = s_am_v[i];
            top = ot;
          }
        }
        s_isum[0] = top;
        s_am_v[0] = tk;
      }
      __syncthreads();
      top = s_isum[0];
      tk = s_am_v[0];
    }
    for (int i = threadIdx.x; i < nsel; i += kSelThreads)
      if (i != top && s_key[i] == tk) s_flag[0] = 1;
    __syncthreads();
    if (threadIdx.x == 0) {
      s_key[top] = -(double)g_val;
      s_sec[top] = gi;
      s_pay[top] = gi;
    }
  }
  __syncthreads();

  // order: score descending; equal scores keep the reference's heap-array order (below)
  sort_kv(s_key, s_sec, s_pay, nsel);
  for (int i = threadIdx.x; i + 1 < nsel; i += kSelThreads)
    if (s_key[i] == s_key[i + 1]) s_flag[0] = 1;
  __syncthreads();

  bool deferred = false;
  if (s_flag[0]) {
    // Exact score ties in the final set: their order is the reference heap's array order, so
    // rebuild that array (heap_replay.h): the heap of the first N pushes with its root replaced by
    // the last record.
    if constexpr (std::is_same<T, float>::value) {
      deferred = a.tie != nullptr && nsel <= kReplayMax;
      if (deferred) {
        // leave the (score, scan index) order and hand the replay to one wave elsewhere: in
        // decode_batch the first workgroups of k_llr run it beside the LLRs (the set of candidates
        // is final; only the order of equal scores changes, which k_compact applies), in
        // ft8_sync_select k_tie_apply runs it and reorders the list
        int32_t* t = a.tie + (int64_t)slot * tie_stride(a.N);
        for (int i = threadIdx.x; i < nsel; i += kSelThreads) {
          t[i] = s_rank[i];
          t[a.N + i] = s_pay[i];
          t[7 * a.N + 2 + i] = __float_as_int(s_val[i]);
        }
        if (threadIdx.x == 0) {
          t[7 * a.N] = has_rec ? gi : -1;
          t[7 * a.N + 1] = __float_as_int(g_val);
        }
      }
    }
    if (!deferred) {
      for (int i = threadIdx.x; i < nsel; i += kSelThreads) {
        s_key[i] = -(double)s_val[i];
        s_sec[i] = s_rank[i];
      }
      __syncthreads();
      if (threadIdx.x < kWave) {
        const int lane = threadIdx.x;
        int tie = 0;
        {
          // float64 scores or N > kReplayMax: lane j holds the j-th ancestor of the new
          // position, a ballot finds how far the item rises
          for (int n = 1; n < nsel; ++n) {
            const double nk = s_key[n];
            const int ni = s_sec[n];
            const int d = 31 - __clz(n + 1);  // ancestors of position n
            double ak = 0.0;
            int ai = 0;
            if (lane < d) {
              const int pj = ((n + 1) >> (lane + 1)) - 1;
              ak = s_key[pj];
              ai = s_sec[pj];
            }
            const bool lt = lane < d && (nk < ak || (nk == ak && ni < ai));
            const int m = __ffsll((long long)~__ballot(lt)) - 1;  // the item passes ancestors 0..m-1
            if (__any(lane < d && lane <= m && nk == ak)) tie = 1;  // a compared parent with an equal key
            if (lane < m) {
              const int dest = lane == 0 ? n : ((n + 1) >> lane) - 1;
              s_key[dest] = ak;
              s_sec[dest] = ai;
            }
            if (lane == 0) {
              const int dest = m == 0 ? n : ((n + 1) >> m) - 1;
              s_key[dest] = nk;
              s_sec[dest] = ni;
            }
            asm volatile("" ::: "memory");  // the next push reads what this one wrote (in-order LDS)
          }
          if (lane == 0 && has_rec) {
            // the records' _siftup compares siblings along the min-child path (same path each time)
            int c = 1;
            while (c < nsel) {
              const int r = c + 1;
              if (r < nsel) {
                if (s_key[c] == s_key[r]) tie = 1;
                const bool cl = s_key[c] < s_key[r] || (s_key[c] == s_key[r] && s_sec[c] < s_sec[r]);
                if (!cl) c = r;
              }
              c = 2 * c + 1;
            }
            s_key[0] = -(double)g_val;
            s_sec[0] = gi;
          }
        }
        if (lane == 0) s_flag[3] = tie;
      }
      __syncthreads();
      // sorted(key=-score) is stable on heap-array order: secondary key = heap position
      for (int i = threadIdx.x; i < nsel; i += kSelThreads) { s_pay[i] = s_sec[i]; s_sec[i] = i; }
      __syncthreads();
      sort_kv(s_key, s_sec, s_pay, nsel);
    }
  }
  if (threadIdx.x == 0) {
    a.cand_count[slot] = nsel;
    a.warn[slot] = (s_flag[3] ? 1 : 0) | (s_flag[0] ? 4 : 0) | (deferred ? 8 : 0);
  }
  for (int i = threadIdx.x; i < nsel; i += kSelThreads) {
    const int idx = s_pay[i];
    a.cand[((int64_t)slot * a.N + i) * 2 + 0] = a.t0 + idx / a.NF;
    a.cand[((int64_t)slot * a.N + i) * 2 + 1] = idx % a.NF;
    a.cand_score[(int64_t)slot * a.N + i] = -s_key[i];
  }
}

// ---------------------------------------------------------------------------------------------
// FT8_FLAG_TOPK selection (build-defined, outside reference parity): the N highest passing scores,
// ties in scan order, sorted by score descending.  MSB-first radix select over order-preserving
// keys (11-bit digits, LDS histogram, early exit once the boundary digit holds exactly the ranks
// still needed), then one ordered compaction (contiguous scan ranges per thread, so equal scores
// at the threshold are taken in scan order) and the bitonic sort shared with k_select.
// ---------------------------------------------------------------------------------------------
constexpr int kTkBits = 11;
constexpr int kTkU = 8;  // grid loads in flight per thread
constexpr int kTkBins = 1 << kTkBits;

template <typename T> struct TkKey;
template <> struct TkKey<float> {
  using K = unsigned;
  static constexpr int kBits = 32;
  __device__ static K of(float v) {
    const unsigned u = __float_as_uint(v);
    return (u >> 31) ? ~u : (u | 0x80000000u);
  }
};
template <> struct TkKey<double> {
  using K = unsigned long long;
  static constexpr int kBits = 64;
  __device__ static K of(double v) { return order_key(v); }
};

template <typename T>
__global__ __launch_bounds__(kSelThreads) void k_topk(SelectArgs a) {
  FT8_RACE_PROLOGUE();
  using K = typename TkKey<T>::K;
  __shared__ double s_key[kMaxCandidates + 2];
  __shared__ int s_sec[kMaxCandidates + 2];
  __shared__ int s_pay[kMaxCandidates + 2];
  __shared__ unsigned s_hist[kTkBins];
  __shared__ int s_isum[kSelWaves + 1];
  __shared__ K s_prefix, s_mask;
  __shared__ int s_need, s_done, s_eqcnt, s_cnt;

  const int slot = blockIdx.x;
  const T* sc = reinterpret_cast<const T*>(a.scores) + (int64_t)slot * a.total;
  const int N = a.N;
  const int total = (int)a.total;
  // passing candidates map to non-zero keys (a key of 0 needs the NaN pattern 0xff..f, excluded)
  auto key = [&](int i) -> K {
    const T v = sc[i];
    return passes(v, a.min_score, a.cmp_f64) ? TkKey<T>::of(v) : (K)0;
  };
  if (threadIdx.x == 0) { s_prefix = 0; s_mask = 0; s_need = N; s_done = 0; s_eqcnt = 0; }
  __syncthreads();
  int total_pass = 0;
  for (int pass = 0;; ++pass) {
    int shift = TkKey<T>::kBits - kTkBits * (pass + 1), width = kTkBits;
    if (shift < 0) { width += shift; shift = 0; }
    const K dmask = ((K)1 << width) - 1;
    const K prefix = s_prefix, mask = s_mask;
    for (int b = threadIdx.x; b < kTkBins; b += kSelThreads) s_hist[b] = 0;
    __syncthreads();
    for (int i0 = threadIdx.x; i0 < total; i0 += kTkU * kSelThreads) {
      K kk[kTkU];
#pragma unroll
      for (int u = 0; u < kTkU; ++u) kk[u] = i0 + u * kSelThreads < total ? key(i0 + u * kSelThreads) : (K)0;
#pragma unroll
      for (int u = 0; u < kTkU; ++u)
        if (kk[u] != 0 && (kk[u] & mask) == prefix) atomicAdd(&s_hist[(unsigned)((kk[u] >> shift) & dmask)], 1u);
    }
    __syncthreads();
    // suffix counts from the top digit: thread t owns digits 2g, 2g+1 of group g = 1023 - t
    const int g = kSelThreads - 1 - (int)threadIdx.x;
    const int hi_c = (int)s_hist[2 * g + 1], lo_c = (int)s_hist[2 * g];
    int in_prefix;
    const int above = block_excl_sum(hi_c + lo_c, s_isum, &in_prefix);
    if (pass == 0) total_pass = in_prefix;
    const int need = s_need;
    if (pass == 0 && total_pass <= N) break;  // every passing candidate is selected
    if (above < need && need <= above + hi_c + lo_c) {
      const bool top = need <= above + hi_c;
      const int b = top ? 2 * g + 1 : 2 * g;
      const int bc = top ? hi_c : lo_c;
      const int rem = need - (top ? above : above + hi_c);  // ranks still needed inside digit b
      s_prefix = prefix | ((K)b << shift);
      s_mask = mask | (dmask << shift);
      s_need = rem;
      s_eqcnt = bc;
      s_done = (bc == rem || shift == 0) ? 1 : 0;
    }
    __syncthreads();
    if (s_done) break;
  }
  const bool take_all = total_pass <= N;
  const K prefix = s_prefix, mask = s_mask;
  const int need_eq = s_need;
  const int nsel = take_all ? total_pass : N;
  int nsort = nsel;
  if (take_all || (N - need_eq) + s_eqcnt <= kMaxCandidates) {
    // everything at or above the threshold fits the sort buffer: collect it unordered (coalesced
    // reads, LDS counter) and let the sort by (-score, scan index) put equal scores in scan order
    nsort = take_all ? total_pass : (N - need_eq) + s_eqcnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    for (int i0 = threadIdx.x; i0 < total; i0 += kTkU * kSelThreads) {
      K kk[kTkU];
#pragma unroll
      for (int u = 0; u < kTkU; ++u) kk[u] = i0 + u * kSelThreads < total ? key(i0 + u * kSelThreads) : (K)0;
#pragma unroll
      for (int u = 0; u < kTkU; ++u) {
        if (kk[u] != 0 && (take_all || (kk[u] & mask) >= prefix)) {
          const int i = i0 + u * kSelThreads;
          const int pos = atomicAdd(&s_cnt, 1);
          s_key[pos] = -(double)sc[i];
          s_sec[pos] = i;
          s_pay[pos] = i;
        }
      }
    }
  } else {
    // many exactly equal scores at the threshold: ordered compaction, thread t scans
    // [t*per, (t+1)*per), equal scores taken in scan order
    const int per = (total + kSelThreads - 1) / kSelThreads;
    const int i_lo = min(total, (int)threadIdx.x * per), i_hi = min(total, i_lo + per);
    int n_above = 0, n_eq = 0;
    for (int i = i_lo; i < i_hi; ++i) {
      const K k = key(i);
      if (k == 0) continue;
      if ((k & mask) > prefix) n_above++;
      else if ((k & mask) == prefix) n_eq++;
    }
    int tot_above, tot_eq;
    int pa = block_excl_sum(n_above, s_isum, &tot_above);
    int pe = block_excl_sum(n_eq, s_isum, &tot_eq);
    for (int i = i_lo; i < i_hi; ++i) {
      const K k = key(i);
      if (k == 0) continue;
      int pos = -1;
      if ((k & mask) > prefix) pos = pa++;
      else if ((k & mask) == prefix) {
        if (pe < need_eq) pos = tot_above + pe;
        pe++;
      }
      if (pos >= 0) {
        s_key[pos] = -(double)sc[i];
        s_sec[pos] = i;
        s_pay[pos] = i;
      }
    }
  }
  __syncthreads();
  sort_kv(s_key, s_sec, s_pay, nsort);
  if (threadIdx.x == 0) {
    a.cand_count[slot] = nsel;
    a.warn[slot] = 0;
  }
  for (int i = threadIdx.x; i < nsel; i += kSelThreads) {
    const int idx = s_pay[i];
    a.cand[((int64_t)slot * a.N + i) * 2 + 0] = a.t0 + idx / a.NF;
    a.cand[((int64_t)slot * a.N + i) * 2 + 1] = idx % a.NF;
    a.cand_score[(int64_t)slot * a.N + i] = -s_key[i];
  }
}


// ---------------------------------------------------------------------------------------------
// FT8_FLAG_TOPK from the compact score layout (k_score2 wrote only each segment's passing scores,
// packed at the segment's start in column order, plus its column masks).  The passing scores of a
// slot, numbered densely d = 0 .. total-1 in segment order, are in scan order (a row's segments
// are its column ranges), so d serves as the scan-order tie key and the grid index of a selected
// candidate is recovered from its segment's mask only for the N outputs.  One 1024-thread
// workgroup per slot: segment offsets by a block scan of the mask popcounts; the passing scores
// staged in LDS (a crowded 12 kHz slot holds ~12.5 k, 50 KB) -- or, past the LDS budget, read
// from HBM by one wave per segment on every pass -- then k_topk's radix select, collection and
// bitonic sort on LDS.  Round 3's k_topk read the full 670 KB grid of every slot per radix pass.
// ---------------------------------------------------------------------------------------------
constexpr int kTkcMaxSeg = 8192;     // segments per slot whose offsets live in LDS
constexpr int kTkcRun = 16;          // staged values per thread and load batch

__device__ __forceinline__ unsigned tk_key(float v) { return TkKey<float>::of(v); }

// the segment holding dense index d: the last seg with off[seg] <= d (empty segments share their
// successor's offset, so the last one is the non-empty one)
__device__ __forceinline__ int tkc_seg(const int* off, int nsegs, int d) {
  int lo = 0, hi = nsegs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= d) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(kSelThreads) void k_topkc(SelectArgs a, int M, int V) {
  FT8_RACE_PROLOGUE();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nsegs = a.NT * a.nseg;
  unsigned* s_hist = reinterpret_cast<unsigned*>(smem);
  int* s_off = reinterpret_cast<int*>(smem + kTkBins * sizeof(unsigned));
  double* s_key = reinterpret_cast<double*>(s_off + ((nsegs + 2) & ~1));
  int* s_sec = reinterpret_cast<int*>(s_key + M);
  int* s_pay = s_sec + M;
  float* s_val = reinterpret_cast<float*>(s_pay + M);
  __shared__ int s_isum[kSelWaves + 1];
  __shared__ unsigned s_prefix, s_mask;
  __shared__ int s_need, s_done, s_eqcnt, s_cnt;

  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid >> 6;
  const int slot = blockIdx.x;  // == the XCD k_score2 wrote this slot's segments from (slot % 8)
  const int64_t seg0 = (int64_t)slot * nsegs;
  const uint64_t* mk = a.smask + 2 * seg0;
  const float* sv = reinterpret_cast<const float*>(a.scores) + seg0 * kSegCols;
  const int N = a.N;

  // ---- segment offsets (dense index of each segment's first passing score); the thread that owns
  // a segment also stages its scores into s_val while they fit (only used when all of them do)
  int carry = 0;
  for (int g0 = 0; g0 < nsegs; g0 += kSelThreads) {
    const int sg = g0 + tid;
    int c = 0;
    if (sg < nsegs) c = __popcll(mk[2 * sg]) + __popcll(mk[2 * sg + 1]);
    int ctot;
    const int ex = block_excl_sum(c, s_isum, &ctot);
    if (sg < nsegs) {
      const int off = carry + ex;
      s_off[sg] = off;
      if (off + c <= V) {
        const float* src = sv + (int64_t)sg * kSegCols;
        for (int j0 = 0; j0 < c; j0 += kTkcRun) {
          float v[kTkcRun];
#pragma unroll
          for (int u = 0; u < kTkcRun; ++u) v[u] = j0 + u < c ? src[j0 + u] : 0.0f;
#pragma unroll
          for (int u = 0; u < kTkcRun; ++u)
            if (j0 + u < c) s_val[off + j0 + u] = v[u];
        }
      }
    }
    carry += ctot;
  }
  const int total = carry;
  if (tid == 0) {
    s_off[nsegs] = total;
    s_prefix = 0;
    s_mask = 0;
    s_need = N;
    s_done = 0;
    s_eqcnt = 0;
    s_cnt = 0;
  }
  __syncthreads();
  // staged (every score fits s_val): the scan above copied them (the barrier after it orders
  // the copies); else every pass reads them from HBM, one wave per segment
  const bool staged = total <= V;
  // every passing score once: (dense index, value)
  auto visit = [&](auto&& fn) {
    if (staged) {
      for (int d = tid; d < total; d += kSelThreads) fn(d, s_val[d]);
    } else {
      for (int sg = w; sg < nsegs; sg += kSelWaves) {
        const int c0 = s_off[sg], c = s_off[sg + 1] - c0;
        for (int j = lane; j < c; j += kWave) fn(c0 + j, sv[(int64_t)sg * kSegCols + j]);
      }
    }
  };

  // ---- radix select of the N-th largest key (k_topk's passes, on the passing scores only)
  const bool take_all = total <= N;
  if (!take_all) {
    for (int pass = 0;; ++pass) {
      int shift = 32 - kTkBits * (pass + 1), width = kTkBits;
      if (shift < 0) { width += shift; shift = 0; }
      const unsigned dmask = (1u << width) - 1u;
      const unsigned prefix = s_prefix, mask = s_mask;
      for (int b = tid; b < kTkBins; b += kSelThreads) s_hist[b] = 0;
      __syncthreads();
      visit([&](int, float v) {
        const unsigned k = tk_key(v);
        if ((k & mask) == prefix) atomicAdd(&s_hist[(k >> shift) & dmask], 1u);
      });
      __syncthreads();
      const int g = kSelThreads - 1 - tid;
      const int hi_c = (int)s_hist[2 * g + 1], lo_c = (int)s_hist[2 * g];
      int in_prefix;
      const int above = block_excl_sum(hi_c + lo_c, s_isum, &in_prefix);
      const int need = s_need;
      if (above < need && need <= above + hi_c + lo_c) {
        const bool top = need <= above + hi_c;
        const int b = top ? 2 * g + 1 : 2 * g;
        const int bc = top ? hi_c : lo_c;
        const int rem = need - (top ? above : above + hi_c);
        s_prefix = prefix | ((unsigned)b << shift);
        s_mask = mask | (dmask << shift);
        s_need = rem;
        s_eqcnt = bc;
        s_done = (bc == rem || shift == 0) ? 1 : 0;
      }
      __syncthreads();
      if (s_done) break;
    }
  }
  const unsigned prefix = s_prefix, mask = s_mask;
  const int need_eq = s_need;
  const int nsel = take_all ? total : N;
  int nsort = take_all ? total : (N - need_eq) + s_eqcnt;
  int m2 = 1;
  while (m2 < nsort) m2 <<= 1;
  if (m2 <= M) {
    // everything at or above the threshold fits the sort buffer: collect unordered, the sort by
    // (-score, dense index) puts equal scores in scan order
    visit([&](int d, float v) {
      if (take_all || (tk_key(v) & mask) >= prefix) {
        const int pos = atomicAdd(&s_cnt, 1);
        s_key[pos] = -(double)v;
        s_sec[pos] = d;
        s_pay[pos] = d;
      }
    });
  } else {
    // many exactly equal scores at the threshold: ordered compaction over contiguous dense runs,
    // equal scores taken in scan order
    nsort = N;
    const int per = (total + kSelThreads - 1) / kSelThreads;
    const int d_lo = min(total, tid * per), d_hi = min(total, d_lo + per);
    const int sg_lo = d_lo < d_hi ? tkc_seg(s_off, nsegs, d_lo) : 0;
    auto walk = [&](auto&& fn) {
      int sg = sg_lo;
      for (int d = d_lo; d < d_hi; ++d) {
        float v;
        if (staged) {
          v = s_val[d];
        } else {
          while (s_off[sg + 1] <= d) ++sg;
          v = sv[(int64_t)sg * kSegCols + (d - s_off[sg])];
        }
        fn(d, v);
      }
    };
    int n_above = 0, n_eq = 0;
    // counters updated arithmetically: an if / else-if on two locals compiled to a store through
    // a selected stack pointer (scratch)
    walk([&](int, float v) {
      const unsigned k = tk_key(v) & mask;
      n_above += k > prefix ? 1 : 0;
      n_eq += k == prefix ? 1 : 0;
    });
    int tot_above, tot_eq;
    int pa = block_excl_sum(n_above, s_isum, &tot_above);
    int pe = block_excl_sum(n_eq, s_isum, &tot_eq);
    walk([&](int d, float v) {
      const unsigned k = tk_key(v) & mask;
      const bool ab = k > prefix, eq = k == prefix;
      const int pos = ab ? pa : (eq && pe < need_eq ? tot_above + pe : -1);
      pa += ab ? 1 : 0;
      pe += eq ? 1 : 0;
      if (pos >= 0) {
        s_key[pos] = -(double)v;
        s_sec[pos] = d;
        s_pay[pos] = d;
      }
    });
  }
  __syncthreads();
  if (tid == 0) {
    a.cand_count[slot] = nsel;
    a.warn[slot] = 0;
  }
  // order by (-score, scan index) (sort_kv: a register network for up to 1024 items)
  sort_kv(s_key, s_sec, s_pay, nsort);
  // dense index -> grid position (row, column) through the segment's column-order mask
  for (int i = tid; i < nsel; i += kSelThreads) {
    const int t_ = i;
    const int d = s_pay[i];
    const int sg = tkc_seg(s_off, nsegs, d);
    const int j = d - s_off[sg];
    const uint64_t e = mk[2 * sg], o = mk[2 * sg + 1];
    const uint64_t c0 = spread32((uint32_t)e) | (spread32((uint32_t)o) << 1);
    const int n0 = __popcll(c0);
    const int col = j < n0 ? select_bit(c0, j)
                           : 64 + select_bit(spread32((uint32_t)(e >> 32)) | (spread32((uint32_t)(o >> 32)) << 1), j - n0);
    const int row = sg / a.nseg;
    a.cand[((int64_t)slot * a.N + i) * 2 + 0] = a.t0 + row;
    a.cand[((int64_t)slot * a.N + i) * 2 + 1] = (sg - row * a.nseg) * kSegCols + col;
    a.cand_score[(int64_t)slot * a.N + i] = -s_key[t_];
  }
}

}  // namespace

// the compact layout needs k_score2 (whole-segment writes); top-k selection reads it through
// k_topkc when the slot's segment offsets fit its LDS (else k_topk on the full grid)
bool score_compact(const SyncLaunch& L) {
  return L.compact && score2_path(L) && (!L.topk || (int64_t)L.NT * n_segments(L.NF) <= kTkcMaxSeg);
}

hipError_t launch_score(const SyncLaunch& L, hipStream_t s) {
  if (L.NT <= 0 || L.NF <= 0 || L.n_slots <= 0) return hipSuccess;
  if (L.wf_f64) return launch_score_t<double, 32>(L, s);
  return launch_score_t<float, 64>(L, s);
}

hipError_t launch_score_list(const void* wf, int wf_f64, int T, int F, int sps, int bpt, const int32_t* cand,
                             int n, void* out, int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  if (wf_f64)
    hipLaunchKernelGGL(k_score_list<double>, dim3(blocks), dim3(256), 0, s, (const double*)wf, T, F, sps, bpt, cand,
                       n, (double*)out, err);
  else
    hipLaunchKernelGGL(k_score_list<float>, dim3(blocks), dim3(256), 0, s, (const float*)wf, T, F, sps, bpt, cand, n,
                       (float*)out, err);
  return hipGetLastError();
}

hipError_t launch_select(const SyncLaunch& L, hipStream_t s) {
  if (L.n_slots <= 0) return hipSuccess;
  SelectArgs a{};
  a.scores = L.scores;
  a.total = (int64_t)max(L.NT, 0) * max(L.NF, 0);
  a.NF = max(L.NF, 1);
  a.t0 = L.t0;
  a.N = L.N;
  a.min_score = L.min_score;
  a.cmp_f64 = L.min_score_f64;
  a.cand = L.cand;
  a.cand_score = L.cand_score;
  a.cand_count = L.cand_count;
  a.warn = L.warn;
  a.rowsum = L.rowsum;
  a.tie = L.tie;
  a.NT = max(L.NT, 0);
  a.smask = L.smask;
  a.nseg = n_segments(a.NF);
  a.compact = score_compact(L) ? 1 : 0;
  if (L.topk && a.compact) {
    // LDS: histogram, segment offsets, the sort buffers (M >= N, a power of two) and as many staged
    // scores as fit beside them in 79 KB (two workgroups per CU: 160 KB less the static words; at
    // 80 KB only one was resident), at least 4096
    int M = 64;
    while (M < L.N) M <<= 1;
    const int nsegs = a.NT * a.nseg;
    const size_t fixed = kTkBins * sizeof(unsigned) + (size_t)((nsegs + 2) & ~1) * sizeof(int) +
                         (size_t)M * (sizeof(double) + 2 * sizeof(int));
    const size_t budget = 79 * 1024;
    const int V = (int)std::max<size_t>(4096, fixed < budget ? (budget - fixed) / sizeof(float) : 0);
    const size_t lds = fixed + (size_t)V * sizeof(float);
    if (lds > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_topkc),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_topkc, dim3(L.n_slots), dim3(kSelThreads), lds, s, a, M, V);
    return hipGetLastError();
  }
  if (L.topk) {
    if (L.wf_f64)
      hipLaunchKernelGGL(k_topk<double>, dim3(L.n_slots), dim3(kSelThreads), 0, s, a);
    else
      hipLaunchKernelGGL(k_topk<float>, dim3(L.n_slots), dim3(kSelThreads), 0, s, a);
    return hipGetLastError();
  }
  if (L.wf_f64)
    hipLaunchKernelGGL(k_select<double>, dim3(L.n_slots), dim3(kSelThreads), 0, s, a);
  else
    hipLaunchKernelGGL(k_select<float>, dim3(L.n_slots), dim3(kSelThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace ft8
