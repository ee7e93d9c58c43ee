// sync.hip -- Costas-7 sync score grid and the reference's candidate selection (gfx950).
//
// k_score replaces ft8_sync_score over the ft8_find_candidates grid (reference
// ft8_decode.py:47-100, 108-131; FT8Candidate.get_log_power ftx_types.py:45-47).  Each thread
// owns one candidate (abs_time, abs_freq) and accumulates its up-to-75 dB differences
// SEQUENTIALLY in the reference order (m, k, then tone-1, tone+1, time-1, time+1): on the float32
// waterfall of a WAV the reference sums in np.float32 (NumPy-2 promotion, ft8_decode.py:57,80-94)
// and any re-association would change the last bit of the score, so the sum is never
// tree-reduced.  A workgroup covers TW consecutive frequency columns of one slot for every time
// row of the grid; the waterfall strip it touches (all rows x (TW + 7*bpt) columns, 58 KB at
// 12 kHz fp32) is staged in LDS once and read conflict-free (lanes = consecutive columns).
// Geometries whose strip does not fit LDS read through L1/L2 instead (same code path, templated).
//
// k_select replaces the heap logic of ft8_find_candidates (ft8_decode.py:113-140), one 1024-thread
// workgroup per slot.  The reference heap stores (-score, cand) and admits a candidate into a full
// heap only when it beats heap[0] -- the CURRENT MAXIMUM -- which it then evicts.  The selected set
// is therefore: the first N passing candidates in scan order (time outer, frequency inner), with
// the maximum of those replaced by each later strict new maximum ("record") in turn.  The kernel
// finds ranks and records with two block scans (count, running max), sorts the set by score, and
// only when two selected scores are exactly equal (where the reference's order depends on heap
// array positions) replays the reference heapq sequence in LDS to reproduce its stable sort.
#include "ft8_internal.h"

namespace ft8 {
namespace {

__constant__ int kCostasD[7] = {3, 1, 4, 0, 6, 5, 2};  // ft8_decode.py:42

constexpr int kScoreThreads = 256;
constexpr size_t kScoreLdsBudget = 64 * 1024;

struct ScoreArgs {
  const void* wf;
  int T, F, sps, bpt, num_blocks;
  int t0, NT, NF;
  int rlo, nrows;    // staged rows [rlo, rlo + nrows)
  void* scores;
};

template <typename T, bool LDS, int TW>
__global__ __launch_bounds__(kScoreThreads) void k_score(ScoreArgs a) {
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
  }
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
  int32_t* rec_idx;
  int32_t* warn;
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
__device__ double block_excl_max(double v, double* sh, double* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    double y = __shfl_up(x, o);
    if (lane >= o) x = fmax(x, y);
  }
  double ex = __shfl_up(x, 1);
  if (lane == 0) ex = -INFINITY;
  if (lane == 63) sh[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    double acc = -INFINITY;
    for (int i = 0; i < kSelWaves; ++i) { double t = sh[i]; sh[i] = acc; acc = fmax(acc, t); }
    sh[kSelWaves] = acc;
  }
  __syncthreads();
  const double r = fmax(sh[w], ex);
  *total = sh[kSelWaves];
  __syncthreads();
  return r;
}

// heap key: (neg score, secondary); equal neg => tie (the reference would compare candidates)
struct HeapCtx {
  double* neg;
  int* idx;
  int tie;
  __device__ bool less(int a, int b) {
    if (neg[a] < neg[b]) return true;
    if (neg[a] > neg[b]) return false;
    tie = 1;
    return idx[a] < idx[b];
  }
  __device__ void mov(int dst, int src) { neg[dst] = neg[src]; idx[dst] = idx[src]; }
};

// CPython heapq _siftdown / _siftup on LDS arrays; slot `tmp` (= capacity) holds newitem
__device__ void h_siftdown(HeapCtx& h, int start, int pos, int tmp) {
  h.mov(tmp, pos);
  while (pos > start) {
    const int pp = (pos - 1) >> 1;
    if (h.less(tmp, pp)) { h.mov(pos, pp); pos = pp; continue; }
    break;
  }
  h.mov(pos, tmp);
}
__device__ void h_siftup(HeapCtx& h, int len, int pos, int tmp) {
  const int start = pos;
  h.mov(tmp + 1, pos);  // newitem
  int c = 2 * pos + 1;
  while (c < len) {
    const int r = c + 1;
    if (r < len && !h.less(c, r)) c = r;
    h.mov(pos, c);
    pos = c;
    c = 2 * pos + 1;
  }
  h.mov(pos, tmp + 1);
  h_siftdown(h, start, pos, tmp);
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

constexpr int kSelV = 4;                        // elements per thread per chunk
constexpr int kSelChunk = kSelThreads * kSelV;  // 4096 scores per chunk

template <typename T>
__global__ __launch_bounds__(kSelThreads) void k_select(SelectArgs a) {
  __shared__ double s_key[kMaxCandidates + 2];
  __shared__ int s_sec[kMaxCandidates + 2];
  __shared__ int s_pay[kMaxCandidates + 2];
  __shared__ int s_rank[kMaxCandidates];  // scan index of passing candidate #rank (rank < N)
  __shared__ int s_isum[kSelWaves + 1];
  __shared__ double s_dmax[kSelWaves + 1];
  __shared__ int s_flag[4];
  __shared__ double s_am_v[kSelWaves];
  __shared__ int s_am_i[kSelWaves];

  const int slot = blockIdx.x;
  const T* sc = reinterpret_cast<const T*>(a.scores) + (int64_t)slot * a.total;
  int32_t* rec = a.rec_idx + (int64_t)slot * kMaxRecords;
  const T ms = (T)a.min_score;
  auto passes = [&](T s) -> bool {
    if (s == (T)-INFINITY) return false;          // ft8_decode.py:127
    if (a.cmp_f64) return !((double)s < a.min_score);
    return !(s < ms);
  };
  const int N = a.N;

  // one ordered sweep in 4096-score chunks: ranks (exclusive count scan), records (new strict
  // maxima after rank N, exclusive max scan), first-occurrence argmax (per thread, strict >)
  int carry_cnt = 0, carry_rec = 0;
  double carry_max = -INFINITY;
  double best_v = -INFINITY;
  int best_i = 0x7fffffff;
  for (int64_t c0 = 0; c0 < a.total; c0 += kSelChunk) {
    T v[kSelV];
    bool p[kSelV];
    int lc = 0;
    double lm = -INFINITY;
    const int64_t i0 = c0 + (int64_t)threadIdx.x * kSelV;
#pragma unroll
    for (int j = 0; j < kSelV; ++j) {
      const int64_t i = i0 + j;
      v[j] = i < a.total ? sc[i] : (T)-INFINITY;
      p[j] = passes(v[j]);
      if (p[j]) {
        lc++;
        lm = fmax(lm, (double)v[j]);
        if ((double)v[j] > best_v) { best_v = (double)v[j]; best_i = (int)i; }
      }
    }
    int chunk_cnt;
    double chunk_max;
    const int ex_cnt = block_excl_sum(lc, s_isum, &chunk_cnt);
    const double ex_max = block_excl_max(lm, s_dmax, &chunk_max);
    int rank = carry_cnt + ex_cnt;
    double rm = fmax(carry_max, ex_max);
    int nrec = 0;
    bool isrec[kSelV];
#pragma unroll
    for (int j = 0; j < kSelV; ++j) {
      isrec[j] = false;
      if (!p[j]) continue;
      if (rank < N) {
        s_rank[rank] = (int)(i0 + j);
      } else if ((double)v[j] > rm) {
        isrec[j] = true;
        nrec++;
      }
      rm = fmax(rm, (double)v[j]);
      rank++;
    }
    if (__syncthreads_or(nrec > 0)) {
      int chunk_rec;
      int r = carry_rec + block_excl_sum(nrec, s_isum, &chunk_rec);
#pragma unroll
      for (int j = 0; j < kSelV; ++j)
        if (isrec[j]) {
          if (r < kMaxRecords) rec[r] = (int)(i0 + j);
          r++;
        }
      carry_rec += chunk_rec;
    }
    carry_cnt += chunk_cnt;
    carry_max = fmax(carry_max, chunk_max);
  }
  const int total_pass = carry_cnt, total_rec = carry_rec;
  const int nsel = min(total_pass, N);

  // first occurrence of the global maximum (the last record, when there are records)
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double bv = best_v;
    int bi = best_i;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(bv, o);
      const int oi = __shfl_xor(bi, o);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { s_am_v[w] = bv; s_am_i[w] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int i = 1; i < kSelWaves; ++i)
        if (s_am_v[i] > s_am_v[0] || (s_am_v[i] == s_am_v[0] && s_am_i[i] < s_am_i[0])) {
          s_am_v[0] = s_am_v[i];
          s_am_i[0] = s_am_i[i];
        }
      s_flag[0] = 0;
      s_flag[1] = total_rec > kMaxRecords;
      s_flag[3] = 0;
    }
    __syncthreads();
  }

  // the heap keeps the first N; each record evicts the current maximum (the top of the first N,
  // then the previous record): the final set is the first N with its top replaced by the last
  // record (ft8_decode.py:134-137)
  for (int i = threadIdx.x; i < nsel; i += kSelThreads) {
    const int idx = s_rank[i];
    s_key[i] = -(double)sc[idx];
    s_sec[i] = idx;
    s_pay[i] = idx;
  }
  __syncthreads();
  if (total_rec > 0 && threadIdx.x == 0) {
    int top = 0;
    for (int i = 1; i < nsel; ++i)
      if (s_key[i] < s_key[top] || (s_key[i] == s_key[top] && s_sec[i] < s_sec[top])) top = i;
    const int gi = s_am_i[0];
    s_key[top] = -(double)sc[gi];
    s_sec[top] = gi;
    s_pay[top] = gi;
  }
  __syncthreads();

  // order: score descending; equal scores keep the reference's heap-array order (below)
  bitonic(s_key, s_sec, s_pay, nsel);
  for (int i = threadIdx.x; i + 1 < nsel; i += kSelThreads)
    if (s_key[i] == s_key[i + 1]) s_flag[0] = 1;
  __syncthreads();

  if (s_flag[0]) {
    // exact score ties in the final set: replay the reference heapq sequence
    for (int i = threadIdx.x; i < nsel; i += kSelThreads) {
      s_key[i] = -(double)sc[s_rank[i]];
      s_sec[i] = s_rank[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      HeapCtx h{s_key, s_sec, 0};
      for (int n = 1; n < nsel; ++n) h_siftdown(h, 0, n, kMaxCandidates);  // heappush x nsel
      const int nr = min(total_rec, kMaxRecords);
      for (int r = 0; r < nr; ++r) {  // heapreplace(heap, record)
        const int i = rec[r];
        s_key[0] = -(double)sc[i];
        s_sec[0] = i;
        h_siftup(h, nsel, 0, kMaxCandidates);
      }
      s_flag[3] = h.tie;
    }
    __syncthreads();
    // sorted(key=-score) is stable on heap-array order: secondary key = heap position
    for (int i = threadIdx.x; i < nsel; i += kSelThreads) { s_pay[i] = s_sec[i]; s_sec[i] = i; }
    __syncthreads();
    bitonic(s_key, s_sec, s_pay, nsel);
  }
  if (threadIdx.x == 0) {
    a.cand_count[slot] = nsel;
    a.warn[slot] = (s_flag[3] ? 1 : 0) | (s_flag[1] && s_flag[0] ? 2 : 0);
  }
  for (int i = threadIdx.x; i < nsel; i += kSelThreads) {
    const int idx = s_pay[i];
    a.cand[((int64_t)slot * a.N + i) * 2 + 0] = a.t0 + idx / a.NF;
    a.cand[((int64_t)slot * a.N + i) * 2 + 1] = idx % a.NF;
    a.cand_score[(int64_t)slot * a.N + i] = -s_key[i];
  }
}

}  // namespace

hipError_t launch_score(const SyncLaunch& L, hipStream_t s) {
  if (L.NT <= 0 || L.NF <= 0 || L.n_slots <= 0) return hipSuccess;
  if (L.wf_f64) return launch_score_t<double, 32>(L, s);
  return launch_score_t<float, 64>(L, s);
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
  a.rec_idx = L.rec_idx;
  a.warn = L.warn;
  if (L.wf_f64)
    hipLaunchKernelGGL(k_select<double>, dim3(L.n_slots), dim3(kSelThreads), 0, s, a);
  else
    hipLaunchKernelGGL(k_select<float>, dim3(L.n_slots), dim3(kSelThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace ft8
