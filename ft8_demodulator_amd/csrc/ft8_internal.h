// ft8_internal.h -- shared device helpers and the internal launch interface between the
// kernel translation units (stft.hip, sync.hip, bp.hip) and the C-ABI (capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <stdint.h>

#include "../../include/ft8hip.h"
#include "ft8_ldpc_tables.h"

namespace ft8 {

constexpr int kWave = 64;

// ---- barrier-race check build (-DFT8_RACE_CHECK; tools/build_race.sh, never the shipped library) --
// FT8_RACE_PROLOGUE() opens every kernel whose workgroup has more than one wave and uses LDS: the
// whole LDS allocation of the workgroup (static + dynamic: the dispatch packet's
// group_segment_size) is filled with 0xffffffff (a NaN / -1 sentinel), a barrier, then one wave of
// the workgroup (rotating with the workgroup id) sleeps ~64 k cycles before it starts.  A read of
// another wave's LDS staging that no barrier orders after the write then sees the sentinel instead
// of a late value, deterministically, and the GPU tests fail.
// tools/probe/race_control.hip is the positive control: a kernel with a deliberately missing
// barrier that must read the sentinel under this prologue (tests/test_gpu_race_control.py).
#ifdef FT8_RACE_CHECK
}  // namespace ft8
#include <hsa/hsa.h>
namespace ft8 {
static_assert(offsetof(hsa_kernel_dispatch_packet_t, group_segment_size) == 28, "dispatch packet layout");
__device__ __forceinline__ void race_prologue() {
  const auto* pkt = (const hsa_kernel_dispatch_packet_t*)__builtin_amdgcn_dispatch_ptr();
  const uint32_t bytes = pkt->group_segment_size;  // static + dynamic LDS of this workgroup
  const uint32_t nt = blockDim.x * blockDim.y * blockDim.z;
  const uint32_t t = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
  for (uint32_t off = 4 * t; off + 4 <= bytes; off += 4 * nt)
    asm volatile("ds_write_b32 %0, %1" ::"v"(off), "v"(0xffffffffu) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  const uint32_t nw = (nt + kWave - 1) / kWave;
  // the test must be wave-uniform in an SGPR: s_sleep is a scalar instruction that the EXEC mask
  // does not gate, so under a per-lane condition (an exec-masked block the compiler does not branch
  // around) every wave slept and none was late -- the positive control caught it
  const uint32_t w = __builtin_amdgcn_readfirstlane(t / kWave);
  if (nw > 1 && w == blockIdx.x % nw)
    for (int i = 0; i < 8; ++i) __builtin_amdgcn_s_sleep(127);
  // a compiler barrier: s_sleep carries no memory semantics, so the kernel's first LDS accesses
  // must not be scheduled above it
  asm volatile("" ::: "memory");
}
#define FT8_RACE_PROLOGUE() ::ft8::race_prologue()
#else
#define FT8_RACE_PROLOGUE() \
  do {                      \
  } while (0)
#endif
constexpr int kMaxCandidates = 4096;   // LDS-resident selection (k_select)
// LDS FFT limits (one (P + P/16 + 1)-point buffer per frame, 256 threads holding P / 256 values each
// per stage): float32 P <= 10240 (87 KB), float64 P <= 8192 (139 KB).  Larger or non-2/3/5/7 lengths
// take the chirp-z transform (its power-of-two convolution on the same LDS FFT), or the direct DFT
// where that convolution would not fit.
constexpr int kMaxFftReal = 20480;     // float32 nfft of the real-input path (half-length FFT <= 10240)
constexpr int kMaxFftComplex = 10240;  // float32 nfft of the complex-input path
constexpr int kMaxFftP64 = 8192;       // float64: FFT points P (real nfft <= 16384, complex <= 8192)
constexpr int kMaxDft = 1 << 18;       // nfft of the direct-DFT fallback (any factorisation)
constexpr int kMaxDftLds = 150 * 1024; // its windowed frame is staged in LDS

__host__ __device__ inline int floordiv(int a, int b) {
  int q = a / b;
  if ((a % b) != 0 && ((a < 0) != (b < 0))) q--;
  return q;
}

template <typename T>
struct cplx {
  T x, y;
};

// ---- STFT plan (host-built tables, device-resident) ----------------------------------------
struct FftPlan {
  int P;              // transform length (nfft/2 for real input, nfft for complex input; nfft if dft;
                      // the convolution length M if blue)
  int dft;            // 1: direct DFT (tw = W_nfft^m): lengths neither the Stockham plans nor the
                      // chirp-z path take (nperseg above its LDS limit)
  int blue;           // 1: chirp-z (Bluestein) transform, for an nfft with a prime factor above 7 or an
                      // odd real nfft: every nfft-point DFT of a frame is a length-P (power of two)
                      // circular convolution, run on the LDS Stockham FFT (stft.hip k_stft_blue)
  int nstages;
  int radix[16];
  const void* tw;     // W_P^m, m in [0, P): cplx<float> or cplx<double>
  const void* post;   // real path: W_N^k, k in [0, P]  (N = 2P)
  // chirp-z (blue): the output bins of a frame are computed in blocks of B = P - nperseg + 1
  int L, B, nblk;     // nperseg the plan is built for, bins per block, blocks covering [0, nfft)
  const void* chirp;  // exp(-i pi k^2 / nfft), k in [0, nfft)
  const void* hspec;  // [nblk][P]: FFT_P of block b's chirp filter conj(chirp(b B + m - (L - 1)))
};
constexpr int kMaxBlueP64 = 8192;       // chirp-z convolution length limits (the LDS FFT's)
constexpr int kMaxBlueP32 = 8192;

struct StftLaunch {
  const void* samples;
  int dtype;               // ft8_dtype
  int64_t n_samples, slot_stride;
  int n_slots;
  int nperseg, hop, nfft;
  int t_lo, t_hi, f_lo, f_hi;
  const void* window;      // float or double [nperseg]
  double scale;            // 1 / (sum w)^2
  void* out;               // float or double [n_slots][t_hi-t_lo][f_hi-f_lo]
  int32_t* argmax;         // non-null: write per-frame argmax over the kept bins instead of `out`
                           // (a direct-DFT plan then writes the dB rows to `out` first)
  int32_t* screen_list;    // non-null (complex128 argmax, 3840-point geometry): float32 screening
  int32_t* screen_count;   // with the uncertain frames listed here and redone in float64
  const void* screen_tw;     // the screening pass's float32 twiddles (W_3840^m) and window
  const void* screen_window;
  FftPlan plan;
};
hipError_t launch_stft(const StftLaunch& a, hipStream_t s);
// the production geometry (real float32 / int16 input, nfft 3840, nperseg 1920, hop 960) with packed
// float32 complex arithmetic (stft3840.hip)
bool stft3840_eligible(const StftLaunch& a);
hipError_t launch_stft3840(const StftLaunch& a, hipStream_t s);
bool stftpk_eligible(const StftLaunch& a);        // stft3840.hip: the packed generic real-input plans
hipError_t launch_stftpk(const StftLaunch& a, hipStream_t s);

// ---- sync score + selection ----------------------------------------------------------------
// Per (slot, time row) summary written by k_score for k_select: how many grid points of the row
// pass the min_score test, and the largest passing score as an order-preserving key (0 = none).
struct RowSummary {
  unsigned count;
  unsigned pad;
  unsigned long long maxkey;
};
static_assert(sizeof(RowSummary) == 16 && offsetof(RowSummary, maxkey) == 8, "k_select reads it as one uint4");
__host__ __device__ inline unsigned long long order_key(double v) {
  union { double d; unsigned long long u; } x{v};
  return (x.u >> 63) ? ~x.u : (x.u | 0x8000000000000000ull);
}
__host__ __device__ inline double key_value(unsigned long long k) {
  union { double d; unsigned long long u; } x;
  x.u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return x.d;
}

struct SyncLaunch {
  const void* wf;          // [n_slots][T][F]
  int wf_f64;
  int n_slots, T, F;
  int sps, bpt;
  int t0, NT, NF;          // abs_time grid = [t0, t0+NT), abs_freq grid = [0, NF)
  void* scores;            // full grid [n_slots][NT][NF] in wf dtype, or (compact) the passing
                           // scores of every segment packed at its start [n_slots][NT][nseg][128]
  uint64_t* smask;         // [n_slots][NT][nseg][2]: passing columns of each 128-column segment
                           // (word 0: even columns 2l -> bit l, word 1: odd columns 2l + 1)
  int compact = 0;         // request the compact score layout (honoured by the k_score2 path)
  int N;                   // max candidates
  double min_score;
  int min_score_f64;
  int32_t* cand;           // [n_slots][N][2]
  double* cand_score;      // [n_slots][N]
  int32_t* cand_count;     // [n_slots]
  int32_t* warn;           // scratch [n_slots] (bit 0: tie reached a heap comparison,
                           //                    bit 2: equal scores in the selected set,
                           //                    bit 3: their order deferred to the LLR kernel)
  RowSummary* rowsum;      // scratch [n_slots][NT][n_segments(NF)]: passing count + max passing score
                           // per (time row, 128-column segment)
  int32_t* tie = nullptr;  // nullable scratch [n_slots][tie_stride(N)]: defer the order of equal
                           // scores to the LLR kernel (warn bit 3); k_compact applies it
  int topk = 0;            // FT8_FLAG_TOPK: k_topk instead of the reference heap selection
};

// deferred tie order, per slot: push order [N] | select order [N] | final order [N] |
// scratch [4N] | last record [1] | its score [1] (float bits) | scores in push order [N]
// (heap_replay.h)
inline __host__ __device__ int64_t tie_stride(int N) { return 8 * (int64_t)N + 2; }
struct TieArgs {
  int n_slots, N;
  const int32_t* cand_count;
  int32_t* warn;           // bit 3 set by k_select: replay this slot's heap; bit 0 set on a tie
  int32_t* tie;            // [n_slots][tie_stride(N)]
  const double* cand_score;  // [n_slots][N] selected scores in select order (float32 values)
};
// the deferred order applied to a candidate list ([n_slots][N][2] + [n_slots][N])
hipError_t launch_tie_apply(const TieArgs& a, int32_t* cand, double* cand_score, hipStream_t s);
hipError_t launch_score(const SyncLaunch& a, hipStream_t s);
// score segments: 128 grid columns of one row; the compact layout holds only passing scores
constexpr int kSegCols = 128;
inline __host__ __device__ int n_segments(int NF) { return (NF + kSegCols - 1) / kSegCols; }
// whether launch_score writes the compact layout for this launch (else the full grid)
bool score_compact(const SyncLaunch& a);
hipError_t launch_select(const SyncLaunch& a, hipStream_t s);
// ft8_sync_score for arbitrary candidates [n][2] = (abs_time, abs_freq); err[i] = 1: IndexError
hipError_t launch_score_list(const void* wf, int wf_f64, int T, int F, int sps, int bpt, const int32_t* cand,
                             int n, void* out, int32_t* err, hipStream_t s);

// ---- LLR + BP + CRC ------------------------------------------------------------------------
// k_bp's work / clock counters: kStatRows rows of kStatStride u64 (one 128-B line each); wave w adds
// to row w % kStatRows and the host sums the rows.  One row for all 4 096 waves put every retiring
// wave's atomics on the same L2 addresses, where they serialise at the launch's tail.
constexpr int kStatRows = 256;
constexpr int kStatStride = 16;   // [0..3] work counters, [4..7] clock (BpLaunch.stats / .clock)
struct BpLaunch {
  // LLR source: either a waterfall + candidate list, or precomputed LLRs
  const void* wf;          // [n_slots][T][F] or null
  int wf_f64, T, F, sps, bpt;
  const int32_t* cand;     // mode A: [n_slots][N][2] + cand_count; mode B: [n][3] (slot, t, f)
  const double* cand_score;
  const int32_t* cand_count;
  int N;                   // per-slot capacity (mode A)
  int n_slots;
  int n_items;             // mode B item count, or n_slots*N in mode A
  int mode;                // 0: waterfall+per-slot candidates, 1: waterfall+explicit list,
                           // 2: LLR input (k_llr: normalise only; k_bp: no candidate metadata)
  const double* llr_in;    // k_bp: always; k_llr: mode 2
  int normalize;           // k_llr only
  int max_iterations;
  double* llr_out;         // k_llr output [n_items][174]
  uint8_t* plain_out;      // nullable [n_items][174]
  ft8_result* res;         // nullable [n_items]
  // k_bp claim counter: 64-bit, never reset.  Launch j claims tickets [base_j, base_j + n_items +
  // waves): every item once, then one ticket >= n_items per wave, so the host advances the base
  // (*work_base, host memory, one per counter) by n_items + waves at each launch -- no reset, no
  // retire counter, nothing a launch cut short could leave behind for the next one to skip over
  unsigned long long* work;
  unsigned long long* work_base;
  unsigned long long* stats = nullptr;  // [candidates, iterations entered, message passes, converged]
  unsigned long long* clock = nullptr;  // timed launches: [wave cycles, wave wall ticks, max wave cycles, waves]
  int slot0 = 0;           // batch index of slot 0 (records carry slot0 + local slot)
  int grid_waves = 4;      // k_bp persistent grid: resident waves per SIMD (clamped to 4)
  // mode 0, nullable: slots whose order of equal scores k_select deferred (warn bit 3) get it
  // replayed by k_llr's first workgroups
  int32_t* tie = nullptr;  // [n_slots][tie_stride(N)]
  int32_t* warn = nullptr; // [n_slots]
};
hipError_t launch_llr(const BpLaunch& a, hipStream_t s);  // k_llr: waterfall -> LLRs
hipError_t launch_bp(const BpLaunch& a, hipStream_t s);   // k_bp: LLRs -> BP + CRC

struct CompactLaunch {
  const ft8_result* res;   // [n_slots][N]
  const int32_t* cand_count;
  int n_slots, N;
  ft8_result* out;         // [n_slots][cap]
  int32_t* counts;
  int cap;
  const int32_t* warn = nullptr;  // with tie: slots with warn bit 3 are read in the final order
  const int32_t* tie = nullptr;
};
hipError_t launch_compact(const CompactLaunch& a, hipStream_t s);

// ft8_pack_decodes (bp.hip): one workgroup packs a batch's decodes for the all-gather
inline __host__ __device__ int64_t pack_header_bytes(int n_slots) { return 8 + ((4 * (int64_t)n_slots + 7) & ~7ll); }
hipError_t launch_pack(const ft8_result* rec, const int32_t* counts, int n_slots, int cap, int capacity,
                       int slot_offset, uint8_t* send, ft8_result* overflow, hipStream_t s);

// ---- transmit chain + subtraction (tx.hip, subtract.hip) -------------------------------------
struct SynthLaunch {
  const uint8_t* tones;        // [n_sig][79]
  const ft8_tx_signal* sig;    // [n_sig], sorted by slot
  int n_sig;
  int nsps, style;
  double fs;
  const double* P;             // cumulative GFSK pulse [3 nsps + 1]
  void* out;                   // [n_slots][slot_stride] of dtype (complex: pairs)
  int dtype;
  int64_t n_samples, slot_stride;
  int n_slots;
};
hipError_t launch_encode(const uint8_t* msg, int msg_bytes, int n, uint8_t* a91, uint8_t* cw, uint8_t* tones,
                         hipStream_t s);
hipError_t launch_synth(const SynthLaunch& a, hipStream_t s);

struct SubLaunch {
  const void* x;               // samples [n_slots][slot_stride], F32 or I16
  int dtype;
  float* residual;             // [n_slots][slot_stride]
  int64_t n_samples, slot_stride;
  int n_slots;
  int fs, nsps, hop, nfft, t_lo, f_lo;
  const ft8_result* res;       // [n_slots][cap] decoded records
  const int32_t* counts;       // [n_slots]
  int cap;
  const double* P;             // cumulative GFSK pulse [3 nsps + 1] (double)
  const float* Pf;             // the same in float
  void* est;                   // scratch [n_slots * cap] SubEst records
  int Q;                       // decimated samples per symbol (nsps % Q == 0)
  int32_t* list;               // scratch [n_slots][cap + 1]: the records to fit (ok, first of their
                               // payload in the slot), in record order, then their count
};
size_t sub_est_bytes();        // sizeof one SubEst record
hipError_t launch_sub_est(const SubLaunch& a, hipStream_t s);    // fits of the records (k_sub_est)
hipError_t launch_sub_apply(const SubLaunch& a, hipStream_t s);  // residual = x - fitted signals

// out[slot] = the pass-1 records out1[slot][0 .. counts1) followed by the pass-2 records
// out2[slot][0 .. counts2) whose payload no pass-1 record carries (pass_index = 1); counts uncapped
hipError_t launch_merge_pass(ft8_result* out, int32_t* counts, int cap, const ft8_result* out1,
                             const int32_t* counts1, int cap1, const ft8_result* out2, const int32_t* counts2,
                             int cap2, int n_slots, hipStream_t s);

// ---- frequency-drift correction (drift.hip) ---------------------------------------------------
struct DriftFitLaunch {
  const int32_t* idx;          // [n_slots][T] per-frame argmax (kept-bin index)
  int n_slots, T, F;
  ft8_drift_params p;
  ft8_drift_result* res;       // [n_slots]
  double* metric;              // [n_slots][T - window + 1] or null
  int32_t* segments;           // [n_slots][max_segments][2] or null
  int max_segments;
  const double* tmpl;          // stage 2: three_sync_correlation_seq [n_tmpl]
  int n_tmpl;
};
constexpr int kDriftMaxT = 16384;   // frames per signal held in LDS by the fit kernels
hipError_t launch_drift_fit(int stage, const DriftFitLaunch& a, hipStream_t s);

struct DerotateLaunch {
  const void* x;               // stage 1: input samples (dtype), row stride slot_stride
  int dtype;
  int64_t slot_stride;
  double* out;                 // complex128 [n_slots][n_samples] (interleaved re, im)
  int64_t n_samples;
  int n_slots;
  const ft8_drift_result* res;
  double fs, inv_fs, inv_2fs2; // fs, fl(1/fs), fl(1/(2 fs^2)) (NumPy divides complex by real via 1/d)
};
// stage 1: out = x * exp(-2 pi i rate1 n^2 / (2 fs^2))  (x itself for FT8_DRIFT_NO_SEGMENT)
hipError_t launch_derotate1(const DerotateLaunch& a, hipStream_t s);
// stage 2: out *= the polynomial carrier of degree deg (1 or 2) where the status is FT8_DRIFT_FULL
hipError_t launch_derotate2(const DerotateLaunch& a, int deg, hipStream_t s);
int drift_max_template();      // LDS capacity of k_drift_fit2: template length, regression points
int drift_max_points();
constexpr int kDriftMaxWindow = 64;  // continuity window (exact int64 sums)

hipError_t launch_crc14(const uint8_t* msg, const int32_t* nbits, int n, uint16_t* crc, hipStream_t s);
hipError_t launch_ldpc_check(const uint8_t* bits, int n, int32_t* err, hipStream_t s);

}  // namespace ft8
