/*
 * ft8hip.h -- C-ABI of libft8hip.so, the MI355X (gfx950) FT8 receive path.
 *
 * Drop-in boundary for the reference's Python decoder (Rintazero/ft8_demodulator,
 * src/ft8_tools/ft8_demodulator).  The reference has no native FFI of its own: every entry point
 * below replaces one Python function on its decode path, cited as file:line relative to
 * src/ft8_tools/ft8_demodulator/.  The Python host layer (ft8_demodulator_amd/) binds these with
 * ctypes and mirrors the reference's functions, names, arguments and error behaviour.
 *
 * Conventions
 *   - All data pointers are device pointers owned by the caller (e.g. torch data_ptr()).  The
 *     library allocates scratch only inside its context and frees only what it allocated.
 *   - Every call is asynchronous on the caller's hipStream_t (passed as void*, NULL = default
 *     stream).  Results are valid after the stream is synchronised.
 *   - Return 0 (FT8_OK) on success, a negative FT8_E_* code otherwise; ft8_last_error() gives the
 *     message.  No C++ exception crosses this boundary.
 *   - One context per device per host thread/stream; a context is not re-entrant.  Its work is
 *     ordered across streams by the library: an entry point that uses the context's scratch, called
 *     on a stream other than the previous such call's, waits (device side) for that call's work, so
 *     two streams sharing one context serialise; independent streams want one context each.
 *     Every such call moves the context's order to its stream -- also one that enqueued nothing
 *     (n_slots = 0) or failed its argument checks: the next call on another stream then waits for
 *     whatever that stream holds at that point (a false dependency, never a missing one).
 */
#ifndef FT8HIP_H
#define FT8HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FT8HIP_ABI_VERSION 2

/* sample dtypes.  The waterfall dtype follows NumPy promotion against complex64 exactly as
 * scipy.signal.spectrogram does (spectrogram_analyse.py:46-56): F32/C64/I16 -> float32 waterfall,
 * F64/C128 -> float64 waterfall.  I16 samples are scaled x/32767 in float32 on the device
 * (from_wave.py:59-67 read_wave_file). */
enum ft8_dtype { FT8_F32 = 0, FT8_F64 = 1, FT8_C64 = 2, FT8_C128 = 3, FT8_I16 = 4 };

enum ft8_status {
  FT8_OK = 0,
  FT8_E_ARG = -1,         /* invalid argument (message in ft8_last_error) */
  FT8_E_HIP = -2,         /* HIP runtime error */
  FT8_E_UNSUPPORTED = -3, /* an input the path does not take (e.g. a dtype a stage does not accept) */
  FT8_E_NOMEM = -4,       /* device allocation failed */
  FT8_E_RANGE = -5        /* a size exceeds a compiled limit (see ft8_limits) */
};

/* Decoder parameters.  Mirrors decode_ft8_message's keyword arguments (ft8_decode.py:288-296);
 * the freq/time masks (ft8_decode.py:322-341) arrive as index ranges computed on the host. */
typedef struct ft8_params {
  int32_t sample_rate;      /* Hz */
  int32_t bins_per_tone;    /* freq_osr */
  int32_t steps_per_symbol; /* time_osr */
  int32_t max_candidates;   /* N of ft8_find_candidates */
  int32_t max_iterations;   /* BP iterations */
  int32_t min_score_f64;    /* 1: compare scores with min_score in float64 even for a float32
                               waterfall (the threshold was an np.float64); 0: in the waterfall
                               dtype (a Python int/float threshold, NumPy-2 rules) */
  double min_score;
  int32_t f_lo, f_hi;       /* kept STFT bins [f_lo, f_hi) after f >= 0 and the band mask */
  int32_t t_lo, t_hi;       /* kept frames [t_lo, t_hi) after the time mask */
  int32_t flags;            /* FT8_FLAG_* (0: the reference's behaviour exactly) */
  int32_t reserved;
  double sample_rate_hz;    /* ABI 2: when > 0, the exact sample rate in Hz, integral or not (the
                               reference takes a float fs: spectrogram_analyse.py:32-34 computes
                               int(0.16 fs) and int(fs / 6.25 bpt) on it, so fs = 12006.3 gives
                               nperseg 1921); sample_rate is then ignored.  0: use sample_rate. */
} ft8_params;

/* ft8_params.flags.  Both are build-defined extensions OUTSIDE reference parity (the reference
 * has neither); with flags = 0 every result is the reference's.
 *   FT8_FLAG_TOPK      candidate selection keeps the max_candidates highest passing scores
 *                      (ties in scan order), sorted by score descending, instead of reproducing
 *                      ft8_find_candidates' heap quirk (ft8_decode.py:131-137, which keeps the
 *                      first N passing candidates in scan order).
 *   FT8_FLAG_SUBTRACT  ft8_decode_batch runs a second pass: every distinct message decoded in
 *                      pass 1 is re-modulated (ft8_encode + GFSK), fitted to the slot (time/
 *                      frequency refinement, per-symbol complex amplitude) and subtracted, and
 *                      the residual is decoded again.  New messages are appended after the
 *                      pass-1 results with pass_index = 1.  F32 and I16 samples only. */
#define FT8_FLAG_TOPK 1
#define FT8_FLAG_SUBTRACT 2

/* One decoded (or attempted) candidate, 40 bytes, 8-byte aligned. */
typedef struct ft8_result {
  double score;            /* sync score; float32 value widened exactly on the float32 path */
  int32_t slot;            /* slot index within the batch */
  int32_t abs_time;        /* candidate time index (frame steps, may be negative) */
  int32_t abs_freq;        /* candidate frequency index (bins from f_lo) */
  uint16_t crc_extracted;  /* FT8DecodeStatus.crc_extracted */
  uint16_t crc_calculated; /* FT8DecodeStatus.crc_calculated (== FT8Message.hash when ok) */
  int16_t ldpc_errors;     /* FT8DecodeStatus.ldpc_errors (min parity errors seen by BP) */
  uint16_t cand_index;     /* position in the reference candidate order */
  uint8_t payload[10];     /* FT8Message.payload (77 bits, [9] & 0xF8) */
  uint8_t ok;              /* 1: LDPC converged and CRC matched (ft8_decode_candidate True) */
  uint8_t pass_index;      /* 0: decoded from the slot; 1: decoded after subtraction (FT8_FLAG_SUBTRACT) */
} ft8_result;

/* One transmitted FT8 signal for ft8_synthesize, 40 bytes. */
typedef struct ft8_tx_signal {
  double f0;               /* Hz, frequency of tone 0 (the reference's f0 + fc, modulator.py:76-90) */
  double amplitude;        /* peak amplitude of the real waveform */
  double phase;            /* radians added to the carrier phase (0: the reference's sin(phi)) */
  int64_t start;           /* first waveform sample within its slot (may be negative) */
  int32_t slot;            /* output row; the signal array must be sorted by slot ascending */
  int32_t reserved;
} ft8_tx_signal;

/* GFSK timing of ft8_synthesize */
enum ft8_tx_style {
  FT8_TX_PROTOCOL = 0,     /* symbol i occupies samples [i nsps, (i+1) nsps); ramp down at the end */
  FT8_TX_REFERENCE = 1     /* modulator.py exactly: freq_seq read without the one-symbol offset
                              (modulator.py:64-68, symbols start one symbol late) and its trailing
                              ramp (modulator.py:72-73) */
};

typedef struct ft8_ctx ft8_ctx;

/* ---- context ------------------------------------------------------------------------------ */
int ft8_create(int device, ft8_ctx** out);
int ft8_destroy(ft8_ctx* ctx);
const char* ft8_last_error(const ft8_ctx* ctx);
int ft8_abi_version(void);
/* compiled limits: max_candidates, max FFT length (real / complex) */
int ft8_limits(int32_t* max_candidates, int32_t* max_fft_real, int32_t* max_fft_complex);

/* STFT geometry of calculate_spectrogram (spectrogram_analyse.py:31-43): window length,
 * hop, FFT length and frame count for n_samples (frames = 0 when n_samples < nperseg). */
int ft8_geometry(int32_t sample_rate, int32_t bins_per_tone, int32_t steps_per_symbol,
                 int64_t n_samples, int32_t* nperseg, int32_t* hop, int32_t* nfft,
                 int32_t* n_frames);
/* The same for a sample rate given in (possibly non-integral) Hz, as ft8_params.sample_rate_hz. */
int ft8_geometry_hz(double sample_rate_hz, int32_t bins_per_tone, int32_t steps_per_symbol,
                    int64_t n_samples, int32_t* nperseg, int32_t* hop, int32_t* nfft,
                    int32_t* n_frames);

/* ---- stage 1: STFT -> dB waterfall ---------------------------------------------------------
 * Replaces calculate_spectrogram (spectrogram_analyse.py:19-66) + the f>=0 / band / time masks
 * (ft8_decode.py:322-341).  d_samples: n_slots rows of n_samples, row stride slot_stride
 * elements.  Output d_wf[n_slots][t_hi-t_lo][f_hi-f_lo] (TIME-major: the transpose of the
 * reference's mag[freq, time]), bins in natural FFT order k in [f_lo, f_hi) of [0, nfft).  For
 * real input bins above nfft/2 are the mirror image (two-sided spectrum of a real signal). */
int ft8_stft(ft8_ctx* ctx, const void* d_samples, int dtype, int64_t n_samples, int32_t n_slots,
             int64_t slot_stride, const ft8_params* p, void* d_wf, void* stream);

/* Which transform ft8_stft / ft8_decode_batch runs for a geometry (introspection for tests and
 * tuning): FT8_STFT_STOCKHAM (LDS mixed-radix FFT), FT8_STFT_PACKED3840 (the production 12 kHz
 * kernel), FT8_STFT_CHIRPZ (Bluestein: nfft with a prime factor above 7, or odd with real input),
 * FT8_STFT_DFT (direct DFT: what neither FFT path takes); negative FT8_E_* on a bad geometry. */
#define FT8_STFT_STOCKHAM 0
#define FT8_STFT_PACKED3840 1
#define FT8_STFT_CHIRPZ 2
#define FT8_STFT_DFT 3
int ft8_stft_method(ft8_ctx* ctx, int32_t sample_rate, int32_t bins_per_tone, int32_t steps_per_symbol,
                    int64_t n_samples, int dtype);
/* Introspection of the last ft8_stft_argmax / drift STFT on complex128 input at the 3840-point
 * geometry, which decides each frame's argmax in float32 where a rounding-error bound settles it
 * and redoes the others in float64: *frames_redone = the float64 frames of that call, *frames =
 * all its frames (0 / 0 when the last call took another path).  Synchronises the device. */
int ft8_stft_screen_stats(ft8_ctx* ctx, int64_t* frames_redone, int64_t* frames);

/* ---- stage 2: Costas sync score grid + candidate selection ---------------------------------
 * Replaces ft8_sync_score / ft8_find_candidates (ft8_decode.py:47-149).  d_wf as produced by
 * ft8_stft: [n_slots][T][F] (row stride F, slot stride T*F), float32 (wf_f64=0) or float64.
 * Outputs per slot s: d_cand[s][max_candidates][2] = (abs_time, abs_freq) in the reference's
 * final order, d_cand_score[s][max_candidates] (double), d_cand_count[s].  d_scores (nullable)
 * receives the full score grid [n_slots][NT][NF] in scan order in the waterfall dtype. */
int ft8_sync_select(ft8_ctx* ctx, const void* d_wf, int wf_f64, int32_t n_slots, int32_t T,
                    int32_t F, const ft8_params* p, int32_t* d_cand, double* d_cand_score,
                    int32_t* d_cand_count, void* d_scores, void* stream);

/* ft8_sync_score itself (ft8_decode.py:47-100) for arbitrary candidates d_cand[n][2] = (abs_time,
 * abs_freq), on or off the search grid: d_out[n] in the waterfall dtype (-inf as the reference
 * returns it), d_err[n] = 1 where the reference's get_log_power (ftx_types.py:45-47) would raise
 * IndexError (NumPy indexing: negative indices count from the end, nothing guards the frequency
 * axis).  d_wf as for ft8_sync_select. */
int ft8_sync_score(ft8_ctx* ctx, const void* d_wf, int wf_f64, int32_t T, int32_t F, int32_t steps_per_symbol,
                   int32_t bins_per_tone, const int32_t* d_cand, int32_t n, void* d_out, int32_t* d_err,
                   void* stream);

/* ---- stage 3: soft LLRs --------------------------------------------------------------------
 * Replaces ft8_extract_likelihood + ftx_normalize_logl (ft8_decode.py:151-198).  d_cand[n][3] =
 * (slot, abs_time, abs_freq).  Output d_llr[n][174] (double). */
int ft8_llr(ft8_ctx* ctx, const void* d_wf, int wf_f64, int32_t T, int32_t F,
            int32_t steps_per_symbol, int32_t bins_per_tone, const int32_t* d_cand, int32_t n,
            int normalize, double* d_llr, void* stream);

/* ftx_normalize_logl alone (ft8_decode.py:190-198): d_out[n][174] = d_in * sqrt(24 / var(d_in)),
 * with NumPy's pairwise summation order for the mean and variance. */
int ft8_normalize(ft8_ctx* ctx, const double* d_in, int32_t n, double* d_out, void* stream);

/* ---- stage 4: LDPC belief propagation + CRC ------------------------------------------------
 * Replaces bp_decode (ldpc_decoder.py:54-113) and the tail of ft8_decode_candidate
 * (ft8_decode.py:236-273, crc.py:11-54).  d_llr[n][174] double.  Outputs (each nullable):
 * d_plain[n][174] hard decisions of the last evaluated iteration, d_res[n] records (score/slot/
 * abs_* left 0). */
int ft8_bp(ft8_ctx* ctx, const double* d_llr, int32_t n, int32_t max_iterations,
           uint8_t* d_plain, ft8_result* d_res, void* stream);

/* ---- whole receive path ---------------------------------------------------------------------
 * Replaces decode_ft8_message (ft8_decode.py:288-394) for a batch of independent slots:
 * STFT -> sync/select -> LLR -> BP -> CRC, all on the device.  Writes, per slot s, the successful
 * decodes in candidate order to d_out[s][0 .. d_counts[s]) (capped at max_results_per_slot;
 * d_counts holds the uncapped count). */
int ft8_decode_batch(ft8_ctx* ctx, const void* d_samples, int dtype, int64_t n_samples,
                     int32_t n_slots, int64_t slot_stride, const ft8_params* p,
                     ft8_result* d_out, int32_t* d_counts, int32_t max_results_per_slot,
                     void* stream);

/* Pipelining of ft8_decode_batch (a context setting).  The batch is cut into chunks of
 * chunk_slots slots, each an independent STFT -> sync/select -> LLR -> BP -> compact chain, and
 * the chunks alternate over n_streams internal streams (forked from and joined back into the
 * caller's stream), so one chunk's BP overlaps the next chunk's STFT/score.  bp_waves_per_simd
 * (1..4) bounds the BP kernel's resident waves per SIMD (chunked or not), leaving room for work on
 * other streams.  n_streams = 0 runs the whole batch as one chain on the caller's stream.  Default
 * (0, 0, 4): one chain, the full BP grid -- on MI355X the BP kernel is FP64-VALU bound and
 * overlapping it with the next chunk's STFT/score measured no gain.  Results do not depend on the
 * setting. */
int ft8_set_pipeline(ft8_ctx* ctx, int32_t chunk_slots, int32_t n_streams, int32_t bp_waves_per_simd);

/* ---- multi-GPU exchange (slot shards, one all-gather of the decodes per batch) --
 * No reference counterpart (the reference is single-process).  Packs the decodes of one
 * ft8_decode_batch (d_records[n_slots][cap], d_counts[n_slots]) into ONE byte buffer that a
 * collective (RCCL all-gather) moves as-is, on the device and without a host sync:
 *   d_send = [int64 total][int32 counts[n_slots], padded to 8 B][capacity x ft8_result]
 * total = sum over slots of min(counts, cap) (counts are copied uncapped); records in slot order,
 * then candidate order, each with ft8_result.slot += slot_offset (global slot ids); rows of the
 * send buffer past total are zeroed.  Rows >= capacity go to d_overflow[row - capacity] when
 * d_overflow (capacity for n_slots * cap - capacity rows) is non-null, else are dropped -- the
 * receiver sees total > capacity either way.  ft8_pack_bytes gives the send-buffer size. */
int64_t ft8_pack_bytes(int32_t n_slots, int32_t capacity);
int ft8_pack_decodes(ft8_ctx* ctx, const ft8_result* d_records, const int32_t* d_counts, int32_t n_slots,
                     int32_t cap, int32_t capacity, int32_t slot_offset, void* d_send, ft8_result* d_overflow,
                     void* stream);

/* Per-slot flags of the last selection (copied device->device into d_out[n_slots]):
 * bit 0: an exact score tie reached a heap comparison (the reference raises TypeError there,
 *        ftx_types.py:37-47; here ties are ordered by scan index), bit 1: unused (0), bit 2
 *        (informational): the selected set held equal scores, so the heap sequence was replayed
 *        to order them, bit 3 (informational): that replay ran outside the selection kernel
 *        (beside the LLRs in ft8_decode_batch). */
int ft8_select_warnings(ft8_ctx* ctx, int32_t* d_out, int32_t n_slots, void* stream);

/* ---- small device utilities used by the Python mirror of crc.py / ldpc_check ---------------- */
/* CRC-14 (crc.py:11-39) of d_msg[n][12] over d_nbits[n] bits -> d_crc[n]. */
int ft8_crc14(ft8_ctx* ctx, const uint8_t* d_msg, const int32_t* d_nbits, int32_t n,
              uint16_t* d_crc, void* stream);
/* parity-check error count (ldpc_decoder.py:33-52) of d_bits[n][174] (0/1) -> d_errors[n]. */
int ft8_ldpc_check(ft8_ctx* ctx, const uint8_t* d_bits, int32_t n, int32_t* d_errors,
                   void* stream);

/* ---- transmit chain (ft8_generator) and subtract-and-redecode ------------------------------ */
/* Replaces crc_generator + ldpc_generator + ft8_encode (ft8_generator/crc.py:25-47,
 * ldpc.py:104-131, encoder.py:15-73).  d_msg[n][msg_bytes]: msg_bytes = 10, a payload (77 bits;
 * [9] & 0xF8 is applied) whose a91 = crc_generator(payload); msg_bytes = 12, an a91 taken as given
 * (ldpc_generator's input).  Outputs d_a91[n][12], d_codeword[n][22], d_tones[n][79] (nullable). */
int ft8_encode(ft8_ctx* ctx, const uint8_t* d_msg, int32_t msg_bytes, int32_t n, uint8_t* d_a91,
               uint8_t* d_codeword, uint8_t* d_tones, void* stream);

/* Replaces gfsk_modulation_waveform_generator + ft8_modulation_waveform_generator + ft8_generator
 * (modulator.py:27-90) for a batch: ADDS amplitude * ramp * sin(phi + phase) of every signal to
 * d_out[slot][start .. start + 79 nsps) (clipped to [0, n_samples)), nsps = int(0.16 fs).
 * out_dtype FT8_F32 / FT8_F64 (real) or FT8_C64 / FT8_C128 (the complex baseband
 * amplitude * ramp * (sin - j cos)(phi + phase) of ft8_baseband_generator).  d_tones[n][79];
 * d_signals sorted by slot.  Signals overlapping in a slot are summed in array order. */
int ft8_synthesize(ft8_ctx* ctx, const uint8_t* d_tones, const ft8_tx_signal* d_signals, int32_t n_signals,
                   int32_t sample_rate, int32_t style, void* d_out, int out_dtype, int64_t n_samples,
                   int32_t n_slots, int64_t slot_stride, void* stream);

/* Subtraction step of FT8_FLAG_SUBTRACT (build-defined; no reference counterpart): for each slot,
 * every distinct ok message among d_res[slot][0 .. min(d_counts[slot], cap)) (the records of a
 * ft8_decode_batch with the same params) is re-modulated, its start and tone-0 frequency refined
 * around the candidate's (abs_time, abs_freq), its complex amplitude fitted per symbol, and the
 * fitted waveform subtracted: d_residual[slot][n] = x[slot][n] - sum of fitted signals (float32,
 * row stride slot_stride).  dtype FT8_F32 or FT8_I16 (x / 32767); d_residual may alias F32
 * d_samples. */
int ft8_subtract(ft8_ctx* ctx, const void* d_samples, int dtype, float* d_residual, int64_t n_samples,
                 int32_t n_slots, int64_t slot_stride, const ft8_params* p, const ft8_result* d_res,
                 const int32_t* d_counts, int32_t cap, void* stream);

/* The signals the last subtraction of this context fitted (ft8_subtract, or pass 1 of an
 * FT8_FLAG_SUBTRACT ft8_decode_batch, whose cap is max_candidates): fit of record r of slot s at
 * d_out[s * cap + r] for r < min(counts[s], cap), copied device -> device.  n_slots and cap must
 * equal that subtraction's.  The residual is x - sum over the active fits of
 * ramp(n) Re(A(n) exp(2 pi i phase(n))), A interpolated linearly between symbol centres. */
typedef struct ft8_sub_fit {
  int32_t active;          /* 1: fitted and subtracted; 0: failed record, or a payload an earlier record carries */
  int32_t reserved;
  int64_t start;           /* refined first sample of the 79-symbol waveform (slot sample index) */
  double f0;               /* refined tone-0 frequency, Hz */
  float amp[79][2];        /* complex amplitude per symbol ([1 2 1]-smoothed), (re, im) */
  float phase0[80];        /* carrier phase in cycles (fractional part) at the start of each symbol */
  uint8_t tones[80];       /* the payload's re-encoded tone sequence (79 used) */
} ft8_sub_fit;
int ft8_subtract_fits(ft8_ctx* ctx, ft8_sub_fit* d_out, int32_t n_slots, int32_t cap, void* stream);

/* ---- frequency-drift correction (ft8_beacon_receiver/frequency_correction.py) -------------
 * Paths below are relative to src/ft8_tools/ft8_beacon_receiver/.  Parameters of
 * correct_frequency_drift (frequency_correction.py:118-163); fields default to the reference's
 * default_params when the Python mirror fills them. */
typedef struct ft8_drift_params {
  double sample_rate;          /* fs, Hz (integral) */
  double sym_bin;              /* symbol frequency spacing, Hz (6.25) */
  double sym_t;                /* symbol time, s (0.16) */
  double max_variance_factor;  /* max_variance = factor * freq_bins^2 */
  int32_t bins_per_tone;       /* freq_osr */
  int32_t steps_per_symbol;    /* time_osr */
  int32_t nsync_sym, ndata_sym;
  int32_t window_size_factor;  /* window_size = factor * steps_per_symbol */
  int32_t fit_middle_percent;
  int32_t poly_degree;
  int32_t precise_sync;
} ft8_drift_params;

/* how correct_frequency_drift returned (frequency_correction.py line of the return) */
enum ft8_drift_status {
  FT8_DRIFT_PENDING = 0,       /* stage 1 done, stage 2 not yet run */
  FT8_DRIFT_NO_SEGMENT = 1,    /* :236  no continuous segment: the input is returned, rate 0 */
  FT8_DRIFT_LINEAR = 2,        /* :359  precise_sync off: linear compensation only */
  FT8_DRIFT_FEW_POINTS = 3,    /* :523  < 10 sync regression points: linear compensation */
  FT8_DRIFT_DEGREE = 4,        /* :631  poly_degree not 1 or 2: linear compensation */
  FT8_DRIFT_FULL = 5,          /* :655  linear + polynomial compensation */
  FT8_DRIFT_UNDERDETERMINED = 6, /* :659 points <= poly_degree + 1: linear compensation */
  FT8_DRIFT_VALUE_ERROR = -1  /* the reference raises ValueError inside LinearRegression.fit
                                 (:337 an empty segment, :539 regression x/y lengths differ) */
};

/* Per-slot outcome, 72 bytes. */
typedef struct ft8_drift_result {
  double rate_per_sample;      /* correct_frequency_drift's second return value */
  double rate1;                /* f_shift_rate of the linear pass, Hz/s (:348) */
  double coef[3];              /* coefs_final[0..2] of the polynomial fit (coef[0] = 0) */
  double intercept;            /* intercept_final */
  int32_t status;              /* ft8_drift_status */
  int32_t n_segments;          /* continuity segments found (detect_signal_continuity) */
  int32_t seg_start, seg_end;  /* longest segment (max by end - start, first on ties) */
  int32_t sync_idx;            /* correlation_peak_time_block_index (:463) */
  int32_t n_points;            /* regression points of the polynomial fit */
} ft8_drift_result;

/* calculate_spectrogram -> kept bins -> np.argmax over frequency per frame, without writing the
 * waterfall (the argmax is fused into the STFT epilogue): d_idx[n_slots][t_hi - t_lo] = the first
 * bin index (relative to f_lo) of the largest dB value of each frame (frequency_correction.py:
 * 190-224, 364-384).  Samples and params as for ft8_stft. */
int ft8_stft_argmax(ft8_ctx* ctx, const void* d_samples, int dtype, int64_t n_samples, int32_t n_slots,
                    int64_t slot_stride, const ft8_params* p, int32_t* d_idx, void* stream);

/* The two estimation stages on per-frame argmax indices d_idx[n_slots][T] (F = kept bins):
 * stage 1: detect_signal_continuity (:42-115) + longest segment + linear fit (:227-348) -> d_res
 *          (d_metric[n_slots][T - window + 1], nullable: the continuity metric; d_segments
 *          [n_slots][max_segments][2], nullable: the first max_segments segments);
 * stage 2: d_idx of the linearly compensated signal -> sync correlation (:386-463) + polynomial
 *          fit (:502-590) -> d_res (which must hold the stage-1 result). */
int ft8_drift_fit(ft8_ctx* ctx, int32_t stage, const int32_t* d_idx, int32_t n_slots, int32_t T, int32_t F,
                  const ft8_drift_params* p, ft8_drift_result* d_res, double* d_metric, int32_t* d_segments,
                  int32_t max_segments, void* stream);

/* Replaces correct_frequency_drift (frequency_correction.py:118-659) for a batch of independent
 * signals: STFT-argmax -> stage 1 -> linear de-rotation -> STFT-argmax -> stage 2 -> polynomial
 * de-rotation, all on the device.  d_samples: dtype F32/F64/C64/C128, row stride slot_stride
 * elements.  d_out: complex128 [n_slots][n_samples] (for FT8_DRIFT_NO_SEGMENT the input converted
 * to complex128).  d_res[n_slots].  De-rotation carriers: :352 and :598-611. */
int ft8_drift_correct(ft8_ctx* ctx, const void* d_samples, int dtype, int64_t n_samples, int32_t n_slots,
                      int64_t slot_stride, const ft8_drift_params* p, void* d_out, ft8_drift_result* d_res,
                      void* stream);

/* ---- build provenance --------------------------------------------------------------------- */
/* SHA-256 prefix of the sources, headers and Makefile the library was compiled from (the Python
 * binding recomputes it from the tree and refuses a stale library), and the effective compile
 * flags of every object.  No reference counterpart. */
const char* ft8_build_id(void);
const char* ft8_build_flags(void);

/* ---- benchmarking: re-launch one kernel of the last ft8_decode_batch -------------------------
 * Re-launches, reps times on `stream`, the kernel of `stage` (0 stft, 1 score, 2 select, 6 llr,
 * 3 bp, 4 compact) exactly as the last single-chain ft8_decode_batch of this context launched it
 * (same buffers, same arguments; every stage is idempotent on its inputs), so a kernel's duration
 * can be measured by wall clock over back-to-back launches, without events between stages.  Valid
 * while the caller's buffers of that call are alive and until any other entry point of this
 * context runs (FT8_E_ARG otherwise).  No reference counterpart. */
int ft8_replay_stage(ft8_ctx* ctx, int32_t stage, int32_t reps, void* stream);

/* ---- per-stage device timing (HIP events on the caller's stream) --------------------------- */
#define FT8_N_STAGES 12 /* 0 stft, 1 score, 2 select, 3 bp, 4 compact, 5 whole decode_batch, 6 llr,
                         7 subtraction fits (k_sub_est), 8 drift STFT-argmax, 9 drift fits,
                         10 drift de-rotation, 11 subtraction of the fitted signals (k_sub_apply) */
int ft8_set_timing(ft8_ctx* ctx, int enable);
/* which stages record events while timing is enabled (bit s = stage s; default all): timing one
 * stage at a time brackets only that kernel, so the rest of the step runs undisturbed */
int ft8_set_timing_stages(ft8_ctx* ctx, uint32_t mask);
/* accumulated milliseconds and launch counts per stage since the last reset; synchronises. */
int ft8_get_timing(ft8_ctx* ctx, double* ms, int64_t* launches, int reset);
/* BP work counters, accumulated while timing is enabled: out4 = {candidates decoded, BP
 * iterations entered, message-passing sweeps executed, candidates converged}; synchronises. */
int ft8_get_counters(ft8_ctx* ctx, int64_t* out4, int reset);
/* k_bp's own clock, accumulated over launches made while timing is enabled (each persistent wave
 * reads the shader-clock and the constant-rate wall-clock counters when it starts and when it
 * retires): out5 = {sum of wave lifetimes in shader cycles, the same in wall-clock ticks, the
 * longest wave lifetime in cycles, waves, wall-clock rate in kHz}.  Cycles per launch do not depend
 * on the box's clock; cycles / wall time is the clock k_bp ran at.  Synchronises.  (No reference
 * counterpart: measurement of ldpc_decoder.py:54-113's replacement.) */
int ft8_get_bp_clock(ft8_ctx* ctx, int64_t* out5, int reset);

#ifdef __cplusplus
}
#endif
#endif /* FT8HIP_H */
