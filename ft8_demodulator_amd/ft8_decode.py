"""Mirror of the reference ft8_decode.py (src/ft8_tools/ft8_demodulator/ft8_decode.py:1-394).

Same public functions, arguments and return values.  The numeric work runs in libft8hip.so:
decode_ft8_message is one ft8_decode_batch call (STFT -> Costas sync -> selection -> LLR -> BP ->
CRC on the GPU); the per-stage functions call the matching stage entry points.

Deliberate differences (DESIGN.md "Parity"):
  * the matplotlib figure (ft8_decode.py:343-380) is opt-in (plot=True) instead of always written
    to ft8_spectrogram_with_candidates.png in the working directory;
  * an input shorter than one symbol, or masks that leave nothing, return [] (the reference
    raises IndexError at ft8_decode.py:346; its own test expects []);
  * exact score ties that reach a heap comparison are ordered by scan position (the reference
    raises TypeError, FT8Candidate being unordered);
  * the reference's progress prints are behind verbose=True;
  * max_candidates is capped at 4096 (ft8_limits(); the selection holds its candidates in LDS):
    a larger value raises ValueError (FT8_E_RANGE) instead of running -- the reference has no cap.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from . import _device, _lib
from ._pipeline import SlotDecoder, device_samples, make_plan, records_to_results
from .crc import compute_crc, extract_crc
from .ftx_types import FT8Candidate, FT8DecodeStatus, FT8Message, FT8Protocol, FT8Waterfall  # noqa: F401
from .spectrogram_analyse import FT8_SYMBOL_DURATION_S, FT8_SYMBOL_FREQ_INTERVAL_HZ, calculate_spectrogram  # noqa: F401

FT8_ND = 58
FT8_NUM_SYNC = 3
FT8_LENGTH_SYNC = 7
FT8_SYNC_OFFSET = 36
FT8_LDPC_N = 174
FT8_LDPC_K = 91
FT8_LDPC_K_BYTES = 12
FT8_Gray_map = [0, 1, 3, 2, 5, 6, 4, 7]
FT8_Costas_pattern = [3, 1, 4, 0, 6, 5, 2]


def ft8_sync_score(wf: FT8Waterfall, candidate: FT8Candidate) -> float:
    """ft8_decode.py:47-100 for any candidate, on or off the search grid (one GPU thread,
    k_score_list): -inf (a Python float) when nothing is comparable, else the waterfall-dtype mean;
    IndexError where the reference's get_log_power (ftx_types.py:45-47) would index past the
    waterfall (negative indices count from the end, as NumPy's do)."""
    s, err = _device.sync_scores(wf, [(candidate.abs_time, candidate.abs_freq)])
    if err[0]:
        raise IndexError("index out of bounds for the waterfall (FT8Candidate.get_log_power)")
    v = s[0]
    return float("-inf") if v == -np.inf else v


def ft8_sync_scores(wf: FT8Waterfall, candidates) -> np.ndarray:
    """Vectorised ft8_sync_score over [(abs_time, abs_freq), ...] (build-defined helper, one launch);
    IndexError if any candidate would raise it."""
    s, err = _device.sync_scores(wf, [(c.abs_time, c.abs_freq) if isinstance(c, FT8Candidate) else tuple(c)
                                      for c in candidates])
    if err.any():
        raise IndexError(f"candidate {int(np.argmax(err))}: index out of bounds for the waterfall")
    return s


def ft8_score_grid(wf: FT8Waterfall) -> np.ndarray:
    """Every ft8_sync_score of the search grid, [time, freq] in scan order (one GPU launch)."""
    _, grid, _ = _device.sync_select(wf, 0, 0, want_grid=True)
    return grid


def ft8_find_candidates(wf: FT8Waterfall, num_candidates: int, min_score, verbose: bool = False, *,
                        selection: str = "reference") -> List[FT8Candidate]:
    """ft8_decode.py:102-149: the reference heap selection, sorted by score descending.

    selection="topk" (build-defined, outside parity) keeps the num_candidates highest passing
    scores instead of the reference heap's first-N-in-scan-order set."""
    if num_candidates <= 0:
        return []
    cands, _, _ = _device.sync_select(wf, num_candidates, min_score, flags=selection_flags(selection))
    out = [FT8Candidate(waterfall=wf, abs_time=a, abs_freq=b, score=s) for a, b, s in cands]
    if verbose:
        print(f"Number of candidates found: {len(out)}")
    return out


def ft8_extract_likelihood(wf: FT8Waterfall, cand: FT8Candidate, log174: np.ndarray) -> None:
    """ft8_decode.py:164-188 (in place)."""
    log174[:FT8_LDPC_N] = _device.llr(wf, [(cand.abs_time, cand.abs_freq)], normalize=False)[0]


def ftx_normalize_logl(log174: np.ndarray) -> None:
    """ft8_decode.py:190-198 (in place): scale to variance 24."""
    log174[:] = _device.normalize(np.asarray(log174, dtype=np.float64))[0]


def pack_bits(bit_array: np.ndarray, num_bits: int) -> bytearray:
    """ft8_decode.py:200-215: bits (zero / non-zero) -> MSB-first bytes."""
    bits = (np.asarray(bit_array[:num_bits]) != 0).astype(np.uint8)
    return bytearray(np.packbits(bits).tobytes())


def ftx_compute_crc(data: bytearray, num_bits: int) -> int:
    return compute_crc(data, num_bits)


def ftx_extract_crc(data: bytearray) -> int:
    return extract_crc(data)


def ft8_decode_candidate(wf: FT8Waterfall, cand: FT8Candidate, max_iterations: int) -> Tuple[bool, FT8Message, FT8DecodeStatus]:
    """ft8_decode.py:225-273: LLR -> normalise -> BP -> CRC for one candidate."""
    log174 = _device.llr(wf, [(cand.abs_time, cand.abs_freq)], normalize=True)
    _, rec = _device.bp(log174, max_iterations)
    r = rec[0]
    message, status = FT8Message(), FT8DecodeStatus()
    status.ldpc_errors = int(r["ldpc_errors"])
    if status.ldpc_errors > 0:
        return False, message, status
    status.crc_extracted = int(r["crc_extracted"])
    status.crc_calculated = int(r["crc_calculated"])
    if not r["ok"]:
        return False, message, status
    message.hash = status.crc_calculated
    message.payload = bytearray(r["payload"].tobytes())
    return True, message, status


def create_waterfall_from_spectrogram(spectrogram: np.ndarray, time_osr: int, freq_osr: int) -> FT8Waterfall:
    """ft8_decode.py:275-286."""
    if len(spectrogram.shape) != 2:
        raise ValueError("spectrogram must be a 2-D array with shape (frequency, time)")
    return FT8Waterfall(mag=spectrogram, time_osr=time_osr, freq_osr=freq_osr)


def selection_flags(selection: str = "reference", subtract: bool = False) -> int:
    """ft8_params.flags for the build-defined options (include/ft8hip.h FT8_FLAG_*)."""
    if selection not in ("reference", "topk"):
        raise ValueError("selection must be 'reference' or 'topk'")
    return (_lib.FT8_FLAG_TOPK if selection == "topk" else 0) | (_lib.FT8_FLAG_SUBTRACT if subtract else 0)


def decode_ft8_message(wave_data, sample_rate: int, bins_per_tone: int = 2, steps_per_symbol: int = 2,
                       max_candidates: int = 20, min_score=10, max_iterations: int = 20,
                       freq_min: float = None, freq_max: float = None, time_min: float = None,
                       time_max: float = None, *, plot: bool = False, verbose: bool = False, device=None,
                       selection: str = "reference", subtract: bool = False):
    """ft8_decode.py:288-394 -> [(FT8Message, FT8DecodeStatus, time_sec, freq_hz, score)].

    time_sec = abs_time / sample_rate and freq_hz = abs_freq / bins_per_tone * 6.25 relative to the
    first kept bin, exactly as the reference reports them (ft8_decode.py:387-388).

    Build-defined options (outside reference parity, defaults reproduce the reference):
    selection="topk" keeps the max_candidates highest scores; subtract=True subtracts the decoded
    signals and decodes the residual once more, appending new messages (float32 input only)."""
    x, code, wf_f64 = device_samples(wave_data, device)
    if x.dim() != 1:
        raise ValueError("wave_data must be one-dimensional")
    plan = make_plan(int(x.shape[0]), sample_rate, bins_per_tone, steps_per_symbol, freq_min, freq_max,
                     time_min, time_max)
    results = []
    if not plan.empty and max_candidates > 0:
        dec = SlotDecoder(sample_rate, bins_per_tone, steps_per_symbol, max_candidates, min_score, max_iterations,
                          freq_min, freq_max, time_min, time_max, device=x.device,
                          flags=selection_flags(selection, subtract))
        recs = dec.records(x.unsqueeze(0), code)[0]
        results = records_to_results(recs, sample_rate, bins_per_tone, wf_f64)
    if plot and not plan.empty:
        _plot(wave_data, sample_rate, bins_per_tone, steps_per_symbol, plan, max_candidates, min_score)
    if verbose:
        print(f"Decoded messages: {results}")
    return results


def _plot(wave_data, sample_rate, bpt, sps, plan, max_candidates, min_score, path="ft8_spectrogram_with_candidates.png"):
    """Opt-in version of the reference's debug figure (ft8_decode.py:343-380)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    wf_t, _, _ = _device.stft(wave_data, sample_rate, bpt, sps, plan.f_lo, plan.f_hi, plan.t_lo, plan.t_hi)
    spec = wf_t.t().contiguous().cpu().numpy()
    f, t = plan.f, plan.t
    plt.figure(figsize=(10, 6))
    plt.imshow(spec, aspect="auto", origin="lower", extent=[t[0], t[-1], f[0], f[-1]])
    plt.colorbar(label="Intensity (dB)")
    plt.title("FT8 Signal Spectrogram")
    plt.xlabel("Time (s)")
    plt.ylabel("Frequency (Hz)")
    wf = create_waterfall_from_spectrogram(spec, sps, bpt)
    for i, cand in enumerate(ft8_find_candidates(wf, max_candidates, min_score)):
        ts = t[0] + (cand.abs_time * (t[-1] - t[0])) / (wf.num_blocks * wf.time_osr)
        fh = f[0] + (cand.abs_freq * (f[-1] - f[0])) / (wf.mag.shape[0])
        plt.plot(ts, fh, "ro", markersize=4)
        plt.annotate(f"{i + 1}:{cand.score:.1f}", (ts, fh), xytext=(5, 5), textcoords="offset points",
                     color="white", fontsize=8, bbox=dict(boxstyle="round,pad=0.3", fc="red", alpha=0.7))
    plt.savefig(path)
    plt.close()
