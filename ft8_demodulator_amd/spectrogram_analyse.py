"""Mirror of the reference spectrogram_analyse.py (spectrogram_analyse.py:1-83), computed on the GPU.

calculate_spectrogram returns the same (spectrogram[nfft, T] in dB, fftshifted; f; t) triple as
the reference; the STFT itself runs in the k_stft HIP kernel (csrc/stft.hip).
"""
from __future__ import annotations

import numpy as np

from . import _device
from ._pipeline import spectrogram_axes

FT8_SYMBOL_DURATION_S = 0.16 / 1
FT8_SYMBOL_FREQ_INTERVAL_HZ = 6.25 * 1
FT8_BAUD_RATE = 1 / FT8_SYMBOL_DURATION_S
SPECTROGRAM_BINS_PER_TONE = 10
SPECTROGRAM_STEPS_PER_SYMBOL = 10
FT8_NUM_SYNC_SEQUENCE = 3
FT8_NUM_SYNC_SYMBOLS_PER_SEQUENCE = 7
FT8_SYNC_PATTERN = [3, 1, 4, 0, 6, 5, 2]
FT8_SYNC_SEQUENCE_OFFSET = 36


def calculate_spectrogram(wave_data, sample_rate: int, bins_per_tone: int = 2, steps_per_symbol: int = 2,
                          device=None) -> tuple:
    """spectrogram_analyse.py:19-66: (10 log10(1e-12 + |STFT|^2/(sum w)^2) fftshifted [nfft, T], f, t)."""
    wf, plan, f64 = _device.stft(wave_data, sample_rate, bins_per_tone, steps_per_symbol, device=device)
    if wf is None:  # signal shorter than one symbol (spectrogram_analyse.py:37-39)
        return np.array([[]]), np.array([]), np.array([])
    spec = wf.t().contiguous().cpu().numpy()
    spec = np.fft.fftshift(spec, axes=0)
    f, t = spectrogram_axes(sample_rate, plan.nperseg, plan.hop, plan.nfft, plan.n_samples)
    return spec, np.fft.fftshift(f), t


def select_frequency_band(spectrogram: np.ndarray, f: np.ndarray, f_min: float, f_max: float) -> tuple:
    """spectrogram_analyse.py:68-82 (inclusive band mask on the frequency axis)."""
    mask = (f >= f_min) & (f <= f_max)
    return spectrogram[mask], f[mask]
