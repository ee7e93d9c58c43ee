"""FT8 data types -- mirror of the reference's ftx_types.py (ftx_types.py:10-60).

Same class names and fields.  FT8Waterfall.mag keeps the reference orientation [freq, time]
(ftx_types.py:17); on the device the waterfall is stored time-major ([time, freq], frequency
fastest) and `mag` may be a transposed view of it.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum

import numpy as np


class FT8Protocol(Enum):
    """FT8 Protocol Type (ftx_types.py:10-12)"""
    FT8 = 1


@dataclass
class FT8Waterfall:
    """Spectrogram waterfall (ftx_types.py:14-34): mag[freq, time], oversampling rates."""
    mag: np.ndarray
    time_osr: int
    freq_osr: int

    def __post_init__(self):
        if len(self.mag.shape) != 2:
            raise ValueError("mag must be a 2D array with shape (frequency, time)")

    @property
    def num_bins(self) -> int:
        return self.mag.shape[0]

    @property
    def num_blocks(self) -> int:
        return self.mag.shape[1] // self.time_osr


@dataclass
class FT8Candidate:
    """Candidate (ftx_types.py:36-47)."""
    waterfall: "FT8Waterfall"
    abs_time: int = 0
    abs_freq: int = 0
    score: float = 0.0

    def get_log_power(self, time_offset: int, freq_offset: int):
        w = self.waterfall
        return w.mag[self.abs_freq + freq_offset * w.freq_osr, self.abs_time + time_offset * w.time_osr]


@dataclass
class FT8Message:
    """Decoded message (ftx_types.py:49-53)."""
    payload: bytearray = field(default_factory=lambda: bytearray(10))
    hash: int = 0


@dataclass
class FT8DecodeStatus:
    """Decode status (ftx_types.py:55-60)."""
    ldpc_errors: int = 0
    crc_extracted: int = 0
    crc_calculated: int = 0
