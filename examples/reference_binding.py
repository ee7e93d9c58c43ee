"""Reference-side binding of libft8hip.so: what a maintainer of Rintazero/ft8_demodulator adds to
use the MI355X receive path from the reference's own code.

Plain ctypes against two shared libraries -- libamdhip64.so (device memory, one stream) and
libft8hip.so (include/ft8hip.h) -- with NumPy on the host: no torch, no package from this
repository.  It provides decode_ft8_message with the reference's signature and return value
(src/ft8_tools/ft8_demodulator/ft8_decode.py:288-394).  Drop it next to ft8_decode.py as
hip_backend.py and route the call as shown in INTEGRATION.md.

Only the whole-path entry point (ft8_decode_batch) is bound here; the per-stage entry points
(ft8_stft, ft8_sync_select, ft8_llr, ft8_bp) bind the same way.
"""
from __future__ import annotations

import ctypes
import os
from collections import namedtuple

import numpy as np

try:  # inside the reference tree: return its own dataclasses
    from .ftx_types import FT8DecodeStatus, FT8Message  # type: ignore
except ImportError:  # standalone use
    FT8Message = namedtuple("FT8Message", "payload hash")
    FT8DecodeStatus = namedtuple("FT8DecodeStatus", "ldpc_errors crc_extracted crc_calculated")

FT8_F32, FT8_F64 = 0, 1
_H2D, _D2H = 1, 2  # hipMemcpyKind


class ft8_params(ctypes.Structure):
    _fields_ = [("sample_rate", ctypes.c_int32), ("bins_per_tone", ctypes.c_int32),
                ("steps_per_symbol", ctypes.c_int32), ("max_candidates", ctypes.c_int32),
                ("max_iterations", ctypes.c_int32), ("min_score_f64", ctypes.c_int32),
                ("min_score", ctypes.c_double), ("f_lo", ctypes.c_int32), ("f_hi", ctypes.c_int32),
                ("t_lo", ctypes.c_int32), ("t_hi", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("sample_rate_hz", ctypes.c_double)]


FT8HIP_ABI_VERSION = 2   # include/ft8hip.h: ft8_params carries sample_rate_hz since ABI 2


class ft8_result(ctypes.Structure):
    _fields_ = [("score", ctypes.c_double), ("slot", ctypes.c_int32), ("abs_time", ctypes.c_int32),
                ("abs_freq", ctypes.c_int32), ("crc_extracted", ctypes.c_uint16),
                ("crc_calculated", ctypes.c_uint16), ("ldpc_errors", ctypes.c_int16),
                ("cand_index", ctypes.c_uint16), ("payload", ctypes.c_uint8 * 10), ("ok", ctypes.c_uint8),
                ("pad", ctypes.c_uint8)]


assert ctypes.sizeof(ft8_result) == 40 and ctypes.sizeof(ft8_params) == 64


class _Backend:
    def __init__(self, lib_path=None, device=0):
        lib_path = lib_path or os.environ.get("FT8HIP_LIB", "libft8hip.so")
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.ft8 = ctypes.CDLL(lib_path)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        self.hip.hipSetDevice.argtypes = [ctypes.c_int]
        self.hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
        self.hip.hipFree.argtypes = [vp]
        self.hip.hipMemcpy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int]
        self.hip.hipDeviceSynchronize.argtypes = []
        self.ft8.ft8_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        self.ft8.ft8_last_error.argtypes = [vp]
        self.ft8.ft8_last_error.restype = ctypes.c_char_p
        self.ft8.ft8_geometry_hz.argtypes = [ctypes.c_double, i32, i32, i64, vp, vp, vp, vp]
        self.ft8.ft8_decode_batch.argtypes = [vp, vp, ctypes.c_int, i64, i32, i64, ctypes.POINTER(ft8_params),
                                              vp, vp, i32, vp]
        if self.ft8.ft8_abi_version() != FT8HIP_ABI_VERSION:
            raise RuntimeError(f"{lib_path}: ABI {self.ft8.ft8_abi_version()}, this binding speaks {FT8HIP_ABI_VERSION}")
        self._check_hip(self.hip.hipSetDevice(device), "hipSetDevice")
        self.ctx = vp()
        rc = self.ft8.ft8_create(device, ctypes.byref(self.ctx))
        if rc != 0:
            raise RuntimeError(f"ft8_create failed ({rc})")

    @staticmethod
    def _check_hip(err, what):
        if err != 0:
            raise RuntimeError(f"{what} failed: hipError {err}")

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.ft8.ft8_last_error(self.ctx).decode()} ({rc})")

    def malloc(self, nbytes):
        p = ctypes.c_void_p()
        self._check_hip(self.hip.hipMalloc(ctypes.byref(p), max(int(nbytes), 1)), "hipMalloc")
        return p

    def geometry(self, fs, bpt, sps, n):
        v = [ctypes.c_int32() for _ in range(4)]
        # the float rate, as spectrogram_analyse.py:32-34 uses it (fs = 10e3 or 12006.3 are legal there)
        self._check(self.ft8.ft8_geometry_hz(float(fs), bpt, sps, n, *[ctypes.byref(x) for x in v]), "ft8_geometry_hz")
        return [x.value for x in v]


_BACKEND = None


def _backend():
    global _BACKEND
    if _BACKEND is None:
        _BACKEND = _Backend()
    return _BACKEND


def _index_range(axis, lo, hi):
    """Inclusive [lo, hi] mask of ft8_decode.py:328-341 as an index range."""
    if lo is None and hi is None:
        return 0, len(axis)
    lo = axis[0] if lo is None else lo
    hi = axis[-1] if hi is None else hi
    idx = np.nonzero((axis >= lo) & (axis <= hi))[0]
    return (int(idx[0]), int(idx[-1]) + 1) if idx.size else (0, 0)


def decode_ft8_message(wave_data, sample_rate, bins_per_tone=2, steps_per_symbol=2, max_candidates=20,
                       min_score=10, max_iterations=20, freq_min=None, freq_max=None, time_min=None,
                       time_max=None):
    """ft8_decode.py:288-394 on the GPU -> [(FT8Message, FT8DecodeStatus, time_s, freq_hz, score)]."""
    b = _backend()
    x = np.asarray(wave_data)
    if x.ndim != 1:
        raise ValueError("wave_data must be one-dimensional")
    # scipy's promotion against complex64 decides the waterfall precision (spectrogram_analyse.py:46-56)
    f64 = np.result_type(x.dtype, np.complex64) == np.complex128
    if np.iscomplexobj(x):
        raise NotImplementedError("complex input: bind FT8_C64/FT8_C128 the same way")
    x = np.ascontiguousarray(x, dtype=np.float64 if f64 else np.float32)
    n = x.shape[0]
    nperseg, hop, nfft, frames = b.geometry(sample_rate, bins_per_tone, steps_per_symbol, n)
    if frames == 0:
        return []
    f = np.fft.fftfreq(nfft, 1 / sample_rate)[: (nfft + 1) // 2]
    t = np.arange(nperseg / 2, n - nperseg / 2 + 1, hop) / float(sample_rate)
    p = ft8_params(sample_rate=int(sample_rate), sample_rate_hz=float(sample_rate),
                   bins_per_tone=bins_per_tone, steps_per_symbol=steps_per_symbol,
                   max_candidates=max_candidates, max_iterations=max_iterations,
                   min_score_f64=int(isinstance(min_score, np.generic)
                                     and np.result_type(np.float32, min_score) == np.float64),
                   min_score=float(min_score))
    p.f_lo, p.f_hi = _index_range(f, freq_min, freq_max)
    p.t_lo, p.t_hi = _index_range(t, time_min, time_max)
    if p.f_hi <= p.f_lo or p.t_hi <= p.t_lo or max_candidates <= 0:
        return []
    cap = max_candidates
    d_x, d_out, d_cnt = b.malloc(x.nbytes), b.malloc(40 * cap), b.malloc(4)
    try:
        b._check_hip(b.hip.hipMemcpy(d_x, x.ctypes.data, x.nbytes, _H2D), "hipMemcpy")
        b._check(b.ft8.ft8_decode_batch(b.ctx, d_x, FT8_F64 if f64 else FT8_F32, n, 1, n, ctypes.byref(p),
                                        d_out, d_cnt, cap, None), "ft8_decode_batch")
        recs = (ft8_result * cap)()
        cnt = ctypes.c_int32()
        b._check_hip(b.hip.hipMemcpy(ctypes.addressof(recs), d_out, 40 * cap, _D2H), "hipMemcpy")
        b._check_hip(b.hip.hipMemcpy(ctypes.byref(cnt), d_cnt, 4, _D2H), "hipMemcpy")
    finally:
        for d in (d_x, d_out, d_cnt):
            b.hip.hipFree(d)
    out = []
    for r in recs[: min(cnt.value, cap)]:
        msg = FT8Message(payload=bytearray(bytes(r.payload)), hash=int(r.crc_calculated))
        st = FT8DecodeStatus(ldpc_errors=int(r.ldpc_errors), crc_extracted=int(r.crc_extracted),
                             crc_calculated=int(r.crc_calculated))
        score = np.float64(r.score) if f64 else np.float32(r.score)
        out.append((msg, st, r.abs_time / sample_rate, (r.abs_freq / bins_per_tone) * 6.25, score))
    return out
