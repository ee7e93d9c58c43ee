"""Host orchestration of the device receive path.

Turns decode_ft8_message's arguments (ft8_decode.py:288-296) into an ft8_params block -- STFT
geometry (spectrogram_analyse.py:31-43), the f >= 0 / band / time masks as index ranges
(ft8_decode.py:322-341) -- launches ft8_decode_batch on the caller's stream, and assembles the
reference's 5-tuples (ft8_decode.py:383-391) from the fixed-size device records.

Only parameter bookkeeping and result formatting happen here; every sample, waterfall, score,
LLR and codeword is processed by the HIP kernels of libft8hip.so.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .ftx_types import FT8DecodeStatus, FT8Message

FT8_SYMBOL_FREQ_INTERVAL_HZ = 6.25  # spectrogram_analyse.py:7


@dataclass
class Plan:
    sample_rate: float  # as the caller gave it (int or float Hz)
    bins_per_tone: int
    steps_per_symbol: int
    n_samples: int
    nperseg: int
    hop: int
    nfft: int
    frames: int
    f_lo: int
    f_hi: int
    t_lo: int
    t_hi: int
    f: np.ndarray  # kept frequencies (Hz)
    t: np.ndarray  # kept frame-centre times (s)

    @property
    def empty(self) -> bool:
        return self.f_hi <= self.f_lo or self.t_hi <= self.t_lo

    @property
    def F(self) -> int:
        return self.f_hi - self.f_lo

    @property
    def T(self) -> int:
        return self.t_hi - self.t_lo


def spectrogram_axes(sample_rate, nperseg, hop, nfft, n_samples):
    """Unshifted two-sided frequency axis and frame times exactly as scipy builds them
    (_spectral_helper: fftfreq(nfft, 1/fs); arange(nperseg/2, n - nperseg/2 + 1, step)/fs)."""
    f = np.fft.fftfreq(nfft, 1 / sample_rate)
    t = np.arange(nperseg / 2, n_samples - nperseg / 2 + 1, hop) / float(sample_rate)
    return f, t


def make_plan(n_samples, sample_rate, bins_per_tone=2, steps_per_symbol=2, freq_min=None, freq_max=None,
              time_min=None, time_max=None) -> Plan:
    nperseg, hop, nfft, frames = _lib.geometry(sample_rate, bins_per_tone, steps_per_symbol, n_samples)
    if frames == 0:  # len(wave_data) < nperseg: empty spectrogram (spectrogram_analyse.py:37-39)
        z = np.zeros(0)
        return Plan(sample_rate, bins_per_tone, steps_per_symbol, n_samples, nperseg, hop, nfft, 0, 0, 0, 0, 0, z, z)
    f_all, t = spectrogram_axes(sample_rate, nperseg, hop, nfft, n_samples)
    npos = (nfft + 1) // 2            # fftshift then f >= 0 keeps natural bins 0..npos-1
    f = f_all[:npos]
    f_lo, f_hi = 0, npos
    if freq_min is not None or freq_max is not None:  # ft8_decode.py:328-333 (inclusive)
        lo = freq_min if freq_min is not None else f[0]
        hi = freq_max if freq_max is not None else f[-1]
        idx = np.nonzero((f >= lo) & (f <= hi))[0]
        f_lo, f_hi = (int(idx[0]), int(idx[-1]) + 1) if idx.size else (0, 0)
    t_lo, t_hi = 0, len(t)
    if time_min is not None or time_max is not None:  # ft8_decode.py:336-341 (inclusive)
        lo = time_min if time_min is not None else t[0]
        hi = time_max if time_max is not None else t[-1]
        idx = np.nonzero((t >= lo) & (t <= hi))[0]
        t_lo, t_hi = (int(idx[0]), int(idx[-1]) + 1) if idx.size else (0, 0)
    return Plan(sample_rate, bins_per_tone, steps_per_symbol, n_samples, nperseg, hop, nfft, frames,
                f_lo, f_hi, t_lo, t_hi, f[f_lo:f_hi], t[t_lo:t_hi])


def min_score_is_f64(min_score) -> bool:
    """NumPy-2 rule for `np.float32 < min_score`: a Python int/float adopts float32; a NumPy scalar
    (np.float64, np.int64, ...) promotes the comparison to float64."""
    if isinstance(min_score, np.generic):
        return np.result_type(np.float32, min_score) == np.float64
    return False


def make_params(plan: Plan, max_candidates, min_score, max_iterations, flags=0) -> _lib.Ft8Params:
    p = _lib.Ft8Params()
    fs = _lib.sample_rate_hz(plan.sample_rate)
    p.sample_rate = int(fs)
    p.sample_rate_hz = fs   # the geometry follows the float rate (spectrogram_analyse.py:32-34)
    p.bins_per_tone = int(plan.bins_per_tone)
    p.steps_per_symbol = int(plan.steps_per_symbol)
    p.max_candidates = int(max_candidates)
    p.max_iterations = int(max_iterations)
    p.min_score_f64 = int(min_score_is_f64(min_score))
    p.min_score = float(min_score)
    p.f_lo, p.f_hi, p.t_lo, p.t_hi = plan.f_lo, plan.f_hi, plan.t_lo, plan.t_hi
    p.flags = int(flags)
    return p


_TORCH_CODES = None


def _torch_codes():
    global _TORCH_CODES
    if _TORCH_CODES is None:
        import torch
        _TORCH_CODES = {torch.float32: _lib.FT8_F32, torch.float64: _lib.FT8_F64,
                        torch.complex64: _lib.FT8_C64, torch.complex128: _lib.FT8_C128,
                        torch.int16: _lib.FT8_I16}
    return _TORCH_CODES


def device_samples(wave_data, device=None, int16_is_pcm=False):
    """-> (tensor on the GPU, ft8 dtype code, waterfall is float64).

    NumPy input follows scipy's promotion against complex64 (spectrogram_analyse.py:46-56): any
    real array that promotes to complex64 is transformed as float32, to complex128 as float64.
    int16 tensors are raw PCM (scaled x/32767 on the device, read_wave_file semantics) only when
    int16_is_pcm is set."""
    torch = _lib.require_gpu()
    dev = torch.device("cuda", _lib.device_index(device))
    if isinstance(wave_data, torch.Tensor):
        x = wave_data
        if x.dtype == torch.int16 and int16_is_pcm:
            code = _lib.FT8_I16
        elif x.dtype in (torch.float32, torch.float64, torch.complex64, torch.complex128):
            code = _torch_codes()[x.dtype]
        else:
            nd = np.result_type(np.dtype(str(x.dtype).replace("torch.", "")), np.complex64)
            x = x.to(torch.float32 if nd == np.complex64 else torch.float64)
            code = _torch_codes()[x.dtype]
        x = x.to(dev).contiguous()
    else:
        a = np.asarray(wave_data)
        rt = np.result_type(a, np.complex64)
        if np.iscomplexobj(a):
            a = a.astype(np.complex64 if rt == np.complex64 else np.complex128, copy=False)
            code = _lib.FT8_C64 if rt == np.complex64 else _lib.FT8_C128
        else:
            a = a.astype(np.float32 if rt == np.complex64 else np.float64, copy=False)
            code = _lib.FT8_F32 if rt == np.complex64 else _lib.FT8_F64
        x = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    wf_f64 = code in (_lib.FT8_F64, _lib.FT8_C128)
    return x, code, wf_f64


def records_to_results(recs: np.ndarray, sample_rate: int, bins_per_tone: int, wf_f64: bool):
    """Device records (ok only, candidate order) -> [(FT8Message, FT8DecodeStatus, time_sec,
    freq_hz, score)] exactly as decode_ft8_message returns them (ft8_decode.py:383-391).

    time_sec = abs_time / sample_rate and freq_hz = (abs_freq / bins_per_tone) * 6.25 as Python
    floats, score as the waterfall dtype's NumPy scalar.  Columns are converted once per call (the
    per-record work is only the object construction)."""
    n = len(recs)
    if n == 0:
        return []
    payload = recs["payload"].tobytes()
    crc_c = recs["crc_calculated"].tolist()
    crc_e = recs["crc_extracted"].tolist()
    errs = recs["ldpc_errors"].tolist()
    tsec = [t / sample_rate for t in recs["abs_time"].tolist()]
    fhz = [(f / bins_per_tone) * FT8_SYMBOL_FREQ_INTERVAL_HZ for f in recs["abs_freq"].tolist()]
    sc = recs["score"].astype(np.float64 if wf_f64 else np.float32)
    out = []
    for i in range(n):
        msg = FT8Message(payload=bytearray(payload[10 * i: 10 * i + 10]), hash=crc_c[i])
        st = FT8DecodeStatus(ldpc_errors=errs[i], crc_extracted=crc_e[i], crc_calculated=crc_c[i])
        out.append((msg, st, tsec[i], fhz[i], sc[i]))
    return out


def warn_truncated(counts: np.ndarray, cap: int, stacklevel: int = 2) -> None:
    """RuntimeWarning when a slot decoded more messages than its record capacity holds (the device
    keeps the first `cap` in candidate order and counts the rest)."""
    over = np.nonzero(counts > cap)[0]
    if over.size:
        import warnings
        warnings.warn(f"{over.size} slot(s) decoded more messages than max_results_per_slot={cap} "
                      f"(e.g. slot {int(over[0])}: {int(counts[over[0]])}); the records beyond it were dropped",
                      RuntimeWarning, stacklevel=stacklevel + 1)


class SlotDecoder:
    """Batched decode of independent slots on one GPU: [B, N] samples -> per-slot decodes.

    The receive path (STFT -> Costas sync -> selection -> LLR -> BP -> CRC) runs as one
    ft8_decode_batch call on the current stream; outputs are fixed-size device records
    (ft8_result, 40 B) plus per-slot counts, ready for an all-gather across ranks.
    """

    def __init__(self, sample_rate=12000, bins_per_tone=2, steps_per_symbol=2, max_candidates=20,
                 min_score=10, max_iterations=20, freq_min=None, freq_max=None, time_min=None,
                 time_max=None, device=None, flags=0, max_results_per_slot=None, context=None):
        self.kw = dict(sample_rate=sample_rate, bins_per_tone=bins_per_tone, steps_per_symbol=steps_per_symbol,
                       freq_min=freq_min, freq_max=freq_max, time_min=time_min, time_max=time_max)
        self.max_candidates = int(max_candidates)
        self.min_score = min_score
        self.max_iterations = int(max_iterations)
        self.flags = flags
        self.device = _lib.device_index(device)
        # the thread's context for the device, or a dedicated one (_lib.Context(device)): decoders
        # that run concurrently on different streams want one context each (the library orders a
        # shared context's work across streams, which serialises them)
        self.ctx = context if context is not None else _lib.context(self.device)
        # a subtract-and-redecode batch appends up to max_candidates pass-2 records after up to
        # max_candidates pass-1 records, so its default capacity holds both passes
        default_cap = max(self.max_candidates, 1) * (2 if flags & _lib.FT8_FLAG_SUBTRACT else 1)
        self.cap = int(max_results_per_slot if max_results_per_slot is not None else default_cap)
        self._plans = {}
        self._out = None
        self._counts = None

    def plan(self, n_samples) -> Plan:
        if n_samples not in self._plans:
            self._plans[n_samples] = make_plan(n_samples, **self.kw)
        return self._plans[n_samples]

    def _buffers(self, n_slots):
        import torch
        dev = torch.device("cuda", self.device)
        need = n_slots * self.cap * _lib.RESULT_DTYPE.itemsize
        if self._out is None or self._out.numel() < max(need, 1):
            self._out = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        if self._counts is None or self._counts.numel() < n_slots:
            self._counts = torch.empty(max(n_slots, 1), dtype=torch.int32, device=dev)
        return self._out, self._counts

    def run(self, samples, code=None, int16_is_pcm=True):
        """Asynchronous launch on the current stream.  samples: GPU tensor [B, N] (or [N]).
        Returns (records uint8 tensor [B*cap*40], counts int32 tensor [B])."""
        import torch
        x = samples
        if code is None:
            x, code, _ = device_samples(samples, self.device, int16_is_pcm=int16_is_pcm)
        if x.dim() == 1:
            x = x.unsqueeze(0)
        if x.dim() != 2:
            raise ValueError("samples must be [n_slots, n_samples]")
        if not x.is_contiguous():
            x = x.contiguous()
        n_slots, n = int(x.shape[0]), int(x.shape[1])
        out, counts = self._buffers(n_slots)
        plan = self.plan(n)
        if plan.empty or n_slots == 0:
            counts[:n_slots].zero_()
            return out, counts[:n_slots]
        p = make_params(plan, self.max_candidates, self.min_score, self.max_iterations, self.flags)
        rc = _lib.lib().ft8_decode_batch(self.ctx.handle, _lib.ptr(x), int(code), n, n_slots, n,
                                         ctypes.byref(p), _lib.ptr(out), _lib.ptr(counts), self.cap,
                                         _lib.stream_handle(torch.device("cuda", self.device)))
        self.ctx.check(rc, "ft8_decode_batch")
        return out, counts[:n_slots]

    def records(self, samples, code=None, int16_is_pcm=True):
        """Synchronous: -> list (per slot) of structured ft8_result arrays (ok decodes, candidate order)."""
        out, counts = self.run(samples, code, int16_is_pcm)
        c = counts.cpu().numpy()
        n_slots = len(c)
        recs = out[: n_slots * self.cap * _lib.RESULT_DTYPE.itemsize].cpu().numpy().view(_lib.RESULT_DTYPE)
        recs = recs.reshape(n_slots, self.cap) if n_slots else recs.reshape(0, self.cap)
        warn_truncated(c, self.cap, stacklevel=3)
        return [recs[s, : min(int(c[s]), self.cap)].copy() for s in range(n_slots)]

    def decode(self, samples, int16_is_pcm=True):
        """-> list (per slot) of the reference's 5-tuples."""
        x, code, wf_f64 = device_samples(samples, self.device, int16_is_pcm=int16_is_pcm)
        per_slot = self.records(x, code)
        return [records_to_results(r, self.kw["sample_rate"], self.kw["bins_per_tone"], wf_f64) for r in per_slot]

    def timing(self, reset=False):
        return self.ctx.timing(reset)


def decode_slots(samples, sample_rate=12000, **kwargs):
    """One-call form of SlotDecoder: samples [B, N] (GPU tensor, float32/int16/...) -> list (per
    slot) of decode_ft8_message's 5-tuples."""
    return SlotDecoder(sample_rate=sample_rate, **kwargs).decode(samples)
