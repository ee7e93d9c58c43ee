"""Mirror of the reference transmit chain (src/ft8_tools/ft8_generator), run on the GPU.

Same names and return types as the reference package (ft8_generator/__init__.py:1-5):
crc_generator, get_crc_from_a91, ldpc_generator, ft8_encode, ft8_baseband_generator,
ft8_generator -- each a call into libft8hip.so (csrc/tx.hip: k_encode, k_synth).  Bit-exact for the
encoder (a91, CRC, codeword, tones); the waveforms match the reference's sequential float64 phase
loop (modulator.py:64-68) to ~1e-10 (closed-form phase, tx_device.h).

Batch entry points for the benchmark and tests: encode_batch (payloads -> a91/codeword/tones on the
device) and synthesize (many signals into many slots, one kernel launch).

Not mirrored: symbolIdSequence_generator / itones_generator / gfsk_modulation_waveform_generator /
ft8_modulation_waveform_generator, the reference's intermediate steps (ft8_encode and the
generators cover them end to end).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

FT8_SYMBOL_NUM = 79
FT8_SYMBOL_TIME_S = 0.16
FT8_SYMBOL_FREQ_INTERVAL_HZ = 6.25


def _u8(a, n):
    a = np.asarray(a, dtype=np.uint8).reshape(-1)
    if a.size < n:
        raise IndexError(f"need at least {n} bytes, got {a.size}")
    return a[:n]


def encode_batch(msgs, msg_bytes: int = 10, device=None):
    """[n, 10] payloads (msg_bytes 10) or [n, 12] a91 (msg_bytes 12), NumPy or torch ->
    (a91 [n, 12], codeword [n, 22], tones [n, 79]) uint8 torch tensors on the GPU."""
    torch = _lib.require_gpu()
    ctx = _lib.context(device)
    dev = torch.device("cuda", ctx.device)
    m = msgs if isinstance(msgs, torch.Tensor) else torch.from_numpy(np.array(msgs, dtype=np.uint8, copy=True))
    m = m.to(device=dev, dtype=torch.uint8).reshape(-1, msg_bytes).contiguous()
    n = m.shape[0]
    a91 = torch.empty((n, 12), dtype=torch.uint8, device=dev)
    cw = torch.empty((n, 22), dtype=torch.uint8, device=dev)
    tones = torch.empty((n, FT8_SYMBOL_NUM), dtype=torch.uint8, device=dev)
    if n:
        ctx.check(_lib.lib().ft8_encode(ctx.handle, _lib.ptr(m), int(msg_bytes), n, _lib.ptr(a91), _lib.ptr(cw),
                                        _lib.ptr(tones), _lib.stream_handle(dev)), "ft8_encode")
    return a91, cw, tones


def crc_generator(payload_10bytes) -> np.ndarray:
    """crc.py:25-47: payload (77 bits) -> a91 (12 bytes) = payload | 5 zero bits dropped | CRC-14."""
    a91, _, _ = encode_batch(_u8(payload_10bytes, 10)[None, :], 10)
    return a91[0].cpu().numpy()


def get_crc_from_a91(a91_12bytes) -> np.uint16:
    """crc.py:49-51."""
    a = _u8(a91_12bytes, 12)
    return np.uint16(((int(a[9]) & 0x07) << 11) | (int(a[10]) << 3) | (int(a[11]) >> 5))


def ldpc_generator(a91_12bytes) -> np.ndarray:
    """ldpc.py:104-131: a91 (taken as given) -> 174-bit codeword (22 bytes)."""
    _, cw, _ = encode_batch(_u8(a91_12bytes, 12)[None, :], 12)
    return cw[0].cpu().numpy()


def ft8_encode(payload) -> np.ndarray:
    """encoder.py:66-73: payload -> 79 channel tones (uint8)."""
    _, _, tones = encode_batch(_u8(payload, 10)[None, :], 10)
    return tones[0].cpu().numpy()


def synthesize(tones, signals, n_slots: int, n_samples: int, sample_rate: int, style: int = _lib.FT8_TX_PROTOCOL,
               out=None, dtype=None, device=None):
    """Add GFSK waveforms to slots on the GPU (ft8_synthesize).

    tones    [n, 79] uint8 (torch on the GPU or NumPy), signal i uses row i
    signals  NumPy array of _lib.TX_SIGNAL_DTYPE (f0, amplitude, phase, start, slot); sorted here
             by slot (stable), with tones permuted to match
    out      optional torch tensor [n_slots, n_samples] (float32/float64/complex64/complex128) that
             the signals are ADDED to; else zeros of `dtype` (default float32) are created.
    """
    torch = _lib.require_gpu()
    ctx = _lib.context(device)
    dev = torch.device("cuda", ctx.device)
    sig = np.ascontiguousarray(signals, dtype=_lib.TX_SIGNAL_DTYPE).reshape(-1)
    t = tones if isinstance(tones, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(tones, dtype=np.uint8))
    t = t.to(device=dev, dtype=torch.uint8).reshape(-1, FT8_SYMBOL_NUM)
    if t.shape[0] != sig.shape[0]:
        raise ValueError("tones and signals differ in length")
    order = np.argsort(sig["slot"], kind="stable")
    if not np.array_equal(order, np.arange(sig.shape[0])):
        sig = sig[order]
        t = t[torch.as_tensor(order, device=dev)]
    t = t.contiguous()
    if sig.size and (sig["slot"].min() < 0 or sig["slot"].max() >= n_slots):
        raise ValueError("signal slot outside [0, n_slots)")
    if out is None:
        out = torch.zeros((n_slots, n_samples), dtype=dtype or torch.float32, device=dev)
    codes = {torch.float32: _lib.FT8_F32, torch.float64: _lib.FT8_F64, torch.complex64: _lib.FT8_C64,
             torch.complex128: _lib.FT8_C128}
    if out.dtype not in codes or out.dim() != 2 or out.stride(1) != 1:
        raise ValueError("out must be a 2-D row-contiguous float32/float64/complex64/complex128 tensor")
    if sig.size:
        d_sig = torch.from_numpy(sig.view(np.uint8).copy()).to(dev)
        ctx.check(_lib.lib().ft8_synthesize(ctx.handle, _lib.ptr(t), _lib.ptr(d_sig), int(sig.shape[0]),
                                            int(sample_rate), int(style), _lib.ptr(out), codes[out.dtype],
                                            int(out.shape[1]), int(out.shape[0]), int(out.stride(0)),
                                            _lib.stream_handle(dev)), "ft8_synthesize")
    return out


def _fs_int(fs) -> int:
    if float(fs) != int(fs) or int(fs) <= 0:
        raise ValueError("sample rate must be a positive integer number of Hz")
    return int(fs)


def _single(payload, fs, f0, style, complex_out):
    torch = _lib.require_gpu()
    fs = _fs_int(fs)
    nsps = int(FT8_SYMBOL_TIME_S * fs)
    n = FT8_SYMBOL_NUM * nsps
    _, _, tones = encode_batch(_u8(payload, 10)[None, :], 10)
    sig = np.zeros(1, dtype=_lib.TX_SIGNAL_DTYPE)
    sig["f0"], sig["amplitude"] = float(f0), 1.0
    out = synthesize(tones, sig, 1, n, fs, style, dtype=torch.complex128 if complex_out else torch.float64)
    return out[0].cpu().numpy()


def ft8_baseband_generator(payload, fs, f0) -> np.ndarray:
    """modulator.py:76-82: complex128 baseband sin(phi) - j cos(phi) with the reference's ramps and
    timing (its one-symbol offset included)."""
    return _single(payload, fs, f0, _lib.FT8_TX_REFERENCE, True)


def ft8_generator(payload, fs, f0, fc) -> np.ndarray:
    """modulator.py:84-90: real float64 waveform = Re(baseband * exp(2j pi fc n / fs))."""
    return _single(payload, fs, float(f0) + float(fc), _lib.FT8_TX_REFERENCE, False)
