"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (parity checker + timed "port" CPU baseline).

Python side of the CPU restatement of the reference FT8 receive path.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the product package
ft8_demodulator_amd never does.

  * STFT: the reference calls scipy.signal.spectrogram (spectrogram_analyse.py:19-66).  SciPy
    1.15.3 is the pinned third-party dependency and is present in this image, so the oracle
    calls exactly that function with exactly the reference's arguments.
  * Sync score, candidate selection, LLR, normalisation, BP and CRC: the C restatement in
    oracle/ft8_oracle.c (built by oracle/Makefile into oracle/_build/libft8oracle.so).
  * Result assembly: ft8_decode.py:383-394.

Pinned against the reference's own outputs in tests/golden/ (tests/test_oracle_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libft8oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i, l, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_double
        for nm in ("orc_score_grid_f32", "orc_score_grid_f64"):
            getattr(L, nm).argtypes = [vp, l, l, i, i, i, i, vp]
            getattr(L, nm).restype = None
        L.orc_select.argtypes = [vp, i, l, l, d, i, vp, vp, vp]
        L.orc_select.restype = l
        for nm in ("orc_llr_f32", "orc_llr_f64"):
            getattr(L, nm).argtypes = [vp, l, l, i, i, i, i, i, vp]
            getattr(L, nm).restype = None
        L.orc_normalize.argtypes = [vp]
        L.orc_pairwise_sum.argtypes = [vp, l]
        L.orc_pairwise_sum.restype = d
        L.orc_bp_decode.argtypes = [vp, i, vp]
        L.orc_bp_decode.restype = i
        L.orc_ldpc_check.argtypes = [vp]
        L.orc_ldpc_check.restype = i
        L.orc_crc14.argtypes = [vp, i]
        L.orc_crc14.restype = i
        L.orc_decode_tail.argtypes = [vp, i, vp, vp, vp]
        L.orc_decode_tail.restype = i
        L.orc_ldpc_encode.argtypes = [vp, vp]
        for nm in ("orc_decode_waterfall_f32", "orc_decode_waterfall_f64"):
            getattr(L, nm).argtypes = [vp, l, l, i, i, i, i, l, d, i, i, vp, vp]
            getattr(L, nm).restype = l
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# ----------------------------------------------------------------------------------------------
# STFT (spectrogram_analyse.py:19-66) and the mask / waterfall step (ft8_decode.py:315-355)
# ----------------------------------------------------------------------------------------------
def calculate_spectrogram(wave_data, sample_rate, bins_per_tone=2, steps_per_symbol=2):
    import scipy.signal

    samples_per_symbol = int(0.16 * sample_rate)
    overlap = samples_per_symbol - samples_per_symbol // steps_per_symbol
    dft_length = int(sample_rate / 6.25 * bins_per_tone)
    if len(wave_data) < samples_per_symbol:
        return np.array([[]]), np.array([]), np.array([])
    if overlap >= samples_per_symbol:
        overlap = samples_per_symbol - 1
    f, t, spec = scipy.signal.spectrogram(
        wave_data, fs=sample_rate, window="hann", nperseg=samples_per_symbol,
        noverlap=overlap, nfft=dft_length, detrend=False, return_onesided=False,
        scaling="spectrum")
    with np.errstate(divide="ignore"):
        spec = 10 * np.log10(1e-12 + np.abs(spec))
    spec = np.fft.fftshift(spec, axes=0)
    f = np.fft.fftshift(f)
    return spec, f, t


def waterfall(wave_data, sample_rate, bins_per_tone=2, steps_per_symbol=2,
              freq_min=None, freq_max=None, time_min=None, time_max=None):
    """mag[freq, time] exactly as decode_ft8_message builds it (ft8_decode.py:315-341)."""
    spec, f, t = calculate_spectrogram(wave_data, sample_rate, bins_per_tone, steps_per_symbol)
    if f.size == 0:
        return None
    keep = f >= 0
    spec, f = spec[keep], f[keep]
    if freq_min is not None or freq_max is not None:
        lo = freq_min if freq_min is not None else f[0]
        hi = freq_max if freq_max is not None else f[-1]
        m = (f >= lo) & (f <= hi)
        spec, f = spec[m], f[m]
    if time_min is not None or time_max is not None:
        lo = time_min if time_min is not None else t[0]
        hi = time_max if time_max is not None else t[-1]
        m = (t >= lo) & (t <= hi)
        spec, t = spec[:, m], t[m]
    return np.ascontiguousarray(spec)


# ----------------------------------------------------------------------------------------------
# stages on a waterfall mag[F, T] (float32 or float64)
# ----------------------------------------------------------------------------------------------
def _strides(mag):
    it = mag.itemsize
    return mag.strides[0] // it, mag.strides[1] // it


def grid_bounds(F, T, sps, bpt):
    nb = T // sps
    return -10 * sps, nb * sps - sps * 59, F - 7 * bpt


def score_grid(mag: np.ndarray, sps: int, bpt: int) -> np.ndarray:
    """All ft8_sync_score values over the ft8_find_candidates grid, scan order [NT, NF]."""
    F, T = mag.shape
    t_lo, t_hi, f_hi = grid_bounds(F, T, sps, bpt)
    NT, NF = max(t_hi - t_lo, 0), max(f_hi, 0)
    out = np.empty((NT, NF), dtype=mag.dtype)
    if NT and NF:
        sf, st = _strides(mag)
        fn = lib().orc_score_grid_f64 if mag.dtype == np.float64 else lib().orc_score_grid_f32
        fn(_p(mag), sf, st, F, T, sps, bpt, _p(out))
    return out


def select(scores: np.ndarray, N: int, min_score, cmp_f64: bool = False):
    """ft8_find_candidates selection on a precomputed score grid -> (scan_idx, score, tie)."""
    flat = np.ascontiguousarray(scores.reshape(-1))
    n = max(int(N), 0)
    idx = np.zeros(max(n, 1), dtype=np.int64)
    sc = np.zeros(max(n, 1), dtype=np.float64)
    tie = ctypes.c_int(0)
    cnt = lib().orc_select(_p(flat), int(flat.dtype == np.float64), flat.size, n, float(min_score),
                           int(cmp_f64), _p(idx), _p(sc), ctypes.byref(tie))
    return idx[:cnt], sc[:cnt], bool(tie.value)


def find_candidates(mag: np.ndarray, sps: int, bpt: int, N: int, min_score, cmp_f64=False):
    """-> list of (abs_time, abs_freq, score) in the reference's final order, tie flag."""
    F, T = mag.shape
    t_lo, _, f_hi = grid_bounds(F, T, sps, bpt)
    sc = score_grid(mag, sps, bpt)
    if sc.size == 0:
        return [], False
    idx, s, tie = select(sc, N, min_score, cmp_f64)
    NF = sc.shape[1]
    return [(int(i // NF) + t_lo, int(i % NF), float(v)) for i, v in zip(idx, s)], tie


def llr(mag: np.ndarray, sps: int, bpt: int, abs_time: int, abs_freq: int, normalize=True):
    F, T = mag.shape
    out = np.zeros(174, dtype=np.float64)
    sf, st = _strides(mag)
    fn = lib().orc_llr_f64 if mag.dtype == np.float64 else lib().orc_llr_f32
    fn(_p(mag), sf, st, T // sps, sps, bpt, int(abs_time), int(abs_freq), _p(out))
    if normalize:
        with np.errstate(all="ignore"):
            lib().orc_normalize(_p(out))
    return out


def normalize(log174: np.ndarray) -> np.ndarray:
    x = np.array(log174, dtype=np.float64, copy=True)
    lib().orc_normalize(_p(x))
    return x


def pairwise_sum(a: np.ndarray) -> float:
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().orc_pairwise_sum(_p(a), a.size)


def bp_decode(llr174: np.ndarray, max_iterations: int):
    x = np.ascontiguousarray(llr174, dtype=np.float64)
    plain = np.zeros(174, dtype=np.uint8)
    err = lib().orc_bp_decode(_p(x), int(max_iterations), _p(plain))
    return plain, err


def ldpc_check(bits: np.ndarray) -> int:
    b = np.ascontiguousarray(bits, dtype=np.uint8)
    return lib().orc_ldpc_check(_p(b))


def crc14(data: bytes, num_bits: int) -> int:
    b = np.frombuffer(bytes(data) + b"\0\0", dtype=np.uint8).copy()
    return lib().orc_crc14(_p(b), int(num_bits))


def decode_tail(plain: np.ndarray, ldpc_errors: int):
    p = np.ascontiguousarray(plain, dtype=np.uint8)
    pay = np.zeros(10, dtype=np.uint8)
    ce, cc = ctypes.c_int(0), ctypes.c_int(0)
    ok = lib().orc_decode_tail(_p(p), int(ldpc_errors), _p(pay), ctypes.byref(ce), ctypes.byref(cc))
    return bool(ok), bytes(pay), ce.value, cc.value


def ldpc_encode(a91: bytes) -> bytes:
    a = np.frombuffer(bytes(a91), dtype=np.uint8).copy()
    out = np.zeros(22, dtype=np.uint8)
    lib().orc_ldpc_encode(_p(a), _p(out))
    return bytes(out)


REC_DTYPE = np.dtype([("score", "<f8"), ("abs_time", "<i4"), ("abs_freq", "<i4"),
                      ("ldpc_errors", "<i4"), ("crc_extracted", "<i4"), ("crc_calculated", "<i4"),
                      ("ok", "<i4"), ("payload", "u1", 10), ("_pad", "u1", 6)])


def decode_waterfall(mag: np.ndarray, sps: int, bpt: int, N: int, min_score, max_iterations: int,
                     cmp_f64: bool = False):
    """Candidates + decode of every candidate (records in candidate order), tie flag."""
    F, T = mag.shape
    rec = np.zeros(max(int(N), 1), dtype=REC_DTYPE)
    tie = ctypes.c_int(0)
    sf, st = _strides(mag)
    fn = lib().orc_decode_waterfall_f64 if mag.dtype == np.float64 else lib().orc_decode_waterfall_f32
    with np.errstate(all="ignore"):
        n = fn(_p(mag), sf, st, F, T, sps, bpt, max(int(N), 0), float(min_score), int(cmp_f64),
               int(max_iterations), _p(rec), ctypes.byref(tie))
    return rec[:n], bool(tie.value)


def decode_ft8_message(wave_data, sample_rate, bins_per_tone=2, steps_per_symbol=2,
                       max_candidates=20, min_score=10, max_iterations=20, freq_min=None,
                       freq_max=None, time_min=None, time_max=None):
    """-> list of (payload bytes, hash, ldpc_errors, crc_ext, crc_calc, time_sec, freq_hz, score)
    following decode_ft8_message (ft8_decode.py:288-394) minus the matplotlib side effect."""
    mag = waterfall(wave_data, sample_rate, bins_per_tone, steps_per_symbol, freq_min, freq_max,
                    time_min, time_max)
    if mag is None or mag.size == 0:
        return []
    cmp_f64 = isinstance(min_score, np.floating) and np.dtype(type(min_score)) == np.float64
    rec, _ = decode_waterfall(mag, steps_per_symbol, bins_per_tone, max_candidates, min_score,
                              max_iterations, cmp_f64=cmp_f64)
    out = []
    for r in rec:
        if not r["ok"]:
            continue
        score = np.float64(r["score"]) if mag.dtype == np.float64 else np.float32(r["score"])
        out.append((bytes(r["payload"]), int(r["crc_calculated"]), int(r["ldpc_errors"]),
                    int(r["crc_extracted"]), int(r["crc_calculated"]),
                    int(r["abs_time"]) / sample_rate,
                    (int(r["abs_freq"]) / bins_per_tone) * 6.25, score))
    return out


# ---- transmit chain (reference src/ft8_tools/ft8_generator) -----------------------------------
# Plain NumPy restatements; the GFSK sequence follows modulator.py's loops term by term.
_COSTAS = np.array([3, 1, 4, 0, 6, 5, 2], dtype=np.uint8)   # encoder.py:11
_GRAY = np.array([0, 1, 3, 2, 5, 6, 4, 7], dtype=np.uint8)  # encoder.py:10


def crc_generator(payload10: bytes) -> bytes:
    """crc.py:25-47: a91 = payload (77 bits) | CRC-14 over 82 bits."""
    a = bytearray(12)
    a[:10] = bytes(payload10)[:10]
    a[9] &= 0xF8
    c = crc14(bytes(a), 82)
    a[9] |= c >> 11
    a[10] = (c >> 3) & 0xFF
    a[11] = (c << 5) & 0xE0
    return bytes(a)


def tx_itones(payload10: bytes) -> np.ndarray:
    """encoder.py:15-73 (ft8_encode): payload -> 79 tones."""
    cw = ldpc_encode(crc_generator(payload10))
    bits = np.unpackbits(np.frombuffer(cw, dtype=np.uint8))[:174]
    sym = _GRAY[(bits[0::3] << 2) | (bits[1::3] << 1) | bits[2::3]]
    return np.concatenate([_COSTAS, sym[:29], _COSTAS, sym[29:], _COSTAS]).astype(np.uint8)


def gauss_window(bt: float, t: np.ndarray) -> np.ndarray:
    """modulator.py:20-25."""
    from scipy.special import erf
    k = np.pi * np.sqrt(2 / np.log(2))
    return 0.5 * (erf(k * bt * (t + 0.5)) - erf(k * bt * (t - 0.5)))


def gfsk_freq_seq(itones: np.ndarray, fs: float) -> np.ndarray:
    """modulator.py:27-50 gfsk_modulation_waveform_generator (same accumulation order)."""
    nsps = int(0.16 * fs)
    t = (np.arange(3 * nsps) - 1.5 * nsps) / nsps
    w = gauss_window(2.0, t)
    nsym = len(itones)
    f = np.zeros((nsym + 2) * nsps, dtype=np.float64)
    for i in range(nsym):
        f[i * nsps:i * nsps + 3 * nsps] += 6.25 * float(itones[i]) * w
    f[:2 * nsps] += 6.25 * float(itones[0]) * w[nsps:3 * nsps]
    f[nsym * nsps:nsym * nsps + 2 * nsps] += 6.25 * float(itones[nsym - 1]) * w[:2 * nsps]
    return f


def gfsk_waveform(itones: np.ndarray, fs: float, f0: float, style: int = 1) -> np.ndarray:
    """Complex baseband sin(phi) - j cos(phi) with ramps (modulator.py:52-74).  style 1: the
    reference (freq_seq read from index 0, its trailing ramp); style 0: protocol timing (symbol i
    at [i nsps, (i+1) nsps), freq_seq read one symbol later) and a falling trailing ramp."""
    nsps = int(0.16 * fs)
    nsym = len(itones)
    L = nsym * nsps
    f = gfsk_freq_seq(itones, fs)
    off = 0 if style == 1 else nsps
    import math
    dphi = (2 * np.pi * f / fs + 2 * np.pi * f0 / fs)[off:off + L].tolist()
    phi = np.empty(L, dtype=np.float64)
    ph, two_pi = 0.0, 2 * np.pi
    for i in range(L):  # modulator.py:64-68, sequential fmod
        phi[i] = ph
        ph = math.fmod(ph + dphi[i], two_pi)
    y = np.sin(phi) - 1j * np.cos(phi)
    nramp = nsps // 8
    i = np.arange(nramp)
    y[:nramp] *= 0.5 * (1 - np.cos(8 * np.pi * i / nsps))
    tail = 0.5 * (1 + np.cos(8 * np.pi * i / nsps)) if style == 1 else 0.5 * (1 - np.cos(8 * np.pi * i / nsps))
    y[L - 1 - i] *= tail
    return y


# ---- FT8_FLAG_TOPK selection (build-defined) --------------------------------------------------
def select_topk(scores: np.ndarray, N: int, min_score, cmp_f64: bool = False):
    """The N highest passing scores (ties in scan order), sorted by score descending.  Passing is
    ft8_find_candidates' test (ft8_decode.py:127): not -inf and score >= min_score, compared in the
    score dtype unless cmp_f64.  -> (scan_idx, score)."""
    flat = np.ascontiguousarray(scores.reshape(-1))
    if cmp_f64 or flat.dtype == np.float64:
        vals, thr = flat.astype(np.float64), np.float64(min_score)
    else:
        vals, thr = flat, flat.dtype.type(min_score)
    with np.errstate(invalid="ignore"):
        ok = ~np.isnan(vals) & ~np.isneginf(vals) & (vals >= thr)
    idx = np.nonzero(ok)[0]
    order = np.lexsort((idx, -flat[idx].astype(np.float64)))
    idx = idx[order][:max(int(N), 0)]
    return idx, flat[idx].astype(np.float64)
