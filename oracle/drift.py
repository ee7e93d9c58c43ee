"""oracle/drift.py -- TEST INFRASTRUCTURE ONLY (parity checker for the drift-correction row).

NumPy restatement of the beacon receiver's frequency-drift correction
(reference src/ft8_tools/ft8_beacon_receiver/frequency_correction.py), SURVEY.md §8(f) item 4.
Only tests/, tools/make_golden_drift.py and bench.py's CPU leg import this module; the product
package ft8_demodulator_amd never does.

The reference depends on scikit-learn (LinearRegression, PolynomialFeatures) and matplotlib
(debug plots written to the CWD).  The restatement keeps the arithmetic and drops the plots:
  * LinearRegression(fit_intercept=True).fit(X, y) centres X and y and solves the centred
    least-squares problem (scipy.linalg.lstsq, gelsd); restated with np.linalg.lstsq (gelsd) on the
    same centred matrices; predict(X) = X @ coef + intercept.
  * PolynomialFeatures(degree=d) on one column: [1, x, x^2, ..., x^d].
Pinned against the reference's own outputs by tests/golden/drift.{json,npz}
(tools/make_golden_drift.py imports the reference in the build container), checked by
tests/test_drift_oracle.py.

Also holds the fixture-input synthesis shared by the golden script and the tests: a complex FT8
beacon (the oracle's pinned GFSK generator, reference timing) mixed to fc, zero-padded on both
sides, given a linear drift and complex white noise at Es/N0 exactly as the reference test builds
its input (src/tests/test_correction/test_correction.py:190-260), but from a seeded generator.
"""
from __future__ import annotations

import numpy as np

from . import oracle as O

DEFAULT_PARAMS = {  # frequency_correction.py:150-163
    "nsync_sym": 7,
    "ndata_sym": 58,
    "zscore_threshold": 5,
    "max_iteration_num": 400,
    "debug_plots": True,
    "window_size_factor": 4,
    "max_variance_factor": 0.0001,
    "fit_middle_percent": 100,
    "bins_per_tone": 2,
    "steps_per_symbol": 2,
    "poly_degree": 2,
    "precise_sync": True,
}


def gfsk_pulse(bt, t):
    """frequency_correction.py:27-40."""
    from scipy.special import erf
    k = np.pi * np.sqrt(2.0 / np.log(2.0))
    return 0.5 * (erf(k * bt * (t + 0.5)) - erf(k * bt * (t - 0.5)))


def _ols(X, y):
    """LinearRegression(fit_intercept=True).fit(X, y) -> (coef, intercept)."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    xo = X.mean(axis=0)
    yo = y.mean()
    coef = np.linalg.lstsq(X - xo, y - yo, rcond=None)[0]
    return coef, yo - xo @ coef


def _poly(x, d):
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    return np.stack([x ** k for k in range(d + 1)], axis=1)


def continuity_metric(max_freq_indices, window_size):
    """The per-window residual variance loop of detect_signal_continuity (:58-80), -variance."""
    m = np.asarray(max_freq_indices)
    n = len(m) - window_size + 1
    out = np.zeros(max(n, 0))
    x = np.arange(window_size).reshape(-1, 1)
    for i in range(n):
        w = m[i:i + window_size]
        coef, b = _ols(x, w)
        res = w - (x @ coef + b)
        out[i] = -np.var(res)
    return out


def detect_signal_continuity(max_freq_indices, window_size=8, max_variance=10.0):
    """frequency_correction.py:42-115 (without the PNG)."""
    if len(max_freq_indices) < window_size:
        return [], np.zeros(len(max_freq_indices))
    metric = continuity_metric(max_freq_indices, window_size)
    segments = []
    is_signal = metric > -max_variance
    in_seg, start = False, 0
    for i in range(len(is_signal)):
        if is_signal[i] and not in_seg:
            in_seg, start = True, i
        elif not is_signal[i] and in_seg:
            in_seg = False
            if i - start >= 1:
                segments.append((start, i))
    if in_seg:
        segments.append((start, len(max_freq_indices) - 1))
    return segments, metric


def column_argmax(wave, fs, bpt, sps):
    """calculate_spectrogram -> f >= 0 -> np.argmax per column (:186-221)."""
    spec, f, _ = O.calculate_spectrogram(wave, fs, bpt, sps)
    spec = spec[f >= 0]
    return np.argmax(spec, axis=0), spec.shape[0]


def sync_template(time_osr, nsync_sym=7, ndata_sym=58):
    """three_sync_correlation_seq (:380-405)."""
    sync_seq = np.array([3, 1, 4, 0, 6, 5, 2]) + 1
    sync_seq = sync_seq - np.mean(sync_seq)
    sps2 = time_osr * 2
    shape = gfsk_pulse(2.0, np.linspace(-1, 1, sps2 + 1))
    one = np.zeros((nsync_sym - 1) * time_osr + sps2 + 1)
    for k in range(nsync_sym):
        one[k * time_osr:k * time_osr + sps2 + 1] += shape * sync_seq[k]
    three = np.zeros((3 * nsync_sym + ndata_sym - 1) * time_osr + 1 + sps2)
    for i in range(3):
        s = i * (nsync_sym + ndata_sym // 2) * time_osr
        three[s:s + len(one)] = one
    return three


def correct_frequency_drift(wave_complex, fs, sym_bin, sym_t, params=None, trace=None):
    """frequency_correction.py:118-659 -> (corrected complex wave, drift rate in Hz per sample).
    `trace` (a dict) receives the intermediate values the GPU path is checked against."""
    p = dict(DEFAULT_PARAMS)
    if params:
        p.update(params)
    tr = trace if trace is not None else {}
    bpt, sps = p["bins_per_tone"], p["steps_per_symbol"]
    nsync, ndata = p["nsync_sym"], p["ndata_sym"]
    window = p["window_size_factor"] * sps
    x = np.asarray(wave_complex)
    n = len(x)
    idx, F = column_argmax(x, fs, bpt, sps)
    time_osr, freq_osr = sps, bpt
    max_variance = p["max_variance_factor"] * (F ** 2)
    segs, metric = detect_signal_continuity(idx, window_size=window, max_variance=max_variance)
    tr.update(argmax1=idx, metric=metric, segments=segs, status=0)
    if not segs:
        tr["status"] = 1
        return x, 0.0
    start, end = max(segs, key=lambda s: s[1] - s[0])
    freq_step = sym_bin / freq_osr
    max_freqs = idx * freq_step
    time_step = sym_t / time_osr
    time_axis = np.arange(len(max_freqs)) * time_step
    seg_t = time_axis[start:end].reshape(-1, 1)
    seg_f = max_freqs[start:end]
    fm = p["fit_middle_percent"]
    if fm < 100:
        trim = int(len(seg_t) * ((100 - fm) / 2 / 100))
        if trim > 0 and 2 * trim < len(seg_t):
            seg_t, seg_f = seg_t[trim:len(seg_t) - trim], seg_f[trim:len(seg_f) - trim]
    coef, _ = _ols(_poly(seg_t, 1), seg_f)
    rate = coef[1] if len(coef) > 1 else 0
    tr["rate1"] = float(rate)
    ar = np.arange(n)
    c1 = np.exp(-2j * np.pi * (rate * ar ** 2 / 2 / fs) / (fs))
    lin = x * c1
    if not p["precise_sync"]:
        tr["status"] = 2
        return lin, rate / fs
    idx2, _ = column_argmax(lin, fs, bpt, sps)
    f2 = idx2 * freq_step
    three = sync_template(time_osr, nsync, ndata)
    sps2 = time_osr * 2
    start, end = max(segs, key=lambda s: s[1] - s[0])
    end = end + window - 2
    masked = np.zeros_like(f2)
    masked[start:end] = f2[start:end]
    masked[start:end] = masked[start:end] - np.mean(masked[start:end])
    corr = np.correlate(masked, three, mode="full")
    peak = int(np.argmax(corr))
    sync_idx = peak - (len(three) - 1) + sps2 // 2
    tr.update(argmax2=idx2, corr=corr, sync_idx=sync_idx)
    rx, ry = np.array([]), np.array([])
    for i in range(3):
        s = i * (nsync + ndata // 2) * time_osr + sync_idx
        e = s + (nsync - 1) * time_osr
        if s < len(masked):
            xs = sym_t / time_osr
            rx = np.append(rx, np.arange(s, min(e, len(masked))) * xs)
            ry = np.append(ry, masked[s:min(e, len(masked))])
    if len(rx) < 10:
        tr["status"] = 3
        return lin, rate / fs
    deg = p["poly_degree"]
    if len(rx) > deg + 1:
        if len(rx) != len(ry):
            raise ValueError("regression x/y length mismatch (the reference's LinearRegression raises here)")
        X = _poly(rx, deg)
        coef2, b2 = _ols(X, ry)
        r2 = coef2[1] if len(coef2) > 1 else 0.0
        a2 = coef2[2] if len(coef2) > 2 else 0.0
        tr.update(coef2=np.asarray(coef2, dtype=np.float64), intercept2=float(b2))
        if deg == 1:
            c2 = np.exp(-2j * np.pi * r2 * ar ** 2 / (2 * fs ** 2))
        elif deg == 2:
            t = ar / fs
            ph = r2 * t ** 2 / 2 + a2 * t ** 3 / 3
            c2 = np.exp(-2j * np.pi * ph)
        else:
            tr["status"] = 4
            return lin, rate / fs
        out = lin * c2
        first = (_poly(rx[:1], deg) @ coef2 + b2)[0]
        last = (_poly(rx[-1:], deg) @ coef2 + b2)[0]
        real = (first - last) / (rx[0] - rx[-1]) + rate
        tr["status"] = 5
        return out, real / fs
    tr["status"] = 6
    return lin, rate / fs


# ---- fixture inputs (shared by tools/make_golden_drift.py and tests) --------------------------
def beacon_input(payload_hex, fs, f0, fc, drift_hz_per_s, esn0_db, seed, pad=1):
    """Complex beacon: baseband (reference GFSK timing) * exp(i 2 pi fc n / fs), `pad` zero-signal
    lengths on both sides, drift carrier exp(i 2 pi k n^2 / (2 fs^2)), complex noise at Es/N0
    (test_correction.py:190-260)."""
    pay = bytes.fromhex(payload_hex)
    bb = O.gfsk_waveform(O.tx_itones(pay), fs, f0, style=1)
    bb = bb * np.exp(1j * 2 * np.pi * fc * np.arange(len(bb)) / fs)
    z = np.zeros(pad * len(bb), dtype=complex)
    w = np.concatenate((z, bb, z))
    n = len(w)
    k = drift_hz_per_s / fs
    t = np.arange(n)
    w = w * np.exp(2j * np.pi * k * t ** 2 / (2 * fs))
    rng = np.random.default_rng(seed)
    if esn0_db is not None:
        es = np.sum(np.abs(w) ** 2) / n
        sd = np.sqrt(es / 10 ** (esn0_db / 10) * fs / 2)
        w = w + (rng.normal(0, sd, n) + 1j * rng.normal(0, sd, n))
    return w
