"""oracle/subtract.py -- TEST INFRASTRUCTURE ONLY: CPU restatement of the build-defined
subtract-and-redecode second pass (FT8_FLAG_SUBTRACT; csrc/subtract.hip k_sub_est / k_sub_apply).

The reference has no second pass (its decode_ft8_message is one pass, ft8_decode.py:288-394), so
this restates the BUILD's algorithm, in float64 NumPy, from the reference's own building blocks:
the encoder (encoder.py:15-73, via oracle.tx_itones) and the GFSK pulse / phase accumulation of the
modulator (modulator.py:20-90) with the protocol timing.  It pins the device's float32 fit within
stated tolerances (tests/test_gpu_subtract_oracle.py), not bit for bit: "parity unpinned" against
the reference, pinned against this restatement.

Per decoded record (ok, payload not seen earlier in the slot):
  1. tones = encode(payload);
  2. z[m] = sum of x[nb + m D + i] exp(-2 pi i fmix n / fs), i < D = nsps / Q: the slot mixed down to
     the centre of the 8-tone band and box-car decimated to Q samples per symbol, around the
     candidate's start s0 = (t_lo + abs_time) hop (tone 0 at ftone = (f_lo + abs_freq) fs / nfft);
  3. metric(dt, df) = sum_k |sum_q z[. + k Q + dt + q] w_k^q|^2 over start offsets dt in [-Mt, Mt]
     (units of D samples) and tone-0 offsets df in [-2, 2] (units of bin / 4): the known tone of
     symbol k coherent within the symbol, power summed over symbols; best point (first maximum),
     refined by a parabola through its neighbours in each direction (clipped to +-0.5);
  4. A_k = 2 sum x r exp(-2 pi i phase) / sum r^2 per symbol against the refined GFSK waveform
     (r the ramp), smoothed [1 2 1] / 4 (ends [2 1] / 3, [1 2] / 3).
Residual = x - sum of r(n) Re(A(n) exp(2 pi i phase(n))), A interpolated linearly between symbol
centres, signals in record order.
"""
from __future__ import annotations

import math

import numpy as np

from . import oracle as O

SYM = 79
KMF = 2  # tone-0 search: 2 KMF + 1 points over +-bin / 2


def sub_q(nsps: int) -> int:
    """Decimated samples per symbol: 32 when nsps allows, else the largest divisor in [8, 32]."""
    for q in range(32, 7, -1):
        if nsps % q == 0:
            return q
    return 0


def pulse_table(nsps: int) -> np.ndarray:
    """Cumulative GFSK frequency pulse P[0 .. 3 nsps] (modulator.py:20-25, 33-34, BT = 2)."""
    from scipy.special import erf
    k = math.pi * math.sqrt(2.0 / math.log(2.0))
    t = (np.arange(3 * nsps, dtype=np.float64) - 1.5 * nsps) / nsps
    w = 0.5 * (erf(k * 2.0 * (t + 0.5)) - erf(k * 2.0 * (t - 0.5)))
    P = np.zeros(3 * nsps + 1)
    P[1:] = np.cumsum(w)
    return P


def _ext_tones(tones):
    """e_{-1} .. e_79 (the first and last tone repeated) and their prefix sums."""
    e = np.asarray(tones, dtype=np.int64)[np.clip(np.arange(SYM + 2) - 1, 0, SYM - 1)]
    return e, np.concatenate([[0], np.cumsum(e)])


def _G(E, PS, P, nsps, u):
    """Integrated frequency pulse train G(u) = sum_j e_j P(u - j nsps) (tx_device.h gfsk_G)."""
    q, r = divmod(u, nsps)
    full = min(max(q - 1, 0), SYM + 2)
    s = PS[full] * P[3 * nsps]
    if 0 <= q - 1 < SYM + 2:
        s += E[q - 1] * P[r + 2 * nsps]
    if q < SYM + 2:
        s += E[q] * P[r + nsps]
    if q + 1 < SYM + 2:
        s += E[q + 1] * P[r]
    return s


def _ramp(n, L, nsps):
    """Protocol-timing amplitude ramp (modulator.py:70-73, falling tail) of sample n (array)."""
    nramp = nsps // 8
    r = np.ones(n.shape)
    a = n < nramp
    r[a] = 0.5 * (1 - np.cos(8 * np.pi * n[a] / nsps))
    i = L - 1 - n
    b = i < nramp
    r[b] = 0.5 * (1 - np.cos(8 * np.pi * i[b] / nsps))
    return r


def _phase(E, PS, P, nsps, f0, fs, start_phase, k, i):
    """Phase in cycles of sample i of symbol k: phase0[k] + i f0 / fs + 6.25 / fs * dG(k, i)."""
    dG = (E[k] * (P[i + 2 * nsps] - P[2 * nsps]) + E[k + 1] * (P[i + nsps] - P[nsps]) + E[k + 2] * (P[i] - P[0]))
    return start_phase[k] + i * (f0 / fs) + (6.25 / fs) * dG


def fit_record(x, rec, fs, nsps, hop, nfft, t_lo, f_lo, P=None):
    """The fit of one record -> dict(start, f0, amp [79] complex, phase0 [80], tones)."""
    Q = sub_q(nsps)
    D, L = nsps // Q, SYM * nsps
    n_samples = len(x)
    tones = O.tx_itones(bytes(rec["payload"]))
    E, PS = _ext_tones(tones)
    if P is None:
        P = pulse_table(nsps)
    Mt = (Q + 2 * (nsps // hop) - 1) // (2 * (nsps // hop))
    Mg = Mt + 1
    Mz = SYM * Q + 2 * Mg
    s0 = (t_lo + int(rec["abs_time"])) * hop
    ftone = (f_lo + int(rec["abs_freq"])) * fs / nfft
    fmix = ftone + 3.5 * 6.25
    # 2. decimated baseband
    nb = s0 - Mg * D
    n = nb + np.arange(Mz * D)
    xv = np.where((n >= 0) & (n < n_samples), x[np.clip(n, 0, n_samples - 1)].astype(np.float64), 0.0)
    z = (xv * np.exp(-2j * np.pi * fmix * n / fs)).reshape(Mz, D).sum(axis=1)
    # 3. hypotheses
    binw = fs / nfft
    fstep = 0.5 * binw / KMF
    nT, nF = 2 * Mt + 1, 2 * KMF + 1
    metric = np.zeros((nT, nF))
    q = np.arange(Q)
    for f in range(nF):
        nu = np.asarray(tones, dtype=np.float64) * 6.25 + (f - KMF) * fstep - 3.5 * 6.25
        w = np.exp(-2j * np.pi * nu * D / fs)                   # per symbol
        wq = w[:, None] ** q[None, :]                           # [79, Q]
        for d in range(nT):
            seg = z[Mg - Mt + d + np.arange(SYM)[:, None] * Q + q[None, :]]
            metric[d, f] = np.sum(np.abs(np.sum(seg * wq, axis=1)) ** 2)
    flat = metric.reshape(-1)
    hb = int(np.argmax(flat))                                   # first maximum, scan order (dt, df)
    dtb, dfb = hb // nF - Mt, hb % nF - KMF

    def parab(m_, m0, mp):
        den = m_ - 2 * m0 + mp
        if not den < 0:
            return 0.0
        return min(0.5, max(-0.5, 0.5 * (m_ - mp) / den))

    ddt = parab(flat[hb - nF], flat[hb], flat[hb + nF]) if -Mt < dtb < Mt else 0.0
    ddf = parab(flat[hb - 1], flat[hb], flat[hb + 1]) if -KMF < dfb < KMF else 0.0
    start = s0 + int(np.rint((dtb + ddt) * D))
    f0 = ftone + (dfb + ddf) * fstep
    # phases at symbol starts (protocol timing)
    G0 = _G(E, PS, P, nsps, nsps)
    ph0 = np.array([(f0 * k * nsps + 6.25 * (_G(E, PS, P, nsps, (k + 1) * nsps) - G0)) / fs for k in range(SYM + 1)])
    ph0 -= np.floor(ph0)
    # 4. amplitude per symbol
    A = np.zeros(SYM, dtype=np.complex128)
    i = np.arange(nsps)
    for k in range(SYM):
        ns = start + k * nsps + i
        ok = (ns >= 0) & (ns < n_samples)
        if not ok.any():
            continue
        r = _ramp(k * nsps + i, L, nsps)[ok]
        cyc = _phase(E, PS, P, nsps, f0, fs, ph0, k, i[ok])
        v = x[ns[ok]].astype(np.float64) * r
        rr = np.sum(r * r)
        if rr > 0:
            A[k] = 2.0 * np.sum(v * np.exp(-2j * np.pi * cyc)) / rr
    S = np.empty_like(A)
    S[0] = (2 * A[0] + A[1]) / 3
    S[-1] = (A[-2] + 2 * A[-1]) / 3
    S[1:-1] = 0.25 * (A[:-2] + 2 * A[1:-1] + A[2:])
    return {"start": start, "f0": f0, "amp": S, "phase0": ph0, "tones": tones, "dt": dtb, "df": dfb,
            "metric": metric}


def fits(x, records, fs, nsps, hop, nfft, t_lo, f_lo):
    """Fits of a slot's records in record order; None for a failed record or a repeated payload."""
    P = pulse_table(nsps)
    seen, out = set(), []
    for r in records:
        pay = bytes(r["payload"])
        if not r["ok"] or pay in seen:
            out.append(None)
            continue
        seen.add(pay)
        out.append(fit_record(x, r, fs, nsps, hop, nfft, t_lo, f_lo, P))
    return out


def waveform(fit, nsps, fs, n_samples, P=None):
    """(sample indices, fitted signal) of one fit: r(n) Re(A(n) exp(2 pi i phase(n)))."""
    if P is None:
        P = pulse_table(nsps)
    L = SYM * nsps
    E, PS = _ext_tones(fit["tones"])
    nr = np.arange(L)
    n = fit["start"] + nr
    ok = (n >= 0) & (n < n_samples)
    nr = nr[ok]
    k, i = nr // nsps, nr % nsps
    cyc = _phase(E, PS, P, nsps, fit["f0"], fs, fit["phase0"], k, i)
    t = (i + 0.5) / nsps - 0.5
    A = fit["amp"]
    prev = A[np.maximum(k - 1, 0)]
    nxt = A[np.minimum(k + 1, SYM - 1)]
    Ak = A[k]
    Ai = np.where(t < 0, Ak + t * (Ak - prev), Ak + t * (nxt - Ak))
    return n[ok], _ramp(nr, L, nsps) * np.real(Ai * np.exp(2j * np.pi * cyc))


def residual(x, fit_list, nsps, fs):
    """x - sum of the fitted signals, in record order (float64)."""
    P = pulse_table(nsps)
    acc = np.zeros(len(x))
    for f in fit_list:
        if f is None:
            continue
        n, s = waveform(f, nsps, fs, len(x), P)
        acc[n] += s
    return x.astype(np.float64) - acc


def decode_topk(x, fs, N, min_score, max_iterations, bpt=2, sps=2):
    """FT8_FLAG_TOPK decode (build-defined selection): the N best passing candidates, decoded by the
    oracle's LLR / BP / CRC -> list of (payload bytes, abs_time, abs_freq) of the successes."""
    mag = O.waterfall(np.asarray(x, dtype=np.float32), fs, bpt, sps)
    F, T = mag.shape
    t_lo, _, _ = O.grid_bounds(F, T, sps, bpt)
    sc = O.score_grid(mag, sps, bpt)
    idx, _ = O.select_topk(sc, N, min_score)
    NF = sc.shape[1]
    out = []
    for i in idx:
        at, af = int(i // NF) + t_lo, int(i % NF)
        plain, err = O.bp_decode(O.llr(mag, sps, bpt, at, af), max_iterations)
        ok, pay, _, _ = O.decode_tail(plain, err)
        if ok:
            out.append((pay, at, af))
    return out
