"""Synthetic FT8 slots for tests and the benchmark (transmit side; not on the decode path).

The reference's transmitter (src/ft8_tools/ft8_generator, crc.py:25-47, ldpc.py:104-131,
encoder.py:15-73, modulator.py:27-90) is out of scope for the build and too slow for batch
synthesis (1.1 s per signal).  This module restates the FT8 transmit chain vectorised in
PyTorch so that 256-slot crowded batches can be synthesised on the GPU in well under a second:

  payload(77 bits) -> CRC-14 -> LDPC(174,91) encode -> Gray map -> 79 tones (Costas at 0/36/72)
  -> GFSK (BT = 2, Gaussian-smoothed frequency pulse, phase continuous) -> raised-cosine ramps

Unlike the reference modulator (modulator.py:66-68 indexes dphi without the +1-symbol offset,
so every reference signal starts one symbol late), the phase here follows the FT8 definition:
symbol i occupies samples [start + i*nsps, start + (i+1)*nsps).

SNR convention is the reference's own (test_ft8_standard.py:51-54): power over white noise in
the full sampled band.  With unit-variance noise a signal at S dB has power 10^(S/10).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from . import _ldpc_tables as T

COSTAS = (3, 1, 4, 0, 6, 5, 2)
GRAY = (0, 1, 3, 2, 5, 6, 4, 7)
_GEN = np.array(T.GEN_ROWS, dtype=np.uint8).reshape(83, 12)


def crc14(data: bytes, num_bits: int) -> int:
    """CRC-14, polynomial 0x2757, MSB first (protocol definition; reference crc.py:11-39)."""
    rem, ib = 0, 0
    for i in range(num_bits):
        if i % 8 == 0:
            rem ^= data[ib] << 6
            ib += 1
        rem = ((rem << 1) ^ 0x2757) if rem & 0x2000 else (rem << 1)
    return rem & 0x3FFF


def add_crc(payload: bytes) -> bytes:
    """77-bit payload (10 bytes) -> a91 (12 bytes): payload | 14-bit CRC over 82 bits."""
    a = bytearray(12)
    a[:10] = payload[:10]
    a[9] &= 0xF8
    c = crc14(bytes(a), 82)
    a[9] |= c >> 11
    a[10] = (c >> 3) & 0xFF
    a[11] = (c << 5) & 0xE0
    return bytes(a)


def ldpc_encode(a91: bytes) -> bytes:
    """a91 -> 174-bit codeword (22 bytes): message bits then 83 parity bits."""
    msg = np.frombuffer(a91, dtype=np.uint8)
    par = np.bitwise_and(_GEN, msg[None, :])
    bits = np.unpackbits(par, axis=1).sum(axis=1) & 1
    cw = bytearray(22)
    cw[:12] = a91
    cw[11] &= 0xE0
    for i, b in enumerate(bits):
        if b:
            k = 91 + i
            cw[k // 8] |= 0x80 >> (k % 8)
    return bytes(cw)


def codeword_bits(payload: bytes) -> np.ndarray:
    cw = ldpc_encode(add_crc(payload))
    return np.unpackbits(np.frombuffer(cw, dtype=np.uint8))[:174]


def itones(payload: bytes) -> np.ndarray:
    """79 channel symbols for a 10-byte payload (reference encoder.py:15-73)."""
    bits = codeword_bits(payload)
    data = [GRAY[(bits[3 * k] << 2) | (bits[3 * k + 1] << 1) | bits[3 * k + 2]] for k in range(58)]
    return np.array(list(COSTAS) + data[:29] + list(COSTAS) + data[29:] + list(COSTAS), dtype=np.uint8)


def random_payload(rng: np.random.Generator) -> bytes:
    p = bytearray(rng.integers(0, 256, size=10, dtype=np.uint8).tobytes())
    p[9] &= 0xF8
    return bytes(p)


def random_payloads(n: int, rng: np.random.Generator) -> np.ndarray:
    """[n, 10] uint8 payloads (77 bits, [9] & 0xF8)."""
    p = rng.integers(0, 256, size=(n, 10), dtype=np.uint8)
    p[:, 9] &= 0xF8
    return p


def codeword_bits_batch(payloads: np.ndarray) -> np.ndarray:
    """[n, 10] payloads -> [n, 174] codeword bits (vectorised add_crc + ldpc_encode)."""
    pay = np.asarray(payloads, dtype=np.uint8).reshape(-1, 10)
    n = pay.shape[0]
    a = np.zeros((n, 12), dtype=np.uint8)
    a[:, :10] = pay
    a[:, 9] &= 0xF8
    bits82 = np.unpackbits(a, axis=1)[:, :82].astype(np.int32)
    rem = np.zeros(n, dtype=np.int32)
    for i in range(82):  # bitwise CRC-14 (poly 0x2757), MSB first
        rem ^= bits82[:, i] << 13
        top = (rem & 0x2000) != 0
        rem = np.where(top, (rem << 1) ^ 0x2757, rem << 1) & 0x3FFF
    a[:, 9] |= (rem >> 11).astype(np.uint8)
    a[:, 10] = ((rem >> 3) & 0xFF).astype(np.uint8)
    a[:, 11] = ((rem << 5) & 0xE0).astype(np.uint8)
    msg = np.unpackbits(a, axis=1)[:, :91].astype(np.int32)
    gen = np.unpackbits(_GEN, axis=1)[:, :91].astype(np.int32)   # [83, 91]
    parity = (msg @ gen.T) & 1
    return np.concatenate([msg, parity], axis=1).astype(np.uint8)


def bp_stress_llrs(n: int, sigma: float = 0.85, mu: float = 1.0, seed: int = 7):
    """BASELINE config 4 input: LLRs (2b - 1) mu + sigma N(0, 1) from the
    codewords of n random payloads (float64 [n, 174], NOT yet normalised) and the bits.  At
    sigma = 0.85 about half of the vectors fail to converge in 50 iterations after
    ftx_normalize_logl (oracle: 47 % converge on 1000 vectors)."""
    rng = np.random.default_rng(seed)
    bits = codeword_bits_batch(random_payloads(n, rng))
    llr = (2.0 * bits - 1.0) * mu + sigma * rng.standard_normal(bits.shape)
    return llr, bits


def _pulse(nsps: int, bt: float = 2.0, device=None) -> torch.Tensor:
    k = math.pi * math.sqrt(2.0 / math.log(2.0))
    t = torch.arange(3 * nsps, dtype=torch.float64, device=device) / nsps - 1.5
    return 0.5 * (torch.special.erf(k * bt * (t + 0.5)) - torch.special.erf(k * bt * (t - 0.5)))


def gfsk_waveforms(tones: torch.Tensor, fs: int, f0: torch.Tensor) -> torch.Tensor:
    """tones [B, 79] (int), f0 [B] Hz -> real unit-amplitude waveforms [B, 79*nsps] float64."""
    B, nsym = tones.shape
    dev = tones.device
    nsps = int(0.16 * fs)
    seg = _pulse(nsps, device=dev).reshape(3, nsps)
    ext = torch.cat([tones[:, :1], tones, tones[:, -1:]], dim=1).to(torch.float64)  # index -1..nsym
    blocks = torch.zeros(B, nsym + 2, nsps, dtype=torch.float64, device=dev)
    for s in range(3):
        # block j gets ext[j - s] * seg[s]; ext position of symbol i is i + 1
        j = torch.arange(nsym + 2, device=dev)
        src = j - s + 1
        ok = (src >= 0) & (src < nsym + 2)
        coef = torch.zeros(B, nsym + 2, dtype=torch.float64, device=dev)
        coef[:, ok] = ext[:, src[ok]]
        blocks += coef[:, :, None] * seg[s][None, None, :]
    dphi_peak = 2.0 * math.pi * 6.25 / fs
    dphi = dphi_peak * blocks.reshape(B, -1) + (2.0 * math.pi / fs) * f0.to(torch.float64)[:, None]
    n = nsym * nsps
    steps = dphi[:, nsps:nsps + n - 1]
    phi = torch.cat([torch.zeros(B, 1, dtype=torch.float64, device=dev), torch.cumsum(steps, 1)], 1)
    sig = torch.sin(torch.remainder(phi, 2.0 * math.pi))
    nramp = nsps // 8
    i = torch.arange(nramp, dtype=torch.float64, device=dev)
    ramp = 0.5 * (1.0 - torch.cos(math.pi * i / nramp))
    sig[:, :nramp] *= ramp
    sig[:, n - nramp:] *= ramp.flip(0)
    return sig


@dataclass
class SlotTruth:
    payloads: list
    f0: list
    start_s: list
    snr_db: list


def make_slots(n_slots: int, n_signals: int, fs: int = 12000, snr_db=(-24.0, -10.0),
               f0_range=(200.0, 2800.0), start_range=(0.0, 2.0), seed: int = 0,
               device="cpu", slot_s: float = 15.0, noise: bool = True, seeds=None):
    """-> (samples float32 [n_slots, int(slot_s*fs)], list[SlotTruth]).

    Slot b uses np.random.default_rng(seeds[b] if seeds else seed + b) for its parameters and a
    torch generator with the same seed for its noise, so slots are reproducible individually.
    """
    N = int(slot_s * fs)
    if torch.device(device).type == "cuda":
        return _make_slots_gpu(n_slots, n_signals, fs, snr_db, f0_range, start_range, seed, device, N, noise, seeds)
    out = torch.empty(n_slots, N, dtype=torch.float32, device=device)
    truths = []
    nsps = int(0.16 * fs)
    for b in range(n_slots):
        sd = int(seeds[b]) if seeds is not None else seed + b
        rng = np.random.default_rng(sd)
        pays = [random_payload(rng) for _ in range(n_signals)]
        lo, hi = (snr_db, snr_db) if np.isscalar(snr_db) else snr_db
        snr = rng.uniform(lo, hi, n_signals) if n_signals else np.zeros(0)
        f0 = rng.uniform(*f0_range, n_signals) if n_signals else np.zeros(0)
        st = rng.uniform(*start_range, n_signals) if n_signals else np.zeros(0)
        g = torch.Generator(device=device)
        g.manual_seed(sd)
        acc = (torch.randn(N, generator=g, device=device, dtype=torch.float64) if noise
               else torch.zeros(N, dtype=torch.float64, device=device))
        if n_signals:
            tones = torch.as_tensor(np.stack([itones(p) for p in pays]), device=device)
            wav = gfsk_waveforms(tones, fs, torch.as_tensor(f0, device=device))
            amp = torch.as_tensor(np.sqrt(2.0 * 10.0 ** (snr / 10.0)), device=device)
            wav *= amp[:, None]
            n = 79 * nsps
            for i in range(n_signals):
                s0 = int(st[i] * fs)
                m = min(n, N - s0)
                acc[s0:s0 + m] += wav[i, :m]
        out[b] = acc.to(torch.float32)
        truths.append(SlotTruth(pays, list(f0), list(st), list(snr)))
    return out, truths


def _make_slots_gpu(n_slots, n_signals, fs, snr_db, f0_range, start_range, seed, device, N, noise, seeds):
    """make_slots on the GPU: the same per-slot parameter draws and noise, the waveforms from the
    HIP transmit chain (ft8_generator.encode_batch / synthesize, protocol timing) in one launch."""
    from . import _lib
    from . import ft8_generator as G
    acc = torch.empty(n_slots, N, dtype=torch.float64, device=device)
    truths, pays_all, sig_rows = [], [], []
    for b in range(n_slots):
        sd = int(seeds[b]) if seeds is not None else seed + b
        rng = np.random.default_rng(sd)
        pays = [random_payload(rng) for _ in range(n_signals)]
        lo, hi = (snr_db, snr_db) if np.isscalar(snr_db) else snr_db
        snr = rng.uniform(lo, hi, n_signals) if n_signals else np.zeros(0)
        f0 = rng.uniform(*f0_range, n_signals) if n_signals else np.zeros(0)
        st = rng.uniform(*start_range, n_signals) if n_signals else np.zeros(0)
        g = torch.Generator(device=device)
        g.manual_seed(sd)
        if noise:
            acc[b] = torch.randn(N, generator=g, device=device, dtype=torch.float64)
        else:
            acc[b].zero_()
        for i in range(n_signals):
            pays_all.append(pays[i])
            sig_rows.append((float(f0[i]), float(np.sqrt(2.0 * 10.0 ** (snr[i] / 10.0))), 0.0, int(st[i] * fs), b, 0))
        truths.append(SlotTruth(pays, list(f0), list(st), list(snr)))
    if sig_rows:
        sig = np.array(sig_rows, dtype=_lib.TX_SIGNAL_DTYPE)
        _, _, tones = G.encode_batch(np.frombuffer(b"".join(pays_all), dtype=np.uint8).reshape(-1, 10), device=device)
        G.synthesize(tones, sig, n_slots, N, fs, _lib.FT8_TX_PROTOCOL, out=acc, device=device)
    return acc.to(torch.float32), truths
