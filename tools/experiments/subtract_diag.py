"""Subtract-and-redecode diagnostics on the GPU (build-defined feature).

  1. clean-signal residual: one noiseless signal at off-grid time/frequency, residual energy in dB
     relative to the signal after decode + ft8_subtract;
  2. crowded batch (the benchmark generator: 50 signals/slot, SNR U(-24, -10) dB): unique true
     decodes per slot for reference selection, top-k selection, top-k + subtraction, and the
     per-stage time of the two-pass decode.

    python tools/subtract_diag.py [--slots 64] [--k 300]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def clean_residual(torch):
    from ft8_demodulator_amd import _lib
    from ft8_demodulator_amd import ft8_generator as G
    from ft8_demodulator_amd._pipeline import SlotDecoder, make_params
    fs, N = 12000, 180000
    out_db = []
    rng = np.random.default_rng(1)
    for trial in range(8):
        pay = rng.integers(0, 256, 10, dtype=np.uint8)
        pay[9] &= 0xF8
        _, _, tones = G.encode_batch(pay[None])
        sig = np.zeros(1, dtype=_lib.TX_SIGNAL_DTYPE)
        sig["f0"], sig["amplitude"] = rng.uniform(300, 2500), 1.0
        sig["phase"], sig["start"] = rng.uniform(0, 6.28), int(rng.uniform(0, 2) * fs)
        x = G.synthesize(tones, sig, 1, N, fs)
        dec = SlotDecoder(fs, 2, 2, max_candidates=20, min_score=2, flags=_lib.FT8_FLAG_TOPK)
        out, counts = dec.run(x)
        res = torch.empty_like(x)
        p = make_params(dec.plan(N), 20, 2, 20, _lib.FT8_FLAG_TOPK)
        dec.ctx.check(_lib.lib().ft8_subtract(dec.ctx.handle, _lib.ptr(x), _lib.FT8_F32, _lib.ptr(res), N, 1, N,
                                              ctypes.byref(p), _lib.ptr(out), _lib.ptr(counts), dec.cap,
                                              _lib.stream_handle()), "ft8_subtract")
        r = 10 * np.log10(float((res.double() ** 2).sum()) / float((x.double() ** 2).sum()))
        out_db.append(r)
    return out_db


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=64)
    ap.add_argument("--k", type=int, default=300)
    a = ap.parse_args()
    import torch
    from ft8_demodulator_amd import _lib
    from ft8_demodulator_amd import synth
    from ft8_demodulator_amd._pipeline import SlotDecoder
    torch.cuda.set_device(0)
    print("clean-signal residual dB:", [round(v, 1) for v in clean_residual(torch)], flush=True)
    x, truths = synth.make_slots(a.slots, 50, seed=0, device="cuda")
    for name, flags in (("reference", 0), ("topk", _lib.FT8_FLAG_TOPK),
                        ("topk+subtract", _lib.FT8_FLAG_TOPK | _lib.FT8_FLAG_SUBTRACT)):
        dec = SlotDecoder(12000, 2, 2, max_candidates=a.k, min_score=2, max_iterations=20, flags=flags)
        recs = dec.records(x, _lib.FT8_F32)
        torch.cuda.synchronize()
        dec.ctx.set_timing(True)
        dec.timing(reset=True)
        t = time.time()
        for _ in range(3):
            dec.run(x, _lib.FT8_F32)
        torch.cuda.synchronize()
        wall = (time.time() - t) / 3 * 1e3
        tm = {k: round(v[0] / max(v[1], 1) * (v[1] / 3), 3) for k, v in dec.timing(reset=True).items() if v[1]}
        dec.ctx.set_timing(False)
        true1 = true2 = false = 0
        for s in range(a.slots):
            tr = set(bytes(p) for p in truths[s].payloads)
            got1 = set(bytes(r["payload"]) for r in recs[s] if r["pass_index"] == 0)
            got2 = set(bytes(r["payload"]) for r in recs[s] if r["pass_index"] == 1)
            true1 += len(got1 & tr)
            true2 += len(got2 & tr)
            false += len((got1 | got2) - tr)
        print(f"{name:14s} unique true decodes/slot pass1 {true1 / a.slots:6.2f} pass2 {true2 / a.slots:6.2f}"
              f"  false {false}  ms/step {wall:7.2f}  stages {tm}", flush=True)


if __name__ == "__main__":
    main()
