"""Capture frequency-drift-correction golden vectors from the REFERENCE (build container only).

Imports /root/reference/src/ft8_tools/ft8_beacon_receiver/frequency_correction.py (read-only;
PYTHONDONTWRITEBYTECODE, scratch CWD because it writes PNGs) and records, for fixed beacon inputs
built by oracle/drift.py's beacon_input (seeded, reproducible on the GPU box from the parameters
alone, so the inputs themselves are not stored):
  * correct_frequency_drift(...)      -> estimated drift rate (Hz/sample) and a strided subsample +
                                         checksums of the corrected complex wave
  * the per-column argmax of the reference's calculate_spectrogram (f >= 0) for both spectrograms
  * detect_signal_continuity(...)     -> segments and the continuity metric
into tests/golden/drift.npz (+ drift.json).  It also checks oracle/drift.py against every value.

Nothing under tests/ imports the reference: tests only read what this script wrote.

Usage:  cd /tmp && python /root/repo/tools/make_golden_drift.py
"""
import contextlib
import io
import json
import logging
import os
import sys
import time

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF_SRC = "/root/reference/src"
GOLD = os.path.join(REPO, "tests", "golden")

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")
sys.path.insert(0, REPO)
sys.path.insert(0, REF_SRC)
with contextlib.redirect_stdout(io.StringIO()):
    from ft8_tools.ft8_beacon_receiver import frequency_correction as RF  # noqa: E402
    from ft8_tools.ft8_demodulator import spectrogram_analyse as RS  # noqa: E402
logging.getLogger(RF.__name__).setLevel(logging.WARNING)
from oracle import drift as OD  # noqa: E402

SUB = 97  # stride of the stored subsample of the corrected wave

# name, payload, fs, f0, fc, drift Hz/s, Es/N0 dB (None = noiseless), seed, correction params
CASES = [
    ("fs12k_sps8_deg2", "1c3f8a6ae207a1e39451", 12000, 300.0, 500.0, 100.0, 28.0, 11,
     {"bins_per_tone": 2, "steps_per_symbol": 8}),
    ("fs12k_sps8_deg2_fast", "5b17c2e09a44d1f03628", 12000, 300.0, 400.0, 200.0, 24.0, 12,
     {"bins_per_tone": 2, "steps_per_symbol": 8}),
    ("fs12k_sps2_default", "aa0203040506070809f8", 12000, 300.0, 600.0, 150.0, 28.0, 13, None),
    ("fs12k_sps8_deg1", "1c3f8a6ae207a1e39451", 12000, 250.0, 700.0, 120.0, 30.0, 14,
     {"bins_per_tone": 2, "steps_per_symbol": 8, "poly_degree": 1}),
    ("fs12k_sps4_no_segment", "1c3f8a6ae207a1e39451", 12000, 250.0, 700.0, -120.0, 30.0, 14,
     {"bins_per_tone": 2, "steps_per_symbol": 4, "poly_degree": 1}),
    ("fs12k_sps8_linear_only", "0123456789abcdef0120", 12000, 300.0, 500.0, 80.0, 28.0, 15,
     {"bins_per_tone": 2, "steps_per_symbol": 8, "precise_sync": False}),
    ("fs12k_sps8_trim80", "fedcba98765432100000", 12000, 300.0, 500.0, 60.0, 26.0, 16,
     {"bins_per_tone": 2, "steps_per_symbol": 8, "fit_middle_percent": 80}),
    ("fs6k_sps8_deg2", "1c3f8a6ae207a1e39451", 6000, 300.0, 200.0, 50.0, 28.0, 17,
     {"bins_per_tone": 2, "steps_per_symbol": 8}),
    ("fs12k_noise_only", "1c3f8a6ae207a1e39451", 12000, 300.0, 500.0, 100.0, -60.0, 18,
     {"bins_per_tone": 2, "steps_per_symbol": 8}),
    # the reference test's own configuration (test_correction.py:121-147): 32 768 Hz, 568 Hz/s,
    # correction at steps_per_symbol 8 -> nfft 10 485 = 3 x 5 x 3 x 233 (the direct-DFT path)
    ("fs32k_reference_test", "1c3f8a6ae207a1e39451", 32768, 300.0, 500.0, 568.0, 28.0, 19,
     {"bins_per_tone": 2, "steps_per_symbol": 8}),
]


def ref_argmax(wave, fs, bpt, sps):
    spec, f, _ = RS.calculate_spectrogram(wave, fs, bpt, sps)
    return np.argmax(spec[f >= 0], axis=0)


def main():
    os.makedirs(GOLD, exist_ok=True)
    arrays, meta = {}, {"numpy": np.__version__, "scipy": __import__("scipy").__version__,
                        "sklearn": __import__("sklearn").__version__, "subsample_stride": SUB, "cases": []}
    for name, hexp, fs, f0, fc, drift, esn0, seed, params in CASES:
        t0 = time.time()
        x = OD.beacon_input(hexp, fs, f0, fc, drift, esn0, seed)
        p_ref = dict(params) if params is not None else None
        if p_ref is not None:
            p_ref.setdefault("debug_plots", False)
        with contextlib.redirect_stdout(io.StringIO()):
            y, rate = RF.correct_frequency_drift(x, fs, 6.25, 0.16, params=p_ref)
        full = dict(OD.DEFAULT_PARAMS)
        full.update(params or {})
        bpt, sps = full["bins_per_tone"], full["steps_per_symbol"]
        window = full["window_size_factor"] * sps
        a1 = ref_argmax(x, fs, bpt, sps)
        F = int(np.sum(RS.calculate_spectrogram(x[:int(0.16 * fs)], fs, bpt, sps)[1] >= 0))
        maxvar = full["max_variance_factor"] * F ** 2
        with contextlib.redirect_stdout(io.StringIO()):
            segs, metric = RF.detect_signal_continuity(a1, window_size=window, max_variance=maxvar)
        # the oracle against the reference, on the same input
        tr = {}
        yo, rate_o = OD.correct_frequency_drift(x, fs, 6.25, 0.16, params=params, trace=tr)
        assert np.array_equal(tr["argmax1"], a1), name
        assert [tuple(map(int, s)) for s in segs] == [tuple(map(int, s)) for s in tr["segments"]], name
        assert np.allclose(tr["metric"], metric, rtol=1e-9, atol=1e-9), name
        r = float(np.asarray(rate).reshape(-1)[0])
        assert abs(rate_o - r) <= 1e-12 * max(1.0, abs(r)), (name, rate_o, rate)
        y = np.asarray(y)
        err = np.max(np.abs(yo - y))
        assert err < 1e-9, (name, err)
        arrays[f"{name}/argmax1"] = a1.astype(np.int32)
        arrays[f"{name}/metric"] = np.asarray(metric, dtype=np.float64)
        arrays[f"{name}/segments"] = np.array(segs, dtype=np.int64).reshape(-1, 2)
        arrays[f"{name}/corrected_sub"] = y[::SUB].astype(np.complex128)
        if "argmax2" in tr:
            yl = x * np.exp(-2j * np.pi * (tr["rate1"] * np.arange(len(x)) ** 2 / 2 / fs) / (fs))
            a2 = ref_argmax(yl, fs, bpt, sps)
            assert np.array_equal(a2, tr["argmax2"]), name
            arrays[f"{name}/argmax2"] = a2.astype(np.int32)
        meta["cases"].append({
            "name": name, "payload": hexp, "fs": fs, "f0": f0, "fc": fc, "drift_hz_per_s": drift,
            "esn0_db": esn0, "seed": seed, "params": params, "n_samples": int(len(x)),
            "rate_per_sample": float(np.asarray(rate).reshape(-1)[0]), "rate_is_array": bool(np.ndim(rate) > 0), "rate1_hz_per_s": float(tr.get("rate1", 0.0)),
            "sync_idx": int(tr["sync_idx"]) if "sync_idx" in tr else None, "status": int(tr["status"]),
            "corrected_abs_sum": float(np.sum(np.abs(y))), "corrected_sum": [float(np.sum(y).real), float(np.sum(y).imag)],
            "oracle_max_abs_err": float(err), "seconds": round(time.time() - t0, 2)})
        print(name, "rate/sample", rate, "est Hz/s", rate * fs, "true", drift, "status", tr["status"],
              "oracle err", err, f"{time.time() - t0:.1f}s", flush=True)
    np.savez_compressed(os.path.join(GOLD, "drift.npz"), **arrays)
    with open(os.path.join(GOLD, "drift.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
