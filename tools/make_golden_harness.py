"""Goldens for the reference's own harness geometries and its one complex I/Q fixture (build
container only: imports /root/reference/src like tools/make_golden.py; nothing under tests/ imports
the reference, tests read only what this script writes).

1. channel  src/tests/channel/doppler_shift_test/down_sampled_signal.npy (complex128, 40 000 samples,
            fs 2000.0 from signal_processing_info.txt), called exactly as
            src/tests/demodulator/test_decode_after_channel.py:51,78-85,104-115 calls it:
              * calculate_spectrogram(x, 2000.0, 2, 2), then the 0 <= f <= 300 Hz mask -> the masked
                complex128-input dB spectrogram (stored), its f and t axes;
              * decode_ft8_message(x, 2000.0) at the reference defaults -> its results;
              * correct_frequency_drift(x, 2000.0, 2, 2, params={...the test's...}) -> the corrected
                wave (stored) and the drift rate, or the exception it raises.
            The fixture is read with np.load(allow_pickle=False) and stored here as data
            (tests/data/down_sampled_signal.npy), since /root/reference does not reach the GPU box.
2. harness  src/tests/demodulator/test_ft8_standard.py:43-68 test_step at every rate of its sweep
            (:70-84, fs 2 000 .. 10 000 Hz step 500): payload -> ft8_generator(payload, fs, f0 = 0,
            fc = 0) -> white noise at `snr_db` of the full band -> decode_ft8_message(bins_per_tone =
            steps_per_symbol = 2, max_candidates 20, min_score 1, max_iterations 20).  Three SNRs per
            rate.  The reference draws payloads and noise from NumPy's unseeded global generator;
            here both come from np.random.default_rng(seed) (bit-reproducible on any host, numpy's
            stream guarantee), so the inputs are NOT stored: the GPU test rebuilds the clean wave
            with oracle.gfsk_waveform (checked bit-identical to the reference generator here, the
            SHA-256 of each clean wave is stored) and the noise from the seed, and checks the input's
            SHA-256 before decoding.  Stored per case: candidate list + scores (the reference's
            ft8_find_candidates on its own waterfall) and decode_ft8_message's results.

Usage:  cd /tmp && python /root/repo/tools/make_golden_harness.py
"""
import contextlib
import hashlib
import io
import json
import logging
import os
import shutil
import sys
import tempfile
import time

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF_SRC = "/root/reference/src"
GOLD = os.path.join(REPO, "tests", "golden")
DATA = os.path.join(REPO, "tests", "data")
FIXTURE = os.path.join(REF_SRC, "tests", "channel", "doppler_shift_test", "down_sampled_signal.npy")

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")
sys.path.insert(0, REPO)
sys.path.insert(0, REF_SRC)
with contextlib.redirect_stdout(io.StringIO()):
    from ft8_tools.ft8_demodulator import ft8_decode as R  # noqa: E402
    from ft8_tools.ft8_demodulator import spectrogram_analyse as RS  # noqa: E402
    from ft8_tools.ft8_demodulator.ftx_types import FT8Waterfall  # noqa: E402
    from ft8_tools.ft8_beacon_receiver import frequency_correction as RF  # noqa: E402
    from ft8_tools import ft8_generator as RG  # noqa: E402
logging.getLogger(RF.__name__).setLevel(logging.WARNING)
from oracle import oracle as O  # noqa: E402

HARNESS_RATES = list(range(2000, 10000 + 500, 500))     # test_ft8_standard.py:70-84
HARNESS_SNRS = (-10.0, -14.0, -17.0)
KW = dict(bins_per_tone=2, steps_per_symbol=2, max_candidates=20, min_score=1, max_iterations=20)
DRIFT_PARAMS = {"nsync_sym": 7, "ndata_sym": 58, "zscore_threshold": 5, "max_iteration_num": 400000,
                "debug_plots": False}                       # test_decode_after_channel.py:88-94


def quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def results_json(res):
    return [{"payload": bytes(m.payload).hex(), "hash": int(m.hash), "ldpc_errors": int(s.ldpc_errors),
             "crc_extracted": int(s.crc_extracted), "crc_calculated": int(s.crc_calculated),
             "time_sec": float(t), "freq_hz": float(f), "score": float(sc),
             "score_dtype": str(np.asarray(sc).dtype)} for (m, s, t, f, sc) in res]


def harness_input(fs, snr_db, seed):
    """test_step's input (test_ft8_standard.py:45-54) with a seeded generator; -> (payload, clean, x)."""
    rng = np.random.default_rng(seed)
    payload = rng.integers(0, 256, size=10, dtype=np.uint8)     # np.random.randint(0, 256, 10, uint8)
    clean = quiet(RG.ft8_generator, payload, fs=fs, f0=0, fc=0)
    signal_power = np.mean(clean ** 2)
    noise_power = signal_power / (10 ** (snr_db / 10))
    noise = np.sqrt(noise_power) * rng.standard_normal(len(clean))
    return payload, clean, clean + noise


def channel_case(arrays):
    x = np.load(FIXTURE, allow_pickle=False)
    assert x.dtype == np.complex128 and x.shape == (40000,), (x.dtype, x.shape)
    os.makedirs(DATA, exist_ok=True)
    shutil.copyfile(FIXTURE, os.path.join(DATA, "down_sampled_signal.npy"))
    fs = 2000.0                                                 # signal_processing_info.txt
    c = {"name": "channel_down_sampled", "fs": fs, "input_sha256": sha(x), "bins_per_tone": 2,
         "steps_per_symbol": 2, "mask_f": [0, 300]}
    spec, f, t = RS.calculate_spectrogram(x, fs, 2, 2)
    m = (f >= 0) & (f <= 300)
    arrays["channel_spec"] = spec[m]
    arrays["channel_f"] = f[m]
    arrays["channel_t"] = t
    c["spec_shape"] = list(spec.shape)
    c["spec_dtype"] = str(spec.dtype)
    c["spec_sha256"] = sha(spec)
    c["masked_rows"] = [int(np.nonzero(m)[0][0]), int(m.sum())]
    try:
        res = quiet(R.decode_ft8_message, x, fs)
        c["decode_defaults"] = {"results": results_json(res)}
    except Exception as e:  # noqa: BLE001 -- the reference's own behaviour is the golden
        c["decode_defaults"] = {"error": type(e).__name__, "message": str(e)}
    try:
        wc, rate = quiet(RF.correct_frequency_drift, x, fs, 2, 2, params=dict(DRIFT_PARAMS))
        arrays["channel_corrected"] = np.asarray(wc)
        c["drift"] = {"rate": float(np.asarray(rate).reshape(-1)[0]), "rate_shape": list(np.shape(rate)), "corrected_sha256": sha(np.asarray(wc)),
                      "corrected_dtype": str(np.asarray(wc).dtype)}
    except Exception as e:  # noqa: BLE001
        c["drift"] = {"error": type(e).__name__, "message": str(e)}
    print("channel:", {k: v for k, v in c.items() if k in ("decode_defaults", "drift")}, flush=True)
    return c


def harness_case(fs, snr_db, seed, arrays):
    t0 = time.time()
    payload, clean, x = harness_input(fs, snr_db, seed)
    # the build's restatement of the generator (oracle/oracle.py) must rebuild the same clean wave
    restated = np.real(O.gfsk_waveform(O.tx_itones(bytes(payload)), fs, 0.0, style=1))
    name = f"h{fs}_{int(round(-snr_db * 10))}"
    c = {"name": name, "fs": fs, "snr_db": snr_db, "seed": seed, "payload": bytes(payload).hex(),
         "n": len(x), "clean_sha256": sha(clean), "x_sha256": sha(x),
         "restated_equal": bool(np.array_equal(restated, clean)),
         "restated_maxdiff": float(np.max(np.abs(restated - clean))), "kwargs": KW,
         "stft_method_expected": None}
    spec, f, _t = RS.calculate_spectrogram(x, fs, KW["bins_per_tone"], KW["steps_per_symbol"])
    mag = spec[f >= 0]
    wf = FT8Waterfall(mag=mag, time_osr=KW["steps_per_symbol"], freq_osr=KW["bins_per_tone"])
    cands = quiet(R.ft8_find_candidates, wf, KW["max_candidates"], KW["min_score"])
    c["cands"] = [[int(q.abs_time), int(q.abs_freq)] for q in cands]
    arrays[f"{name}_scores"] = np.array([q.score for q in cands], dtype=np.float64)
    c["waterfall_shape"] = list(mag.shape)
    res = quiet(R.decode_ft8_message, x, fs, **KW)
    c["results"] = results_json(res)
    c["seconds"] = round(time.time() - t0, 2)
    print(name, len(cands), "cands,", len(res), "decodes,", c["seconds"], "s, restated_equal",
          c["restated_equal"], flush=True)
    return c


def main():
    scratch = tempfile.mkdtemp(prefix="ft8gold_")
    os.chdir(scratch)
    arrays = {}
    meta = {"numpy": np.__version__, "scipy": __import__("scipy").__version__, "python": sys.version.split()[0],
            "channel": channel_case(arrays), "harness": []}
    seed = 50500
    for fs in HARNESS_RATES:
        for snr in HARNESS_SNRS:
            meta["harness"].append(harness_case(fs, snr, seed, arrays))
            seed += 1
    np.savez_compressed(os.path.join(GOLD, "harness.npz"), **arrays)
    with open(os.path.join(GOLD, "harness.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(GOLD, "harness.{json,npz}"))


if __name__ == "__main__":
    main()
