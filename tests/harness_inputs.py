"""Inputs of the reference-harness goldens (tools/make_golden_harness.py), rebuilt from their seeds.

test_ft8_standard.py:45-54 test_step: payload -> ft8_generator(payload, fs, f0 = 0, fc = 0) -> white
noise at snr_db of the full band.  The payload and the noise come from np.random.default_rng(seed)
(the golden script's stand-in for NumPy's unseeded global generator); the clean wave from the oracle's
restatement of the reference generator (oracle.gfsk_waveform, style 1), which the golden script
checked bit-identical to the reference's own output."""
import hashlib
import json
import os

import numpy as np

from conftest import DATA, GOLD


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load():
    with open(os.path.join(GOLD, "harness.json")) as f:
        meta = json.load(f)
    return meta, np.load(os.path.join(GOLD, "harness.npz"), allow_pickle=False)


def harness_input(case, O):
    """-> (clean, x) for one golden case; O is oracle.oracle (the generator restatement)."""
    rng = np.random.default_rng(case["seed"])
    payload = rng.integers(0, 256, size=10, dtype=np.uint8)
    assert bytes(payload).hex() == case["payload"]
    clean = np.real(O.gfsk_waveform(O.tx_itones(bytes(payload)), case["fs"], 0.0, style=1))
    signal_power = np.mean(clean ** 2)
    noise_power = signal_power / (10 ** (case["snr_db"] / 10))
    noise = np.sqrt(noise_power) * rng.standard_normal(len(clean))
    return clean, clean + noise


def channel_input():
    return np.load(os.path.join(DATA, "down_sampled_signal.npy"), allow_pickle=False)
