"""Capture transmit-chain golden vectors from the REFERENCE generator (build container only).

Imports /root/reference/src/ft8_tools/ft8_generator (read-only; PYTHONDONTWRITEBYTECODE) and
records, for fixed payloads/rates/frequencies:
  * gfsk_modulation_waveform_generator  (modulator.py:27-50)  -> the GFSK frequency sequence
  * ft8_baseband_generator              (modulator.py:76-82)  -> complex baseband
  * ft8_generator                       (modulator.py:84-90)  -> real waveform (f0 + fc)
into tests/golden/tx_wave.npz (+ the inputs in tx_wave.json).  Encoder known answers (a91, CRC,
codeword, itones) are already in golden.json ("tx", tools/make_golden.py).

Nothing under tests/ imports the reference: tests only read what this script wrote.

Usage:  cd /tmp && python /root/repo/tools/make_golden_tx.py
"""
import contextlib
import io
import json
import os
import sys
import time

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF_SRC = "/root/reference/src"
GOLD = os.path.join(REPO, "tests", "golden")

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")
sys.path.insert(0, REF_SRC)
with contextlib.redirect_stdout(io.StringIO()):
    from ft8_tools.ft8_generator import encoder as RE  # noqa: E402
    from ft8_tools.ft8_generator import modulator as RM  # noqa: E402

CASES = [
    # name, payload hex, fs, f0, fc, kind, segment (None = whole waveform)
    ("freq_1k", "1c3f8a6ae207a1e39451", 1000, 0.0, 0.0, "freq", None),
    ("bb_2k", "aa0203040506070809f8", 2000, 100.0, 0.0, "baseband", None),
    ("real_6k", "1c3f8a6ae207a1e39451", 6000, 1000.0, 0.0, "real", None),
    ("real_12k", "5b17c2e09a44d1f03628", 12000, 500.0, 250.0, "real", (0, 30000, 141680, 151680)),
]


def main():
    os.makedirs(GOLD, exist_ok=True)
    arrays, meta = {}, {"numpy": np.__version__, "scipy": __import__("scipy").__version__, "cases": []}
    for name, hexp, fs, f0, fc, kind, seg in CASES:
        t = time.time()
        pay = np.frombuffer(bytes.fromhex(hexp), dtype=np.uint8).copy()
        it = RE.ft8_encode(pay)
        if kind == "freq":
            y = RM.gfsk_modulation_waveform_generator(it, fs)
        elif kind == "baseband":
            y = RM.ft8_baseband_generator(pay, fs, f0)
        else:
            y = RM.ft8_generator(pay, fs, f0, fc)
        y = np.asarray(y)
        full_len = int(y.shape[0])
        if seg is not None:
            a0, a1, b0, b1 = seg
            y = np.concatenate([y[a0:a1], y[b0:b1]])
        arrays[name] = y
        meta["cases"].append({"name": name, "payload": hexp, "fs": fs, "f0": f0, "fc": fc, "kind": kind,
                              "segment": seg, "length": full_len, "dtype": str(y.dtype)})
        print(name, kind, full_len, y.dtype, round(time.time() - t, 1), "s", flush=True)
    np.savez_compressed(os.path.join(GOLD, "tx_wave.npz"), **arrays)
    with open(os.path.join(GOLD, "tx_wave.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", GOLD)


if __name__ == "__main__":
    main()
