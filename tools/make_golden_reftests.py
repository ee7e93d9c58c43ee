"""Golden vectors for the geometries of the reference's OWN decode tests (runs only in the build
container, like tools/make_golden.py, whose reference-import recipe it shares):

  ref_noise  test_decode_with_noise (src/tests/demodulator/test_spectrogram_analyse.py:128-163):
             12 kHz, f0 = 500 Hz, payload 1c3f8a6ae207a1e39451, noise 0.1 N(0, 1), bins_per_tone =
             steps_per_symbol = 10 (nfft 19 200, hop 192), max_candidates 20, min_score 5
  ref_6k     test_decode_ft8_message (:92-126): fs 6000, f0 = 0 (tones at DC), payload
             1c3f8a6ae207a1e39450, noise at 0 dB SNR, bins_per_tone = steps_per_symbol = 2,
             max_candidates 20, min_score 1

The reference draws its noise from the unseeded global generator; here np.random.seed(seed) makes
the inputs reproducible, and the noisy input itself is stored (float64) so every consumer sees
the reference's exact bytes.  Stored per case: the input, the reference waterfall's SHA-256 (and
shape), its score grid's SHA-256 (ref_6k: full grid; ref_noise: the rows around the signal, also
pinned by hash only), the candidate list with scores, normalised LLRs of the first candidates, and
decode_ft8_message's results.

  nochan_*   test_ft8_without_channel.py:30-57: fs = 10e3 (a FLOAT), f0 = 550 Hz, fc = 0, payload
             np.random.randint(0, 255, 10) with [9] &= 0xF8, noise at the full-band SNR (-19 / -17 /
             -15 dB), bins_per_tone = steps_per_symbol = 4 (nperseg 1600, hop 400, nfft 6400),
             max_candidates 20, min_score 1, 20 iterations; several seeds
  ref_fs_frac  the same decode call at a NON-INTEGRAL sample rate, fs = 12006.3 (f0 = 1000 Hz,
             bpt = sps = 2, -15 dB): the reference computes int(0.16 fs) = 1921 and int(fs / 6.25 * 2)
             = 3842 on the float (spectrogram_analyse.py:32-34)

  bad_*      non-finite and silent input at the production geometry (12 kHz, bpt = sps = 2, K = 40,
             min_score 2, FLOAT32 samples as read_wave_file returns them): three signals (-12 / -10
             / -8 dB full-band SNR) in unit noise with a NaN burst near the slot's end (bad_nan_tail),
             +inf and -inf at its start (bad_inf_head), or exact zeros before the signals and after
             them (bad_zero_half: a -120 dB waterfall there).  NaN frames make every score touching them NaN -> -inf
             (ft8_decode.py:97-98) and every LLR vector touching them NaN after the normalisation,
             which bp_decode ends at once (sum(plain) == 0)

Usage:  cd /tmp && python /root/repo/tools/make_golden_reftests.py [nochannel | nonfinite]
        (nochannel / nonfinite: add / replace only those cases in the existing files)
"""
import contextlib
import hashlib
import io
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF_SRC = "/root/reference/src"
GOLD = os.path.join(REPO, "tests", "golden")

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")
sys.path.insert(0, REF_SRC)

with contextlib.redirect_stdout(io.StringIO()):
    from ft8_tools.ft8_demodulator import ft8_decode as R  # noqa: E402
    from ft8_tools.ft8_demodulator import spectrogram_analyse as RS  # noqa: E402
    from ft8_tools.ft8_demodulator.ftx_types import FT8Waterfall, FT8Candidate  # noqa: E402
    from ft8_tools import ft8_generator as RG  # noqa: E402


def quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def grid_rows(mag, sps, bpt, rows):
    """ft8_sync_score over the ft8_find_candidates grid, restricted to the given time rows."""
    wf = FT8Waterfall(mag=mag, time_osr=sps, freq_osr=bpt)
    fr = range(0, mag.shape[0] - 7 * bpt)
    out = np.empty((len(rows), len(fr)), dtype=mag.dtype)
    for i, t in enumerate(rows):
        for j, f in enumerate(fr):
            out[i, j] = R.ft8_sync_score(wf, FT8Candidate(waterfall=wf, abs_time=t, abs_freq=f))
    return out


def case(name, x, fs, kw, arrays, sub_rows=None):
    bpt, sps = kw["bins_per_tone"], kw["steps_per_symbol"]
    t0 = time.time()
    spec, f, t = RS.calculate_spectrogram(x, fs, bpt, sps)
    mag = spec[f >= 0]
    wf = FT8Waterfall(mag=mag, time_osr=sps, freq_osr=bpt)
    nb = wf.num_blocks
    trange = list(range(-10 * sps, nb * sps - sps * 59))
    c = {"name": name, "fs": fs, "kwargs": kw, "waterfall_shape": list(mag.shape), "waterfall_dtype": str(mag.dtype),
         "waterfall_sha256": sha(mag), "grid_t0": trange[0], "grid_nt": len(trange),
         "grid_nf": mag.shape[0] - 7 * bpt}
    rows = trange if sub_rows is None else [r for r in sub_rows if trange[0] <= r <= trange[-1]]
    g = grid_rows(mag, sps, bpt, rows)
    c["grid_rows"] = [rows[0], len(rows)]
    c["grid_rows_sha256"] = sha(g)
    cands = quiet(R.ft8_find_candidates, wf, kw["max_candidates"], kw["min_score"])
    c["cands"] = [[int(q.abs_time), int(q.abs_freq)] for q in cands]
    arrays[f"{name}_scores"] = np.array([q.score for q in cands], dtype=mag.dtype)
    llrs = []
    for q in cands[:4]:
        v = np.zeros(174)
        R.ft8_extract_likelihood(wf, q, v)
        with np.errstate(all="ignore"):
            R.ftx_normalize_logl(v)
        llrs.append(v)
    arrays[f"{name}_llr"] = np.array(llrs)
    res = quiet(R.decode_ft8_message, x, fs, **kw)
    c["results"] = [{"payload": bytes(m.payload).hex(), "hash": int(m.hash), "ldpc_errors": int(s.ldpc_errors),
                     "crc_extracted": int(s.crc_extracted), "crc_calculated": int(s.crc_calculated),
                     "time_sec": float(tt), "freq_hz": float(ff), "score": float(sc),
                     "score_dtype": str(np.asarray(sc).dtype)} for (m, s, tt, ff, sc) in res]
    arrays[f"{name}_x"] = x
    c["seconds"] = time.time() - t0
    print(name, "done", round(c["seconds"], 1), "s,", len(cands), "candidates,", len(res), "decodes", flush=True)
    return c


NOCHAN = [(-19, 11), (-17, 12), (-17, 13), (-15, 14)]   # (snr_db, np.random.seed)


def nochannel_cases(arrays):
    """test_ft8_without_channel.py:30-57 with np.random.seed(seed) before its draws, in its order:
    payload (randint(0, 255, 10), [9] &= 0xF8), then the noise (randn)."""
    out = []
    for snr_db, seed in NOCHAN:
        np.random.seed(seed)
        p = np.random.randint(0, 255, size=10, dtype=np.uint8)
        p[9] &= 0xF8
        fs = 10e3
        w = quiet(RG.ft8_generator, p, fs=fs, f0=550, fc=0)
        noise = np.sqrt(np.mean(w ** 2) / (10 ** (snr_db / 10))) * np.random.randn(len(w))
        x = w + noise
        kw = dict(bins_per_tone=4, steps_per_symbol=4, max_candidates=20, min_score=1, max_iterations=20)
        c = case(f"nochan_{-snr_db}db_s{seed}", x, fs, kw, arrays)
        c["payload_sent"] = p.tobytes().hex()
        out.append(c)
    # a non-integral sample rate through the same call
    np.random.seed(15)
    p = np.random.randint(0, 255, size=10, dtype=np.uint8)
    p[9] &= 0xF8
    fs = 12006.3
    w = quiet(RG.ft8_generator, p, fs=fs, f0=1000, fc=0)
    x = w + np.sqrt(np.mean(w ** 2) / (10 ** (-15 / 10))) * np.random.randn(len(w))
    kw = dict(bins_per_tone=2, steps_per_symbol=2, max_candidates=20, min_score=1, max_iterations=20)
    c = case("ref_fs_frac", x, fs, kw, arrays, sub_rows=list(range(-20, 30)))
    c["payload_sent"] = p.tobytes().hex()
    out.append(c)
    return out


BAD = (("bad_nan_tail", 31), ("bad_inf_head", 32), ("bad_zero_half", 33))


def nonfinite_cases(arrays):
    """Three reference-generator signals in unit noise, float32, with the slot partly non-finite or
    silent (module docstring)."""
    out = []
    fs, n = 12000, 180000
    for name, seed in BAD:
        np.random.seed(seed)
        x = np.random.randn(n)
        sent = []
        for f0, snr_db in ((600.0, -12), (1350.0, -10), (2100.0, -8)):
            p = np.random.randint(0, 255, size=10, dtype=np.uint8)
            p[9] &= 0xF8
            w = quiet(RG.ft8_generator, p, fs=fs, f0=f0, fc=0)
            w = w * np.sqrt(10 ** (snr_db / 10) / np.mean(w ** 2))
            m = min(n, len(w))
            x[:m] += w[:m]
            sent.append(p.tobytes().hex())
        x = x.astype(np.float32)
        if name == "bad_nan_tail":
            x[174000:174100] = np.nan
        elif name == "bad_inf_head":
            x[0:10] = np.inf
            x[10:20] = -np.inf
        else:
            x[:5000] = 0.0
            x[160000:] = 0.0
        kw = dict(bins_per_tone=2, steps_per_symbol=2, max_candidates=40, min_score=2, max_iterations=20)
        with np.errstate(all="ignore"):
            c = case(name, x, fs, kw, arrays, sub_rows=list(range(-20, 30)) + list(range(150, 176)))
        c["payloads_sent"] = sent
        out.append(c)
    return out


def main():
    scratch = tempfile.mkdtemp(prefix="ft8gold_")
    os.chdir(scratch)
    if sys.argv[1:] in (["nochannel"], ["nonfinite"]):
        with open(os.path.join(GOLD, "reftests.json")) as f:
            meta = json.load(f)
        old = np.load(os.path.join(GOLD, "reftests.npz"), allow_pickle=False)
        arrays = {k: old[k] for k in old.files}
        new = nochannel_cases(arrays) if sys.argv[1] == "nochannel" else nonfinite_cases(arrays)
        names = {c["name"] for c in new}
        meta["cases"] = [c for c in meta["cases"] if c["name"] not in names] + new
        np.savez_compressed(os.path.join(GOLD, "reftests.npz"), **arrays)
        with open(os.path.join(GOLD, "reftests.json"), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        print("updated", os.path.join(GOLD, "reftests.{json,npz}"))
        return
    arrays, cases = {}, []

    # test_decode_with_noise (:128-163)
    np.random.seed(20260)
    p = np.array([0x1C, 0x3F, 0x8A, 0x6A, 0xE2, 0x07, 0xA1, 0xE3, 0x94, 0x51], dtype=np.uint8)
    w = quiet(RG.ft8_generator, p, fs=12000, f0=500, fc=0)
    x = w + 0.1 * np.random.randn(len(w))
    kw = dict(bins_per_tone=10, steps_per_symbol=10, max_candidates=20, min_score=5, max_iterations=20)
    # the signal sits at abs_time ~ 10 (one-symbol late reference timing): rows -100 .. 40 of the grid
    cases.append(case("ref_noise", x, 12000, kw, arrays, sub_rows=list(range(-100, 41))))

    # test_decode_ft8_message (:92-126)
    np.random.seed(20261)
    p = np.array([0x1C, 0x3F, 0x8A, 0x6A, 0xE2, 0x07, 0xA1, 0xE3, 0x94, 0x50], dtype=np.uint8)
    w = quiet(RG.ft8_generator, p, fs=6000, f0=0, fc=0)
    noise = np.sqrt(np.mean(w ** 2) / 10 ** (0 / 10)) * np.random.randn(len(w))
    x = w + noise
    kw = dict(bins_per_tone=2, steps_per_symbol=2, max_candidates=20, min_score=1, max_iterations=20)
    cases.append(case("ref_6k", x, 6000, kw, arrays))

    meta = {"numpy": np.__version__, "scipy": __import__("scipy").__version__, "python": sys.version.split()[0],
            "cases": cases}
    np.savez_compressed(os.path.join(GOLD, "reftests.npz"), **arrays)
    with open(os.path.join(GOLD, "reftests.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(GOLD, "reftests.{json,npz}"))


if __name__ == "__main__":
    main()
