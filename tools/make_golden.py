"""Capture golden vectors from the REFERENCE implementation (runs only in the build container).

Imports /root/reference/src (read-only; PYTHONDONTWRITEBYTECODE, scratch CWD because
decode_ft8_message writes a PNG into CWD) and records its outputs stage by stage into
tests/golden/.  Inputs are either the reference's own data file (the bundled 20 kHz WAV, copied
to tests/data/) or synthetic data made by ft8_demodulator_amd.synth and stored as 16-bit WAV
files so that every consumer reads bit-identical float32 samples (from_wave.py:24-69 semantics).

Nothing under tests/ imports the reference: tests only read what this script wrote.

Usage:  cd /tmp && python /root/repo/tools/make_golden.py
"""
import contextlib
import hashlib
import io
import json
import os
import shutil
import sys
import tempfile
import time
import wave

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF_SRC = "/root/reference/src"
GOLD = os.path.join(REPO, "tests", "golden")
DATA = os.path.join(REPO, "tests", "data")
WAV_REF = os.path.join(REF_SRC, "ft8_tools", "ft8_beacon_receiver", "data", "raw", "ft8_fs20k_f0_550_id_1.wav")

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")
sys.path.insert(0, REPO)
sys.path.insert(0, REF_SRC)
sys.path.insert(0, os.path.join(REF_SRC, "tests", "demodulator"))

with contextlib.redirect_stdout(io.StringIO()):
    from ft8_tools.ft8_demodulator import ft8_decode as R  # noqa: E402
    from ft8_tools.ft8_demodulator import spectrogram_analyse as RS  # noqa: E402
    from ft8_tools.ft8_demodulator import ldpc_decoder as RL  # noqa: E402
    from ft8_tools.ft8_demodulator import crc as RC  # noqa: E402
    from ft8_tools.ft8_demodulator.ftx_types import FT8Waterfall, FT8Candidate  # noqa: E402
    from ft8_tools import ft8_generator as RG  # noqa: E402
    # the package-level get_crc_from_a91 recurses into itself (ft8_generator/__init__.py:20-27)
    from ft8_tools.ft8_generator import crc as RGC  # noqa: E402
    from from_wave import read_wave_file  # noqa: E402

from ft8_demodulator_amd import synth as S  # noqa: E402


def quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def write_wav(path, x_float, fs):
    q = np.clip(np.round(np.asarray(x_float, dtype=np.float64) * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(fs)
        w.writeframes(q.tobytes())


def ref_candidates(mag, sps, bpt, N, min_score):
    wf = FT8Waterfall(mag=mag, time_osr=sps, freq_osr=bpt)
    try:
        c = quiet(R.ft8_find_candidates, wf, N, min_score)
    except TypeError as e:  # exact score tie reached a heap comparison
        return None, str(e), wf
    return [(int(x.abs_time), int(x.abs_freq), x.score) for x in c], None, wf


def ref_score_grid(mag, sps, bpt):
    wf = FT8Waterfall(mag=mag, time_osr=sps, freq_osr=bpt)
    nb = wf.num_blocks
    tr = range(-10 * sps, nb * sps - sps * 59)
    fr = range(0, mag.shape[0] - 7 * bpt)
    out = np.empty((len(tr), len(fr)), dtype=mag.dtype)
    for i, t in enumerate(tr):
        for j, f in enumerate(fr):
            out[i, j] = R.ft8_sync_score(wf, FT8Candidate(waterfall=wf, abs_time=t, abs_freq=f))
    return out


def ref_llr(wf, at, af, normalize):
    x = np.zeros(174)
    R.ft8_extract_likelihood(wf, FT8Candidate(waterfall=wf, abs_time=at, abs_freq=af), x)
    if normalize:
        with np.errstate(all="ignore"):
            R.ftx_normalize_logl(x)
    return x


# ----------------------------------------------------------------------------------------------
def gold_tx(out):
    rng = np.random.default_rng(11)
    pays = [bytes.fromhex("1c3f8a6ae207a1e39451"), bytes.fromhex("aa0203040506070809f8")]
    pays += [bytes(rng.integers(0, 256, 10, dtype=np.uint8)) for _ in range(8)]
    rows = []
    for p in pays:
        a91 = quiet(RG.crc_generator, np.frombuffer(p, dtype=np.uint8).copy())
        cw = quiet(RG.ldpc_generator, a91)
        it = quiet(RG.ft8_encode, np.frombuffer(p, dtype=np.uint8).copy())
        rows.append({"payload": p.hex(), "a91": bytes(a91).hex(), "codeword": bytes(cw).hex(),
                     "crc": int(RGC.get_crc_from_a91(a91)), "itones": "".join(str(int(v)) for v in it)})
    # CRC / bit packing known answers (crc.py:11-79, ft8_decode.py:200-215)
    crc_rows = []
    for k in range(24):
        nb = int(rng.integers(1, 97))
        data = bytes(rng.integers(0, 256, 12, dtype=np.uint8))
        crc_rows.append({"data": data.hex(), "nbits": nb, "crc": int(RC.compute_crc(bytearray(data), nb)),
                         "extract": int(RC.extract_crc(bytearray(data)))})
        bits = rng.integers(0, 2, 174).astype(np.uint8)
        crc_rows[-1]["bits"] = "".join(map(str, bits))
        crc_rows[-1]["packed91"] = bytes(R.pack_bits(bits, 91)).hex()
    out["tx"] = rows
    out["crc"] = crc_rows


def gold_stft(arrays, meta):
    rng = np.random.default_rng(5)
    cases = []
    for name, fs, n, kind, bpt, sps in [("r32_2k", 2000, 8000, "f32", 2, 2), ("r64_2k", 2000, 8000, "f64", 2, 2),
                                         ("c64_2k", 2000, 6000, "c64", 2, 2), ("c128_2k", 2000, 6000, "c128", 2, 2),
                                         ("r32_12k", 12000, 12000, "f32", 2, 2), ("r32_6k_b4", 6000, 9000, "f32", 4, 4),
                                         ("r64_10k_b3", 10000, 9000, "f64", 3, 3), ("r32_2k_b1", 2000, 5000, "f32", 1, 1)]:
        x = rng.standard_normal(n) + 0.5 * np.sin(2 * np.pi * 300.0 * np.arange(n) / fs)
        if kind == "f32":
            x = x.astype(np.float32)
        elif kind == "c64":
            x = (x + 1j * rng.standard_normal(n)).astype(np.complex64)
        elif kind == "c128":
            x = x + 1j * rng.standard_normal(n)
        spec, f, t = RS.calculate_spectrogram(x, fs, bpt, sps)
        arrays[f"stft_{name}_x"] = x
        arrays[f"stft_{name}_spec"] = spec
        arrays[f"stft_{name}_f"] = f
        arrays[f"stft_{name}_t"] = t
        cases.append({"name": name, "fs": fs, "bpt": bpt, "sps": sps, "dtype": str(spec.dtype)})
    meta["stft"] = cases


def gold_sync(arrays, meta):
    rng = np.random.default_rng(7)
    cases = []

    def add(name, mag, sps, bpt, selections, grid=True, llr_top=6):
        c = {"name": name, "sps": sps, "bpt": bpt, "dtype": str(mag.dtype), "sel": []}
        arrays[f"sync_{name}_mag"] = mag
        if grid:
            g = ref_score_grid(mag, sps, bpt)
            arrays[f"sync_{name}_grid"] = g
        for (N, ms) in selections:
            cands, err, wf = ref_candidates(mag, sps, bpt, N, ms)
            e = {"N": N, "min_score": ms, "error": err}
            if cands is not None:
                e["cands"] = [[a, b] for a, b, _ in cands]
                arrays[f"sync_{name}_N{N}_ms{ms}_scores"] = np.array([s for _, _, s in cands], dtype=mag.dtype)
                # LLRs (raw + normalised) for the first few selected candidates
                llrs = [ref_llr(wf, a, b, False) for a, b, _ in cands[:llr_top]]
                nl = [ref_llr(wf, a, b, True) for a, b, _ in cands[:llr_top]]
                if llrs:
                    arrays[f"sync_{name}_N{N}_ms{ms}_llr_raw"] = np.array(llrs)
                    arrays[f"sync_{name}_N{N}_ms{ms}_llr"] = np.array(nl)
            c["sel"].append(e)
        cases.append(c)

    base = (-60 + 8 * rng.standard_normal((100, 186))).astype(np.float32)
    add("rand32", base, 2, 2, [(20, 10), (50, 2), (7, -1000), (300, 0.5), (40, 3.25)])
    add("rand64", base.astype(np.float64) + 1e-9 * rng.standard_normal(base.shape), 2, 2,
        [(20, 10), (25, -1000), (200, 1.0)])
    # scores rising along the scan order: new maxima after the heap is full (heapreplace path)
    ramp = (base + np.linspace(0, 30, 186, dtype=np.float32)[None, :] * (np.arange(100)[:, None] % 9 == 0)).astype(np.float32)
    add("ramp32", ramp, 2, 2, [(5, -1000), (12, 0.0), (30, 2)])
    # other oversampling factors
    add("b4s4_32", (-50 + 6 * rng.standard_normal((120, 372))).astype(np.float32), 4, 4, [(20, 3), (60, 1)])
    add("b1s1_64", (-50 + 6 * rng.standard_normal((40, 93))), 1, 1, [(20, 1), (10, -1000)])
    add("b3s3_32", (-50 + 6 * rng.standard_normal((70, 280))).astype(np.float32), 3, 3, [(25, 2)])
    # short waterfall: few blocks, the time grid is still non-empty
    add("short32", (-50 + 6 * rng.standard_normal((40, 120))).astype(np.float32), 2, 2, [(30, -1000)])
    # quantised values: exact score ties (the reference may raise TypeError)
    add("quant32", np.round(-50 + 3 * rng.standard_normal((30, 186))).astype(np.float32), 2, 2,
        [(10, 1), (10, 100), (5, -1000)], llr_top=3)
    # silence: constant -120 dB -> every score exactly 0.0
    add("silence32", np.full((30, 186), -120, dtype=np.float32), 2, 2, [(10, 1), (10, 0)], llr_top=2)
    meta["sync"] = cases


def gold_bp(arrays, meta):
    rng = np.random.default_rng(9)
    vecs, iters = [], []
    for i in range(90):
        p = S.random_payload(rng)
        bits = S.codeword_bits(p).astype(np.float64)
        mu = 1.0
        sigma = [0.4, 0.7, 0.9, 1.0, 1.1, 1.3][i % 6]
        llr = (2 * bits - 1) * mu + sigma * rng.standard_normal(174)
        with np.errstate(all="ignore"):
            R.ftx_normalize_logl(llr)
        vecs.append(llr)
        iters.append([20, 20, 20, 50, 5, 1][i % 6] if i < 60 else 20)
    # edge cases: zero vector (NaN after normalisation), all-negative, exact codeword, zero iterations
    with np.errstate(all="ignore"):
        z = np.zeros(174)
        R.ftx_normalize_logl(z)
    vecs.append(z); iters.append(20)
    vecs.append(-np.abs(rng.standard_normal(174)) - 0.1); iters.append(20)
    cw = S.codeword_bits(bytes.fromhex("aa0203040506070809f8")).astype(np.float64)
    vecs.append(4.0 * (2 * cw - 1)); iters.append(20)
    vecs.append(4.0 * (2 * cw - 1)); iters.append(0)
    plains, errs = [], []
    t0 = time.time()
    for v, it in zip(vecs, iters):
        pl, e = RL.bp_decode(np.array(v), it)
        plains.append(np.asarray(pl, dtype=np.uint8))
        errs.append(int(e))
    arrays["bp_llr"] = np.array(vecs)
    arrays["bp_iters"] = np.array(iters, dtype=np.int32)
    arrays["bp_plain"] = np.array(plains)
    arrays["bp_errors"] = np.array(errs, dtype=np.int32)
    # decode tail for each (ft8_decode.py:239-273)
    tails = []
    for pl, e in zip(plains, errs):
        ok = False
        pay, ce, cc = b"", 0, 0
        if e == 0:
            a91 = R.pack_bits(pl, 91)
            ce = RC.extract_crc(a91)
            buf = bytearray(12)
            buf[:10] = a91[:10]
            buf[9] &= 0xF8
            cc = RC.compute_crc(buf, 82)
            ok = ce == cc
            if ok:
                pp = bytearray(a91[:10])
                pp[9] &= 0xF8
                pay = bytes(pp)
        tails.append({"ok": bool(ok), "payload": pay.hex(), "crc_extracted": int(ce), "crc_calculated": int(cc)})
    meta["bp_tail"] = tails
    meta["bp_seconds"] = time.time() - t0


def decode_record(res):
    return [{"payload": bytes(m.payload).hex(), "hash": int(m.hash), "ldpc_errors": int(s.ldpc_errors),
             "crc_extracted": int(s.crc_extracted), "crc_calculated": int(s.crc_calculated),
             "time_sec": float(t), "freq_hz": float(f), "score": float(sc), "score_dtype": str(np.asarray(sc).dtype)}
            for (m, s, t, f, sc) in res]


def gold_e2e(arrays, meta):
    os.makedirs(DATA, exist_ok=True)
    shutil.copyfile(WAV_REF, os.path.join(DATA, "ft8_fs20k_f0_550_id_1.wav"))
    cases = []

    def run(name, wav, kwargs):
        x, fs = quiet(read_wave_file, wav)
        try:
            res = quiet(R.decode_ft8_message, x, fs, **kwargs)
            rec, err = decode_record(res), None
        except Exception as e:  # noqa: BLE001
            rec, err = None, f"{type(e).__name__}: {e}"
        cases.append({"name": name, "wav": os.path.basename(wav), "kwargs": kwargs, "results": rec, "error": err})

    wavp = os.path.join(DATA, "ft8_fs20k_f0_550_id_1.wav")
    run("wav_default", wavp, {})
    run("wav_band", wavp, {"freq_min": 400.0, "freq_max": 700.0})
    run("wav_time", wavp, {"time_min": 0.5, "time_max": 12.0, "max_candidates": 10})
    run("wav_k50_ms5", wavp, {"max_candidates": 50, "min_score": 5, "max_iterations": 30})

    # WAV waterfall + candidate + LLR details (stage pins on real data)
    x, fs = quiet(read_wave_file, wavp)
    spec, f, t = RS.calculate_spectrogram(x, fs, 2, 2)
    mag = spec[f >= 0]
    meta["wav_waterfall"] = {"shape": list(mag.shape), "dtype": str(mag.dtype), "sha256": sha(mag)}
    g = ref_score_grid(mag, 2, 2)
    meta["wav_grid"] = {"shape": list(g.shape), "sha256": sha(g)}
    arrays["wav_grid_max"] = np.array([np.max(g)])
    cands, _, wf = ref_candidates(mag, 2, 2, 20, 10)
    arrays["wav_cands"] = np.array([[a, b] for a, b, _ in cands], dtype=np.int32)
    arrays["wav_scores"] = np.array([s for _, _, s in cands], dtype=np.float32)
    arrays["wav_llr"] = np.array([ref_llr(wf, a, b, True) for a, b, _ in cands])
    arrays["wav_llr_raw"] = np.array([ref_llr(wf, a, b, False) for a, b, _ in cands])
    outs = []
    for a, b, _ in cands:
        ok, m, s = R.ft8_decode_candidate(wf, FT8Candidate(waterfall=wf, abs_time=a, abs_freq=b), 20)
        outs.append([int(ok), int(s.ldpc_errors), int(s.crc_extracted), int(s.crc_calculated)])
    arrays["wav_cand_status"] = np.array(outs, dtype=np.int32)

    # synthetic slots from our own transmitter, stored as 16-bit WAV (scaled by 1/8 to avoid clipping)
    def synth_wav(name, n_sig, snr, seed, f0r=(200.0, 2800.0), str_=(0.0, 2.0)):
        xs, tr = S.make_slots(1, n_sig, snr_db=snr, f0_range=f0r, start_range=str_, seed=seed)
        p = os.path.join(DATA, f"{name}.wav")
        write_wav(p, xs[0].numpy().astype(np.float64) / 8.0, 12000)
        meta.setdefault("synth_truth", {})[name] = [q.hex() for q in tr[0].payloads]
        return p

    p1 = synth_wav("synth_cfg1", 1, 10.0, 1, (1000.0, 1000.0), (0.5, 0.5))
    run("cfg1_default", p1, {})
    p2 = synth_wav("synth_cfg2", 50, (-24.0, -10.0), 2026)
    run("cfg2_k300_ms2", p2, {"max_candidates": 300, "min_score": 2, "max_iterations": 20})
    run("cfg2_k20_ms10", p2, {"max_candidates": 20, "min_score": 10})
    p3 = synth_wav("synth_few", 4, (-12.0, 0.0), 77)
    run("few_k60_ms6", p3, {"max_candidates": 60, "min_score": 6, "max_iterations": 25})
    # float64 input path (scores are np.float64)
    xs, _ = quiet(read_wave_file, p1)
    res = quiet(R.decode_ft8_message, xs.astype(np.float64), 12000)
    cases.append({"name": "cfg1_f64", "wav": "synth_cfg1.wav", "kwargs": {}, "as_float64": True,
                  "results": decode_record(res), "error": None})
    # complex128 input (analytic signal): two-sided spectrum, f >= 0 half
    import scipy.signal
    z = scipy.signal.hilbert(xs.astype(np.float64))
    arrays["cfg1_complex_x"] = z[:0]  # recomputed by the test from the WAV (scipy is in the image)
    res = quiet(R.decode_ft8_message, z, 12000)
    cases.append({"name": "cfg1_c128", "wav": "synth_cfg1.wav", "kwargs": {}, "as_analytic": True,
                  "results": decode_record(res), "error": None})
    # edge cases (test_spectrogram_analyse.py:165-198): the reference raises IndexError
    for nm, n in (("zeros1000", 1000), ("zeros10", 10)):
        try:
            res = quiet(R.decode_ft8_message, np.zeros(n), 12000, bins_per_tone=2, steps_per_symbol=2)
            cases.append({"name": nm, "results": decode_record(res), "error": None})
        except Exception as e:  # noqa: BLE001
            cases.append({"name": nm, "results": None, "error": f"{type(e).__name__}: {e}"})
    meta["e2e"] = cases


def main():
    os.makedirs(GOLD, exist_ok=True)
    scratch = tempfile.mkdtemp(prefix="ft8gold_")
    os.chdir(scratch)
    meta, arrays = {"numpy": np.__version__, "scipy": __import__("scipy").__version__,
                    "python": sys.version.split()[0]}, {}
    for step in (lambda: gold_tx(meta), lambda: gold_stft(arrays, meta), lambda: gold_sync(arrays, meta),
                 lambda: gold_bp(arrays, meta), lambda: gold_e2e(arrays, meta)):
        t = time.time()
        step()
        print("step done", round(time.time() - t, 1), "s", flush=True)
    np.savez_compressed(os.path.join(GOLD, "golden.npz"), **arrays)
    with open(os.path.join(GOLD, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    shutil.rmtree(scratch, ignore_errors=True)
    print("wrote", GOLD)


if __name__ == "__main__":
    main()
