"""The reference's OWN decode-test geometries (src/tests/demodulator/test_spectrogram_analyse.py):

  ref_noise  test_decode_with_noise (:128-163): 12 kHz, bins_per_tone = steps_per_symbol = 10
             (nfft 19 200: the direct-DFT STFT, the generic float64 score kernel), K = 20, min_score 5
  ref_6k     test_decode_ft8_message (:92-126): fs 6000, f0 = 0 (tones at DC), bpt = sps = 2,
             K = 20, min_score 1
  nochan_*   test_ft8_without_channel.py:30-57: fs = 10e3 as a float, f0 = 550 Hz, -19..-15 dB,
             bpt = sps = 4 (nfft 6400), K = 20, min_score 1
  ref_fs_frac  a non-integral sample rate, fs = 12006.3: nperseg 1921, nfft 3842 (chirp-z), computed
             on the float as spectrogram_analyse.py:32-34 does
  bad_*      the production geometry (12 kHz, bpt = sps = 2, float32 samples: k_stft3840p, k_score2)
             on a slot with a NaN burst, with +-inf samples, or with exact zeros at both ends
             (-120 dB waterfall regions); NaN scores become -inf and NaN LLR vectors end BP at once

Goldens from the reference itself (tools/make_golden_reftests.py -> tests/golden/reftests.*), inputs
stored as the reference's float64 samples.  CPU tests pin the oracle (waterfall SHA-256, score-grid
rows, candidates, LLRs, decodes); GPU tests run the same inputs through the HIP path: stage parity on
the (SHA-pinned) reference waterfall, and the whole decode_ft8_message end to end."""
import json
import os

import numpy as np
import pytest

from conftest import GOLD


@pytest.fixture(scope="module")
def reft():
    with open(os.path.join(GOLD, "reftests.json")) as f:
        meta = json.load(f)
    arr = np.load(os.path.join(GOLD, "reftests.npz"), allow_pickle=False)
    return {c["name"]: c for c in meta["cases"]}, arr


def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


CASES = ("ref_noise", "ref_6k", "nochan_19db_s11", "nochan_17db_s12", "nochan_17db_s13", "nochan_15db_s14",
         "ref_fs_frac", "bad_nan_tail", "bad_inf_head", "bad_zero_half")


@pytest.mark.parametrize("name", CASES)
def test_oracle_pinned_on_reference_test_geometry(reft, oracle, name):
    cases, arr = reft
    c = cases[name]
    kw = c["kwargs"]
    x = arr[f"{name}_x"]
    mag = oracle.waterfall(x, c["fs"], kw["bins_per_tone"], kw["steps_per_symbol"])
    assert list(mag.shape) == c["waterfall_shape"] and _sha(mag) == c["waterfall_sha256"]
    g = oracle.score_grid(mag, kw["steps_per_symbol"], kw["bins_per_tone"])
    assert g.shape == (c["grid_nt"], c["grid_nf"])
    r0, nr = c["grid_rows"]
    assert _sha(g[r0 - c["grid_t0"]: r0 - c["grid_t0"] + nr]) == c["grid_rows_sha256"]
    idx, sc, _ = oracle.select(g, kw["max_candidates"], kw["min_score"])
    t0, NF = c["grid_t0"], c["grid_nf"]
    assert [[int(i // NF) + t0, int(i % NF)] for i in idx] == c["cands"]
    assert np.array_equal(np.asarray(sc, dtype=arr[f"{name}_scores"].dtype), arr[f"{name}_scores"])
    for j, (at, af) in enumerate(c["cands"][:len(arr[f"{name}_llr"])]):
        # (bad_*: a candidate whose symbols touch a NaN frame has an all-NaN LLR vector)
        assert np.array_equal(oracle.llr(mag, kw["steps_per_symbol"], kw["bins_per_tone"], at, af),
                              arr[f"{name}_llr"][j], equal_nan=True)
    got = oracle.decode_ft8_message(x, c["fs"], **kw)
    exp = [(r["payload"], r["crc_calculated"], r["time_sec"], r["freq_hz"], r["score"]) for r in c["results"]]
    assert [(bytes(p).hex(), h, t, f, float(s)) for (p, h, _e, _ce, _cc, t, f, s) in got] == exp


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_stages_on_reference_test_geometry(reft, oracle, gpu, name):
    """Injection: the SHA-pinned reference waterfall through the GPU score / selection / LLR stages."""
    from ft8_demodulator_amd import FT8Waterfall, ft8_extract_likelihood, ft8_find_candidates, ftx_normalize_logl
    cases, arr = reft
    c = cases[name]
    kw = c["kwargs"]
    mag = oracle.waterfall(arr[f"{name}_x"], c["fs"], kw["bins_per_tone"], kw["steps_per_symbol"])
    assert _sha(mag) == c["waterfall_sha256"]
    wf = FT8Waterfall(mag=mag, time_osr=kw["steps_per_symbol"], freq_osr=kw["bins_per_tone"])
    cands = ft8_find_candidates(wf, kw["max_candidates"], kw["min_score"])
    assert [[q.abs_time, q.abs_freq] for q in cands] == c["cands"]
    assert np.array_equal(np.array([q.score for q in cands], dtype=arr[f"{name}_scores"].dtype),
                          arr[f"{name}_scores"])
    for j, q in enumerate(cands[:len(arr[f"{name}_llr"])]):
        v = np.zeros(174)
        ft8_extract_likelihood(wf, q, v)
        ftx_normalize_logl(v)
        assert np.array_equal(v, arr[f"{name}_llr"][j], equal_nan=True), j
    # every candidate's LLRs (GPU) through GPU BP == oracle BP, bit for bit
    from ft8_demodulator_amd import bp_decode
    for q in cands:
        v = np.zeros(174)
        ft8_extract_likelihood(wf, q, v)
        ftx_normalize_logl(v)
        p_gpu, e_gpu = bp_decode(v, kw["max_iterations"])
        p_ref, e_ref = oracle.bp_decode(v, kw["max_iterations"])
        assert e_gpu == e_ref and np.array_equal(p_gpu, p_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_decode_on_reference_test_geometry(reft, gpu, name):
    """End to end: decode_ft8_message on the reference test's input == the reference's results
    (payload, CRCs, LDPC errors, time, frequency exact; score within the STFT tolerance)."""
    from ft8_demodulator_amd import decode_ft8_message
    cases, arr = reft
    c = cases[name]
    got = decode_ft8_message(arr[f"{name}_x"], c["fs"], **c["kwargs"])
    # ref_noise: the reference itself decodes nothing there (its test only prints "Failed to
    # decode"), so the parity is an empty list; ref_6k decodes its payload
    assert len(got) == len(c["results"])
    for (m, s, t, f, sc), r in zip(got, c["results"]):
        assert (m.payload.hex(), m.hash, s.ldpc_errors, s.crc_extracted, s.crc_calculated, t, f) == \
            (r["payload"], r["hash"], r["ldpc_errors"], r["crc_extracted"], r["crc_calculated"], r["time_sec"],
             r["freq_hz"])
        assert type(sc).__name__ == r["score_dtype"]
        # float64 input: a float64 FFT (1e-9); float32: a float32 FFT's rounding (1e-4)
        assert abs(float(sc) - r["score"]) <= (1e-9 if r["score_dtype"] == "float64" else 1e-4)


def test_geometry_follows_the_float_sample_rate():
    """spectrogram_analyse.py:32-34 on the float fs: int(0.16 * 12006.3) = 1921 (not 1920) and
    int(12006.3 / 6.25 * 2) = 3842; fs = 10e3 as a float equals the integer rate."""
    from ft8_demodulator_amd import _lib
    from ft8_demodulator_amd._pipeline import make_plan
    assert _lib.geometry(12006.3, 2, 2, 180000) == (1921, 960, 3842, (180000 - 961) // 960)
    assert _lib.geometry(12006, 2, 2, 180000) == (1920, 960, 3841, (180000 - 960) // 960)
    assert _lib.geometry(10e3, 4, 4, 126400) == _lib.geometry(10000, 4, 4, 126400) == (1600, 400, 6400, 313)
    p = make_plan(180000, 12006.3)
    assert (p.nperseg, p.nfft, p.F) == (1921, 3842, 1921)
    for bad in (0, -1.0, float("nan"), float("inf")):
        with pytest.raises(ValueError):
            _lib.geometry(bad, 2, 2, 1000)


@pytest.mark.gpu
def test_gpu_batch_with_nonfinite_slots(reft, gpu):
    """The bad_* slots and a clean one (ref_fs_frac is another rate, so a synthetic clean slot) in
    ONE SlotDecoder batch: every slot's decodes equal its reference golden -- a NaN / inf slot
    changes nothing in its neighbours (slot isolation through the compact score layout, the
    selection, the LLR gathers and the persistent BP), in any order of the batch."""
    import torch
    from ft8_demodulator_amd import SlotDecoder, decode_ft8_message
    cases, arr = reft
    names = ["bad_nan_tail", "bad_inf_head", "bad_zero_half"]
    clean = np.nan_to_num(arr["bad_nan_tail_x"], nan=0.0).astype(np.float32)
    exp_clean = [(m.payload.hex(), t, f) for (m, _s, t, f, _sc) in
                 decode_ft8_message(clean, 12000, **cases["bad_nan_tail"]["kwargs"])]
    kw = cases[names[0]]["kwargs"]
    dec = SlotDecoder(12000, kw["bins_per_tone"], kw["steps_per_symbol"], kw["max_candidates"], kw["min_score"],
                      kw["max_iterations"])
    for order in ([0, 1, 2, 3], [3, 2, 1, 0], [1, 3, 0, 2]):
        xs = [arr[f"{n}_x"] for n in names] + [clean]
        batch = torch.from_numpy(np.stack([xs[i] for i in order])).cuda()
        got = dec.decode(batch)
        for pos, i in enumerate(order):
            g = [(m.payload.hex(), t, f) for (m, _s, t, f, _sc) in got[pos]]
            if i < 3:
                c = cases[names[i]]
                assert g == [(r["payload"], r["time_sec"], r["freq_hz"]) for r in c["results"]], (order, names[i])
            else:
                assert g == exp_clean, order
