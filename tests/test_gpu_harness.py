"""The HIP path on the reference's own harness geometries and its complex I/Q fixture.

tests/golden/harness.* hold the reference's outputs (tools/make_golden_harness.py imported it in the
build container; tests/test_harness_golden.py pins the oracle to the same goldens on the CPU):

  * harness (test_ft8_standard.py:43-68 test_step, every rate of its sweep :70-84): float64 input at
    fs = 2 000 .. 10 000 Hz step 500, f0 = fc = 0 (tones at DC), bins_per_tone = steps_per_symbol =
    2, K = 20, min_score 1.  Four rates have an FFT length with a prime factor above 7 and take the
    chirp-z STFT (5.5 / 6.5 / 8.5 / 9.5 kHz: P = 880 / 1 040 / 1 360 / 1 520 = 16 * 5 * 11/13/17/19),
    the others the LDS Stockham plans.  Checked: the transform each rate runs, the GPU waterfall's
    candidate list and scores against the reference's (the reference's own waterfall), and
    decode_ft8_message end to end (payload, CRCs, LDPC errors, time, frequency exact; float64 scores
    within 1e-9).
  * channel (test_decode_after_channel.py:78-115 on down_sampled_signal.npy, complex128, 2 kHz):
    calculate_spectrogram's 0-300 Hz rows within the float64 STFT tolerance, decode_ft8_message at
    the defaults (the reference decodes nothing), correct_frequency_drift with the test's parameters
    (rate and corrected wave)."""
import numpy as np
import pytest

import harness_inputs as H

pytestmark = pytest.mark.gpu

META, ARR = H.load()
CASES = META["harness"]
ST, P38, CZ, DFT = 0, 1, 2, 3  # ft8_stft_method: Stockham, packed 3840, chirp-z, direct DFT
CHIRP_Z_RATES = {5500, 6500, 8500, 9500}


@pytest.mark.parametrize("fs", sorted({c["fs"] for c in CASES}))
def test_stft_method_per_harness_rate(gpu, fs):
    from ft8_demodulator_amd import _lib
    n = next(c["n"] for c in CASES if c["fs"] == fs)
    m = _lib.lib().ft8_stft_method(_lib.context().handle, fs, 2, 2, n, _lib.FT8_F64)
    assert m == (CZ if fs in CHIRP_Z_RATES else ST), (fs, m)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_matches_reference_harness(gpu, oracle, case):
    from ft8_demodulator_amd import FT8Waterfall, calculate_spectrogram, decode_ft8_message, ft8_find_candidates
    kw = case["kwargs"]
    clean, x = H.harness_input(case, oracle)
    assert H.sha(x) == case["x_sha256"], "the rebuilt input differs from the reference's bytes"
    # the GPU's own waterfall -> GPU selection == the reference's candidates on its waterfall
    spec, f, _t = calculate_spectrogram(x, case["fs"], kw["bins_per_tone"], kw["steps_per_symbol"])
    mag = np.ascontiguousarray(spec[f >= 0])
    assert list(mag.shape) == case["waterfall_shape"]
    wf = FT8Waterfall(mag=mag, time_osr=kw["steps_per_symbol"], freq_osr=kw["bins_per_tone"])
    cands = ft8_find_candidates(wf, kw["max_candidates"], kw["min_score"])
    assert [[q.abs_time, q.abs_freq] for q in cands] == case["cands"]
    assert np.allclose([float(q.score) for q in cands], ARR[f"{case['name']}_scores"], rtol=0, atol=1e-9)
    # end to end, samples on the device
    got = decode_ft8_message(x, case["fs"], **kw)
    assert len(got) == len(case["results"]), (len(got), case["results"])
    for (m, s, t, fq, sc), r in zip(got, case["results"]):
        assert (m.payload.hex(), m.hash, s.ldpc_errors, s.crc_extracted, s.crc_calculated, t, fq) == \
            (r["payload"], r["hash"], r["ldpc_errors"], r["crc_extracted"], r["crc_calculated"], r["time_sec"],
             r["freq_hz"])
        assert type(sc).__name__ == r["score_dtype"] and abs(float(sc) - r["score"]) <= 1e-9


def test_gpu_batch_matches_reference_harness(gpu, oracle):
    """All cases of one rate decoded as one batch (SlotDecoder, float64) give the same decodes."""
    import torch
    from ft8_demodulator_amd import _lib
    from ft8_demodulator_amd._pipeline import SlotDecoder
    for fs in sorted({c["fs"] for c in CASES}):
        cs = [c for c in CASES if c["fs"] == fs]
        x = torch.from_numpy(np.stack([H.harness_input(c, oracle)[1] for c in cs])).cuda()
        kw = cs[0]["kwargs"]
        dec = SlotDecoder(fs, kw["bins_per_tone"], kw["steps_per_symbol"], kw["max_candidates"], kw["min_score"],
                          kw["max_iterations"])
        recs = dec.records(x, _lib.FT8_F64)
        for c, r in zip(cs, recs):
            assert [bytes(p).hex() for p in r["payload"]] == [e["payload"] for e in c["results"]], c["name"]


def test_gpu_channel_fixture_spectrogram_and_decode(gpu):
    from ft8_demodulator_amd import calculate_spectrogram, decode_ft8_message
    c = META["channel"]
    x = H.channel_input()
    assert H.sha(x) == c["input_sha256"]
    spec, f, t = calculate_spectrogram(x, c["fs"], c["bins_per_tone"], c["steps_per_symbol"])
    assert list(spec.shape) == c["spec_shape"] and spec.dtype == np.float64
    m = (f >= c["mask_f"][0]) & (f <= c["mask_f"][1])
    assert np.array_equal(f[m], ARR["channel_f"]) and np.array_equal(t, ARR["channel_t"])
    ref = ARR["channel_spec"]
    d = np.abs(spec[m] - ref)
    strong = ref >= ref.max(axis=0, keepdims=True) - 60.0
    assert d[strong].max() <= 1e-6 and d.max() <= 1e-3, (d[strong].max(), d.max())
    assert decode_ft8_message(x, c["fs"]) == []


def test_gpu_channel_fixture_drift_correction(gpu):
    from ft8_demodulator_amd.frequency_correction import correct_frequency_drift
    c = META["channel"]
    x = H.channel_input()
    params = {"nsync_sym": 7, "ndata_sym": 58, "zscore_threshold": 5, "max_iteration_num": 400000,
              "debug_plots": False}
    y, rate = correct_frequency_drift(x, c["fs"], 2, 2, params=params)
    assert abs(float(np.asarray(rate).reshape(-1)[0]) - c["drift"]["rate"]) <= 1e-9 * abs(c["drift"]["rate"])
    ref = ARR["channel_corrected"]
    y = np.asarray(y)
    assert y.shape == ref.shape and y.dtype == np.complex128
    assert np.max(np.abs(y - ref)) <= 1e-9 * np.max(np.abs(ref))


def test_gpu_sensitivity_points_match_reference(gpu, oracle):
    """The reference's own sensitivity harness (test_ft8_standard.py:43-123) at seven of its rates,
    run here with the reference deciding success (tools/make_golden_sensitivity.py ->
    tests/golden/sensitivity_ref.json, 20 seeded rounds per SNR point): the GPU decodes the same
    float64 inputs and reaches the same verdict on every slot -- so the GPU sweep's thresholds
    (bench.py `sensitivity`) are the reference decoder's."""
    import json
    import os
    import torch
    from conftest import GOLD
    from ft8_demodulator_amd import _lib
    from ft8_demodulator_amd._pipeline import SlotDecoder
    path = os.path.join(GOLD, "sensitivity_ref.json")
    if not os.path.exists(path):
        pytest.skip("tests/golden/sensitivity_ref.json not generated")
    with open(path) as f:
        ref = json.load(f)
    kw = ref["kwargs"]
    for pt in ref["points"]:
        cases = [{"seed": s, "fs": pt["fs"], "snr_db": pt["snr_db"]} for s in pt["seeds"]]
        xs = []
        for c in cases:
            rng = np.random.default_rng(c["seed"])
            payload = rng.integers(0, 256, size=10, dtype=np.uint8)
            clean = np.real(oracle.gfsk_waveform(oracle.tx_itones(bytes(payload)), c["fs"], 0.0, style=1))
            noise = np.sqrt(np.mean(clean ** 2) / (10 ** (c["snr_db"] / 10))) * rng.standard_normal(len(clean))
            xs.append(clean + noise)
        dec = SlotDecoder(pt["fs"], kw["bins_per_tone"], kw["steps_per_symbol"], kw["max_candidates"],
                          kw["min_score"], kw["max_iterations"])
        recs = dec.records(torch.from_numpy(np.stack(xs)).cuda(), _lib.FT8_F64)
        got = [len(r) > 0 for r in recs]
        assert got == pt["success"], (pt["fs"], pt["snr_db"], got, pt["success"])
