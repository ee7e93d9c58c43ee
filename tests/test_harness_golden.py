"""The oracle against the reference's own harness geometries and its complex I/Q fixture (CPU).

tests/golden/harness.{json,npz} were written by tools/make_golden_harness.py, which imported the
reference in the build container:
  * harness: test_ft8_standard.py:43-68 test_step at every rate of its sweep (2 000 .. 10 000 Hz step
    500; f0 = fc = 0, bins_per_tone = steps_per_symbol = 2, K = 20, min_score 1), three SNRs each.
    The inputs are rebuilt here from their seeds (tests/harness_inputs.py) and must hash to the
    reference's bytes; the oracle's candidate lists, scores and decodes must equal the reference's.
  * channel: src/tests/channel/doppler_shift_test/down_sampled_signal.npy (complex128, 2 kHz) as
    test_decode_after_channel.py:78-115 uses it: the masked spectrogram, decode_ft8_message at the
    defaults ([]), correct_frequency_drift with the test's parameters."""
import numpy as np
import pytest

import harness_inputs as H

META, ARR = H.load()
CASES = META["harness"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_harness(oracle, case):
    kw = case["kwargs"]
    clean, x = H.harness_input(case, oracle)
    assert H.sha(clean) == case["clean_sha256"] and H.sha(x) == case["x_sha256"]
    mag = oracle.waterfall(x, case["fs"], kw["bins_per_tone"], kw["steps_per_symbol"])
    assert list(mag.shape) == case["waterfall_shape"]
    cands, _tie = oracle.find_candidates(mag, kw["steps_per_symbol"], kw["bins_per_tone"], kw["max_candidates"],
                                         kw["min_score"])
    assert [[at, af] for at, af, _ in cands] == case["cands"]
    assert np.array_equal(np.array([s for _, _, s in cands], dtype=np.float64), ARR[f"{case['name']}_scores"])
    got = oracle.decode_ft8_message(x, case["fs"], **kw)
    exp = [(r["payload"], r["crc_calculated"], r["time_sec"], r["freq_hz"], r["score"]) for r in case["results"]]
    assert [(bytes(p).hex(), h, t, f, float(s)) for (p, h, _e, _ce, _cc, t, f, s) in got] == exp


def test_harness_goldens_cover_the_sweep():
    rates = sorted({c["fs"] for c in CASES})
    assert rates == list(range(2000, 10001, 500))
    assert all(c["restated_equal"] for c in CASES)        # the generator restatement is bit-identical
    assert sum(len(c["results"]) for c in CASES) >= 30     # most cases decode; the -17 dB ones mostly not


def test_oracle_matches_reference_channel_fixture(oracle):
    from oracle import drift as OD
    c = META["channel"]
    x = H.channel_input()
    assert x.dtype == np.complex128 and H.sha(x) == c["input_sha256"]
    spec, f, t = oracle.calculate_spectrogram(x, c["fs"], c["bins_per_tone"], c["steps_per_symbol"])
    assert list(spec.shape) == c["spec_shape"] and H.sha(spec) == c["spec_sha256"]
    m = (f >= c["mask_f"][0]) & (f <= c["mask_f"][1])
    assert np.array_equal(spec[m], ARR["channel_spec"]) and np.array_equal(f[m], ARR["channel_f"])
    assert np.array_equal(t, ARR["channel_t"])
    assert c["decode_defaults"] == {"results": []}
    assert oracle.decode_ft8_message(x, c["fs"]) == []
    params = {"nsync_sym": 7, "ndata_sym": 58, "zscore_threshold": 5, "max_iteration_num": 400000,
              "debug_plots": False}
    y, rate = OD.correct_frequency_drift(x, c["fs"], 2, 2, params=params)
    assert abs(float(np.asarray(rate).reshape(-1)[0]) - c["drift"]["rate"]) <= 1e-12 * abs(c["drift"]["rate"])
    ref = ARR["channel_corrected"]
    assert np.max(np.abs(np.asarray(y) - ref)) <= 1e-9 * np.max(np.abs(ref))
