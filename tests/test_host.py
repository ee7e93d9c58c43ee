"""Host-side logic that needs no GPU: spectrogram axes and masks, dtype promotion, result assembly,
WAV reading, the LDPC tables and the transmit chain used for synthesis."""
import json
import os

import numpy as np
import pytest

from conftest import DATA, ROOT


def test_plan_axes_match_reference(golden):
    from ft8_demodulator_amd._pipeline import make_plan, spectrogram_axes
    meta, arr = golden
    for c in meta["stft"]:
        x = arr[f"stft_{c['name']}_x"]
        plan = make_plan(len(x), c["fs"], c["bpt"], c["sps"])
        f, t = spectrogram_axes(c["fs"], plan.nperseg, plan.hop, plan.nfft, len(x))
        assert np.array_equal(np.fft.fftshift(f), arr[f"stft_{c['name']}_f"])
        assert np.array_equal(t, arr[f"stft_{c['name']}_t"])
        assert plan.frames == arr[f"stft_{c['name']}_spec"].shape[1]
        fs_ = np.fft.fftshift(f)
        assert np.array_equal(plan.f, fs_[fs_ >= 0])


def test_masks_are_the_reference_masks():
    from ft8_demodulator_amd._pipeline import make_plan
    n = 252800
    p = make_plan(n, 20000, freq_min=400.0, freq_max=700.0)
    f = np.fft.fftshift(np.fft.fftfreq(6400, 1 / 20000))
    f = f[f >= 0]
    m = (f >= 400.0) & (f <= 700.0)
    assert (p.f_lo, p.f_hi) == (int(np.nonzero(m)[0][0]), int(np.nonzero(m)[0][-1]) + 1)
    p = make_plan(n, 20000, time_min=0.5, time_max=12.0)
    t = np.arange(1600, n - 1600 + 1, 1600) / 20000.0
    m = (t >= 0.5) & (t <= 12.0)
    assert (p.t_lo, p.t_hi) == (int(np.nonzero(m)[0][0]), int(np.nonzero(m)[0][-1]) + 1)
    assert make_plan(n, 20000, freq_min=5000.0, freq_max=4000.0).empty
    assert make_plan(100, 12000).empty


def test_min_score_promotion_rules():
    from ft8_demodulator_amd._pipeline import min_score_is_f64
    assert not min_score_is_f64(10) and not min_score_is_f64(10.2) and not min_score_is_f64(np.float32(3))
    assert min_score_is_f64(np.float64(10.2)) and min_score_is_f64(np.int64(3))
    s = np.float32(10.2)
    assert (s < 10.2) is np.False_ and (s < np.float64(10.2)) is np.True_  # the rule being mirrored


def test_result_assembly():
    from ft8_demodulator_amd import _lib
    from ft8_demodulator_amd._pipeline import records_to_results
    r = np.zeros(1, dtype=_lib.RESULT_DTYPE)
    r["score"] = np.float64(np.float32(29.03573))
    r["abs_time"], r["abs_freq"] = 2, 177
    r["crc_extracted"] = r["crc_calculated"] = 11187
    r["payload"] = np.frombuffer(bytes.fromhex("aa0203040506070809f8"), dtype=np.uint8)
    r["ok"] = 1
    (m, s, t, f, sc), = records_to_results(r, 20000, 2, False)
    assert (m.payload.hex(), m.hash, s.ldpc_errors, s.crc_extracted, t, f) == (
        "aa0203040506070809f8", 11187, 0, 11187, 0.0001, 553.125)
    assert type(sc) is np.float32 and sc == np.float32(29.03573)
    assert _lib.RESULT_DTYPE.itemsize == 40


def test_read_wave_file_semantics():
    import wave
    from ft8_demodulator_amd import read_wave_file
    x, fs = read_wave_file(os.path.join(DATA, "ft8_fs20k_f0_550_id_1.wav"))
    with wave.open(os.path.join(DATA, "ft8_fs20k_f0_550_id_1.wav")) as w:
        raw = np.frombuffer(w.readframes(w.getnframes()), dtype=np.int16)
    ref = raw.astype(np.float32)
    ref /= np.iinfo(np.int16).max
    assert fs == 20000 and x.dtype == np.float32 and np.array_equal(x, ref)


def test_ldpc_tables(oracle):
    from ft8_demodulator_amd import _ldpc_tables as T, constants, synth
    src = open(os.path.join(ROOT, "ft8_demodulator_amd", "csrc", "ft8_ldpc_tables.h")).read()
    assert T.SHA256 in src
    assert len(T.EDGE_VAR) == 522 and T.CHK_START[-1] == 522
    assert sorted(constants.kFTX_LDPC_Num_rows) == [6] * 59 + [7] * 24  # 59*6 + 24*7 = 522 edges
    # every variable in exactly 3 checks, Mn is the transpose of Nm
    for n, row in enumerate(constants.kFTX_LDPC_Mn):
        assert len(set(row)) == 3
        for m in row:
            assert n + 1 in constants.kFTX_LDPC_Nm[m - 1]
    # H * codeword = 0 for codewords of the generator: the two tables describe one code
    rng = np.random.default_rng(1)
    for _ in range(200):
        bits = synth.codeword_bits(synth.random_payload(rng))
        assert oracle.ldpc_check(bits) == 0
        flip = bits.copy()
        flip[rng.integers(0, 174)] ^= 1
        assert oracle.ldpc_check(flip) == 3


def test_tx_known_answers(golden):
    from ft8_demodulator_amd import synth
    meta, _ = golden
    for t in meta["tx"]:
        p = bytes.fromhex(t["payload"])
        assert synth.add_crc(p).hex() == t["a91"]
        assert synth.ldpc_encode(synth.add_crc(p)).hex() == t["codeword"]
        assert "".join(map(str, synth.itones(p))) == t["itones"]


def test_synth_slot_properties():
    from ft8_demodulator_amd import synth
    x, tr = synth.make_slots(2, 3, seed=4)
    assert x.shape == (2, 180000) and x.dtype.is_floating_point
    assert len(tr) == 2 and len(tr[0].payloads) == 3
    for p in tr[0].payloads:
        assert p[9] & 0x07 == 0
    y, _ = synth.make_slots(1, 0, seed=4)
    assert abs(float(y.std()) - 1.0) < 0.01


def test_codeword_bits_batch_matches_scalar(oracle):
    from ft8_demodulator_amd import synth
    rng = np.random.default_rng(9)
    pay = synth.random_payloads(64, rng)
    got = synth.codeword_bits_batch(pay)
    for i in range(64):
        assert np.array_equal(got[i], synth.codeword_bits(bytes(pay[i])))
        assert oracle.ldpc_check(got[i]) == 0


def test_drift_params_host_logic():
    """frequency_correction mirror: default filling mutates the caller's dict like the reference
    (frequency_correction.py:165-171), the C struct carries every field, short inputs return
    before touching the GPU, and the GPU path fails loudly without one (no CPU fallback)."""
    import torch
    from ft8_demodulator_amd import _lib
    from ft8_demodulator_amd import frequency_correction as FC
    p = {"steps_per_symbol": 8}
    out = FC._fill_params(p)
    assert out is p and p["steps_per_symbol"] == 8 and p["poly_degree"] == 2 and p["window_size_factor"] == 4
    c = FC._drift_params(p, 12000, 6.25, 0.16)
    assert (c.sample_rate, c.sym_bin, c.sym_t, c.max_variance_factor) == (12000.0, 6.25, 0.16, 0.0001)
    assert (c.bins_per_tone, c.steps_per_symbol, c.nsync_sym, c.ndata_sym, c.window_size_factor,
            c.fit_middle_percent, c.poly_degree, c.precise_sync) == (2, 8, 7, 58, 4, 100, 2, 1)
    assert ctypes_size(_lib.Ft8DriftParams) == 64 and _lib.DRIFT_RESULT_DTYPE.itemsize == 72
    segs, m = FC.detect_signal_continuity(np.arange(5), window_size=8)
    assert segs == [] and m.shape == (5,)
    if not torch.cuda.is_available():
        import pytest
        with pytest.raises(_lib.Ft8Error):
            FC.correct_frequency_drift(np.zeros(100000, complex), 12000, 6.25, 0.16)


def ctypes_size(t):
    import ctypes
    return ctypes.sizeof(t)
