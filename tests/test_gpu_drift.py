"""Frequency-drift correction on the GPU (csrc/drift.hip + the STFT argmax epilogue) against the
reference's outputs (tests/golden/drift.*, pinned by tools/make_golden_drift.py) and the oracle
(oracle/drift.py, itself checked against those goldens in test_drift_oracle.py).

Tolerances: per-frame argmax indices, segments, statuses and sync indices exact; continuity metric
1e-9 absolute (the kernel evaluates it exactly in integers, the reference in floating point);
rates 1e-9 relative (closed-form least squares vs scikit-learn's SVD solver); corrected waveform
16 ulp(theta_max) x max|x| absolute: the carrier phase theta = pi rate n^2 / fs reaches 1e6..3e6
rad (one float64 ulp there is 1.2e-10..4.7e-10 rad), and the device's sincos / pow and NumPy's
complex exp / power each round the phase and the carrier differently."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu



def _full(params):
    from oracle import drift as OD
    p = dict(OD.DEFAULT_PARAMS)
    p.update(params or {})
    return p


def test_stft_argmax_equals_argmax_of_waterfall(gpu):
    """The fused epilogue picks np.argmax (first maximum) of the dB row ft8_stft writes."""
    from ft8_demodulator_amd import _lib
    import ctypes
    rng = np.random.default_rng(5)
    for dtype, fs, sps in ((np.complex128, 12000, 8), (np.complex64, 6000, 4), (np.float64, 12000, 8),
                           (np.float32, 12000, 2)):
        n = int(0.16 * fs) * 20
        x = rng.normal(size=(3, n))
        if np.iscomplexobj(np.zeros(1, dtype)):
            x = x + 1j * rng.normal(size=(3, n))
        x = x.astype(dtype)
        # a constant tone in part of the slot makes long runs of equal argmax
        x[:, : n // 2] += (5 * np.cos(2 * np.pi * 700 * np.arange(n // 2) / fs)).astype(x.real.dtype)
        ctx = _lib.context()
        nperseg, hop, nfft, T = _lib.geometry(fs, 2, sps, n)
        F = (nfft + 1) // 2
        t = gpu.from_numpy(x).cuda()
        code = {np.complex128: 3, np.complex64: 2, np.float64: 1, np.float32: 0}[dtype]
        p = _lib.Ft8Params(sample_rate=fs, bins_per_tone=2, steps_per_symbol=sps, f_lo=0, f_hi=F, t_lo=0, t_hi=T)
        f64 = code in (1, 3)
        wf = gpu.empty((3, T, F), dtype=gpu.float64 if f64 else gpu.float32, device="cuda")
        idx = gpu.empty((3, T), dtype=gpu.int32, device="cuda")
        s = gpu.cuda.current_stream().cuda_stream
        ctx.check(_lib.lib().ft8_stft(ctx.handle, t.data_ptr(), code, n, 3, n, ctypes.byref(p), wf.data_ptr(), s), "stft")
        ctx.check(_lib.lib().ft8_stft_argmax(ctx.handle, t.data_ptr(), code, n, 3, n, ctypes.byref(p), idx.data_ptr(), s),
                  "argmax")
        assert np.array_equal(idx.cpu().numpy(), np.argmax(wf.cpu().numpy(), axis=2)), (dtype, fs, sps)


def test_screened_complex128_argmax_equals_float64(gpu):
    """complex128 STFT-argmax at the 3840-point geometry decides frames in float32 where its error
    bound settles them and redoes the rest in float64 (round 4): the result equals np.argmax of the
    float64 dB rows on frames built to defeat the screen -- all-zero stretches (every level equal),
    tones exactly between two bins and a pair of equal-power tones (near-equal top levels), a tone
    far below the 1e-12 floor, huge amplitudes -- and plain noise; the split is reported."""
    from ft8_demodulator_amd import _lib
    import ctypes
    fs, sps, n = 12000, 8, 1920 * 40
    nperseg, hop, nfft, T = _lib.geometry(fs, 2, sps, n)
    F = (nfft + 1) // 2
    rng = np.random.default_rng(77)
    tt = np.arange(n) / fs
    x = np.zeros((5, n), np.complex128)
    x[0] = rng.normal(size=n) + 1j * rng.normal(size=n)                     # noise
    x[1, n // 3:] = np.exp(2j * np.pi * (1000.0 + 6.25 / 2 * 0.5) * tt[n // 3:])  # between bins, then silence before
    x[2] = np.exp(2j * np.pi * 500.0 * tt) + np.exp(2j * np.pi * 1500.0 * tt)   # two equal tones
    x[2] += 1e-3 * (rng.normal(size=n) + 1j * rng.normal(size=n))
    x[3] = 1e-9 * np.exp(2j * np.pi * 800.0 * tt)                               # below the level floor
    x[4] = 1e150 * (rng.normal(size=n) + 1j * rng.normal(size=n))               # float32 overflows
    ctx = _lib.context()
    p = _lib.Ft8Params(sample_rate=fs, bins_per_tone=2, steps_per_symbol=sps, f_lo=0, f_hi=F, t_lo=0, t_hi=T)
    s = gpu.cuda.current_stream().cuda_stream
    redone = []
    # one slot per call, so the split is known per kind of input
    for k in range(5):
        t = gpu.from_numpy(x[k:k + 1].copy()).cuda()
        wf = gpu.empty((1, T, F), dtype=gpu.float64, device="cuda")
        idx = gpu.empty((1, T), dtype=gpu.int32, device="cuda")
        ctx.check(_lib.lib().ft8_stft(ctx.handle, t.data_ptr(), _lib.FT8_C128, n, 1, n, ctypes.byref(p), wf.data_ptr(), s),
                  "stft")
        ctx.check(_lib.lib().ft8_stft_argmax(ctx.handle, t.data_ptr(), _lib.FT8_C128, n, 1, n, ctypes.byref(p),
                                             idx.data_ptr(), s), "argmax")
        got, want = idx.cpu().numpy()[0], np.argmax(wf.cpu().numpy()[0], axis=1)
        assert np.array_equal(got, want), (k, np.flatnonzero(got != want)[:5])
        r, fr = ctypes.c_int64(), ctypes.c_int64()
        ctx.check(_lib.lib().ft8_stft_screen_stats(ctx.handle, ctypes.byref(r), ctypes.byref(fr)), "stats")
        assert fr.value == T
        redone.append(r.value)
    print("frames redone in float64 per slot (of %d):" % T, redone)
    silent = (n // 3 - nperseg) // hop + 1
    assert redone[0] <= T // 20                 # noise: float32 settles almost every frame
    assert redone[1] >= silent                  # all-zero frames: every level equal
    assert redone[4] == T                       # float32 overflows
    assert redone[2] < T                        # equal tones: the noise separates most frames


def test_argmax_matches_reference_goldens(gpu, drift_golden, drift_inputs):
    from ft8_demodulator_amd import _lib
    import ctypes
    meta, arr = drift_golden
    for c in meta["cases"]:
        p = _full(c["params"])
        x = drift_inputs[c["name"]]
        n = len(x)
        _, _, nfft, T = _lib.geometry(c["fs"], p["bins_per_tone"], p["steps_per_symbol"], n)
        sp = _lib.Ft8Params(sample_rate=c["fs"], bins_per_tone=p["bins_per_tone"], steps_per_symbol=p["steps_per_symbol"],
                            f_lo=0, f_hi=(nfft + 1) // 2, t_lo=0, t_hi=T)
        ctx = _lib.context()
        t = gpu.from_numpy(x).cuda()
        idx = gpu.empty(T, dtype=gpu.int32, device="cuda")
        ctx.check(_lib.lib().ft8_stft_argmax(ctx.handle, t.data_ptr(), _lib.FT8_C128, n, 1, n, ctypes.byref(sp),
                                             idx.data_ptr(), gpu.cuda.current_stream().cuda_stream), "argmax")
        got, want = idx.cpu().numpy(), arr[f"{c['name']}/argmax1"]
        # the FFT is not pocketfft: only a frame whose two largest bins are within rounding may differ
        assert np.mean(got == want) >= 0.995, (c["name"], np.flatnonzero(got != want)[:10])


def test_detect_signal_continuity_vs_oracle(gpu):
    from ft8_demodulator_amd import frequency_correction as FC
    from oracle import drift as OD
    rng = np.random.default_rng(3)
    for trial in range(6):
        T = int(rng.integers(20, 3000))
        idx = rng.integers(0, 1920, T)
        for _ in range(int(rng.integers(1, 5))):  # straight runs (signal) inside noise
            a = int(rng.integers(0, T - 10))
            b = min(T, a + int(rng.integers(10, 400)))
            idx[a:b] = np.clip(300 + (np.arange(b - a) * rng.uniform(-2, 2)).astype(int) + rng.integers(-1, 2, b - a), 0, 1919)
        for w, mv in ((8, 368.64), (32, 368.64), (16, 10.0), (64, 1e4)):
            segs, m = FC.detect_signal_continuity(idx, window_size=w, max_variance=mv)
            s2, m2 = OD.detect_signal_continuity(idx, window_size=w, max_variance=mv)
            assert segs == [tuple(map(int, s)) for s in s2], (trial, w)
            assert np.allclose(m, m2, rtol=1e-9, atol=1e-9), (trial, w)
    assert FC.detect_signal_continuity(np.arange(5), window_size=8)[0] == []


def test_correct_frequency_drift_goldens(gpu, drift_golden, drift_inputs):
    from ft8_demodulator_amd import frequency_correction as FC
    meta, arr = drift_golden
    for c in meta["cases"]:
        nm = c["name"]
        x = drift_inputs[nm]
        params = dict(c["params"]) if c["params"] else None
        y, rate = FC.correct_frequency_drift(x, c["fs"], 6.25, 0.16, params=params)
        if c["status"] == 1:
            assert y is x and rate == 0.0, nm
            continue
        assert isinstance(rate, np.ndarray) == c["rate_is_array"], nm
        r = float(np.asarray(rate).reshape(-1)[0])
        assert abs(r - c["rate_per_sample"]) <= 1e-9 * abs(c["rate_per_sample"]), (nm, r, c["rate_per_sample"])
        assert y.dtype == np.complex128 and y.shape == x.shape
        err = np.max(np.abs(y[::meta["subsample_stride"]] - arr[f"{nm}/corrected_sub"]))
        theta_max = np.pi * abs(c["rate_per_sample"]) * len(x) ** 2 / c["fs"]
        tol = 16 * theta_max * 2.0 ** -52 * np.max(np.abs(x)) + 1e-12
        assert err < tol, (nm, err, tol)


def test_stages_vs_oracle_trace(gpu, drift_golden, drift_inputs):
    """Per-signal records (status, segments, sync index, fit) against the oracle's trace."""
    from ft8_demodulator_amd import frequency_correction as FC
    from oracle import drift as OD
    meta, _ = drift_golden
    for c in meta["cases"]:
        tr = {}
        OD.correct_frequency_drift(drift_inputs[c["name"]], c["fs"], 6.25, 0.16, params=c["params"], trace=tr)
        _, res = FC.correct_frequency_drift_batch(drift_inputs[c["name"]], c["fs"], 6.25, 0.16,
                                                  params=dict(c["params"]) if c["params"] else None)
        r = res[0]
        assert int(r["status"]) == tr["status"], c["name"]
        if tr["status"] == 1:
            continue
        longest = max(tr["segments"], key=lambda s: s[1] - s[0])
        assert (int(r["seg_start"]), int(r["seg_end"])) == tuple(longest)
        assert int(r["n_segments"]) == len(tr["segments"])
        assert abs(r["rate1"] - tr["rate1"]) <= 1e-9 * abs(tr["rate1"])
        if "sync_idx" in tr:
            assert int(r["sync_idx"]) == tr["sync_idx"], c["name"]
        if "coef2" in tr:
            assert np.allclose(r["coef"][1:len(tr["coef2"])], tr["coef2"][1:], rtol=1e-7, atol=1e-12), c["name"]


def test_batch_equals_single_and_dtypes(gpu, drift_golden, drift_inputs):
    from ft8_demodulator_amd import frequency_correction as FC
    meta, _ = drift_golden
    cs = [c for c in meta["cases"] if c["fs"] == 12000 and (c["params"] or {}).get("steps_per_symbol") == 8
          and c["params"].get("precise_sync", True)][:4]
    X = np.stack([drift_inputs[c["name"]] for c in cs])
    p = dict(cs[0]["params"])
    outb, resb = FC.correct_frequency_drift_batch(X, 12000, 6.25, 0.16, params=p)
    for i in range(len(cs)):
        o1, r1 = FC.correct_frequency_drift_batch(X[i], 12000, 6.25, 0.16, params=p)
        assert gpu.equal(o1[0], outb[i]) and r1[0].tobytes() == resb[i].tobytes()
    # a torch tensor in -> a GPU tensor out, identical values
    yt, rt = FC.correct_frequency_drift(gpu.from_numpy(X[0]).cuda(), 12000, 6.25, 0.16, params=dict(p))
    assert yt.is_cuda and gpu.equal(yt, outb[0])
    # complex64 input: the first spectrogram in float32, results close to the complex128 run
    y64, r64 = FC.correct_frequency_drift(X[0].astype(np.complex64), 12000, 6.25, 0.16, params=dict(p))
    assert abs(float(np.asarray(r64).reshape(-1)[0]) - float(resb[0]["rate_per_sample"])) < 1e-3 * abs(resb[0]["rate_per_sample"])


def test_decode_after_correction(gpu, drift_golden, drift_inputs):
    """The reference test's end-to-end check (test_correction.py:300-330): the corrected signal
    decodes (here with the GPU decoder) while the drifting one does not."""
    from ft8_demodulator_amd import frequency_correction as FC
    from ft8_demodulator_amd.ft8_decode import decode_ft8_message
    meta, _ = drift_golden
    for c in meta["cases"]:
        if c["status"] != 5 or c["fs"] not in (12000, 32768):
            continue
        x = drift_inputs[c["name"]]
        y, _ = FC.correct_frequency_drift(x, c["fs"], 6.25, 0.16, params=dict(c["params"]) if c["params"] else None)
        want = bytearray(bytes.fromhex(c["payload"]))
        want[9] &= 0xF8
        got = decode_ft8_message(np.real(y), c["fs"], 2, 2, 100, 6, 40, time_min=10)
        assert any(m.payload == want for m, *_ in got), c["name"]
        assert not decode_ft8_message(np.real(x), c["fs"], 2, 2, 100, 6, 40, time_min=10), c["name"]


def test_errors(gpu):
    from ft8_demodulator_amd import frequency_correction as FC
    with pytest.raises(ValueError):
        FC.correct_frequency_drift(np.zeros(100, complex), 12000, 6.25, 0.16)  # shorter than one symbol
    with pytest.raises(ValueError):
        FC.correct_frequency_drift(np.zeros(100000, complex), 12000, 6.25, 0.16,
                                   params={"steps_per_symbol": 32})  # window 128 > 64
    with pytest.raises(NotImplementedError):
        FC.correct_frequency_drift(np.zeros(100000, complex), 12000.5, 6.25, 0.16)


def test_reference_test_configuration(gpu, drift_golden, drift_inputs):
    """test_correction.py's own setup (32 768 Hz, 568 Hz/s, steps_per_symbol 8): nfft 10 485 runs
    the direct-DFT STFT; the estimated rate matches the reference's and the result decodes."""
    from ft8_demodulator_amd import frequency_correction as FC
    meta, arr = drift_golden
    c = [c for c in meta["cases"] if c["name"] == "fs32k_reference_test"][0]
    x = drift_inputs[c["name"]]
    y, rate = FC.correct_frequency_drift(x, 32768, 6.25, 0.16, params=dict(c["params"]))
    assert abs(float(rate[0]) - c["rate_per_sample"]) <= 1e-9 * c["rate_per_sample"]
    # drift estimate error of the reference test (test_correction.py:294): < 1 Hz over the signal
    assert abs((float(rate[0]) - 568.0 / 32768) * len(x)) < 5000.0
