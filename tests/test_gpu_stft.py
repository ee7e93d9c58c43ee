"""GPU STFT vs the reference's scipy spectrogram (golden vectors).  Not bit-exact (a different FFT
than pocketfft), bounded: |dB error| <= 1e-3 dB where the bin is within 60 dB of the frame peak,
<= 0.25 dB elsewhere for float32 (the reference's own float32 FFT differs from float64 by up to
0.136 dB on weak bins); float64 input: <= 1e-6 dB / 1e-3 dB."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_calculate_spectrogram_matches_reference(golden, gpu):
    from ft8_demodulator_amd import calculate_spectrogram
    meta, arr = golden
    for c in meta["stft"]:
        x = arr[f"stft_{c['name']}_x"]
        spec, f, t = calculate_spectrogram(x, c["fs"], c["bpt"], c["sps"])
        ref = arr[f"stft_{c['name']}_spec"]
        assert spec.dtype == ref.dtype, c["name"]
        assert spec.shape == ref.shape, c["name"]
        assert np.array_equal(f, arr[f"stft_{c['name']}_f"]), c["name"]
        assert np.array_equal(t, arr[f"stft_{c['name']}_t"]), c["name"]
        strong = ref >= (ref.max(axis=0, keepdims=True) - 60.0)
        d = np.abs(spec.astype(np.float64) - ref.astype(np.float64))
        tight, loose = (1e-3, 0.25) if ref.dtype == np.float32 else (1e-6, 1e-3)
        assert d[strong].max() <= tight, (c["name"], d[strong].max())
        assert d.max() <= loose, (c["name"], d.max())


def test_short_input_empty(gpu):
    from ft8_demodulator_amd import calculate_spectrogram
    s, f, t = calculate_spectrogram(np.zeros(10), 12000)
    assert s.shape == (1, 0) and f.size == 0 and t.size == 0


ST, P38, CZ, DFT = 0, 1, 2, 3  # ft8_stft_method: Stockham, packed 3840, chirp-z, direct DFT


@pytest.mark.parametrize("fs,bpt,sps,cplx,dt,method", [
    (32768, 2, 2, False, np.float64, CZ),    # nfft 10485 = 3^2 5 233: odd, a prime factor 233 (reference test rate)
    (32768, 2, 8, True, np.complex128, CZ),  # the reference drift test's geometry
    (32768, 2, 2, False, np.float32, CZ),
    (11025, 3, 2, False, np.float32, ST),    # nfft 5292 = 2^2 3^3 7^2 ... P = 2646 = 2 3^3 7^2: FFT path
    (9973, 1, 2, False, np.float32, CZ),     # prime-ish rate: nfft 1595 = 5 x 11 x 29, odd real
    (9973, 2, 2, True, np.complex64, CZ),    # nfft 3191, a prime
    (12000, 10, 10, False, np.float32, ST),  # nfft 19200: k_stft_sp's 16 x 8 x 15 x 5 plan (P 9600)
    (20000, 2, 2, False, np.float32, ST),    # the bundled recording's rate: k_stft_sp, 16 x 8 x 5 x 5 (P 3200)
    (6000, 2, 2, False, np.float32, ST),     # the reference decode test's 6 kHz: k_stft_sp, 16 x 4 x 15 (P 960)
    (20000, 2, 2, False, np.float64, ST),    # float64 at the same plan: the generic k_stft
    (12000, 5, 2, True, np.complex64, ST),   # complex nfft 9600 in (8192, 10240]: the same variant
    (12000, 2, 2, False, np.float32, P38),   # the production geometry
    (12000, 2, 2, True, np.complex64, ST),   # complex input, nfft 3840: k_stftc3840 dB epilogue (hop 960)
    (12000, 2, 8, True, np.complex64, ST),   # ... hop 240 (the beacon receiver's geometry), float32
    (12000, 2, 8, True, np.complex128, ST),  # ... float64
])
def test_any_fft_length_matches_scipy(gpu, oracle, fs, bpt, sps, cplx, dt, method):
    """Lengths without a 2/3/5/7 factorisation (or odd real nfft) take the chirp-z transform (or the
    direct DFT, where the chirp-z convolution would not fit the LDS FFT); every geometry matches
    scipy within the same tolerances as the golden cases."""
    from ft8_demodulator_amd import _lib, calculate_spectrogram
    code = {np.float32: _lib.FT8_F32, np.float64: _lib.FT8_F64, np.complex64: _lib.FT8_C64,
            np.complex128: _lib.FT8_C128}[dt]
    ctx = _lib.context()
    assert _lib.lib().ft8_stft_method(ctx.handle, fs, bpt, sps, int(0.16 * fs) * 12, code) == method
    rng = np.random.default_rng(fs + sps)
    n = int(0.16 * fs) * 12
    x = rng.normal(size=n) + (1j * rng.normal(size=n) if cplx else 0)
    x = x + 3 * np.exp(2j * np.pi * 1000.0 * np.arange(n) / fs) if cplx else x + 3 * np.cos(2 * np.pi * 1000.0 * np.arange(n) / fs)
    x = x.astype(dt)
    spec, f, t = calculate_spectrogram(x, fs, bpt, sps)
    ref, fr, tr = oracle.calculate_spectrogram(x, fs, bpt, sps)
    assert spec.dtype == ref.dtype and spec.shape == ref.shape
    assert np.array_equal(f, fr) and np.array_equal(t, tr)
    strong = ref >= (ref.max(axis=0, keepdims=True) - 60.0)
    d = np.abs(spec.astype(np.float64) - ref.astype(np.float64))
    tight, loose = (1e-3, 0.25) if ref.dtype == np.float32 else (1e-6, 1e-3)
    assert d[strong].max() <= tight, d[strong].max()
    assert d.max() <= loose, d.max()


@pytest.mark.parametrize("frames", [1, 2, 3, 5, 6, 7, 11, 12, 13, 23, 25])
def test_production_stft_ragged_frame_counts(gpu, oracle, frames):
    """k_stft3840p transforms two frames per pass in runs of 12: runs that end on an odd frame (the
    second frame of the last pass absent) and runs shorter than a chunk match scipy like full ones."""
    from ft8_demodulator_amd import _lib, calculate_spectrogram
    fs, n = 12000, (frames - 1) * 960 + 1920
    ctx = _lib.context()
    assert _lib.lib().ft8_stft_method(ctx.handle, fs, 2, 2, n, _lib.FT8_F32) == P38
    rng = np.random.default_rng(frames)
    x = (rng.normal(size=n) + 3 * np.cos(2 * np.pi * 1234.5 * np.arange(n) / fs)).astype(np.float32)
    spec, f, t = calculate_spectrogram(x, fs, 2, 2)
    ref, fr, tr = oracle.calculate_spectrogram(x, fs, 2, 2)
    assert spec.shape == ref.shape and t.size in spec.shape  # frame counts of both parities across the cases
    strong = ref >= (ref.max(axis=0, keepdims=True) - 60.0)
    d = np.abs(spec.astype(np.float64) - ref.astype(np.float64))
    assert d[strong].max() <= 1e-3, d[strong].max()
    assert d.max() <= 0.25, d.max()


@pytest.mark.parametrize("fs,bpt,sps", [(20000, 2, 2), (12000, 10, 10), (6000, 2, 2), (12000, 2, 2)])
def test_int16_stft_equals_float_of_scaled_samples(gpu, fs, bpt, sps):
    """16-bit PCM into the packed plans (k_stft_pk; k_stft3840p at 12 kHz) reads each sample as
    float32(x) / 32767 (read_wave_file's scaling): the dB rows equal, bit for bit, those of the float32
    path given those floats -- the int16 instantiations transform the same values."""
    from ft8_demodulator_amd import _lib
    import ctypes
    n = int(0.16 * fs) * 20
    nperseg, hop, nfft, T = _lib.geometry(fs, bpt, sps, n)
    F = nfft // 2
    rng = np.random.default_rng(fs + bpt)
    xi = rng.integers(-20000, 20000, size=(2, n)).astype(np.int16)
    xf = (xi.astype(np.float32) / np.float32(32767.0)).astype(np.float32)
    ctx = _lib.context()
    s = gpu.cuda.current_stream().cuda_stream
    p = _lib.Ft8Params(sample_rate=fs, bins_per_tone=bpt, steps_per_symbol=sps, f_lo=0, f_hi=F, t_lo=0, t_hi=T)
    out = []
    for x, code in ((xi, _lib.FT8_I16), (xf, _lib.FT8_F32)):
        t = gpu.from_numpy(x).cuda()
        wf = gpu.empty((2, T, F), dtype=gpu.float32, device="cuda")
        ctx.check(_lib.lib().ft8_stft(ctx.handle, t.data_ptr(), code, n, 2, n, ctypes.byref(p), wf.data_ptr(), s), "stft")
        out.append(wf.cpu().numpy())
    assert np.array_equal(out[0], out[1])
