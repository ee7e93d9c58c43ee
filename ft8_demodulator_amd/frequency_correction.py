"""Mirror of the reference beacon receiver's frequency-drift correction, computed on the GPU.

Reference: src/ft8_tools/ft8_beacon_receiver/frequency_correction.py (gfsk_pulse :27-40,
detect_signal_continuity :42-115, correct_frequency_drift :118-659).  Same names, arguments,
defaults and return values; every numerical step runs in libft8hip.so (csrc/drift.hip and the STFT
kernel's argmax epilogue, include/ft8hip.h ft8_drift_correct / ft8_drift_fit):

  * the two spectrograms are never materialised: the STFT kernel reduces each frame to its argmax;
  * the continuity metric, segment scan, linear fit, sync correlation and polynomial fit run in one
    workgroup per signal; the de-rotations are element-wise float64 kernels.

Differences from the reference: no matplotlib debug plots (`debug_plots` is accepted and ignored;
the reference writes PNG files into the CWD); scikit-learn is not used (LinearRegression is the
centred least-squares solution, computed directly).  `correct_frequency_drift_batch` is the batched
entry point (one call for many independent signals).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._pipeline import device_samples

DEFAULT_PARAMS = {  # frequency_correction.py:150-163
    "nsync_sym": 7,
    "ndata_sym": 58,
    "zscore_threshold": 5,
    "max_iteration_num": 400,
    "debug_plots": True,
    "window_size_factor": 4,
    "max_variance_factor": 0.0001,
    "fit_middle_percent": 100,
    "bins_per_tone": 2,
    "steps_per_symbol": 2,
    "poly_degree": 2,
    "precise_sync": True,
}


def gfsk_pulse(bt, t):
    """frequency_correction.py:27-40 (a host-side helper: the device builds its own template)."""
    from scipy.special import erf
    k = np.pi * np.sqrt(2.0 / np.log(2.0))
    return 0.5 * (erf(k * bt * (np.asarray(t) + 0.5)) - erf(k * bt * (np.asarray(t) - 0.5)))


def _fill_params(params):
    """The reference fills missing keys into the caller's dict (:165-171)."""
    if params is None:
        params = dict(DEFAULT_PARAMS)
    else:
        for k, v in DEFAULT_PARAMS.items():
            if k not in params:
                params[k] = v
    return params


def _drift_params(params, fs, sym_bin, sym_t) -> _lib.Ft8DriftParams:
    p = _lib.Ft8DriftParams()
    if float(fs) != int(fs):
        raise NotImplementedError("the GPU spectrogram needs an integral sample rate")
    p.sample_rate = float(fs)
    p.sym_bin = float(sym_bin)
    p.sym_t = float(sym_t)
    p.max_variance_factor = float(params["max_variance_factor"])
    p.bins_per_tone = int(params["bins_per_tone"])
    p.steps_per_symbol = int(params["steps_per_symbol"])
    p.nsync_sym = int(params["nsync_sym"])
    p.ndata_sym = int(params["ndata_sym"])
    p.window_size_factor = int(params["window_size_factor"])
    fm = params["fit_middle_percent"]
    if int(fm) != fm:
        raise NotImplementedError("fit_middle_percent must be an integer")
    p.fit_middle_percent = int(fm)
    p.poly_degree = int(params["poly_degree"])
    p.precise_sync = int(bool(params["precise_sync"]))
    return p


def detect_signal_continuity(max_freq_indices, window_size=8, max_variance=10.0):
    """frequency_correction.py:42-115 -> (segments [(start, end)], continuity metric), on the GPU
    (ft8_drift_fit stage 1; the PNG of :84-93 is not written)."""
    idx = np.asarray(max_freq_indices)
    n = len(idx)
    if n < window_size:  # :57-58
        return [], np.zeros(n)
    torch = _lib.require_gpu()
    if idx.size and (idx.min() < 0 or idx.max() >= 8192):
        raise ValueError("argmax indices must lie in [0, 8192)")
    ctx = _lib.context()
    dev = torch.device("cuda", ctx.device)
    nwin = n - window_size + 1
    max_seg = nwin // 2 + 1
    d_idx = torch.from_numpy(idx.astype(np.int32)).to(dev)
    d_res = torch.zeros(_lib.DRIFT_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_metric = torch.zeros(nwin, dtype=torch.float64, device=dev)
    d_seg = torch.zeros(max_seg * 2, dtype=torch.int32, device=dev)
    p = _drift_params(dict(DEFAULT_PARAMS, steps_per_symbol=int(window_size), window_size_factor=1,
                           bins_per_tone=1, nsync_sym=1, max_variance_factor=float(max_variance)), 1, 1.0, 1.0)
    s = torch.cuda.current_stream(dev).cuda_stream
    ctx.check(_lib.lib().ft8_drift_fit(ctx.handle, 1, d_idx.data_ptr(), 1, n, 1, ctypes.byref(p), d_res.data_ptr(),
                                       d_metric.data_ptr(), d_seg.data_ptr(), max_seg, s), "ft8_drift_fit")
    r = d_res.cpu().numpy().view(_lib.DRIFT_RESULT_DTYPE)[0]
    nseg = int(r["n_segments"])
    seg = d_seg.cpu().numpy().reshape(-1, 2)[:nseg]
    return [(int(a), int(b)) for a, b in seg], d_metric.cpu().numpy()


def correct_frequency_drift_batch(waves, fs, sym_bin, sym_t, params=None, device=None):
    """Batched correct_frequency_drift: waves [n_signals, n_samples] (NumPy or torch; float32/64,
    complex64/128) -> (corrected complex128 torch tensor [n_signals, n_samples] on the GPU,
    per-signal records of _lib.DRIFT_RESULT_DTYPE)."""
    torch = _lib.require_gpu()
    params = _fill_params(params)
    if isinstance(waves, torch.Tensor):
        x2 = waves if waves.dim() == 2 else waves.reshape(1, -1)
    else:
        a = np.asarray(waves)
        x2 = a if a.ndim == 2 else a.reshape(1, -1)
    n_sig, n = int(x2.shape[0]), int(x2.shape[1])
    x, code, _ = device_samples(x2, device)
    if code == _lib.FT8_I16:
        raise NotImplementedError("int16 input is not a complex baseband signal")
    ctx = _lib.context(x.device)
    out = torch.empty((n_sig, n), dtype=torch.complex128, device=x.device)
    res = torch.zeros(n_sig * _lib.DRIFT_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=x.device)
    p = _drift_params(params, fs, sym_bin, sym_t)
    s = torch.cuda.current_stream(x.device).cuda_stream
    ctx.check(_lib.lib().ft8_drift_correct(ctx.handle, x.data_ptr(), code, n, n_sig, n, ctypes.byref(p),
                                           out.data_ptr(), res.data_ptr(), s), "ft8_drift_correct")
    return out, res.cpu().numpy().view(_lib.DRIFT_RESULT_DTYPE)


def correct_frequency_drift(wave_complex, fs: float, sym_bin: float, sym_t: float, params=None):
    """frequency_correction.py:118-659 -> (corrected signal, estimated drift rate per sample).

    Returns NumPy for NumPy input (complex128, as the reference's carrier multiplication
    promotes) and a GPU tensor for tensor input.  As in the reference: with no continuous segment
    the input object itself and 0.0; after the polynomial stage the rate is a 1-element array."""
    torch = _lib.require_gpu()
    is_tensor = isinstance(wave_complex, torch.Tensor)
    out, res = correct_frequency_drift_batch(wave_complex, fs, sym_bin, sym_t, params)
    r = res[0]
    st = int(r["status"])
    if st == _lib.FT8_DRIFT_VALUE_ERROR:
        raise ValueError("LinearRegression.fit: inconsistent or empty regression inputs (reference raises here)")
    if st == _lib.FT8_DRIFT_NO_SEGMENT:
        return wave_complex, 0.0  # :235-236 returns the caller's array unchanged
    y = out[0] if is_tensor else out[0].cpu().numpy()
    if st == _lib.FT8_DRIFT_FULL:
        return y, np.array([r["rate_per_sample"]], dtype=np.float64)
    return y, np.float64(r["rate_per_sample"])

