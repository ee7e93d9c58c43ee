"""ctypes binding of libft8hip.so (include/ft8hip.h) and the device/stream plumbing.

The library is the product: every numeric stage of the receive path runs in its HIP kernels.  If
the library or a ROCm GPU is missing, every entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FT8HIP_LIB", os.path.join(_HERE, "lib", "libft8hip.so"))

FT8_F32, FT8_F64, FT8_C64, FT8_C128, FT8_I16 = 0, 1, 2, 3, 4
FT8_OK, FT8_E_ARG, FT8_E_HIP, FT8_E_UNSUPPORTED, FT8_E_NOMEM, FT8_E_RANGE = 0, -1, -2, -3, -4, -5
FT8_FLAG_TOPK, FT8_FLAG_SUBTRACT = 1, 2
FT8_TX_PROTOCOL, FT8_TX_REFERENCE = 0, 1
FT8_STFT_STOCKHAM, FT8_STFT_PACKED3840, FT8_STFT_CHIRPZ, FT8_STFT_DFT = 0, 1, 2, 3
N_STAGES = 12
STAGE_NAMES = ("stft", "score", "select", "bp", "compact", "decode_batch", "llr", "sub_est",
               "drift_stft_argmax", "drift_fit", "drift_derotate", "sub_apply")
# ft8_drift_status
(FT8_DRIFT_PENDING, FT8_DRIFT_NO_SEGMENT, FT8_DRIFT_LINEAR, FT8_DRIFT_FEW_POINTS, FT8_DRIFT_DEGREE,
 FT8_DRIFT_FULL, FT8_DRIFT_UNDERDETERMINED) = range(7)
FT8_DRIFT_VALUE_ERROR = -1


class Ft8Params(ctypes.Structure):
    _fields_ = [("sample_rate", ctypes.c_int32), ("bins_per_tone", ctypes.c_int32),
                ("steps_per_symbol", ctypes.c_int32), ("max_candidates", ctypes.c_int32),
                ("max_iterations", ctypes.c_int32), ("min_score_f64", ctypes.c_int32),
                ("min_score", ctypes.c_double), ("f_lo", ctypes.c_int32), ("f_hi", ctypes.c_int32),
                ("t_lo", ctypes.c_int32), ("t_hi", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("sample_rate_hz", ctypes.c_double)]


class Ft8DriftParams(ctypes.Structure):
    _fields_ = [("sample_rate", ctypes.c_double), ("sym_bin", ctypes.c_double), ("sym_t", ctypes.c_double),
                ("max_variance_factor", ctypes.c_double), ("bins_per_tone", ctypes.c_int32),
                ("steps_per_symbol", ctypes.c_int32), ("nsync_sym", ctypes.c_int32), ("ndata_sym", ctypes.c_int32),
                ("window_size_factor", ctypes.c_int32), ("fit_middle_percent", ctypes.c_int32),
                ("poly_degree", ctypes.c_int32), ("precise_sync", ctypes.c_int32)]


# ft8_drift_result (72 bytes)
DRIFT_RESULT_DTYPE = np.dtype({
    "names": ["rate_per_sample", "rate1", "coef", "intercept", "status", "n_segments", "seg_start", "seg_end",
              "sync_idx", "n_points"],
    "formats": ["<f8", "<f8", ("<f8", (3,)), "<f8", "<i4", "<i4", "<i4", "<i4", "<i4", "<i4"],
    "offsets": [0, 8, 16, 40, 48, 52, 56, 60, 64, 68],
    "itemsize": 72,
})

# ft8_result (40 bytes) as a NumPy structured dtype
RESULT_DTYPE = np.dtype({
    "names": ["score", "slot", "abs_time", "abs_freq", "crc_extracted", "crc_calculated",
              "ldpc_errors", "cand_index", "payload", "ok", "pass_index"],
    "formats": ["<f8", "<i4", "<i4", "<i4", "<u2", "<u2", "<i2", "<u2", ("u1", (10,)), "u1", "u1"],
    "offsets": [0, 8, 12, 16, 20, 22, 24, 26, 28, 38, 39],
    "itemsize": 40,
})

# ft8_sub_fit (1056 bytes)
SUB_FIT_DTYPE = np.dtype({
    "names": ["active", "start", "f0", "amp", "phase0", "tones"],
    "formats": ["<i4", "<i8", "<f8", ("<f4", (79, 2)), ("<f4", (80,)), ("u1", (80,))],
    "offsets": [0, 8, 16, 24, 656, 976],
    "itemsize": 1056,
})

# ft8_tx_signal (40 bytes)
TX_SIGNAL_DTYPE = np.dtype({
    "names": ["f0", "amplitude", "phase", "start", "slot", "reserved"],
    "formats": ["<f8", "<f8", "<f8", "<i8", "<i4", "<i4"],
    "offsets": [0, 8, 16, 24, 32, 36],
    "itemsize": 40,
})

_lib = None
_lock = threading.Lock()
_tls = threading.local()


class Ft8Error(RuntimeError):
    pass


def lib():
    """Load libft8hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise Ft8Error(
                f"libft8hip.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        P = ctypes.POINTER(Ft8Params)
        DP = ctypes.POINTER(Ft8DriftParams)
        sig = {
            "ft8_create": ([ctypes.c_int, ctypes.POINTER(vp)], ctypes.c_int),
            "ft8_destroy": ([vp], ctypes.c_int),
            "ft8_last_error": ([vp], ctypes.c_char_p),
            "ft8_abi_version": ([], ctypes.c_int),
            "ft8_limits": ([vp, vp, vp], ctypes.c_int),
            "ft8_geometry": ([i32, i32, i32, i64, vp, vp, vp, vp], ctypes.c_int),
            "ft8_geometry_hz": ([dbl, i32, i32, i64, vp, vp, vp, vp], ctypes.c_int),
            "ft8_stft": ([vp, vp, ctypes.c_int, i64, i32, i64, P, vp, vp], ctypes.c_int),
            "ft8_sync_select": ([vp, vp, ctypes.c_int, i32, i32, i32, P, vp, vp, vp, vp, vp], ctypes.c_int),
            "ft8_llr": ([vp, vp, ctypes.c_int, i32, i32, i32, i32, vp, i32, ctypes.c_int, vp, vp], ctypes.c_int),
            "ft8_normalize": ([vp, vp, i32, vp, vp], ctypes.c_int),
            "ft8_bp": ([vp, vp, i32, i32, vp, vp, vp], ctypes.c_int),
            "ft8_decode_batch": ([vp, vp, ctypes.c_int, i64, i32, i64, P, vp, vp, i32, vp], ctypes.c_int),
            "ft8_select_warnings": ([vp, vp, i32, vp], ctypes.c_int),
            "ft8_crc14": ([vp, vp, vp, i32, vp, vp], ctypes.c_int),
            "ft8_ldpc_check": ([vp, vp, i32, vp, vp], ctypes.c_int),
            "ft8_set_timing": ([vp, ctypes.c_int], ctypes.c_int),
            "ft8_get_timing": ([vp, vp, vp, ctypes.c_int], ctypes.c_int),
            "ft8_get_counters": ([vp, vp, ctypes.c_int], ctypes.c_int),
            "ft8_get_bp_clock": ([vp, vp, ctypes.c_int], ctypes.c_int),
            "ft8_set_pipeline": ([vp, i32, i32, i32], ctypes.c_int),
            "ft8_encode": ([vp, vp, i32, i32, vp, vp, vp, vp], ctypes.c_int),
            "ft8_synthesize": ([vp, vp, vp, i32, i32, i32, vp, ctypes.c_int, i64, i32, i64, vp], ctypes.c_int),
            "ft8_subtract": ([vp, vp, ctypes.c_int, vp, i64, i32, i64, P, vp, vp, i32, vp], ctypes.c_int),
            "ft8_stft_argmax": ([vp, vp, ctypes.c_int, i64, i32, i64, P, vp, vp], ctypes.c_int),
            "ft8_drift_fit": ([vp, i32, vp, i32, i32, i32, DP, vp, vp, vp, i32, vp], ctypes.c_int),
            "ft8_drift_correct": ([vp, vp, ctypes.c_int, i64, i32, i64, DP, vp, vp, vp], ctypes.c_int),
            "ft8_build_id": ([], ctypes.c_char_p),
            "ft8_build_flags": ([], ctypes.c_char_p),
            "ft8_replay_stage": ([vp, i32, i32, vp], ctypes.c_int),
            "ft8_set_timing_stages": ([vp, ctypes.c_uint32], ctypes.c_int),
            "ft8_sync_score": ([vp, vp, ctypes.c_int, i32, i32, i32, i32, vp, i32, vp, vp, vp], ctypes.c_int),
            "ft8_pack_bytes": ([i32, i32], i64),
            "ft8_subtract_fits": ([vp, vp, i32, i32, vp], ctypes.c_int),
            "ft8_stft_method": ([vp, i32, i32, i32, i64, ctypes.c_int], ctypes.c_int),
            "ft8_stft_screen_stats": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i64)], ctypes.c_int),
            "ft8_pack_decodes": ([vp, vp, vp, i32, i32, i32, i32, vp, vp, vp], ctypes.c_int),
        }
        stale_ok = os.environ.get("FT8HIP_ALLOW_STALE") == "1"
        for name, (args, res) in sig.items():
            if stale_ok and not hasattr(L, name):
                continue  # an older build under A/B (tools/build_ref_variant.sh): entry points it predates
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _ = dbl
        built, want = L.ft8_build_id().decode(), source_hash()
        # FT8HIP_ALLOW_STALE=1: A/B tooling only (tools/ab_variants.py loads older builds on purpose)
        if want is not None and built != want and os.environ.get("FT8HIP_ALLOW_STALE") != "1":
            raise Ft8Error(
                f"stale {LIB_PATH}: built from sources {built}, the tree holds {want}; rebuild with "
                "`python -c 'import __graft_entry__ as g; g.build()'`")
        _lib = L
    return _lib


# csrc files hashed into FT8_BUILD_ID, in the Makefile's ID_FILES order
_ID_FILES = ("capi.hip", "stft.hip", "stft3840.hip", "sync.hip", "bp.hip", "tx.hip", "subtract.hip", "drift.hip",
             "ft8_internal.h", "ft8_ldpc_tables.h", "tx_device.h", "heap_replay.h", "../../include/ft8hip.h",
             "Makefile")


def source_hash():
    """SHA-256 prefix of the library's sources as the Makefile computes FT8_BUILD_ID, or None when
    the sources are not beside the library (an installed copy)."""
    import hashlib
    csrc = os.path.join(_HERE, "csrc")
    paths = [os.path.normpath(os.path.join(csrc, f)) for f in _ID_FILES]
    if not all(os.path.exists(p) for p in paths):
        return None
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:32]


EXPORTED_SYMBOLS = (
    "ft8_create", "ft8_destroy", "ft8_last_error", "ft8_abi_version", "ft8_limits", "ft8_geometry",
    "ft8_geometry_hz",
    "ft8_stft", "ft8_sync_select", "ft8_llr", "ft8_normalize", "ft8_bp", "ft8_decode_batch", "ft8_select_warnings",
    "ft8_crc14", "ft8_ldpc_check", "ft8_set_timing", "ft8_get_timing", "ft8_get_counters", "ft8_get_bp_clock", "ft8_set_pipeline",
    "ft8_encode", "ft8_synthesize", "ft8_subtract", "ft8_stft_argmax", "ft8_drift_fit", "ft8_drift_correct",
    "ft8_build_id", "ft8_build_flags", "ft8_replay_stage", "ft8_set_timing_stages", "ft8_sync_score",
    "ft8_pack_bytes", "ft8_pack_decodes", "ft8_subtract_fits", "ft8_stft_method", "ft8_stft_screen_stats")


def limits():
    a, b, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    lib().ft8_limits(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return {"max_candidates": a.value, "max_fft_real": b.value, "max_fft_complex": c.value}


def sample_rate_hz(sample_rate) -> float:
    """The sample rate as the reference uses it: any positive finite number of Hz, integral or not
    (spectrogram_analyse.py:32-34 computes int(0.16 fs) and int(fs / 6.25 bpt) on the value given)."""
    fs = float(sample_rate)
    if not (0.0 < fs < 2e9):
        raise ValueError(f"sample_rate must be a positive finite number of Hz, got {sample_rate!r}")
    return fs


def geometry(sample_rate, bins_per_tone: int, steps_per_symbol: int, n_samples: int):
    """(nperseg, hop, nfft, frames) of calculate_spectrogram (spectrogram_analyse.py:31-43), computed
    by the library from the float sample rate."""
    v = [ctypes.c_int32() for _ in range(4)]
    rc = lib().ft8_geometry_hz(sample_rate_hz(sample_rate), int(bins_per_tone), int(steps_per_symbol),
                               int(n_samples), *[ctypes.byref(x) for x in v])
    if rc != FT8_OK:
        raise ValueError("invalid spectrogram geometry (nfft must be greater than or equal to nperseg, "
                         "positive sample rate and oversampling factors)")
    return tuple(x.value for x in v)


def require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise Ft8Error("ft8_demodulator_amd runs on a ROCm GPU (MI355X / gfx950); none is visible. "
                       "There is no CPU fallback.")
    return torch


class Context:
    """One libft8hip context per (host thread, device)."""

    def __init__(self, device: int):
        h = ctypes.c_void_p()
        rc = lib().ft8_create(int(device), ctypes.byref(h))
        if rc != FT8_OK:
            raise Ft8Error(f"ft8_create(device={device}) failed with code {rc}")
        self.handle = h
        self.device = int(device)

    def check(self, rc: int, what: str):
        if rc == FT8_OK:
            return
        msg = lib().ft8_last_error(self.handle).decode(errors="replace")
        text = f"{what}: {msg}"
        if rc in (FT8_E_ARG, FT8_E_RANGE):
            raise ValueError(text)
        if rc == FT8_E_UNSUPPORTED:
            raise NotImplementedError(text)
        if rc == FT8_E_NOMEM:
            raise MemoryError(text)
        raise Ft8Error(text)

    def set_timing(self, on: bool, stages=None):
        """Per-stage HIP events on/off; `stages` (names) limits which kernels are bracketed."""
        mask = 0xFFFFFFFF if stages is None else sum(1 << STAGE_NAMES.index(s) for s in stages)
        self.check(lib().ft8_set_timing_stages(self.handle, mask), "ft8_set_timing_stages")
        lib().ft8_set_timing(self.handle, int(bool(on)))

    def timing(self, reset: bool = False):
        ms = (ctypes.c_double * N_STAGES)()
        cnt = (ctypes.c_int64 * N_STAGES)()
        self.check(lib().ft8_get_timing(self.handle, ms, cnt, int(reset)), "ft8_get_timing")
        return {STAGE_NAMES[i]: (ms[i], cnt[i]) for i in range(N_STAGES)}

    def set_pipeline(self, chunk_slots: int = 0, n_streams: int = 0, bp_waves_per_simd: int = 4):
        """ft8_decode_batch chunking over internal streams (n_streams = 0: one chain) and the BP
        grid's resident waves per SIMD (1..4)."""
        self.check(lib().ft8_set_pipeline(self.handle, int(chunk_slots), int(n_streams), int(bp_waves_per_simd)),
                   "ft8_set_pipeline")

    def replay(self, stage: str, reps: int = 1, stream=None):
        """ft8_replay_stage: re-launch one kernel of the last ft8_decode_batch `reps` times."""
        self.check(lib().ft8_replay_stage(self.handle, STAGE_NAMES.index(stage), int(reps),
                                          stream if stream is not None else stream_handle(self.device)),
                   "ft8_replay_stage")

    def counters(self, reset: bool = False):
        v = (ctypes.c_int64 * 4)()
        self.check(lib().ft8_get_counters(self.handle, v, int(reset)), "ft8_get_counters")
        return {"candidates": v[0], "iterations": v[1], "passes": v[2], "converged": v[3]}

    def bp_clock(self, reset: bool = False):
        """ft8_get_bp_clock: k_bp's waves' own shader-clock cycles and wall-clock time, summed over
        the launches made while timing was enabled."""
        v = (ctypes.c_int64 * 5)()
        self.check(lib().ft8_get_bp_clock(self.handle, v, int(reset)), "ft8_get_bp_clock")
        return {"wave_cycles": v[0], "wave_wall_ticks": v[1], "max_wave_cycles": v[2], "waves": v[3],
                "wall_clock_khz": v[4]}

    def __del__(self):
        try:
            if getattr(self, "handle", None) and _lib is not None:
                _lib.ft8_destroy(self.handle)
        except Exception:  # noqa: BLE001
            pass


def device_index(device=None) -> int:
    torch = require_gpu()
    if device is None:
        return torch.cuda.current_device()
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


def context(device=None) -> Context:
    dev = device_index(device)
    cache = getattr(_tls, "ctx", None)
    if cache is None:
        cache = _tls.ctx = {}
    if dev not in cache:
        cache[dev] = Context(dev)
    return cache[dev]


def stream_handle(device=None):
    torch = require_gpu()
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())
