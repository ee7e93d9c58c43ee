"""Device-side helpers shared by the mirror modules (waterfall upload, stage calls)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def waterfall_to_device(wf):
    """FT8Waterfall.mag [freq, time] (NumPy or torch) -> time-major device tensor [T, F].

    float32 stays float32 (the reference's np.float32 score path); every other dtype is scored in
    float64."""
    torch = _lib.require_gpu()
    mag = wf.mag
    if isinstance(mag, torch.Tensor):
        t = mag
        if t.dtype not in (torch.float32, torch.float64):
            t = t.to(torch.float64)
        t = t.t().contiguous().cuda()
    else:
        a = np.asarray(mag)
        if a.dtype not in (np.float32, np.float64):
            a = a.astype(np.float64)
        t = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    F, T = int(t.shape[1]), int(t.shape[0])
    return t, t.dtype == torch.float64, T, F


def sync_params(wf, max_candidates, min_score, flags=0):
    from ._pipeline import min_score_is_f64
    p = _lib.Ft8Params()
    p.flags = int(flags)
    p.sample_rate = 1
    p.bins_per_tone = int(wf.freq_osr)
    p.steps_per_symbol = int(wf.time_osr)
    p.max_candidates = int(max_candidates)
    p.max_iterations = 0
    p.min_score_f64 = int(min_score_is_f64(min_score))
    p.min_score = float(min_score)
    return p


def grid_shape(T, F, sps, bpt):
    nb = T // sps
    t0 = -10 * sps
    NT = max(nb * sps - sps * 59 - t0, 0)
    NF = max(F - 7 * bpt, 0)
    return t0, NT, NF


def sync_select(wf, max_candidates, min_score, want_grid=False, flags=0):
    """-> (cands [(abs_time, abs_freq, score)], score grid or None, warning flags)."""
    torch = _lib.require_gpu()
    ctx = _lib.context()
    d, f64, T, F = waterfall_to_device(wf)
    N = max(int(max_candidates), 0)
    sps, bpt = int(wf.time_osr), int(wf.freq_osr)
    t0, NT, NF = grid_shape(T, F, sps, bpt)
    dev = d.device
    cand = torch.zeros(max(N, 1) * 2, dtype=torch.int32, device=dev)
    cs = torch.zeros(max(N, 1), dtype=torch.float64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    grid = torch.empty(max(NT * NF, 1), dtype=d.dtype, device=dev) if want_grid else None
    p = sync_params(wf, max(N, 1) if want_grid else N, min_score, flags)
    rc = _lib.lib().ft8_sync_select(ctx.handle, _lib.ptr(d), int(f64), 1, T, F, ctypes.byref(p),
                                    _lib.ptr(cand), _lib.ptr(cs), _lib.ptr(cnt),
                                    _lib.ptr(grid) if grid is not None else None, _lib.stream_handle())
    ctx.check(rc, "ft8_sync_select")
    warn = torch.zeros(1, dtype=torch.int32, device=dev)
    if NT > 0 and NF > 0 and p.max_candidates > 0:
        ctx.check(_lib.lib().ft8_select_warnings(ctx.handle, _lib.ptr(warn), 1, _lib.stream_handle()),
                  "ft8_select_warnings")
    n = int(cnt.item()) if N > 0 else 0
    c = cand.cpu().numpy().reshape(-1, 2)
    s = cs.cpu().numpy()
    sc_t = np.float64 if f64 else np.float32
    cands = [(int(c[i, 0]), int(c[i, 1]), sc_t(s[i])) for i in range(n)]
    g = None
    if want_grid:
        g = grid[: NT * NF].cpu().numpy().reshape(NT, NF) if NT * NF else np.zeros((NT, NF), d.cpu().numpy().dtype)
    return cands, g, int(warn.item())


def sync_scores(wf, cand_list):
    """ft8_sync_score of arbitrary (abs_time, abs_freq) pairs (k_score_list) -> (scores in the
    waterfall dtype, IndexError flags)."""
    torch = _lib.require_gpu()
    ctx = _lib.context()
    d, f64, T, F = waterfall_to_device(wf)
    n = len(cand_list)
    c = torch.tensor([[int(a), int(b)] for a, b in cand_list] or [[0, 0]], dtype=torch.int32, device=d.device)
    out = torch.empty(max(n, 1), dtype=d.dtype, device=d.device)
    err = torch.zeros(max(n, 1), dtype=torch.int32, device=d.device)
    rc = _lib.lib().ft8_sync_score(ctx.handle, _lib.ptr(d), int(f64), T, F, int(wf.time_osr), int(wf.freq_osr),
                                   _lib.ptr(c), n, _lib.ptr(out), _lib.ptr(err), _lib.stream_handle())
    ctx.check(rc, "ft8_sync_score")
    return out.cpu().numpy()[:n], err.cpu().numpy()[:n].astype(bool)


def llr(wf, cand_list, normalize):
    """cand_list [(abs_time, abs_freq)] -> LLRs [n, 174] (float64)."""
    torch = _lib.require_gpu()
    ctx = _lib.context()
    d, f64, T, F = waterfall_to_device(wf)
    n = len(cand_list)
    if n == 0:
        return np.zeros((0, 174))
    c = torch.tensor([[0, int(a), int(b)] for a, b in cand_list], dtype=torch.int32, device=d.device)
    out = torch.empty(n, 174, dtype=torch.float64, device=d.device)
    rc = _lib.lib().ft8_llr(ctx.handle, _lib.ptr(d), int(f64), T, F, int(wf.time_osr), int(wf.freq_osr),
                            _lib.ptr(c), n, int(bool(normalize)), _lib.ptr(out), _lib.stream_handle())
    ctx.check(rc, "ft8_llr")
    return out.cpu().numpy()


def normalize(x):
    torch = _lib.require_gpu()
    ctx = _lib.context()
    a = torch.from_numpy(np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1, 174))).cuda()
    out = torch.empty_like(a)
    ctx.check(_lib.lib().ft8_normalize(ctx.handle, _lib.ptr(a), a.shape[0], _lib.ptr(out), _lib.stream_handle()),
              "ft8_normalize")
    return out.cpu().numpy()


def bp(llrs, max_iterations):
    """LLRs [n, 174] -> (plain uint8 [n, 174], records structured [n])."""
    torch = _lib.require_gpu()
    ctx = _lib.context()
    a = torch.from_numpy(np.ascontiguousarray(np.asarray(llrs, dtype=np.float64).reshape(-1, 174))).cuda()
    n = a.shape[0]
    plain = torch.zeros(n, 174, dtype=torch.uint8, device=a.device)
    res = torch.zeros(n * _lib.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=a.device)
    ctx.check(_lib.lib().ft8_bp(ctx.handle, _lib.ptr(a), n, int(max_iterations), _lib.ptr(plain), _lib.ptr(res),
                                _lib.stream_handle()), "ft8_bp")
    return plain.cpu().numpy(), res.cpu().numpy().view(_lib.RESULT_DTYPE)


def crc14(msgs, nbits):
    torch = _lib.require_gpu()
    ctx = _lib.context()
    n = len(msgs)
    buf = np.zeros((max(n, 1), 12), dtype=np.uint8)
    for i, m in enumerate(msgs):
        b = bytes(m)[:12]
        buf[i, :len(b)] = np.frombuffer(b, dtype=np.uint8)
    d = torch.from_numpy(buf).cuda()
    nb = torch.tensor(list(nbits) or [0], dtype=torch.int32, device=d.device)
    out = torch.zeros(max(n, 1), dtype=torch.int16, device=d.device)
    ctx.check(_lib.lib().ft8_crc14(ctx.handle, _lib.ptr(d), _lib.ptr(nb), n, _lib.ptr(out), _lib.stream_handle()),
              "ft8_crc14")
    return [int(v) & 0xFFFF for v in out.cpu().numpy()[:n]]


def ldpc_check(bits):
    torch = _lib.require_gpu()
    ctx = _lib.context()
    b = torch.from_numpy(np.ascontiguousarray((np.asarray(bits).reshape(-1, 174) != 0).astype(np.uint8))).cuda()
    n = b.shape[0]
    out = torch.zeros(n, dtype=torch.int32, device=b.device)
    ctx.check(_lib.lib().ft8_ldpc_check(ctx.handle, _lib.ptr(b), n, _lib.ptr(out), _lib.stream_handle()),
              "ft8_ldpc_check")
    return out.cpu().numpy()


def stft(wave_data, sample_rate, bins_per_tone, steps_per_symbol, f_lo=None, f_hi=None, t_lo=None, t_hi=None,
         device=None):
    """-> (waterfall tensor [T, F] time-major on the device, plan, wf_f64)."""
    torch = _lib.require_gpu()
    from ._pipeline import device_samples, make_plan
    x, code, f64 = device_samples(wave_data, device)
    if x.dim() != 1:
        raise ValueError("wave_data must be one-dimensional")
    n = int(x.shape[0])
    plan = make_plan(n, sample_rate, bins_per_tone, steps_per_symbol)
    if plan.frames == 0:
        return None, plan, f64
    ctx = _lib.context(x.device)
    p = _lib.Ft8Params()
    p.sample_rate_hz = _lib.sample_rate_hz(sample_rate)
    p.sample_rate, p.bins_per_tone, p.steps_per_symbol = int(p.sample_rate_hz), int(bins_per_tone), int(steps_per_symbol)
    p.f_lo = 0 if f_lo is None else int(f_lo)
    p.f_hi = plan.nfft if f_hi is None else int(f_hi)
    p.t_lo = 0 if t_lo is None else int(t_lo)
    p.t_hi = plan.frames if t_hi is None else int(t_hi)
    out = torch.empty(max(p.t_hi - p.t_lo, 0), max(p.f_hi - p.f_lo, 0),
                      dtype=torch.float64 if f64 else torch.float32, device=x.device)
    rc = _lib.lib().ft8_stft(ctx.handle, _lib.ptr(x), int(code), n, 1, n, ctypes.byref(p), _lib.ptr(out),
                             _lib.stream_handle(x.device))
    ctx.check(rc, "ft8_stft")
    return out, plan, f64
