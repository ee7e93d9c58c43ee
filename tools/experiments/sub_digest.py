"""Digest of ft8_subtract on a seeded crowded batch: sha256 of the residual samples and of the fits
(ft8_subtract_fits).  Run it under two library builds (FT8HIP_LIB=... FT8HIP_ALLOW_STALE=1) to check
that a kernel change leaves the second pass bit-identical."""
import ctypes
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ft8_demodulator_amd import SlotDecoder, _lib, synth  # noqa: E402
from ft8_demodulator_amd._pipeline import make_params  # noqa: E402

if __name__ == "__main__":
    S, K, MS, IT = 64, 300, 2, 20
    x, _ = synth.make_slots(S, 50, seed=4242, device="cuda", snr_db=(-24.0, -10.0))
    n = x.shape[1]
    dec = SlotDecoder(12000, 2, 2, K, MS, IT, flags=_lib.FT8_FLAG_TOPK)
    out, counts = dec.run(x)
    p = make_params(dec.plan(n), K, MS, IT, _lib.FT8_FLAG_TOPK)
    ctx, L, st = dec.ctx, _lib.lib(), _lib.stream_handle()
    resid = torch.empty_like(x)
    ctx.check(L.ft8_subtract(ctx.handle, _lib.ptr(x), _lib.FT8_F32, _lib.ptr(resid), n, S, n, ctypes.byref(p),
                             _lib.ptr(out), _lib.ptr(counts), dec.cap, st), "ft8_subtract")
    fits = torch.empty(S * dec.cap * _lib.SUB_FIT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    ctx.check(L.ft8_subtract_fits(ctx.handle, _lib.ptr(fits), S, dec.cap, st), "ft8_subtract_fits")
    torch.cuda.synchronize()
    f = fits.cpu().numpy().view(_lib.SUB_FIT_DTYPE).reshape(S, dec.cap)
    c = counts.cpu().numpy()
    fh = hashlib.sha256()
    for s in range(S):
        r = f[s, : min(int(c[s]), dec.cap)]
        r = r[r["active"] == 1]  # an inactive record's other fields are not written
        for name in ("active", "start", "f0", "amp", "phase0", "tones"):  # not the unwritten `reserved`
            fh.update(r[name].tobytes())
    print(json.dumps({"lib": os.environ.get("FT8HIP_LIB", "default"), "slots": S, "decodes": int(c.sum()),
                      "residual_sha256": hashlib.sha256(resid.cpu().numpy().tobytes()).hexdigest(),
                      "fits_sha256": fh.hexdigest()}))
