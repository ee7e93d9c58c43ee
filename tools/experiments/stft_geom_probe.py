"""Time calculate_spectrogram + decode_ft8_message on the reference test geometry (12 kHz, bpt = sps =
10: nfft 19200) for the library in FT8HIP_LIB."""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import numpy as np, torch
from ft8_demodulator_amd import calculate_spectrogram, decode_ft8_message, synth
x, _ = synth.make_slots(1, 20, seed=7, device="cpu")
x = x[0].numpy()
for name, fn in (("spectrogram", lambda: calculate_spectrogram(x, 12000, 10, 10)),
                 ("decode", lambda: decode_ft8_message(x, 12000, 10, 10, max_candidates=50, min_score=2))):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5): fn()
    torch.cuda.synchronize()
    print(os.path.basename(os.environ.get("FT8HIP_LIB", "lib")), name, "ms", (time.perf_counter() - t) / 5 * 1e3)
