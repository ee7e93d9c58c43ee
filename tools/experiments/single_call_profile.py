"""Host-side breakdown of one decode_ft8_message call (cProfile over warm calls)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ft8_demodulator_amd import decode_ft8_message, synth  # noqa: E402

x, _ = synth.make_slots(1, 50, seed=100000, device="cpu")
slot = x[0].numpy()
for kw in ({}, dict(max_candidates=300, min_score=2)):
    for _ in range(10):
        decode_ft8_message(slot, 12000, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        decode_ft8_message(slot, 12000, **kw)
    print(kw, "%.3f ms per call" % ((time.perf_counter() - t0) / 50 * 1e3), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        decode_ft8_message(slot, 12000, **kw)
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(18)
