"""Consecutive headline steps alternated over two contexts on two streams (step k+1's STFT / score
may start while step k's k_bp retires its last waves) against the one-stream loop, interleaved
rounds on the same data.  Experiment only."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ft8_demodulator_amd import SlotDecoder, synth, _lib  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    x, _ = synth.make_slots(256, 50, seed=100000, device="cuda")
    d1 = SlotDecoder(12000, 2, 2, 300, 2, 20)
    d2 = SlotDecoder(12000, 2, 2, 300, 2, 20)
    d2.ctx = _lib.Context(0)
    S = [torch.cuda.Stream(), torch.cuda.Stream()]
    K = 50

    def one():
        for _ in range(K):
            d1.run(x)

    def two():
        for k in range(K):
            with torch.cuda.stream(S[k % 2]):
                (d1 if k % 2 == 0 else d2).run(x)

    for f in (one, two):
        for _ in range(15):
            f()
    torch.cuda.synchronize()
    # same decodes on both contexts
    _, c1 = d1.run(x)
    with torch.cuda.stream(S[1]):
        _, c2 = d2.run(x)
    torch.cuda.synchronize()
    same = bool(torch.equal(c1, c2))
    for rnd in range(4):
        for name, f in (("one", one), ("two", two)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / K
            print(json.dumps({"round": rnd, "mode": name, "ms_per_step": dt * 1e3, "slots_per_s": 256 / dt,
                              "counts_equal": same}), flush=True)
