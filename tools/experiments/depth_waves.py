"""Headline steps alternated over D contexts / streams with the BP grid at W resident waves per
SIMD (ft8_set_pipeline(0, 0, W)), against one chain at 4, interleaved rounds.  Experiment only.
    python tools/experiments/depth_waves.py D:W [D:W ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ft8_demodulator_amd import SlotDecoder, synth, _lib  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    x, _ = synth.make_slots(256, 50, seed=100000, device="cuda")
    cfgs = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or [(1, 4), (2, 4), (2, 3), (3, 3), (2, 2)]
    Dmax = max(d for d, _ in cfgs)
    decs = [SlotDecoder(12000, 2, 2, 300, 2, 20) for _ in range(Dmax)]
    for d in decs[1:]:
        d.ctx = _lib.Context(0)
    S = [torch.cuda.Stream() for _ in range(Dmax)]
    K = 50

    def run(D, W):
        for d in decs[:D]:
            d.ctx.set_pipeline(0, 0, W)
        torch.cuda.synchronize()
        for k in range(20):
            with torch.cuda.stream(S[k % D]):
                decs[k % D].run(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            with torch.cuda.stream(S[k % D]):
                _, c = decs[k % D].run(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        return dt, int(c.sum())

    for rnd in range(3):
        for D, W in cfgs:
            dt, n = run(D, W)
            print(json.dumps({"round": rnd, "depth": D, "bp_waves": W, "ms_per_step": dt * 1e3,
                              "slots_per_s": 256 / dt, "decodes": n}), flush=True)
