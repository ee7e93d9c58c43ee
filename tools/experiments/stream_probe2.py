"""Which part of bench.main's sequence slows the streaming leg down (diagnostic)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from ft8_demodulator_amd import SlotDecoder, synth  # noqa: E402

kw = dict(max_candidates=300, min_score=2, max_iterations=20)

if __name__ == "__main__":
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    x, _ = synth.make_slots(256, 50, seed=0, device=dev)
    print("fresh                  %.2f" % bench.h2d_stream(x, 10, kw)["ms_per_batch"], flush=True)
    dec = SlotDecoder(12000, 2, 2, device=dev, **kw)
    for _ in range(23):
        dec.run(x)
    torch.cuda.synchronize()
    print("after 23 f32 decodes   %.2f" % bench.h2d_stream(x, 10, kw)["ms_per_batch"], flush=True)
    ctx = dec.ctx
    ctx.set_timing(True)
    ctx.timing(reset=True)
    for _ in range(20):
        dec.run(x)
    torch.cuda.synchronize()
    ctx.set_timing(False)
    ctx.timing(reset=True)
    print("after timing on/off    %.2f" % bench.h2d_stream(x, 10, kw)["ms_per_batch"], flush=True)
    r = bench.bp_stress(ctx, dev)
    print("after bp_stress        %.2f" % bench.h2d_stream(x, 10, kw)["ms_per_batch"], flush=True)
