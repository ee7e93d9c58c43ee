"""The PCIe-inclusive streaming leg (bench.h2d_stream) at StreamDecoder depth 1 / 2 / 3, interleaved
on one box, with the upload alone as its bound."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from ft8_demodulator_amd import synth  # noqa: E402

kw = dict(max_candidates=300, min_score=2, max_iterations=20)

if __name__ == "__main__":
    x, _ = synth.make_slots(256, 50, seed=100000, device="cuda")
    torch.cuda.synchronize()
    for rnd in range(2):
        for depth in (1, 2, 3):
            r = bench.h2d_stream(x, 40, kw, depth=depth)
            print(json.dumps({"round": rnd, "depth": depth, "ms_per_batch": round(r["ms_per_batch"], 4),
                              "slots_per_s": round(r["slots_per_s"]),
                              "steady_ms": round(r["steady"]["ms_per_batch"], 4),
                              "borrow_ms": round(r["borrow"]["ms_per_batch"], 4),
                              "borrow_steady_ms": round(r["borrow"]["steady_ms_per_batch"], 4),
                              "upload_alone_ms": round(r["upload_alone"]["ms_per_batch"], 4)}), flush=True)
