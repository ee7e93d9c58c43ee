"""The bench's drift leg alone (256 complex128 beacons, bench.drift_correct), for counter passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

r = bench.drift_correct(torch.device("cuda", 0), n_sig=256, reps=2)
print({k: r[k] for k in ("ms_per_launch", "stages_ms")})
