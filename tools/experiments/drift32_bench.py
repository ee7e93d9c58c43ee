"""bench.drift_32k alone (the chirp-z drift geometry), for A/B runs of library builds
(FT8HIP_LIB=... FT8HIP_ALLOW_STALE=1)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    bench.drift_32k(dev, reps=1)
    print(json.dumps(bench.drift_32k(dev, n_sig=int(sys.argv[1]) if len(sys.argv) > 1 else 16, reps=5)), flush=True)
