"""The bench's geometry legs alone (bench.geometry_legs: 20 kHz bpt 2, 12 kHz bpt 10), for A/B runs
of library builds (FT8HIP_LIB=... FT8HIP_ALLOW_STALE=1)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    r = bench.geometry_legs(torch.device("cuda", 0))
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk in ("slots_per_s", "stages_ms")} for k, v in r.items()
                      if isinstance(v, dict)}), flush=True)
