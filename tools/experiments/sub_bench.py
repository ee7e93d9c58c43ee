"""The subtract-and-redecode bench leg alone (bench.subtract_redecode), for profiling."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    r = bench.subtract_redecode(torch.device("cuda", 0))
    print(json.dumps({k: v for k, v in r.items() if k != "workload"}), flush=True)
