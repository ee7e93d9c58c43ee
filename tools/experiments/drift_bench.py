"""The drift-correction bench leg alone (bench.drift_correct), for profiling:
    rocprofv3 --kernel-trace --stats -d gpurun_out/pd -o run -- python3 tools/drift_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    torch.cuda.set_device(0)
    print(json.dumps(bench.drift_correct(torch.device("cuda", 0), n_sig=n)), flush=True)
