"""The reference's sensitivity harness (test_ft8_standard.py:43-123) on one GPU, standalone:
bench.sensitivity with a chosen number of rounds per SNR point; prints one JSON object.

    python tools/sensitivity_sweep.py [--rounds 20] [--rates 2000,2500,...] [--step 0.2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--step", type=float, default=0.2)
    ap.add_argument("--lo", type=float, default=-24.0)
    ap.add_argument("--hi", type=float, default=-5.0)
    ap.add_argument("--rates", default="")
    ap.add_argument("--oracle-per-rate", type=int, default=2)
    ap.add_argument("--seed", type=int, default=31337)
    a = ap.parse_args()
    import bench
    procs = bench.host_cores()[0]
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rates = [int(r) for r in a.rates.split(",") if r] or None
    t0 = time.perf_counter()
    out = bench.sensitivity(dev, rates=rates, snr_lo=a.lo, snr_hi=a.hi, step=a.step, rounds=a.rounds, seed=a.seed,
                            oracle_per_rate=a.oracle_per_rate, procs=procs)
    out["wall_s"] = time.perf_counter() - t0
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
