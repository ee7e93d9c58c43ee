"""Small driver for profiling: synthesise a config-3 batch, run the decode a few times."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=256)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import torch
    from ft8_demodulator_amd import SlotDecoder, synth
    x, _ = synth.make_slots(a.slots, 50, seed=100000, device="cuda")
    dec = SlotDecoder(12000, 2, 2, 300, 2, 20)
    for _ in range(a.iters):
        dec.run(x)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
