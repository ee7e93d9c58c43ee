"""k_topkc phase timestamps (variants/TKP.so: s_memrealtime, 10 ns ticks, printed by three
workgroups) on the subtract leg's top-k decode of 334 crowded slots.
    FT8HIP_LIB=$PWD/variants/TKP.so FT8HIP_ALLOW_STALE=1 python tools/experiments/topkc_phases.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ft8_demodulator_amd import SlotDecoder, _lib, synth  # noqa: E402

x, _ = synth.make_slots(334, 50, seed=200000, device="cuda")
dec = SlotDecoder(12000, 2, 2, 300, 2, 20, flags=_lib.FT8_FLAG_TOPK)
for _ in range(3):
    dec.run(x)
    torch.cuda.synchronize()
print("ok", flush=True)
