"""How many slots of the bench workload take k_select's tie (heap replay) path?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from ft8_demodulator_amd import SlotDecoder, synth, _lib
    x, _ = synth.make_slots(256, 50, seed=100000, device="cuda")
    dec = SlotDecoder(12000, 2, 2, 300, 2, 20)
    dec.run(x)
    w = torch.zeros(256, dtype=torch.int32, device="cuda")
    dec.ctx.check(_lib.lib().ft8_select_warnings(dec.ctx.handle, _lib.ptr(w), 256, _lib.stream_handle()), "warn")
    w = w.cpu().numpy()
    print("heap-tie(bit0)", int((w & 1).sum()), "overflow(bit1)", int(((w >> 1) & 1).sum()),
          "replay(bit2)", int(((w >> 2) & 1).sum()), "of", len(w))


if __name__ == "__main__":
    main()
