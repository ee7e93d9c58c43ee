"""A/B the ft8_decode_batch pipeline settings on the bench workload; checks identical records."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from ft8_demodulator_amd import SlotDecoder, synth
    x, _ = synth.make_slots(256, 50, seed=100000, device="cuda")
    dec = SlotDecoder(12000, 2, 2, 300, 2, 20)
    ctx = dec.ctx
    cfgs = [(0, 0, 4), (32, 2, 3), (64, 2, 3), (128, 2, 3), (64, 2, 4), (128, 2, 4), (64, 3, 3), (32, 2, 2)]
    ref = None
    for rnd in range(2):
        for cfg in cfgs:
            ctx.set_pipeline(*cfg)
            for _ in range(15 if rnd == 0 else 5):
                out, cnt = dec.run(x)
            torch.cuda.synchronize()
            if rnd == 0:
                recs = out.cpu().numpy().tobytes(), cnt.cpu().numpy().tobytes()
                if ref is None:
                    ref = recs
                same = recs == ref
            t0 = time.perf_counter()
            for _ in range(20):
                out, cnt = dec.run(x)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 20
            print(json.dumps({"cfg": cfg, "ms": dt * 1e3, "slots_per_s": 256 / dt, "same": same if rnd == 0 else None}),
                  flush=True)


if __name__ == "__main__":
    main()
