"""Does per-stage event timing perturb the step time?"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from ft8_demodulator_amd import SlotDecoder, synth
    x, _ = synth.make_slots(256, 50, seed=100000, device="cuda")
    dec = SlotDecoder(12000, 2, 2, 300, 2, 20)
    ctx = dec.ctx
    ctx.set_pipeline(0, 0, 4)
    for rnd in range(3):
        for timing in (False, True):
            ctx.set_timing(timing)
            for _ in range(3):
                dec.run(x)
            torch.cuda.synchronize()
            ctx.timing(reset=True)
            t0 = time.perf_counter()
            for _ in range(10):
                dec.run(x)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            tm = ctx.timing(reset=True)
            print(json.dumps({"timing": timing, "ms": dt * 1e3,
                              "stages": {k: round(v[0] / max(v[1], 1), 4) for k, v in tm.items() if v[1]}}), flush=True)


if __name__ == "__main__":
    main()
