"""Front-end slot chunks (ft8_set_pipeline(chunk, 0, 4): STFT -> score/select -> LLR per chunk of
`chunk` slots, one BP over the whole batch) against the plain step, at depth 1 and 2, interleaved
rounds on one box; every configuration's records must equal the plain step's.  Experiment only:
the front-chunk mode of decode_pass it measured (round 6, profiles/r6_b_front_chunks.log: no gain)
was removed again, so on the current library every chunk runs the plain step.
    python tools/experiments/front_chunks.py [chunk ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ft8_demodulator_amd import SlotDecoder, synth, _lib  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    x, _ = synth.make_slots(256, 50, seed=100000, device="cuda")
    chunks = [int(a) for a in sys.argv[1:]] or [0, 128, 64, 32]
    decs = [SlotDecoder(12000, 2, 2, 300, 2, 20), SlotDecoder(12000, 2, 2, 300, 2, 20, context=_lib.Context(0))]
    S = [torch.cuda.Stream(), torch.cuda.Stream()]
    K = 40
    ref = None

    def run(D, ch):
        for d in decs:
            d.ctx.set_pipeline(ch, 0, 4)
        torch.cuda.synchronize()
        for k in range(16):
            with torch.cuda.stream(S[k % D]):
                decs[k % D].run(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            with torch.cuda.stream(S[k % D]):
                out, c = decs[k % D].run(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        return dt, out, c

    for rnd in range(3):
        for D in (1, 2):
            for ch in chunks:
                dt, out, c = run(D, ch)
                key = (out.cpu().numpy().tobytes(), c.cpu().numpy().tobytes())
                if ref is None:
                    ref = key
                print(json.dumps({"round": rnd, "depth": D, "chunk": ch, "ms_per_step": dt * 1e3,
                                  "slots_per_s": 256 / dt, "decodes": int(c.sum()), "same": key == ref}), flush=True)
