"""Where the PCIe-inclusive streaming leg loses time: resident decode vs upload vs StreamDecoder,
with and without the host-side result conversion."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ft8_demodulator_amd import synth  # noqa: E402
from ft8_demodulator_amd.stream import StreamDecoder  # noqa: E402

kw = dict(max_candidates=300, min_score=2, max_iterations=20)


def timeit(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


if __name__ == "__main__":
    x, _ = synth.make_slots(256, 50, seed=0, device="cuda")
    pcm = torch.clamp(torch.round(x / x.abs().amax() * 30000.0), -32767, 32767).to(torch.int16).cpu().pin_memory()
    sd = StreamDecoder(pcm.shape[1], max_batch=256, **kw)
    dpcm = pcm.cuda()
    print("resident int16 decode  %.2f ms" % timeit(lambda: sd.dec.run(dpcm, code=4)), flush=True)
    d = torch.empty_like(dpcm)
    print("upload only            %.2f ms" % timeit(lambda: d.copy_(pcm, non_blocking=True)), flush=True)

    def stream(n=8):
        for _ in sd.decode_batches([pcm] * n):
            pass
    t = timeit(lambda: stream(8), reps=2) / 8
    print("stream decoder         %.2f ms per batch" % t, flush=True)
    orig = sd._collect
    sd._collect = lambda i, nb: (sd.ready[i].synchronize(), [])[1]
    t = timeit(lambda: stream(8), reps=2) / 8
    print("stream, no conversion  %.2f ms per batch" % t, flush=True)
    sd._collect = orig
    t0 = time.perf_counter()
    for _ in range(8):
        orig(0, 256)
    print("host conversion alone  %.2f ms per batch" % ((time.perf_counter() - t0) / 8 * 1e3), flush=True)
    import bench  # noqa: E402
    r = bench.h2d_stream(x, 10, kw)
    print("bench.h2d_stream       %.2f ms per batch" % r["ms_per_batch"], flush=True)
    t = timeit(lambda: stream(8), reps=2) / 8
    print("stream decoder again   %.2f ms per batch" % t, flush=True)
