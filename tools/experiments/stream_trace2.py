"""12 pinned int16 batches through StreamDecoder(depth=2) after a warm pass: the process a kernel +
memory-copy trace is taken of (tools/experiments/gpu_stream_trace2.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ft8_demodulator_amd import synth  # noqa: E402
from ft8_demodulator_amd.stream import StreamDecoder  # noqa: E402

if __name__ == "__main__":
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    x, _ = synth.make_slots(256, 50, seed=100000, device="cuda")
    pcm = torch.clamp(torch.round(x / x.abs().amax() * 30000.0), -32767, 32767).to(torch.int16).cpu().pin_memory()
    sd = StreamDecoder(pcm.shape[1], max_batch=256, depth=depth, max_candidates=300, min_score=2, max_iterations=20)
    for _ in range(2):
        for _ in sd.decode_batches([pcm] * 12):
            pass
    torch.cuda.synchronize()
    print("done", flush=True)
