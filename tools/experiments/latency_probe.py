import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
from ft8_demodulator_amd import decode_ft8_message, synth, read_wave_file, decode_ft8_from_wave
x, _ = synth.make_slots(1, 50, seed=100000, device="cpu")
x = x[0].numpy()
for kw in (dict(), dict(max_candidates=300, min_score=2)):
    for _ in range(5): decode_ft8_message(x, 12000, **kw)
    torch.cuda.synchronize()
    t = time.perf_counter(); n = 50
    for _ in range(n): r = decode_ft8_message(x, 12000, **kw)
    print(kw, "decode_ft8_message ms/call:", (time.perf_counter() - t) / n * 1e3, "decodes", len(r))
wav = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests", "data", "synth_cfg1.wav")
for _ in range(3): decode_ft8_from_wave(wav)
t = time.perf_counter()
for _ in range(20): decode_ft8_from_wave(wav)
print("decode_ft8_from_wave ms/call:", (time.perf_counter() - t) / 20 * 1e3)
