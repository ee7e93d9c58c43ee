"""A/B several libft8hip.so builds on the same data in one process family (one subprocess per
variant, interleaved rounds).  Usage: python tools/ab_variants.py lib1.so lib2.so ..."""
import json
import os
import subprocess
import sys

CHILD = r'''
import os, sys, json, time
sys.path.insert(0, os.environ["REPO"])
import torch
from ft8_demodulator_amd import SlotDecoder, synth
torch.manual_seed(0)
x, _ = synth.make_slots(256, 50, seed=100000, device="cuda")
dec = SlotDecoder(12000, 2, 2, 300, 2, 20)
for _ in range(20): dec.run(x)   # k_bp settles over ~15 launches
torch.cuda.synchronize()
ctx = dec.ctx
t0 = time.perf_counter()
for _ in range(30): out, cnt = dec.run(x)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 30
tm = {}
for st in ("stft", "score", "select", "llr", "bp"):
    ctx.set_timing(True, stages=[st]); ctx.timing(reset=True)
    for _ in range(8): dec.run(x)
    torch.cuda.synchronize()
    ctx.set_timing(False)
    tm[st] = ctx.timing(reset=True)[st]
# the top-k selection (k_topkc) on the same batch
dk = SlotDecoder(12000, 2, 2, 300, 2, 20, flags=1)
for _ in range(3): dk.run(x)
ctx.set_timing(True, stages=["select"]); ctx.timing(reset=True)
for _ in range(8): dk.run(x)
torch.cuda.synchronize()
ctx.set_timing(False)
tk = ctx.timing(reset=True)["select"]
print(json.dumps({"lib": os.environ["FT8HIP_LIB"], "ms_step": dt * 1e3, "decodes": int(cnt.sum()),
                  "stages": {k: v[0] / max(v[1], 1) for k, v in tm.items() if v[1]},
                  "topk_select": tk[0] / max(tk[1], 1)}))
'''


def main():
    libs = sys.argv[1:]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {l: [] for l in libs}
    for rnd in range(2):
        for l in libs:
            env = dict(os.environ, FT8HIP_LIB=l, REPO=repo, FT8HIP_ALLOW_STALE="1")
            out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in out.stdout.splitlines() if x.startswith("{")]
            if not line:
                print("FAILED", l, out.stderr[-2000:])
                continue
            d = json.loads(line[-1])
            res[l].append(d)
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
