"""The reference's own sensitivity harness run here at seven of its rates (build container only; imports
/root/reference/src like tools/make_golden_harness.py): test_ft8_standard.py:43-68 test_step,
`ROUNDS` rounds per SNR point, the reference's decode_ft8_message deciding success.  Inputs are
seeded exactly as in make_golden_harness.py (np.random.default_rng(seed): payload, then noise; the
clean wave from the reference generator), so the GPU test rebuilds the same float64 bytes and must
reach the same per-slot verdicts (tests/test_gpu_harness.py::test_gpu_sensitivity_points_match_reference).

This checks BASELINE.md section 1's table (snr_vs_freq_analysis.xlsx: -9 dB at B = 1 000 Hz, -13 dB at
B = 3 000 Hz) against the committed harness and decoder: the success ratio per point is stored.

Usage:  cd /tmp && python /root/repo/tools/make_golden_sensitivity.py [extend]
        (extend: add only the rates not yet in tests/golden/sensitivity_ref.json)
"""
import json
import multiprocessing
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden_harness as MH  # noqa: E402  (reference import recipe, harness_input, KW)

POINTS = {2000: (-14.0, -13.0, -12.0, -11.0, -10.0), 6000: (-20.0, -19.0, -18.0, -17.0, -16.0, -15.0, -14.0),
          # round 6: a chirp-z rate (nfft 1760 = 2^5 * 5 * 11) and one >= 9 kHz, around the GPU table's
          # thresholds (-18.2 dB at 5 500 Hz, -20.6 dB at 10 000 Hz)
          5500: (-19.5, -19.0, -18.5, -18.0, -17.5), 10000: (-21.5, -21.0, -20.5, -20.0, -19.5),
          # round 6, later: 3 000, 8 000 and 12 000 Hz around the 200-round GPU thresholds
          # (-15.4, -19.6 and -21.4 dB, profiles/r6_y_sensitivity_200rounds.json)
          3000: (-16.5, -16.0, -15.5, -15.0, -14.5), 8000: (-20.5, -20.0, -19.5, -19.0, -18.5),
          12000: (-22.5, -22.0, -21.5, -21.0, -20.5)}
ROUNDS = 20
SEED0 = 70000


def _verdict(job):
    """One test_step of the harness: the reference's decode_ft8_message decides success."""
    fs, snr, seed = job
    _p, _c, x = MH.harness_input(fs, snr, seed)
    return len(MH.quiet(MH.R.decode_ft8_message, x, fs, **MH.KW)) > 0


def main():
    import tempfile
    os.chdir(tempfile.mkdtemp(prefix="ft8gold_"))
    out = {"rounds": ROUNDS, "kwargs": MH.KW, "points": []}
    seed = SEED0
    path = os.path.join(MH.GOLD, "sensitivity_ref.json")
    done = set()
    if sys.argv[1:] == ["extend"]:
        # keep the rates already stored (and their seeds); add the others, seeds continuing after
        with open(path) as f:
            out = json.load(f)
        done = {p["fs"] for p in out["points"]}
        seed = max(s_ for p in out["points"] for s_ in p["seeds"]) + 1
    for fs, snrs in POINTS.items():
        if fs in done:
            continue
        for snr in snrs:
            t0 = time.time()
            seeds = list(range(seed, seed + ROUNDS))
            seed += ROUNDS
            with multiprocessing.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
                ok = pool.map(_verdict, [(fs, snr, s_) for s_ in seeds])
            out["points"].append({"fs": fs, "snr_db": snr, "seeds": seeds, "success": ok,
                                  "ratio": sum(ok) / ROUNDS})
            print(fs, snr, sum(ok), "/", ROUNDS, round(time.time() - t0, 1), "s", flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(MH.GOLD, "sensitivity_ref.json"))


if __name__ == "__main__":
    main()
