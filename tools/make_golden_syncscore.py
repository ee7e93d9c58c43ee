"""Golden ft8_sync_score values for candidates OFF the ft8_find_candidates grid, from the reference
itself (build container only; same import recipe as tools/make_golden.py).  Waterfalls: the
golden sync cases rand32 (float32) and b1s1_64 (float64) of tests/golden/golden.npz.  Candidates
include negative frequencies (NumPy wraps them), frequencies whose tone +1 lies past the last bin
(IndexError), times before / after the grid.  -> tests/golden/syncscore.json

Usage:  cd /tmp && python /root/repo/tools/make_golden_syncscore.py
"""
import contextlib
import io
import json
import os
import sys

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")
sys.path.insert(0, "/root/reference/src")
with contextlib.redirect_stdout(io.StringIO()):
    from ft8_tools.ft8_demodulator import ft8_decode as R  # noqa: E402
    from ft8_tools.ft8_demodulator.ftx_types import FT8Waterfall, FT8Candidate  # noqa: E402


def main():
    g = np.load(os.path.join(REPO, "tests", "golden", "golden.npz"), allow_pickle=False)
    out = []
    for name, sps, bpt in (("rand32", 2, 2), ("b1s1_64", 1, 1)):
        mag = g[f"sync_{name}_mag"]
        F, T = mag.shape
        wf = FT8Waterfall(mag=mag, time_osr=sps, freq_osr=bpt)
        cands = [(0, -1), (0, -5), (3, -14 * bpt), (-25 * sps, 3), (-11 * sps, 10), (-200, 4), (T - 2, 5),
                 (T // 2, F - 8 * bpt), (T // 2, F - 7 * bpt), (T // 2, F - 6 * bpt), (5, F + 3),
                 (T - 30 * sps, 2), (T + 50, 1), (-3 * sps - 1, F // 2), (7, -F), (7, -F - 1)]
        for at, af in cands:
            try:
                v = R.ft8_sync_score(wf, FT8Candidate(waterfall=wf, abs_time=at, abs_freq=af))
                rec = {"score": float(v), "dtype": type(v).__name__, "error": None}
            except Exception as e:  # noqa: BLE001
                rec = {"score": None, "dtype": None, "error": type(e).__name__}
            out.append(dict(case=name, sps=sps, bpt=bpt, abs_time=at, abs_freq=af, **rec))
    with open(os.path.join(REPO, "tests", "golden", "syncscore.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(len(out), "cases;", sum(o["error"] is not None for o in out), "raise")


if __name__ == "__main__":
    main()
