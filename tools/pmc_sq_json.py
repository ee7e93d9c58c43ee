"""SQ/GRBM counter pass (tools/experiments/gpu_pmc_all.sh) -> profiles/<name>.json: per kernel, the last dispatch's
counters plus derived fractions.  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
summed over waves; GRBM_GUI_ACTIVE counts cycles summed over the 8 XCDs (MI355X_MICROARCH.md), so

    valu_busy_per_simd = 4 * SQ_ACTIVE_INST_VALU / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8)
    resident_waves_per_cu = 4 * SQ_WAVE_CYCLES / 256 CUs / (GRBM_GUI_ACTIVE / 8)

    python3 tools/pmc_sq_json.py gpurun_out/sqpmc profiles/r1_v13_pmc.json "<source text>"
"""
import collections
import csv
import glob
import json
import sys


def build_id():
    """FT8_BUILD_ID of the library in this tree (the build the counters were collected on: the
    passes run from the same tree, right before this script); bench.py reports the counters only
    when it equals the id of the library it loads."""
    import ctypes
    import os
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ft8_demodulator_amd", "lib",
                       "libft8hip.so")
    L = ctypes.CDLL(lib)
    L.ft8_build_id.restype = ctypes.c_char_p
    return L.ft8_build_id().decode()


def main():
    last = collections.defaultdict(dict)
    for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            k = k.replace("ft8::", "")
            d = int(r["Dispatch_Id"])
            c = r["Counter_Name"]
            prev = last[k].get(c)
            if prev is None or d >= prev[0]:
                last[k][c] = (d, float(r["Counter_Value"]))
    out = {}
    for k, cs in last.items():
        v = {c: x for c, (_, x) in cs.items()}
        wc = v.get("SQ_WAVE_CYCLES", 0.0)
        g = v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if wc > 0:
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if c in v:
                    v["frac_" + c[3:].lower() + "_per_wave"] = v[c] / wc
        if g > 0:
            if "SQ_ACTIVE_INST_VALU" in v:
                v["valu_busy_per_simd"] = 4.0 * v["SQ_ACTIVE_INST_VALU"] / 1024.0 / g
            v["resident_waves_per_cu"] = 4.0 * wc / 256.0 / g
            v["kernel_cycles"] = g
        out[k] = v
    json.dump({"build_id": build_id(), "source": sys.argv[3] if len(sys.argv) > 3 else sys.argv[1], "kernels": out},
              open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
