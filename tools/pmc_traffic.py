"""HBM traffic per launch from rocprofv3 PMC passes (MI355X_MICROARCH.md "HBM [CDNA4]"): FETCH_SIZE
and WRITE_SIZE in separate passes (they do not fit one pass), kilobytes -> bytes, averaged over the
dispatches of each kernel.  gfx950 reports FETCH_SIZE at half the bytes of wide coalesced streaming
reads; both the raw and the doubled figure are kept.  Writes profiles/<name>.json for bench.py.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/f -o run -- python3 tools/bp_only.py
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/w -o run -- python3 tools/bp_only.py
    python3 tools/pmc_traffic.py /tmp/f /tmp/w profiles/r1_pmc_traffic.json
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


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            acc[k].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("ft8::"):
            continue
        f, w = fetch.get(k), write.get(k)
        out[k] = {"fetch_bytes_raw": f, "fetch_bytes_x2": 2 * f if f is not None else None, "write_bytes": w,
                  "hbm_bytes": (2 * f if f is not None else 0) + (w or 0)}
    what = sys.argv[4] if len(sys.argv) > 4 else "tools/bp_only.py (256 slots, config 3)"
    json.dump({"build_id": build_id(), "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of {what}; "
                         "FETCH_SIZE doubled per the gfx950 correction; bytes per launch (mean over dispatches)",
               "kernels": out}, open(sys.argv[3], "w"), indent=1)
    for k, v in out.items():
        print(k, {a: (round(b / 1e6, 2) if b else b) for a, b in v.items()}, "MB")


if __name__ == "__main__":
    main()
