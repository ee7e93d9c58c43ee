"""rocprofv3 --kernel-trace csv -> per-kernel dispatch count and mean / min / max duration (ms),
stamped with this tree's FT8_BUILD_ID.

    python3 tools/kernel_summary.py <trace dir> <out.json> "<source text>"
"""
import collections
import csv
import glob
import json
import statistics as st
import sys

from pmc_traffic import build_id


def main():
    dur = collections.defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    out = {k: {"dispatches": len(v), "mean_ms": st.mean(v), "min_ms": min(v), "max_ms": max(v), "total_ms": sum(v)}
           for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))}
    json.dump({"build_id": build_id(), "source": sys.argv[3] if len(sys.argv) > 3 else sys.argv[1], "kernels": out},
              open(sys.argv[2], "w"), indent=1)
    for k, v in out.items():
        print(f"{v['total_ms']:9.3f} ms  {v['dispatches']:5d} x {v['mean_ms']:.4f}  {k}")


if __name__ == "__main__":
    main()
