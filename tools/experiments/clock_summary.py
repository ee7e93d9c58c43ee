"""Effective clock per kernel from a rocprofv3 run with --pmc GRBM_GUI_ACTIVE ... --kernel-trace
(MI355X_MICROARCH.md 'DVFS give-back': clock = GRBM_GUI_ACTIVE / 8 / kernel wall time)."""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    dur = {}
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            agg[k][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
    for k, cs in agg.items():
        g = cs.get("GRBM_GUI_ACTIVE")
        if not g:
            continue
        clk = []
        for did, v in g:
            if did in dur and dur[did][0] > 0:
                clk.append(v / 8 / dur[did][0])
        ns = [dur[did][0] for did, _ in g if did in dur]
        line = f"{k:40s} n={len(g)} dur_us={sum(ns) / max(len(ns), 1) / 1e3:9.1f} clock_GHz={sum(clk) / max(len(clk), 1):.3f}"
        for c, vals in sorted(cs.items()):
            line += f" {c}={sum(v for _, v in vals) / len(vals):.4g}"
        print(line)


if __name__ == "__main__":
    main()
