"""Summarise rocprofv3 --pmc CSVs per kernel (averaged over dispatches)."""
import collections
import csv
import glob
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in sys.argv[1:]:
        for f in glob.glob(path):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
                k = k.split("(")[0]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    for k, v in agg.items():
        print(k)
        for c, x in sorted(v.items()):
            n = len(disp[(k, c)])
            print(f"   {c:28s} {x / n:16.0f}  (n={n})")


if __name__ == "__main__":
    main()
