"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one or more passes).
usage: python tools/pmc_table.py DIR [name-filter]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            k = (r["Dispatch_Id"], r["Counter_Name"])
            per[k] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in per.items():
            n = names[d]
            if filt in n:
                acc[n.split("(")[0][:70]][c].append(v)
    for n, cs in acc.items():
        print(n)
        for c in sorted(cs):
            v = cs[c]
            print(f"   {c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")


if __name__ == "__main__":
    main()
