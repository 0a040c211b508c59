"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel totals per step.

usage: python tools/prof_summary.py <kernel_stats.csv> [steps]
"""
import csv
import re
import sys


def short(name: str) -> str:
    m = re.match(r"_ZN5vitmi\d+(\w+?)I", name)
    if name.startswith("_ZN5vitmi"):
        return name[:110]
    return name.split("(")[0][:110]


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'ms/step':>9} {'%':>6} {'calls/step':>10} {'avg us':>9}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"]) / 1e6 / steps
        if t < 0.01:
            continue
        print(f"{t:9.3f} {float(r['Percentage']):6.2f} {float(r['Calls']) / steps:10.1f} "
              f"{float(r['AverageNs']) / 1e3:9.1f}  {short(r['Name'])}")
    print(f"total kernel time per step: {tot / 1e6 / steps:.3f} ms")


if __name__ == "__main__":
    main()
