"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel totals per step.

usage: python tools/prof_summary.py <kernel_stats.csv> [steps]
"""
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import _demangle  # noqa: E402


def short(name: str) -> str:
    if name.startswith("_Z"):       # rocprofv3's demangler gives up on __bf16 (DF16b) templates
        name = _demangle([name])[name]
    if name.startswith("void "):
        name = name[5:]
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
