#!/usr/bin/env python
"""Compact per-kernel table from a rocprofv3 --stats kernel_stats.csv.

usage: python tools/prof_summary.py <kernel_stats.csv> [steps]
"""
import csv
import re
import sys


def short(name):
    name = name.replace("wgsr::(anonymous namespace)::", "").replace("void ", "")
    return re.split(r"[(<]", name, maxsplit=1)[0]


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = list(csv.DictReader(open(path)))
    print(f"{'kernel':32s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'pct':>6s}" +
          (f" {'us/step':>9s}" if steps else ""))
    for r in rows:
        tot = float(r["TotalDurationNs"]) / 1e6
        line = (f"{short(r['Name']):32s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} "
                f"{tot:9.3f} {float(r['Percentage']):6.2f}")
        if steps:
            line += f" {1e3 * tot / steps:9.1f}"
        print(line)


if __name__ == "__main__":
    main()
