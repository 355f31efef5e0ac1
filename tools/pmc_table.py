#!/usr/bin/env python
"""Per-kernel per-wave averages of every counter in a rocprofv3 --pmc run.

usage: python tools/pmc_table.py gpurun_out/pmc_<name> [kernel-substring ...]
"""
import collections
import csv
import os
import re
import sys


def short(name):
    name = name.replace("wgsr::(anonymous namespace)::", "").replace("void ", "")
    return re.split(r"[(]", name, maxsplit=1)[0]


def main():
    root = sys.argv[1]
    pats = sys.argv[2:]
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(os.path.join(root, "run_counter_collection.csv"))):
        d[(short(r["Kernel_Name"]), int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key, cs in sorted(d.items()):
        if pats and not any(p in key[0] for p in pats):
            continue
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        waves = avg.get("SQ_WAVES") or 1.0
        cols = "  ".join(f"{c}={avg[c] / waves:.0f}" for c in sorted(avg) if c != "SQ_WAVES")
        print(f"{key[0][:40]:40s} grid={key[1]:8d} waves={waves:.0f}  per-wave: {cols}")


if __name__ == "__main__":
    main()
