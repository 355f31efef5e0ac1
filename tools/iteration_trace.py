#!/usr/bin/env python
"""One graph-replayed mapping iteration's kernels from a rocprofv3 kernel
trace of tools/bench_online.py (the span between two consecutive
k_gather_rows launches, the iteration's first kernel, taken mid-run).
usage: python tools/iteration_trace.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_gather_rows" in r["Kernel_Name"]]
i0, i1 = idx[len(idx) // 2], idx[len(idx) // 2 + 1]
t0 = int(rows[i0]["Start_Timestamp"])
busy = 0.0
print("start_us  dur_us  kernel")
for r in rows[i0:i1]:
    n = r["Kernel_Name"].replace("wgsr::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy += d
    print(f"{s:8.1f} {d:7.1f}  {n}")
print(f"iteration span {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.1f} us, {i1 - i0} kernels, "
      f"{busy:.1f} us busy (under kernel tracing)")
