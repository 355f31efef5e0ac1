"""Print the top kernels of rocprofv3 --stats CSVs: python tools/kstat.py <csv> [n]"""
import csv
import sys

for f in sys.argv[1:]:
    if f.isdigit():
        continue
    n = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 14
    rows = list(csv.DictReader(open(f)))
    print(f)
    for r in rows[:n]:
        name = r["Name"].replace("wgsr::(anonymous namespace)::", "").replace("void ", "")
        print(f"  {name[:44]:44s} {r['Calls']:>5s} avg {float(r['AverageNs']) / 1000:8.1f} us"
              f"  min {float(r['MinNs']) / 1000:7.1f}  max {float(r['MaxNs']) / 1000:7.1f}")
