"""Per-frame kernel times from a rocprofv3 --stats kernel_stats.csv (one frame at a time, bench.py
--inflight 1): python tools/kstats.py <kernel_stats.csv> [frames] [substring ...]"""
import csv
import sys

path = sys.argv[1]
frames = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 17
keep = [a for a in sys.argv[2:] if not a.isdigit()]
rows = list(csv.DictReader(open(path)))
tot = 0.0
for r in rows:
    n = r["Name"].split("(")[0].replace("void ", "")
    if keep and not any(k in n for k in keep):
        continue
    us = int(r["TotalDurationNs"]) / frames / 1e3
    tot += us
    print("%-44s %5.1f launches %9.1f us/frame  avg %8.1f us" % (n[:44], int(r["Calls"]) / frames, us,
                                                               float(r["AverageNs"]) / 1e3))
print("total %.1f us/frame" % tot)
