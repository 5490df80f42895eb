"""Per-launch durations of the tree-filter kernels of the LAST step in a rocprofv3 kernel trace."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = ("walk", "chain", "up_pre")
w = [r for r in rows if any(k in r["Kernel_Name"] for k in keys)]
# the last step = everything after the last k_bor_local
last_bor = max(i for i, r in enumerate(rows) if "k_bor_local" in r["Kernel_Name"])
t0 = int(rows[last_bor]["Start_Timestamp"])
w = [r for r in w if int(r["Start_Timestamp"]) >= t0]
tot = {}
for r in w:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    tot[name] = tot.get(name, 0) + d
    print("%-28s grid %9s x %s  %9.1f us" % (name, r["Grid_Size_X"], r["Grid_Size_Y"], d))
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print("TOTAL %-28s %9.1f us" % (k, v))
