"""Per-launch timeline of the last frame in a rocprofv3 kernel trace (tools/gpu_trace.sh output).
Usage: python tools/trace_frame.py gpurun_out/<dir>/run_kernel_trace.csv [substring filter...]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_prep" in r["Kernel_Name"]]
last = rows[idx[-1]:]
t0 = int(last[0]["Start_Timestamp"])
prev = t0
keep = sys.argv[2:] or ["up_", "down_"]
for r in last:
    s, e, n = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]
    if any(k in n for k in keep):
        print("%8.1f %7.1f gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, n[:60]))
    prev = e
print("frame %.1f us" % ((int(last[-1]["End_Timestamp"]) - t0) / 1e3))
