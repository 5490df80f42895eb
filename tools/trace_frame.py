"""Per-launch timeline of one frame in a rocprofv3 kernel trace (tools/gpu_trace.sh output).
Usage: python tools/trace_frame.py gpurun_out/<dir>/run_kernel_trace.csv [--frame K] [substring filter...]
--frame K: the K-th frame (negative: from the end; default -1).  bench.py runs warmup, timed, 2
diagnostic frames (every launch timed with HIP events) and 3 wall-clock frames (one at a time, no
per-launch events; then the host-I/O frames unless --no-host-io): with --no-host-io, -1 is the last
wall-clock frame and -6 the last timed one."""
import csv
import sys

args = sys.argv[2:]
frame = -1
if len(args) >= 2 and args[0] == "--frame":
    frame = int(args[1])
    args = args[2:]
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_prep" in r["Kernel_Name"]]
k = idx[frame] if frame < 0 else idx[frame]
nxt = [i for i in idx if i > k]
last = rows[k:nxt[0]] if nxt else rows[k:]
t0 = int(last[0]["Start_Timestamp"])
prev = t0
keep = args or ["up_", "down_"]
for r in last:
    s, e, n = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]
    if any(k in n for k in keep):
        print("%8.1f %7.1f gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, n[:60]))
    prev = e
print("frame %.1f us" % ((int(last[-1]["End_Timestamp"]) - t0) / 1e3))
