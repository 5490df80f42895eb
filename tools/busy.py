"""GPU busy fraction of a rocprofv3 kernel trace: union of kernel intervals over a window of the
last K frames' span, and per-kernel-family summed durations.  Usage:
python tools/busy.py <run_kernel_trace.csv> [skip_first_fraction]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
t0, t1 = iv[0][0], iv[-1][1]
w0 = t0 + (t1 - t0) * skip  # skip warmup / setup
sel = [x for x in iv if x[0] >= w0]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in sel:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = sel[-1][1] - sel[0][0]
fam = defaultdict(int)
for s, e, n in sel:
    fam[n.split("(")[0].replace("void ", "")[:40]] += e - s
print("window %.3f ms, busy (any kernel running) %.3f ms = %.1f %%, summed kernel time %.3f ms (%.2fx overlap)" %
      (span / 1e6, busy / 1e6, 100.0 * busy / span, sum(fam.values()) / 1e6, sum(fam.values()) / max(busy, 1)))
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:14]:
    print("  %-40s %8.3f ms" % (k, v / 1e6))
