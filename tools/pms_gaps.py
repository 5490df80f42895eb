"""Per-queue busy time and launch gaps of the MST_PMS later calls from a rocprofv3 kernel trace:
python tools/pms_gaps.py run_kernel_trace.csv.  The later calls are the k_pms_guess launches' spans."""
import collections
import csv
import gzip
import sys

rows = list(csv.DictReader((gzip.open if sys.argv[1].endswith(".gz") else open)(sys.argv[1], "rt")))
key_q = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
by_q = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    by_q[r.get(key_q, "0")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
for q, ks in sorted(by_q.items()):
    ks.sort()
    guess = [k for k in ks if "k_pms_guess" in k[2]]
    if len(guess) < 2:
        continue
    t0, t1 = guess[0][0], ks[-1][1]  # from the first speculative pass to the queue's last kernel
    sel = [k for k in ks if k[0] >= t0]
    busy = 0
    last = t0
    gaps = []
    names = collections.Counter()
    dur = collections.Counter()
    for s, e, n in sel:
        if s > last:
            gaps.append(s - last)
        busy += max(0, e - max(s, last))
        last = max(last, e)
        short = n
        names[short] += 1
        dur[short] += e - s
    span = t1 - t0
    print("queue %s: later-call span %.2f ms, kernels %d, busy %.2f ms (%.0f%%), gaps %.2f ms (mean %.1f us)" % (
        q, span / 1e6, len(sel), busy / 1e6, 100.0 * busy / span, sum(gaps) / 1e6, (sum(gaps) / max(1, len(gaps))) / 1e3))
    for n, c in names.most_common(12):
        print("   %-40s %6d launches  %8.2f ms  mean %6.1f us" % (n[:40], c, dur[n] / 1e6, dur[n] / c / 1e3))
