"""Per-kernel launch statistics of bench.py's timed region, from a rocprofv3 --kernel-trace of the same
command: bench.py prints the region's clock span on stderr ("# timed region rank 0 boottime_ns A B
monotonic_ns C D"); the launches whose start falls inside it are the ones its HIP-event timing covers
(the run's other phases -- parity check, warm-up, the one-frame-at-a-time diagnostic pass -- are left
out, unlike rocprofv3's --stats summary, which averages over all of them).
Usage: python tools/timed_region.py <kernel_trace.csv> <bench log> [kernel substring ...]"""
import csv
import re
import sys


def main():
    trace, log = sys.argv[1], sys.argv[2]
    names = sys.argv[3:] or ["k_up_walk", "k_down_walk", "k_up_chain", "k_down_chain"]
    span = None
    for ln in open(log):
        m = re.match(r"# timed region rank 0 boottime_ns (\d+) (\d+) monotonic_ns (\d+) (\d+)", ln)
        if m:
            span = [int(x) for x in m.groups()]
    if span is None:
        sys.exit("no timed-region line in %s" % log)
    rows = list(csv.DictReader(open(trace)))
    starts = [int(r["Start_Timestamp"]) for r in rows]
    clock = None
    for cname, a, b in (("boottime", span[0], span[1]), ("monotonic", span[2], span[3])):
        if any(a <= t <= b for t in starts):
            clock = (cname, a, b)
            break
    if clock is None:
        sys.exit("no launch inside the timed region on either clock")
    cname, a, b = clock
    print("timed region: %.3f ms (%s clock)" % ((b - a) / 1e6, cname))
    for n in names:
        sel = [r for r in rows if n in r["Kernel_Name"].split("(")[0]]
        inr = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel if a <= int(r["Start_Timestamp"]) <= b]
        alld = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel]
        if not sel:
            continue
        print("%-14s timed region: %4d launches, avg %7.1f us | whole run: %4d launches, avg %7.1f us" % (
            n, len(inr), sum(inr) / max(len(inr), 1) / 1e3, len(alld), sum(alld) / len(alld) / 1e3))


if __name__ == "__main__":
    main()
