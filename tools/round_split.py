"""Per-round launch times of the last frame in a rocprofv3 kernel trace of tools/round_probe.py.

    python tools/round_split.py <run_kernel_trace.csv> <round_probe stderr log>

Rounds come from the library's SM_LAYOUT_DEBUG lines of the last frame (per view: long / short paths,
nodes, longest path); launches are assigned to rounds in start order (the streams are joined at every
round boundary, so a round's launches all start after the previous round's end).
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
preps = [i for i, r in enumerate(rows) if "k_prep" in r["Kernel_Name"]]
frame = rows[preps[-1]:]
fam = ("k_up_pre", "k_up_chain", "k_up_walk", "k_down_chain", "k_down_walk")
L = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in frame
     if any(f in r["Kernel_Name"] for f in fam)]

blocks = open(sys.argv[2]).read().split("# frame ")
rx = re.compile(r"view (\d) round (\d+): long (\d+) paths (\d+) nodes maxlen (\d+) \| short (\d+) paths (\d+) nodes maxlen (\d+)")
last = [b for b in blocks if rx.search(b)][-1]
st = {}
for m in rx.finditer(last):
    v, r = int(m.group(1)), int(m.group(2))
    st.setdefault(r, []).append(tuple(int(m.group(k)) for k in range(3, 9)))
nr = max(st) + 1


def agg(r):
    s = st.get(r, [])
    return (sum(x[0] for x in s), sum(x[1] for x in s), max([x[2] for x in s] or [0]),
            sum(x[3] for x in s), sum(x[4] for x in s), max([x[5] for x in s] or [0]))


pos = 0
tot = {"up": [0, 0, 0], "down": [0, 0, 0]}
prev_end = None
for pas, order in (("up", range(nr - 1, -1, -1)), ("down", range(nr))):
    print("%s pass: round | long paths nodes maxlen | short paths nodes maxlen | chain us walk us | span us gap us" % pas)
    for r in order:
        lp, ln, lm, sp, sn, sm_ = agg(r)
        k = (1 if lp else 0) + (1 if sp else 0)
        got = []
        while len([g for g in got if "pre" not in g[0]]) < k and pos < len(L):
            got.append(L[pos])
            pos += 1
        ch = sum((e - s) for n, s, e in got if "chain" in n or "pre" in n) / 1e3
        wk = sum((e - s) for n, s, e in got if "walk" in n) / 1e3
        if not got:
            continue
        s0 = min(g[1] for g in got)
        e0 = max(g[2] for g in got)
        gap = (s0 - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e0
        tot[pas][0] += (e0 - s0) / 1e3
        tot[pas][1] += ch
        tot[pas][2] += wk
        print("  %3d | %6d %8d %6d | %7d %8d %4d | %7.1f %7.1f | %7.1f %6.1f" % (r, lp, ln, lm, sp, sn, sm_, ch, wk,
                                                                             (e0 - s0) / 1e3, gap))
    print("  %s: sum of round spans %.1f us, chain launches %.1f us, walker launches %.1f us" % (pas, *tot[pas]))
span = (L[-1][2] - L[0][1]) / 1e3 if L else 0
print("filter span (first up launch start .. last down launch end): %.1f us; rounds %d; launches %d" % (span, nr, len(L)))
