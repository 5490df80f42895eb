"""Chain-engine occupancy from a -DSM_CHAIN_TIMES build's device prints ("CT U|D view item len M
t0 t1", 100 MHz): per launch, its span, the summed workgroup time / (256 CUs x span) (one chain
workgroup per CU), the item count and the longest item.  Usage: python tools/chain_times.py <log>"""
import sys

rows = []
for ln in open(sys.argv[1]):
    p = ln.split()
    if len(p) == 8 and p[0] == "CT":
        rows.append((p[1], int(p[2]), int(p[3]), int(p[4]), int(p[5]), int(p[6]), int(p[7])))
fin = [r for r in rows if r[0] in "WR"]  # up pieces: W = waiting for the piece below, R = repair walk
dfin = [r for r in rows if r[0] in "cpwr"]  # down pieces: p = prologue, w = wait for the piece above, r = repair
rows = [r for r in rows if r[0] in "UD"]
if fin:
    for tag, what in (("W", "wait for the piece below"), ("R", "repair walk")):
        f = sorted([r for r in fin if r[0] == tag], key=lambda r: r[5] - r[6])
        print("%s: %d pieces, max %.1f us, mean %.1f us; longest: merge at node %s" % (
            what, len(f), (f[0][6] - f[0][5]) / 100.0 if f else 0, sum(r[6] - r[5] for r in f) / 100.0 / max(len(f), 1),
            [(r[3], round((r[6] - r[5]) / 100.0, 1)) for r in f[:5]]))
for tag, what in (("c", "down prologue to its own aggregate"), ("p", "down prologue (aggregate + guess)"),
                  ("w", "down wait for the piece above"),
                  ("r", "down repair walk")):
    f = sorted([r for r in dfin if r[0] == tag], key=lambda r: r[5] - r[6])
    if f:
        print("%s: %d pieces, max %.1f us, mean %.1f us; longest: (len|merge node, us) %s" % (
            what, len(f), (f[0][6] - f[0][5]) / 100.0, sum(r[6] - r[5] for r in f) / 100.0 / len(f),
            [(r[3], round((r[6] - r[5]) / 100.0, 1)) for r in f[:5]]))
rows.sort(key=lambda r: r[5])
launches, cur, end = [], [], 0
for r in rows:
    if cur and (r[5] >= end or r[0] != cur[0][0]):
        launches.append(cur)
        cur = []
    cur.append(r)
    end = max(end if cur[1:] else 0, r[6])
if cur:
    launches.append(cur)
tot = {"U": [0.0, 0.0], "D": [0.0, 0.0]}
for L in launches:
    t0 = min(r[5] for r in L)
    t1 = max(r[6] for r in L)
    span = (t1 - t0) / 100.0  # us
    busy = sum(r[6] - r[5] for r in L) / 100.0
    longest = max(L, key=lambda r: r[6] - r[5])
    nodes = sum(r[3] for r in L)
    tot[L[0][0]][0] += span
    tot[L[0][0]][1] += busy
    print("%s items %4d nodes %7d span %7.1f us  util %4.0f%%  longest %6.1f us (len %d, M %d)  mean %5.1f us" % (
        L[0][0], len(L), nodes, span, 100 * busy / (256 * span) if span else 0, (longest[6] - longest[5]) / 100.0,
        longest[3], longest[4], busy / len(L)))
for k, (sp, bu) in tot.items():
    print("%s total span %.1f us, busy/256 %.1f us" % (k, sp, bu / 256))
