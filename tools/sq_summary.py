"""Sum rocprofv3 SQ counters per kernel family: python tools/sq_summary.py <dir> [<dir>...]"""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:int(__import__("os").environ.get("TOP", "12"))]:
    w = c.get("SQ_WAVES", 1) or 1
    wc = c.get("SQ_WAVE_CYCLES", 0)
    print("%-28s waves %9.0f  cyc/wave %9.0f  wait %4.0f%%  waitinst %4.0f%%  active %4.0f%%  valu/w %7.0f vmem/w %6.0f lds/w %6.0f"
          % (k[:28], w, wc / w, 100 * c.get("SQ_WAIT_ANY", 0) / max(wc, 1), 100 * c.get("SQ_WAIT_INST_ANY", 0) / max(wc, 1),
             100 * c.get("SQ_ACTIVE_INST_ANY", 0) / max(wc, 1), c.get("SQ_INSTS_VALU", 0) / w, c.get("SQ_INSTS_VMEM_RD", 0) / w,
             c.get("SQ_INSTS_LDS", 0) / w))
    extra = {n: v for n, v in c.items() if n not in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                     "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS")}
    if extra:
        print("      " + "  ".join("%s=%.3g" % (n.replace("SQ_", ""), v / w) for n, v in sorted(extra.items())))
