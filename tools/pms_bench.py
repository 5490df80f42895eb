"""MST_PMS (SM_AGG_PMS) timing at a given size: the GPU's per-call times (first call serial, later calls
speculative) and, optionally, the oracle's (serial CPU restatement) for one call per view.

python tools/pms_bench.py W H D ITERS [--oracle] [--c 5000 --min-size 200]"""
import argparse
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import stereomatch_amd as sm  # noqa: E402
from tools.synth import make_pair  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("W", type=int)
ap.add_argument("H", type=int)
ap.add_argument("D", type=int)
ap.add_argument("iters", type=int)
ap.add_argument("--c", type=float, default=5000.0)
ap.add_argument("--min-size", type=int, default=200)
ap.add_argument("--oracle", action="store_true")
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
left, right, _ = make_pair(a.W, a.H, a.D, index=0)
ctx = sm.Context(0)
p = sm.default_params(aggregator=sm.SM_AGG_PMS, c=a.c, min_size=a.min_size, pms_iters=a.iters, disp_total=a.D)
res = {}
for rep in range(a.reps):
    t = time.time()
    out = ctx.match(left, right, a.D, p)
    wall = (time.time() - t) * 1e3
    st = ctx.pms_stats()
    print("rep %d wall %.1f ms %s" % (rep, wall, json.dumps(st)), flush=True)
res["gpu"] = st
res["gpu"]["wall_ms"] = wall
if a.iters > 1:
    res["gpu"]["ms_per_later_call_per_view"] = st["iters_ms"] / (2 * (a.iters - 1))
res["gpu"]["ms_first_call_per_view"] = st["iter0_ms"] / 2
if a.oracle:
    from oracle import oracle as O
    import os
    t = time.time()
    ref = O.stereo3dmst_pms(left, right, a.D, iters=1, c=a.c, min_size=a.min_size)
    res["oracle_one_call_both_views_s"] = time.time() - t
    labs = ctx.labels() if a.iters == 1 else None
    if labs is not None:
        res["bitexact_1call"] = all(np.array_equal(labs[v].view(np.uint32), ref[v]["abc"].view(np.uint32)) for v in ("left", "right"))
print(json.dumps(res), flush=True)
