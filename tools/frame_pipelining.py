"""Wall time per frame with and without a host synchronisation after every frame (C2).
Usage (GPU box): python tools/frame_pipelining.py"""
import time

import numpy as np

import stereomatch_amd as sm
from tools.synth import make_pair

W, H, D = 1920, 1200, 128
left, right, _ = make_pair(W, H, D, index=0)
ctx = sm.Context(0)
ctx.upload(left, right)
params = sm.default_params(disp_begin=0, disp_total=D)
for _ in range(3):
    ctx.match_async(D, params)
    ctx.synchronize()
for mode in ("sync", "async", "sync+stats", "dom-events", "dom-events+stats", "sync", "async", "sync+stats", "dom-events", "dom-events+stats"):
    ctx.set_kernel_timing(["k_up_walk"] if mode.startswith("dom") else [])
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        ctx.match_async(D, params)
        if mode != "async":
            ctx.synchronize()
        if mode.endswith("stats"):
            ctx.stage_times()
            ctx.kernel_stats()
    ctx.synchronize()
    print(mode, "%.3f ms/frame" % ((time.perf_counter() - t0) * 1e3 / 20))
ctx.close()
