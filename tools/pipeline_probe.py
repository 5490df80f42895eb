"""Frames in flight: one context (frame after frame) vs two contexts on two streams whose frames
interleave (frame n+1's prep/MST/layout on one stream while frame n's filter runs on the other).
Usage (GPU box): python tools/pipeline_probe.py [W H D]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
import stereomatch_amd as sm  # noqa: E402
from tools.synth import make_pair  # noqa: E402

W, H, D = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (1920, 1200, 128)
left, right, _ = make_pair(W, H, D, index=0)
params = sm.default_params(disp_begin=0, disp_total=D)
NC = int(os.environ.get("NCTX", "3"))
ctxs = [sm.Context(0) for _ in range(NC)]
for c in ctxs:
    c.upload(left, right)
    c.set_kernel_timing([])
    for _ in range(2):
        c.match_async(D, params)
        c.synchronize()
K = 30
for rep in range(2):
    t0 = time.perf_counter()
    for _ in range(K):
        ctxs[0].match_async(D, params)
        ctxs[0].synchronize()
    t1 = time.perf_counter()
    print("one context: %.3f ms/frame" % ((t1 - t0) * 1e3 / K), flush=True)
    for n in range(2, NC + 1):
        t0 = time.perf_counter()
        for i in range(K):
            ctxs[i % n].match_async(D, params)  # returns after this frame's layout; its filter is queued
            if i >= n - 1:
                ctxs[(i - n + 1) % n].synchronize()
        for i in range(max(0, K - n + 1), K):
            ctxs[i % n].synchronize()
        t1 = time.perf_counter()
        print("%d contexts interleaved: %.3f ms/frame" % (n, (t1 - t0) * 1e3 / K), flush=True)
r = [c.results() for c in ctxs]
import numpy as np  # noqa: E402
assert all(np.array_equal(r[0][v]["idx"], r[1][v]["idx"]) for v in ("left", "right"))
print("results of both contexts identical")
