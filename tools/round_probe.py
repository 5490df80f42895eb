"""Per-round structure of the tree filter, one frame at a time (GPU only).

Runs `--frames` frames of one share (views, slices) with SM_LAYOUT_DEBUG set, so the library prints the
per-round path statistics of each frame on stderr; run it under `rocprofv3 --kernel-trace` and feed the
trace and the log to tools/round_split.py for per-round launch times.

    python tools/round_probe.py [--views 1|2|3] [--D 64] [--d0 0] [--dtotal 256] [--frames 2]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
import stereomatch_amd as sm  # noqa: E402
from tools.synth import make_pair  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--views", type=int, default=1)
ap.add_argument("--D", type=int, default=64)
ap.add_argument("--d0", type=int, default=0)
ap.add_argument("--dtotal", type=int, default=256)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1200)
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--warmup", type=int, default=3)
a = ap.parse_args()
left, right, _ = make_pair(a.width, a.height, a.dtotal, index=0)
ctx = sm.Context(0)
ctx.upload(left, right)
p = sm.default_params(disp_begin=a.d0, disp_total=a.dtotal, views=a.views)
ctx.set_kernel_timing([])
for _ in range(a.warmup):
    ctx.match_async(a.D, p)
    ctx.synchronize()
sm.set_knob("SM_LAYOUT_DEBUG", "1")  # knobs only through sm_set_knob (round 6)
for i in range(a.frames):
    print("# frame %d" % i, file=sys.stderr, flush=True)
    t = time.perf_counter()
    ctx.match_async(a.D, p)
    ctx.synchronize()
    st = ctx.stage_times()
    print("# frame %d wall %.3f ms up %.3f down %.3f" % (i, (time.perf_counter() - t) * 1e3, st["up_ms"], st["down_ms"]),
          file=sys.stderr, flush=True)
ctx.close()
