"""Repair statistics of the long-path pieces (knob SM_PIECE_DEBUG: per call on stderr) for one C2 frame.
python tools/piece_stats.py [W H D]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stereomatch_amd as sm  # noqa: E402
from tools.synth import make_pair  # noqa: E402

W, H, D = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (1920, 1200, 128)))
left, right, _ = make_pair(W, H, D, index=0)
ctx = sm.Context(0)
ctx.upload(left, right)
sm.set_knob("SM_PIECE_DEBUG", "1")
for _ in range(2):
    ctx.match_async(D, sm.default_params())
    ctx.synchronize()
ctx.close()
