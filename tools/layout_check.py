"""Tree-layout metadata invariants on the GPU box without running any filter (sm_build_tree with the
SM_LAYOUT_CHECK knob: compact A rows, head parent words).  python tools/layout_check.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import stereomatch_amd as sm  # noqa: E402
from tools.synth import make_pair  # noqa: E402

sm.set_knob("SM_LAYOUT_CHECK", "1")
ctx = sm.Context(0)
bad = 0
for (W, H, D, idx) in [(160, 120, 24, 7), (96, 64, 16, 1), (1920, 1200, 128, 0)]:
    left, right, _ = make_pair(W, H, D, index=idx)
    for name, img in (("left", left), ("right", right)):
        try:
            t = ctx.build_tree(img)
            print("%dx%d %s: ok (root slot %d)" % (W, H, name, int(t["slot_of_pix"][0])), flush=True)
        except sm.StereoMSTError as e:
            bad += 1
            print("%dx%d %s: %s" % (W, H, name, e), flush=True)
for c in (5000.0, 300.0):
    left, _, _ = make_pair(320, 240, 32, index=3)
    try:
        ctx.build_tree(left, sm.default_params(c=c, min_size=20))
        print("segment c=%g: ok" % c, flush=True)
    except sm.StereoMSTError as e:
        bad += 1
        print("segment c=%g: %s" % (c, e), flush=True)
ctx.close()
sys.exit(1 if bad else 0)
