"""How many WTA indices would change if the AGD cost (PatchMatchStereoGPU.cu:1529-1540) were
contracted the way nvcc's default --fmad=true does (the reference's CMakeLists.txt:19-20 sets no
--fmad flag), against the uncontracted restatement this repo ships.  Oracle only (CPU):
    python tools/agd_contraction.py [W H D]
Prints the cost-volume differences and the per-view WTA index flips."""
import sys
import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from tools.synth import make_pair  # noqa: E402

W, H, D = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (1920, 1200, 128)
left, right, _ = make_pair(W, H, D, index=0)
res = {}
for mode in (0, 1):
    O.set_agd_contract(mode)
    res[mode] = O.match(left, right, D)
O.set_agd_contract(0)
for v in ("left", "right"):
    a, b = res[0][v], res[1][v]
    dv = np.count_nonzero(a["vol"] != b["vol"])
    flips = np.count_nonzero(a["idx"] != b["idx"])
    print("%s: cost voxels differing %d of %d (%.3f%%), max |diff| %.3g; WTA indices flipped %d of %d (%.4f%%)" % (
        v, dv, a["vol"].size, 100.0 * dv / a["vol"].size, float(np.max(np.abs(a["vol"] - b["vol"]))), flips, W * H,
        100.0 * flips / (W * H)))
