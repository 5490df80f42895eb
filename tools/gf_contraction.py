"""How many guided-filter WTA indices would change if the helper kernels
(colorGuidedFilterHelper1-5, PatchMatchStereoGPU.cu:8185-8248) were contracted the way nvcc's
default --fmad=true does (the reference's CMakeLists.txt:19-20 sets no --fmad flag), against the
uncontracted restatement this repo ships (sm_guided.hip).  Oracle only (CPU):
    python tools/gf_contraction.py [W H D]
The contraction convention is orc_set_agd_contract's: in a*b + c*d the first product is fused."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from tools.synth import make_pair  # noqa: E402

W, H, D = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (1920, 1200, 128)
left, right, _ = make_pair(W, H, D, index=0)
res = {}
for mode in (0, 1):
    O.set_gf_contract(mode)
    res[mode] = O.guided_match(left, right, D)
O.set_gf_contract(0)
for v in ("left", "right"):
    a, b = res[0][v], res[1][v]
    dv = np.count_nonzero(a["vol"] != b["vol"])
    rel = np.abs(a["vol"] - b["vol"]) / np.maximum(np.abs(a["vol"]), 1e-30)
    flips = np.count_nonzero(a["idx"] != b["idx"])
    print("%s: filtered voxels differing %d of %d (%.3f%%), max rel diff %.3g; WTA indices flipped %d of %d (%.4f%%)" % (
        v, dv, a["vol"].size, 100.0 * dv / a["vol"].size, float(rel.max()), flips, W * H, 100.0 * flips / (W * H)))
