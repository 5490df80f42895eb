"""Host segmentation timing (sm_segment_forest, segment mode's serial part) on a synthetic C2 view:
python tools/seg_bench.py [W H] [reps].  CPU only; checks the forest against the oracle's once."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from stereomatch_amd import _lib as L  # noqa: E402
from tools.synth import make_pair  # noqa: E402


def main():
    W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1920, 1200)
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    left, _, _ = make_pair(W, H, 128, index=0)
    wR, wD = O.edge_weights(O.median3(left))
    wR = np.ascontiguousarray(wR, np.uint16)
    wD = np.ascontiguousarray(wD, np.uint16)
    lib = ctypes.CDLL(L.LIB_PATH)
    f = lib.sm_segment_forest
    P = ctypes.c_void_p
    f.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, P, P, P, P]
    N = W * H
    mR, mD = np.zeros(N, np.uint8), np.zeros(N, np.uint8)
    fR, fD = np.zeros(N, np.uint16), np.zeros(N, np.uint16)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        k = f(wR.ctypes.data, wD.ctypes.data, W, H, 5000.0, 200, mR.ctypes.data, mD.ctypes.data, fR.ctypes.data,
              fD.ctypes.data)
        ts.append(time.perf_counter() - t)
    print("trees %d  ms %s" % (k, " ".join("%.1f" % (1e3 * x) for x in ts)))
    if os.environ.get("CHECK", "1") == "1":
        mask, _ = O.segment(W, H, wR, wD, 5000.0, 200)
        print("oracle trees", O.bfs(W, H, wR, wD, mask)["ntrees"])


if __name__ == "__main__":
    main()
