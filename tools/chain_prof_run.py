"""One C2 match through the library named by $SM_LIB (diagnostic builds)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (HIP runtime first, as bench.py)
from stereomatch_amd import _lib  # noqa: E402
from tools.synth import make_pair  # noqa: E402

D = int(os.environ.get("D", "128"))
l, r, _ = make_pair(1920, 1200, 128)
ctx = _lib.Context(0)
ctx.match(l, r, D)
print("stages", ctx.stage_times(), flush=True)
fn = getattr(_lib.lib(), "sm_chain_times_dump", None)  # -DSM_CHAIN_TIMES builds only
if fn is not None:
    import ctypes
    fn(ctypes.cast(None, ctypes.POINTER(ctypes.c_ulonglong)), 0)  # drop the first call's entries
    ctx.match(l, r, D)
    buf = (ctypes.c_ulonglong * (4 * 65536))()
    n = fn(buf, 65536)
    for k in range(max(n, 0)):
        a, t0, t1, item = buf[4 * k], buf[4 * k + 1], buf[4 * k + 2], buf[4 * k + 3]
        print("CT %s %d %d %d %d %d %d" % (("pcwr" if a & 8 else "UDWR")[a & 3], (a >> 2) & 1, item, a >> 32, (a >> 8) & 0xFFFFFF, t0, t1))

