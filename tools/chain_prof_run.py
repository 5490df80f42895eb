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
