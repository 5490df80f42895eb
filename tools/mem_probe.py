"""Device memory of one context after a frame (GPU only): hipMemGetInfo's used bytes before the context
and after one full frame of W x H x D, both views.  python tools/mem_probe.py [W H D]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import stereomatch_amd as sm  # noqa: E402
from tools.synth import make_pair  # noqa: E402

W, H, D = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (3840, 2160, 256)))
torch.cuda.init()
free0, tot = torch.cuda.mem_get_info(0)
left, right, _ = make_pair(W, H, D, index=0)
ctx = sm.Context(0)
ctx.upload(left, right)
for _ in range(2):
    ctx.match_async(D, sm.default_params())
    ctx.synchronize()
free1, _ = torch.cuda.mem_get_info(0)
print("context %dx%d D=%d: %.2f GB of device memory (total %.1f GB)" % (W, H, D, (free0 - free1) / 1e9, tot / 1e9), flush=True)
ctx.close()
