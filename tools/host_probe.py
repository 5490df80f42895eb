"""Host time per C2 frame in the streamed loop (3 contexts, split calls): how long the host spends
inside match_begin, match_finish and the retire waits, against the frame period.
python tools/host_probe.py [frames]"""
import sys
import time

sys.path.insert(0, ".")
import stereomatch_amd as sm  # noqa: E402
from tools.synth import make_pair  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
W, H, D = 1920, 1200, 128
left, right, _ = make_pair(W, H, D, index=0)
ctxs = [sm.Context(0) for _ in range(3)]
for c in ctxs:
    c.upload(left, right)
p = sm.default_params(disp_total=D)
for c in ctxs:
    c.match_async(D, p)
    c.synchronize()
tb = tf = tr = 0.0
n = len(ctxs)
t0 = time.perf_counter()
for i in range(steps):
    a = time.perf_counter()
    ctxs[i % n].match_begin(D, p)
    b = time.perf_counter()
    if i >= 1:
        ctxs[(i - 1) % n].match_finish()
    c_ = time.perf_counter()
    if i >= n - 1:
        ctxs[(i - n + 1) % n].synchronize()
    d = time.perf_counter()
    tb += b - a
    tf += c_ - b
    tr += d - c_
ctxs[(steps - 1) % n].match_finish()
for c in ctxs:
    c.synchronize()
el = time.perf_counter() - t0
print("period %.3f ms/frame; host per frame: begin %.3f, finish %.3f (incl. layout wait), retire wait %.3f ms"
      % (el * 1e3 / steps, tb * 1e3 / steps, tf * 1e3 / steps, tr * 1e3 / steps))
