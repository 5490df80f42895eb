import os, sys
sys.path.insert(0, os.getcwd())
import torch
import stereomatch_amd as sm
from tools.synth import make_pair
l, r, _ = make_pair(1920, 1200, 128, index=0)
ctx = sm.Context(0)
ctx.match(l, r, 128)
ctx.match(l, r, 128)
print(ctx.stage_times(), flush=True)
