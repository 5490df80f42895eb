"""Per-round MST statistics (SM_MST_DEBUG) on the bench workload; GPU only."""
import os, sys
os.environ[os.environ.get("DBG", "SM_MST_DEBUG")] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stereomatch_amd as sm
from bench import make_pair
left, right, _ = make_pair(1920, 1200, 128, index=0)
ctx = sm.Context(0)
ctx.upload(left, right)
ctx.match_async(8, sm.default_params())
ctx.synchronize()
