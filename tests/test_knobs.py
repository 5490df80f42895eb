"""The product library reads no environment variable: its tuning / diagnostic knobs come only from
sm_set_knob (include/stereomst.h), and the experiment switches that skip work exist only in -DSM_DEV
builds.  bench.py refuses to print a headline with any SM_* variable set.  CPU only (no GPU call)."""
import glob
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "stereomatch_amd", "libstereomst.so")
CSRC = os.path.join(ROOT, "stereomatch_amd", "csrc")
# switches that skip or corrupt work, and settled A/B paths: SM_DEV builds only
DEV_ONLY = ["SM_EXP_SKIP", "SM_EXP_FILTER_ONLY", "SM_GF_DBG", "SM_WALK_LDS_PAD", "SM_NO_PIECES", "SM_NO_HALF_WAVE",
            "SM_NO_DPAD32", "SM_EVENT_FENCE", "SM_NO_KTIMING", "SM_RUN_DIV", "SM_RUN_CAP", "SM_SEG_SYNC",
            "SM_WALK_FILL"]


def test_product_library_has_no_experiment_switches():
    data = open(LIB, "rb").read()
    assert data.count(b"SM_EXP") == 0
    for name in DEV_ONLY:
        assert re.search(re.escape(name.encode()) + rb"[^A-Z_]", data) is None, name


def test_no_environment_reads_outside_the_dev_build():
    """getenv appears only in sm_knob.h / sm_knob.cpp, and there only under SM_DEV."""
    for f in glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(CSRC, "*.hip")) + \
            glob.glob(os.path.join(CSRC, "*.h")):
        src = open(f).read()
        if os.path.basename(f) in ("sm_knob.h", "sm_knob.cpp"):
            for m in re.finditer(r"getenv\(", src):
                assert src.rfind("#ifdef SM_DEV", 0, m.start()) > src.rfind("#endif", 0, m.start()), f
            continue
        assert "getenv(" not in src, f


def test_set_knob_accepts_knobs_and_rejects_others():
    import stereomatch_amd as sm
    names = sm.knob_names()
    assert "SM_PIECE_LEN" in names and "SM_TEST_PMS_CYCLE" in names
    for name in DEV_ONLY:
        assert name not in names
    sm.set_knob("SM_PIECE_LEN", 64)
    sm.set_knob("SM_PIECE_LEN", None)
    with pytest.raises(sm.StereoMSTError):
        sm.set_knob("SM_EXP_SKIP", "mst")
    with pytest.raises(sm.StereoMSTError):
        sm.set_knob("NOT_A_KNOB", "1")


@pytest.mark.parametrize("var", ["SM_EXP_SKIP=mst", "SM_LIB=/tmp/variant.so", "SM_PIECE_LEN=64"])
def test_bench_refuses_sm_environment(var):
    k, v = var.split("=", 1)
    env = dict(os.environ, **{k: v})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--plan-only"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 2
    assert "refusing to print a headline" in r.stderr and k in r.stderr
    assert not r.stdout.strip()
