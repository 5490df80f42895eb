"""The drop-in shim (stereomatch_amd/shim) against the reference's link contract:
stereo3dmst exported unmangled, startTimer/getTimer with C++ linkage (_Z10startTimerv,
_Z8getTimerv), all resolved from libstereomst.so.  Compiled here against a minimal cv::Mat stub
(tests/shim_stub) because the image has no OpenCV; the real build is stereomatch_amd/shim/Makefile."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shim_compiles_and_exports_reference_symbols(tmp_path):
    so = tmp_path / "libstereo3dmst_shim.so"
    cmd = ["g++", "-std=c++17", "-O1", "-fPIC", "-shared", "-I", os.path.join(ROOT, "tests", "shim_stub"),
           os.path.join(ROOT, "stereomatch_amd", "shim", "stereo3dmst_shim.cpp"), "-o", str(so),
           "-L", os.path.join(ROOT, "stereomatch_amd"), "-lstereomst"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    syms = subprocess.run(["nm", "-D", "--defined-only", str(so)], capture_output=True, text=True).stdout.split()
    for s in ("stereo3dmst", "_Z10startTimerv", "_Z8getTimerv"):
        assert s in syms, s
    undef = subprocess.run(["nm", "-D", "--undefined-only", str(so)], capture_output=True, text=True).stdout
    for s in ("sm_match", "sm_create", "sm_default_params", "sm_start_timer", "sm_get_timer_ms", "sm_upload_cost_volumes"):
        assert s in undef, s
