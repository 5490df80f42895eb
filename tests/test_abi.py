"""CPU: the C-ABI library loads and exports every symbol include/stereomst.h declares.
No compute calls: without a GPU every entry must fail loudly (no CPU fallback)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "stereomst.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sm_[a-z_]+)\s*\(", txt)))


def test_library_exports_all_declared_symbols():
    import stereomatch_amd as sm
    L = sm.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_library_is_gfx950_code_object(tmp_path):
    import shutil
    import subprocess
    # --offloading extracts the bundles next to its input: work on a copy in a temp dir
    so = str(tmp_path / "libstereomst.so")
    shutil.copy(os.path.join(ROOT, "stereomatch_amd", "libstereomst.so"), so)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", so], capture_output=True, text=True,
                         cwd=str(tmp_path))
    assert "gfx950" in (out.stdout + out.stderr)


def test_no_device_fails_loudly():
    import stereomatch_amd as sm
    if sm.device_count() > 0:
        pytest.skip("a device is present")
    with pytest.raises(sm.StereoMSTError):
        sm.Context(0)


def test_default_params_match_reference_constants():
    import math
    import stereomatch_amd as sm
    p = sm.default_params()
    assert p.gamma == float.fromhex("0x1.5555560000000p-4")  # 1.0f/12.f (Stereo3DMST.cpp:830)
    assert math.isinf(p.c) and p.min_size == 200 and p.median_ksize == 3
