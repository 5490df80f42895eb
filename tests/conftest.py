"""Test configuration.  Markers: `gpu` = needs an MI355X (run with -m gpu on the GPU box)."""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); parity tests through the C-ABI")
    # the oracle (test infrastructure) is a tiny C library: make sure it is built
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)


def golden_cases():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load_case(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def flir_pair():
    """The FLIR 000020 pair (BGR, 2048x1536), decode-checked against the committed sums."""
    from PIL import Image
    d = os.path.join(GOLDEN, "flir")
    L = np.ascontiguousarray(np.array(Image.open(os.path.join(d, "000020_191400042.jpg")).convert("RGB"))[:, :, ::-1])
    R = np.ascontiguousarray(np.array(Image.open(os.path.join(d, "000020_191400039.jpg")).convert("RGB"))[:, :, ::-1])
    with np.load(os.path.join(d, "decode_check.npz")) as chk:
        assert int(L.astype(np.int64).sum()) == int(chk["left_sum"])
        assert int(R.astype(np.int64).sum()) == int(chk["right_sum"])
    return L, R


@pytest.fixture(scope="session")
def gpu_ctx():
    import stereomatch_amd as sm
    if sm.device_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    ctx = sm.Context(0)
    yield ctx
    ctx.close()


class Knobs:
    """Library knobs (sm_set_knob) with monkeypatch's setenv / delenv surface; every knob set through it
    is restored to its default when the test ends.  The product library never reads the environment."""

    def __init__(self):
        self.touched = set()

    def setenv(self, name, value):
        import stereomatch_amd as sm
        sm.set_knob(name, value)
        self.touched.add(name)

    def delenv(self, name, raising=True):
        import stereomatch_amd as sm
        sm.set_knob(name, None)
        self.touched.add(name)

    def restore(self):
        import stereomatch_amd as sm
        for n in self.touched:
            sm.set_knob(n, None)


@pytest.fixture
def knobs():
    k = Knobs()
    yield k
    k.restore()
