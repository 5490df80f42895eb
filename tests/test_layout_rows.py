"""Compact A rows of the GPU tree layout (round 6, sm_common.h SmMeta): every light children's parent
holds a distinct row below n_has_light in its fourth child word, every path head's parent word is
SM_HEAD | its parent's row, every other node's the previous slot.  The library's own host check
(knob SM_LAYOUT_CHECK, sm_api.cpp layout_check) reads the metadata back after sm_build_tree and fails
the call on any violation; these cases cover image sizes that are not multiples of the 32x32 layout
tiles (partial tile waves), a single row / column and the constant-image comb."""
import numpy as np
import pytest

import stereomatch_amd as sm
from tools.synth import make_pair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sm.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("W,H,idx", [(160, 120, 7), (97, 61, 2), (33, 31, 5), (1920, 1200, 0)])
def test_rows_textured(ctx, knobs, W, H, idx):
    knobs.setenv("SM_LAYOUT_CHECK", "1")
    left, right, _ = make_pair(W, H, 16, index=idx)
    for img in (left, right):
        t = ctx.build_tree(img)
        assert int(t["slot_of_pix"][0]) == 0  # the root (pixel 0) is slot 0


@pytest.mark.parametrize("W,H", [(1, 777), (777, 1), (64, 64), (95, 70)])
def test_rows_constant(ctx, knobs, W, H):
    knobs.setenv("SM_LAYOUT_CHECK", "1")
    img = np.full((H, W, 3), 128, np.uint8)
    t = ctx.build_tree(img)
    assert int(t["slot_of_pix"][0]) == 0


def test_rows_segment_forest(ctx, knobs):
    knobs.setenv("SM_LAYOUT_CHECK", "1")
    left, _, _ = make_pair(320, 240, 32, index=3)
    for c in (5000.0, 300.0):
        ctx.build_tree(left, sm.default_params(c=c, min_size=20))
