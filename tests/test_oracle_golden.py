"""CPU: the oracle restatement against the committed golden fixtures.

ref_* fields are outputs of the reference's own segment-graph.h/disjoint-set.h
(compiled from /root/reference into oracle/_ref, tests/golden/make_golden.py); the rest
are oracle regression vectors.  Also pins the S/S2 tables independently of any libm.
"""
import decimal
import fractions
import struct

import numpy as np
import pytest

from conftest import golden_cases, load_case
from oracle import oracle as O

CASES = golden_cases()


@pytest.mark.parametrize("name", CASES)
def test_oracle_mst_matches_reference_segment_graph(name):
    z = load_case(name)
    H, W, _ = z["left"].shape
    for v in ("left", "right"):
        wR, wD = z[v + "_wR"], z[v + "_wD"]
        mask, ncomp = O.segment(W, H, wR, wD, float("inf"), 200)
        assert ncomp == 1
        np.testing.assert_array_equal(mask, z[v + "_ref_mst_mask"])
        # spanning tree: N-1 edges
        assert int(np.unpackbits(mask[:, None], axis=1)[:, -2:].sum()) == W * H - 1
        # segment mode (c=5000, segment_graph alone) against the reference too
        seg, nseg = O.segment(W, H, wR, wD, 5000.0, -1)
        np.testing.assert_array_equal(seg, z[v + "_ref_seg_mask"])
        assert nseg == int(z[v + "_ref_seg_nsets"])


@pytest.mark.parametrize("name", CASES)
def test_oracle_regression(name):
    z = load_case(name)
    D = int(z["D"])
    res = O.match(z["left"], z["right"], D, want_volumes=("left_Aup" in z))
    for v in ("left", "right"):
        t = res[v]["tree"]
        np.testing.assert_array_equal(t["med"], z[v + "_median"])
        np.testing.assert_array_equal(t["wR"], z[v + "_wR"])
        np.testing.assert_array_equal(t["node_pix"], z[v + "_node_pix"])
        np.testing.assert_array_equal(t["node_parent"], z[v + "_node_parent"])
        np.testing.assert_array_equal(res[v]["vol"], z[v + "_vol"])
        np.testing.assert_array_equal(res[v]["idx"], z[v + "_idx"])
        assert np.array_equal(res[v]["minc"].view(np.uint64), z[v + "_minc"].view(np.uint64))
        if v + "_Aup" in z:
            assert np.array_equal(res[v]["Aup"].view(np.uint64), z[v + "_Aup"].view(np.uint64))
            assert np.array_equal(res[v]["A"].view(np.uint64), z[v + "_A"].view(np.uint64))


def test_s_tables_correctly_rounded():
    """S(w)=exp(-w*(double)(1.0f/12.f)) correctly rounded (glibc 2.23 semantics), S2=fma(-S,S,1)."""
    S, S2 = O.s_lut(), O.s2_lut()
    g = struct.unpack("f", struct.pack("f", 1.0 / 12.0))[0]
    decimal.getcontext().prec = 70
    for w in range(766):
        x = (-float(w)) * g
        assert S[w] == float(decimal.Decimal(x).exp()), w
        exact = fractions.Fraction(1) - fractions.Fraction(S[w]) * fractions.Fraction(S[w])
        assert S2[w] == float(exact), w
    assert S[0] == 1.0 and S2[0] == 0.0


def test_agd_color_term_table():
    """0.11f*fminf((float)(l1*0.33333333333), 7.0f) in IEEE single precision."""
    f32 = np.float32
    for l1 in range(766):
        exp = f32(0.11) * min(f32(l1 * 0.33333333333), f32(7.0))
        assert O.lib().orc_agd_color_term(l1) == exp
