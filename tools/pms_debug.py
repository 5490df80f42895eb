"""Debug helper: GPU vs oracle MST_PMS labels on one golden case; prints the distinct differing label
pairs and an exact-arithmetic recomputation of the first tree's refinement labels."""
import sys
from fractions import Fraction

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import stereomatch_amd as sm  # noqa: E402
from conftest import load_case  # noqa: E402
from oracle import oracle as O  # noqa: E402

f32 = np.float32


def rnd32(fr):
    c = f32(float(fr))
    best = None
    for cand in (np.nextafter(c, f32(-np.inf)), c, np.nextafter(c, f32(np.inf))):
        e = abs(Fraction(float(cand)) - fr)
        key = (e, int(np.array(cand, np.float32).view(np.uint32)) & 1)
        if best is None or key < best[0]:
            best = (key, cand)
    return f32(best[1])


def F(x):
    return Fraction(float(x))


def fma(a, b, c):
    return rnd32(F(a) * F(b) + F(c))


def div(a, b):
    return rnd32(F(a) / F(b))


def sqrt(a):
    # correctly rounded sqrt of a float32: candidates around float64 sqrt
    c = f32(np.sqrt(np.float64(a)))
    best = None
    for cand in (np.nextafter(c, f32(-np.inf)), c, np.nextafter(c, f32(np.inf))):
        e = abs(F(cand) * F(cand) - F(a))
        if best is None or e < best[0]:
            best = (e, cand)
    return f32(best[1])


name = sys.argv[1] if len(sys.argv) > 1 else "smooth_64x48"
z = load_case(name)
D = int(z["D"])
ctx = sm.Context(0)
p = sm.default_params(aggregator=sm.SM_AGG_PMS, c=5000.0, min_size=200, pms_iters=1, disp_total=D)
out = ctx.match(z["left"], z["right"], D, p)
labs = ctx.labels()
ref = O.stereo3dmst_pms(z["left"], z["right"], D, iters=1, c=5000.0, min_size=200)
H, W, _ = z["left"].shape
for v in ("left", "right"):
    g, o = labs[v], ref[v]["abc"]
    diff = np.any(g.view(np.uint32) != o.view(np.uint32), axis=1)
    print(v, "differing pixels", int(diff.sum()))
    pairs = {}
    for i in np.nonzero(diff)[0]:
        pairs.setdefault((tuple(o[i]), tuple(g[i])), 0)
        pairs[(tuple(o[i]), tuple(g[i]))] += 1
    for k, n in list(pairs.items())[:6]:
        print("  oracle", k[0], "gpu", k[1], "x", n)
# exact recomputation of view 0 tree 0's refinement (1 tree, no neighbours)
tree = ref["left"]["tree"]
K = tree["ntrees"]
rnd = O.glibc_random(1, 6 * W * H, K)
dice = O.pms_dice(200)
abc0 = ref["abc0"]
ts = tree["tree_start"]
sz = ts[1] - ts[0]
tp = tree["node_pix"][ts[0] + (int(rnd[0]) % sz)]
la, lb, lc = abc0[tp]
px, py = f32(tp % W), f32(tp // W)
nz = div(f32(1.0), sqrt(f32(fma(la, la, f32(lb * lb)) + f32(1.0))))
nx, ny = f32(-la * nz), f32(-lb * nz)
d = f32(fma(la, px, f32(lb * py)) + lc)
print("tp", tp, "nz nx ny d", nz, nx, ny, d)
max_n, max_d, k = f32(1.0), f32(0.5) * f32(D), 0
while max_d > f32(0.1):
    rd = fma(dice[k], max_d, d); k += 1
    if not (rd < 0 or rd > f32(D)):
        rnx = fma(max_n, dice[k], nx); rny = fma(max_n, dice[k + 1], ny); rnz = fma(max_n, dice[k + 2], nz); k += 3
        ni = div(f32(1.0), sqrt(fma(rnz, rnz, fma(rnx, rnx, f32(rny * rny)))))
        rnx, rny, rnz = f32(rnx * ni), f32(rny * ni), abs(f32(rnz * ni))
        a, b = div(-rnx, rnz), div(-rny, rnz)
        c = div(fma(rd, rnz, fma(rnx, px, f32(rny * py))), rnz)
        print("  exact label", (a, b, c))
    max_d = f32(max_d * f32(0.5)); max_n = f32(max_n * f32(0.5))
