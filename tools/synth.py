"""Seeded synthetic stereo pairs (SURVEY.md §8(d) "Synthetic inputs").

left  : 3-octave value noise + uniform +-4 noise, BGR uint8
disp  : K slanted planes d = a*x + b*y + c on Voronoi cells, clipped to [0, D-1]
right : right(x, y) = left(x + d(x, y), y) by backward warp; out-of-image holes = noise
seed  : 20261015 + pair index
"""
import numpy as np

BASE_SEED = 20261015


def _value_noise(rng, H, W, cell):
    gh, gw = H // cell + 2, W // cell + 2
    g = rng.uniform(0, 1, (gh, gw, 3))
    ys = np.arange(H) / cell
    xs = np.arange(W) / cell
    y0 = ys.astype(np.int64); x0 = xs.astype(np.int64)
    fy = (ys - y0)[:, None, None]; fx = (xs - x0)[None, :, None]
    fy = fy * fy * (3 - 2 * fy); fx = fx * fx * (3 - 2 * fx)
    a = g[y0][:, x0]; b = g[y0][:, x0 + 1]; c = g[y0 + 1][:, x0]; d = g[y0 + 1][:, x0 + 1]
    return (a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy


def make_pair(W, H, D, index=0, planes=None):
    rng = np.random.default_rng(BASE_SEED + index)
    Wp = W + D + 2
    tex = 0.55 * _value_noise(rng, H, Wp, 64) + 0.3 * _value_noise(rng, H, Wp, 16) + 0.15 * _value_noise(rng, H, Wp, 4)
    tex = tex * 255.0 + rng.uniform(-4, 4, tex.shape)
    big = np.clip(tex, 0, 255).astype(np.uint8)
    left = np.ascontiguousarray(big[:, :W])
    K = planes or (64 if W * H <= 2304000 else 256)
    cy = rng.uniform(0, H, K); cx = rng.uniform(0, W, K)
    pa = rng.uniform(-0.02, 0.02, K); pb = rng.uniform(-0.02, 0.02, K); pc = rng.uniform(0, D - 1, K)
    # nearest seed per pixel, computed on a coarse grid and upsampled (Voronoi cells)
    step = 4
    gy, gx = np.mgrid[0:H:step, 0:W:step]
    best = np.full(gy.shape, np.inf); lab = np.zeros(gy.shape, np.int64)
    for k in range(K):
        dd = (gy - cy[k]) ** 2 + (gx - cx[k]) ** 2
        m = dd < best
        best[m] = dd[m]; lab[m] = k
    lab = np.repeat(np.repeat(lab, step, 0), step, 1)[:H, :W]
    yy, xx = np.mgrid[0:H, 0:W]
    disp = np.clip(pa[lab] * (xx - cx[lab]) + pb[lab] * (yy - cy[lab]) + pc[lab], 0, D - 1)
    src = np.rint(xx + disp).astype(np.int64)
    right = big[yy, np.clip(src, 0, Wp - 1)]
    hole = src >= Wp
    right[hole] = rng.integers(0, 256, (int(hole.sum()), 3))
    return left, np.ascontiguousarray(right), disp.astype(np.float32)
