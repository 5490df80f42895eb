"""Pin the MST_PMS random streams (Stereo3DMST.cpp:390-430, :554, :584, :72-80) against the C/C++
runtimes of this container, and write tests/golden/pms/rng_streams.npz.

The reference draws from two third-party generators (not in /root/reference; published algorithms):
  * std::default_random_engine = minstd_rand0 (libstdc++; the shipped build/StereoYin names
    linear_congruential_engine<unsigned long,16807,0,2147483647> in MST_PMS's signature) through
    std::uniform_real_distribution<float>, bound with std::bind to a copy of a default-seeded engine;
  * glibc rand()/random() (random_rgb's 3 draws per pixel and MST_PMS's one draw per tree).
This script compiles a small C++ program of its own against this container's libstdc++ (g++), calls
glibc's random() through ctypes, and checks the oracle's restatements (oracle/sm_oracle_pms.c) against
both.  One known difference is allowed and asserted: GCC >= 7's generate_canonical clamps a result of
exactly 1.0f to nextafter(1, 0); the shipped GCC 5.4 code has no clamp (its disassembly,
build/StereoYin 0x40ff38-0x40ff63, multiplies by 2^-31 and uses the result), and the oracle follows the
binary.  In the minstd_rand0 stream from seed 1 the first such draw is index 32,807,962 (of 2e9: 56),
far beyond what one MST_PMS call consumes; the init labels of a 3840x2160 image use ~29.5M draws.

Run from the repo root:  python tests/golden/make_rng_golden.py
"""
import ctypes
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

N = 200000
CPP = r"""
#include <cstdio>
#include <functional>
#include <random>
int main(int argc, char** argv) {
    long n = atol(argv[1]);
    std::default_random_engine g0;                       // default seed (1)
    std::uniform_real_distribution<float> d01(0.0f, 1.0f);
    auto dice01 = std::bind(d01, g0);                    // Stereo3DMST.cpp:390-392
    std::default_random_engine g1;
    std::uniform_real_distribution<float> d11(-1.0f, 1.0f);
    auto dice11 = std::bind(d11, g1);                    // :554 / :851-852
    std::minstd_rand0 raw;
    for (long k = 0; k < n; ++k) {
        float a = dice01(), b = dice11();
        unsigned long u = raw();
        std::fwrite(&a, 4, 1, stdout); std::fwrite(&b, 4, 1, stdout); std::fwrite(&u, 8, 1, stdout);
    }
    return 0;
}
"""


def libstdcxx_streams(n):
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "rng.cpp")
        exe = os.path.join(td, "rng")
        with open(src, "w") as f:
            f.write(CPP)
        subprocess.run(["g++", "-O2", "-std=c++11", "-o", exe, src], check=True)
        out = subprocess.run([exe, str(n)], check=True, stdout=subprocess.PIPE).stdout
    rec = np.frombuffer(out, dtype=np.dtype([("a", "<f4"), ("b", "<f4"), ("u", "<u8")]))
    return rec["a"].copy(), rec["b"].copy(), rec["u"].copy()


def main():
    a01, a11, raw = libstdcxx_streams(N)
    # minstd_rand0 itself
    s = 1
    mine_raw = np.empty(N, np.uint64)
    for k in range(N):
        s = (s * 16807) % 2147483647
        mine_raw[k] = s
    assert np.array_equal(raw, mine_raw), "minstd_rand0 restatement differs from libstdc++"
    # the oracle's canonical floats and dice (the clamp never triggers in this prefix)
    canon = ((raw - 1).astype(np.int64).astype(np.float32) * np.float32(2.0 ** -31)).astype(np.float32)
    assert not (canon >= 1.0).any()
    assert np.array_equal(a01.view(np.uint32), canon.view(np.uint32)), "uniform(0,1) differs from libstdc++"
    dice = O.pms_dice(N)
    assert np.array_equal(a11.view(np.uint32), dice.view(np.uint32)), "uniform(-1,1) dice differ from libstdc++"
    # glibc random() (rand() returns the same stream)
    libc = ctypes.CDLL("libc.so.6")
    libc.random.restype = ctypes.c_long
    libc.srandom(1)
    g = np.array([libc.random() for _ in range(50000)], np.int64)
    mine = O.glibc_random(1, 0, 50000)
    assert np.array_equal(g, mine), "glibc random() restatement differs"
    skip = O.glibc_random(1, 40000, 1000)
    assert np.array_equal(skip, g[40000:41000])
    # init labels of a small image from the libstdc++ (0,1) stream, restated in numpy float32 with the
    # binary's operation order (fma where build/StereoYin has vfmadd)
    W, H, D = 16, 12, 64
    init = O.pms_init_labels(W, H, D)
    f32 = np.float32
    k = 0
    ref = np.empty((H * W, 3), np.float32)

    from fractions import Fraction

    def fma(x, y, z):  # fused multiply-add of float32 values: the exact value, rounded once to float32
        r = Fraction(float(x)) * Fraction(float(y)) + Fraction(float(z))
        c = f32(float(r))
        best = None
        for cand in (np.nextafter(c, f32(-np.inf)), c, np.nextafter(c, f32(np.inf))):
            e = abs(Fraction(float(cand)) - r)
            key = (e, int(np.array(cand, np.float32).view(np.uint32)) & 1)  # ties to even
            if best is None or key < best[0]:
                best = (key, cand)
        return f32(best[1])

    for y in range(H):
        for x in range(W):
            d = f32(a01[k] * f32(D)); k += 1
            while True:
                x1 = a01[k]; x2 = a01[k + 1]; k += 2
                s1 = f32(x1 * x1); s2 = f32(x2 * x2)
                if f32(s1 + s2) < f32(1.0):
                    break
            root = f32(np.sqrt(f32(f32(f32(1.0) - s1) - s2)))
            nx = f32(f32(x1 + x1) * root); ny = f32(f32(x2 + x2) * root)
            nz = f32(np.sqrt(fma(-ny, ny, fma(-nx, nx, f32(1.0)))))
            ref[y * W + x] = (f32(-nx / nz), f32(-ny / nz), f32(fma(nz, d, fma(f32(x), nx, f32(ny * f32(y)))) / nz))
    assert np.array_equal(init.view(np.uint32), ref.view(np.uint32)), "init labels differ from the restated loop"
    out = os.path.join(ROOT, "tests", "golden", "pms", "rng_streams.npz")
    np.savez_compressed(out, dice=a11[:8192], canon01=a01[:8192], glibc=g[:8192].astype(np.int32),
                        glibc_skip40000=skip, init_16x12_d64=ref)
    print("rng streams pinned (libstdc++ %s, glibc); wrote %s" % (subprocess.run(["g++", "-dumpversion"],
          stdout=subprocess.PIPE, text=True).stdout.strip(), out))


if __name__ == "__main__":
    main()
