// sm_guided.hip -- the guided-filter cost aggregator: the reference's colour
// guided filter of the AGD cost volume, each view guided by its own BGR image, then selectDisparity
// (PatchMatchStereoGPU.cu:8251-8470 costVolumeColorGuidedFilterCUDA2Streams, box means :495-580,
// WTA :1688-1737; radius 9 and eps = 0.01^2 * 255^2 at :9000-9001).  A second aggregator behind the
// same C-ABI (sm_params.aggregator = SM_AGG_GUIDED): no tree, no MST.
//
// Arithmetic (the reference's float operations in source order, uncontracted):
//   box mean  : per 32-pixel block (the reference kernels' block width) a sliding sum -- the first
//               output sums in[x0-r .. x0+r] in ascending order (0 outside the image), then
//               t += in[x+r]; t -= in[x-r-1]; out = t * (1.0f / (2r+1)) -- x pass, then y pass;
//   guide     : mean_c = box(c); var_cc' = box(c*c') - mean_c*mean_c' (+ eps on the diagonal);
//               inv = adjugate / det with det = inv_rr*var_rr + inv_rg*var_rg + inv_rb*var_rb;
//   per slice : mean_p = box(p), mean_Ip_c = box(c*p), cov_c = mean_Ip_c - mean_c*mean_p,
//               a = inv * cov, b = mean_p - a_r*mean_r - a_g*mean_g - a_b*mean_b,
//               q = box(b) + box(a_r)*r + box(a_g)*g + box(a_b)*b;
//   WTA       : strict < from 1e10f over ascending d, optional parabola (selectDisparity).
//
// Layout: planes [k][N] f32 in HBM; a batch of S slices moves through the box passes as 4*S planes
// (grid.z).  The x pass runs one thread per (row, 32-column block), the y pass one thread per
// (column, 32-row block) -- adjacent lanes read adjacent columns, so it is coalesced.  All passes
// are HBM-streaming kernels (no MFMA: per-pixel scalar arithmetic).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "sm_launch.h"

#define GF_BLOCK 32

// x pass of nplanes planes (plane stride N): thread = (row, 32-column block, plane)
__global__ __launch_bounds__(64) void k_gf_box_x(const float* __restrict__ in, float* __restrict__ out, int W, int H, int r,
                                                 size_t N) {
    const int y = blockIdx.x * 64 + threadIdx.x;
    if (y >= H) return;
    const int x0 = blockIdx.y * GF_BLOCK;
    const float* row = in + (size_t)blockIdx.z * N + (size_t)y * W;
    float* o = out + (size_t)blockIdx.z * N + (size_t)y * W;
    const float scale = 1.0f / (float)((r << 1) + 1);
    float t = 0.0f;
    for (int i = x0 - r; i <= x0 + r; ++i) t += (i < 0 || i >= W) ? 0.0f : row[i];
    o[x0] = t * scale;
    const int end = W - x0 < GF_BLOCK ? W : x0 + GF_BLOCK;
    for (int x = x0 + 1; x < end; ++x) {
        t += (x + r >= W) ? 0.0f : row[x + r];
        t -= (x - r - 1 < 0) ? 0.0f : row[x - r - 1];
        o[x] = t * scale;
    }
}

// x pass through LDS: a workgroup stages `rows` whole rows of one plane (coalesced loads), each
// thread runs one (row, 32-column block) sliding sum out of LDS -- the same operations in the same
// order as k_gf_box_x -- and the results leave through LDS again as coalesced stores.  Rows are
// padded by one float per 32 (index i + i/32), so the 64 lanes' block starts (stride 33) hit 64
// different banks.  grid = (ceil(H / rows), planes).
__global__ __launch_bounds__(256) void k_gf_box_x_lds(const float* __restrict__ in, float* __restrict__ out, int W, int H, int r,
                                                      size_t N, int rows) {
    extern __shared__ float lds[];
    const int nblk = (W + GF_BLOCK - 1) / GF_BLOCK;
    const int rl = W + nblk;  // padded row length
    float* li = lds;
    float* lo = lds + rows * rl;
    const int ya = blockIdx.x * rows;
    const int nr = H - ya < rows ? H - ya : rows;
    const float* src = in + (size_t)blockIdx.y * N + (size_t)ya * W;
    float* dst = out + (size_t)blockIdx.y * N + (size_t)ya * W;
    const int tot = nr * W;
    for (int i = threadIdx.x; i < tot; i += 256) {
        const int y = i / W, x = i - y * W;
        li[y * rl + x + (x >> 5)] = src[i];
    }
    __syncthreads();
    const int t_id = threadIdx.x;
    if (t_id < nr * nblk) {
        const int y = t_id / nblk, blk = t_id - y * nblk;
        const float* row = li + y * rl;
        float* o = lo + y * rl;
        const int x0 = blk * GF_BLOCK;
        const float scale = 1.0f / (float)((r << 1) + 1);
        float t = 0.0f;
        for (int i = x0 - r; i <= x0 + r; ++i) t += (i < 0 || i >= W) ? 0.0f : row[i + (i >> 5)];
        o[x0 + blk] = t * scale;
        const int end = W - x0 < GF_BLOCK ? W : x0 + GF_BLOCK;
        for (int x = x0 + 1; x < end; ++x) {
            const int a = x + r, b = x - r - 1;
            t += (a >= W) ? 0.0f : row[a + (a >> 5)];
            t -= (b < 0) ? 0.0f : row[b + (b >> 5)];
            o[x + blk] = t * scale;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < tot; i += 256) {
        const int y = i / W, x = i - y * W;
        dst[i] = lo[y * rl + x + (x >> 5)];
    }
}

// y pass: thread = (column, 32-row block, plane)
__global__ __launch_bounds__(256) void k_gf_box_y(const float* __restrict__ in, float* __restrict__ out, int W, int H, int r,
                                                  size_t N) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= W) return;
    const int y0 = blockIdx.y * GF_BLOCK;
    const float* col = in + (size_t)blockIdx.z * N + x;
    float* o = out + (size_t)blockIdx.z * N + x;
    const float scale = 1.0f / (float)((r << 1) + 1);
    float t = 0.0f;
    for (int i = y0 - r; i <= y0 + r; ++i) t += (i < 0 || i >= H) ? 0.0f : col[(size_t)i * W];
    o[(size_t)y0 * W] = t * scale;
    const int end = H - y0 < GF_BLOCK ? H : y0 + GF_BLOCK;
    for (int y = y0 + 1; y < end; ++y) {
        t += (y + r >= H) ? 0.0f : col[(size_t)(y + r) * W];
        t -= (y - r - 1 < 0) ? 0.0f : col[(size_t)(y - r - 1) * W];
        o[(size_t)y * W] = t * scale;
    }
}

__device__ __forceinline__ void guide_of(uint32_t bgrx, float& r, float& g, float& b) {
    b = (float)(bgrx & 255u);
    g = (float)((bgrx >> 8) & 255u);
    r = (float)((bgrx >> 16) & 255u);
}

// the 9 guide planes r, g, b, rr, gg, bb, rg, rb, gb (pointWiseMul: one rounding each)
__global__ void k_gf_guide_in(const uint32_t* __restrict__ bgrx, float* __restrict__ pl, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    float r, g, b;
    guide_of(bgrx[i], r, g, b);
    pl[i] = r;
    pl[N + i] = g;
    pl[2 * N + i] = b;
    pl[3 * N + i] = r * r;
    pl[4 * N + i] = g * g;
    pl[5 * N + i] = b * b;
    pl[6 * N + i] = r * g;
    pl[7 * N + i] = r * b;
    pl[8 * N + i] = g * b;
}

// guide statistics from the 9 box means m[]: st = mean_r, mean_g, mean_b, inv_rr, inv_rg, inv_rb,
// inv_gg, inv_gb, inv_bb (colorGuidedFilterHelper0 / 1 / 2, pointWiseDivison)
__global__ void k_gf_stats(const float* __restrict__ m, float* __restrict__ st, size_t N, float eps) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float mr = m[i], mg = m[N + i], mb = m[2 * N + i];
    const float vrr = m[3 * N + i] - mr * mr + eps;
    const float vgg = m[4 * N + i] - mg * mg + eps;
    const float vbb = m[5 * N + i] - mb * mb + eps;
    const float vrg = m[6 * N + i] - mr * mg;
    const float vrb = m[7 * N + i] - mr * mb;
    const float vgb = m[8 * N + i] - mg * mb;
    const float irr = vgg * vbb - vgb * vgb;
    const float igg = vrr * vbb - vrb * vrb;
    const float ibb = vrr * vgg - vrg * vrg;
    const float irg = vgb * vrb - vrg * vbb;
    const float irb = vrg * vgb - vgg * vrb;
    const float igb = vrb * vrg - vrr * vgb;
    const float det = irr * vrr + irg * vrg + irb * vrb;
    st[i] = mr;
    st[N + i] = mg;
    st[2 * N + i] = mb;
    st[3 * N + i] = irr / det;
    st[4 * N + i] = irg / det;
    st[5 * N + i] = irb / det;
    st[6 * N + i] = igg / det;
    st[7 * N + i] = igb / det;
    st[8 * N + i] = ibb / det;
}

// per slice s of the batch: planes [0..S) p, [S..2S) r*p, [2S..3S) g*p, [3S..4S) b*p
__global__ void k_gf_slice_in(const float* __restrict__ cost, const uint32_t* __restrict__ bgrx, float* __restrict__ pl,
                              size_t N, int S) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int s = blockIdx.y;
    float r, g, b;
    guide_of(bgrx[i], r, g, b);
    const float p = cost[(size_t)s * N + i];
    pl[(size_t)s * N + i] = p;
    pl[(size_t)(S + s) * N + i] = r * p;
    pl[(size_t)(2 * S + s) * N + i] = g * p;
    pl[(size_t)(3 * S + s) * N + i] = b * p;
}

// means -> a_r, a_g, a_b, b (colorGuidedFilterHelper3 / 2 / 4), in place over the 4S planes
__global__ void k_gf_ab(float* __restrict__ pl, const float* __restrict__ st, size_t N, int S) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int s = blockIdx.y;
    float* mp = pl + (size_t)s * N;
    float* mIr = pl + (size_t)(S + s) * N;
    float* mIg = pl + (size_t)(2 * S + s) * N;
    float* mIb = pl + (size_t)(3 * S + s) * N;
    const float m_p = mp[i];
    const float mr = st[i], mg = st[N + i], mb = st[2 * N + i];
    const float irr = st[3 * N + i], irg = st[4 * N + i], irb = st[5 * N + i];
    const float igg = st[6 * N + i], igb = st[7 * N + i], ibb = st[8 * N + i];
    const float cr = mIr[i] - mr * m_p;
    const float cg = mIg[i] - mg * m_p;
    const float cb = mIb[i] - mb * m_p;
    const float ar = irr * cr + irg * cg + irb * cb;
    const float ag = irg * cr + igg * cg + igb * cb;
    const float ab = irb * cr + igb * cg + ibb * cb;
    const float bb = m_p - ar * mr - ag * mg - ab * mb;
    mIr[i] = ar;
    mIg[i] = ag;
    mIb[i] = ab;
    mp[i] = bb;
}

// q = box(b) + box(a_r)*r + box(a_g)*g + box(a_b)*b (colorGuidedFilterHelper5), fused with the
// strict-< WTA over the batch's slices in ascending order (selectDisparity), state per pixel:
// min (1e10f), best (-1), pre / next of best (the parabola's neighbours), q of the previous slice
struct GfState {
    float* mn;
    int32_t* best;
    float* pre;
    float* nxt;
    float* prevq;
};

__global__ void k_gf_q_wta(const float* __restrict__ pl, const uint32_t* __restrict__ bgrx, GfState st, size_t N, int S,
                           int dloc0, int dtot_loc) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    float r, g, b;
    guide_of(bgrx[i], r, g, b);
    float mn = st.mn[i], pre = st.pre[i], nxt = st.nxt[i], pq = st.prevq[i];
    int best = st.best[i];
    for (int s = 0; s < S; ++s) {
        const int d = dloc0 + s;
        const float q = pl[(size_t)s * N + i] + pl[(size_t)(S + s) * N + i] * r + pl[(size_t)(2 * S + s) * N + i] * g +
                        pl[(size_t)(3 * S + s) * N + i] * b;
        if (best >= 0 && best == d - 1) nxt = q;  // the winner's right neighbour (until replaced)
        if (q < mn) {
            mn = q;
            best = d;
            pre = d == 0 ? 0.0f : pq;
            nxt = 0.0f;
        }
        pq = q;
    }
    (void)dtot_loc;
    st.mn[i] = mn;
    st.best[i] = best;
    st.pre[i] = pre;
    st.nxt[i] = nxt;
    st.prevq[i] = pq;
}

// final maps: idx (global), min, disp with the optional parabola (0 at the total range's ends)
__global__ void k_gf_out(GfState st, size_t N, int dglob0, int dtot, int sub, int32_t* __restrict__ idx,
                         double* __restrict__ minc, float* __restrict__ disp) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int best = st.best[i];
    const float mn = st.mn[i];
    minc[i] = (double)mn;
    if (best < 0) {
        idx[i] = 0;
        disp[i] = 0.0f;
        return;
    }
    const int g = dglob0 + best;
    idx[i] = g;
    float dd = (float)g;
    if (sub) {
        const float pre = g == 0 ? 0.0f : st.pre[i];
        const float nxt = g == dtot - 1 ? 0.0f : st.nxt[i];
        const float s = (nxt - pre) * 0.5f / (nxt - 2.0f * mn + pre);
        if (fabsf(s) < 1.0f) dd = (float)g - s;
    }
    disp[i] = dd;
}

__global__ void k_gf_init(GfState st, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    st.mn[i] = 1e10f;
    st.best[i] = -1;
    st.pre[i] = 0.0f;
    st.nxt[i] = 0.0f;
    st.prevq[i] = 0.0f;
}

// ---------------------------------------------------------------------------------------------
// Fused tile path (radius 9, the reference's constant).  The unfused chain above moves every slice
// through HBM ten times (slice_in, 2 x (box x, box y), ab, q); here two kernels do it over 2-D tiles
// with the box passes in LDS:
//   k_gf_box1_ab : cost slice + guide -> (p, r*p, g*p, b*p) -> x pass over the tile's 32 + 2r rows ->
//                  y pass of its 32 rows -> (b, a_r, a_g, a_b) (colorGuidedFilterHelper3/2/4) -> HBM;
//   k_gf_box2_q  : (b, a_r, a_g, a_b) -> x pass -> y pass -> q (colorGuidedFilterHelper5) -> HBM;
//   k_gf_wta     : q of the batch's slices in ascending order -> the running strict-< WTA.
// The four planes of a pixel travel together as one float4 (in LDS and, between the kernels, in HBM
// as [slice][pixel] float4), so a sliding-sum step is two 16-byte LDS reads and four independent
// add chains.  A tile is TX (a multiple of 32) columns x one 32-row block, so the x pass runs the
// unfused kernels' per-32-column-block sliding sums and the y pass their per-32-row-block ones, with
// the same float operations in the same order: the staged halo (r columns each side, r rows above and
// below) holds 0.0f outside the image exactly where the unfused kernels add 0.0f, and x-pass rows
// outside the image are 0.0f for the y pass likewise.  Bit-identical to the unfused chain
// (tests/test_gpu_parity.py::test_guided_fused_tiles_match_unfused).
//
// Work order: the work items (tile, slice) -- a tile's slices back to back, tiles in raster order --
// are cut into one contiguous range per workgroup, and the ranges dealt to the 8 XCDs in contiguous
// eighths (workgroup b runs on XCD b % 8): neighbouring tiles' halos and a tile's statistics / guide
// stay in that XCD's L2 and in registers.
template <int RR, int TX>
struct GfTile {
    static constexpr int R = 32 + 2 * RR;   // x-pass rows of a 32-row block
    static constexpr int C = TX + 2 * RR;   // staged columns (from x0 - RR)
    static constexpr int SP = C | 1;        // staging pitch in float4 (odd: 16-byte lanes on consecutive rows
                                            // cover all banks)
    static constexpr int XP = TX | 1;       // x-pass output pitch in float4
    static constexpr int NB = TX / 32;      // 32-column blocks per tile
    static constexpr int NT = 4 * TX;       // threads
    static constexpr int NS = R * C;        // staged pixels
    static constexpr int NPER = (NS + NT - 1) / NT;  // staged pixels per thread
    static constexpr int PU = 32 * TX / NT; // output pixels per thread
    static_assert(TX % 32 == 0, "tiles are whole 32-column blocks");
    static_assert(R * SP >= 32 * XP, "the y pass writes its means over the staging rows");
    static constexpr size_t LDS = (size_t)(R * SP + R * XP) * 16;
};

__device__ __forceinline__ float4 f4add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 f4sub(float4 a, float4 b) { return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
__device__ __forceinline__ float4 f4mul(float4 a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }

// the two box passes of a staged tile: x pass (job = (row, 32-column block), consecutive lanes on
// consecutive rows) into xo, then y pass (thread = column) into the staging rows (means of tile row
// yy at sp[yy * SP + j])
template <int RR, int TX>
__device__ __forceinline__ void gf_box_tile(float4* sp, float4* xo, int x0, int y0, int W, int H) {
    using T = GfTile<RR, TX>;
    const float scale = 1.0f / (float)(2 * RR + 1);
    const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int job = threadIdx.x; job < T::NB * T::R; job += T::NT) {
        const int bb = job / T::R, rr = job - bb * T::R;
        const int xb = x0 + 32 * bb, gy = y0 - RR + rr;
        if (xb >= W) continue;
        const int nout = W - xb < 32 ? W - xb : 32;
        float4* o = xo + rr * T::XP + 32 * bb;
        if (gy < 0 || gy >= H) {
            for (int x = 0; x < nout; ++x) o[x] = z4;
            continue;
        }
        const float4* row = sp + rr * T::SP + 32 * bb + RR;  // staged column of the block start
        float4 t = z4;
        {
            float4 w[2 * RR + 1];  // the first window's reads issued together
#pragma unroll
            for (int i = 0; i <= 2 * RR; ++i) w[i] = row[i - RR];
#pragma unroll
            for (int i = 0; i <= 2 * RR; ++i) t = f4add(t, w[i]);
        }
        o[0] = f4mul(t, scale);
        if (nout == 32) {
            // steps in groups of GS: the group's 2 x GS LDS reads are issued before its dependent adds
            constexpr int GS = 8;
#pragma unroll
            for (int xg = 1; xg < 32; xg += GS) {
                float4 ah[GS], bh[GS];
#pragma unroll
                for (int k = 0; k < GS; ++k)
                    if (xg + k < 32) {
                        ah[k] = row[xg + k + RR];
                        bh[k] = row[xg + k - RR - 1];
                    }
#pragma unroll
                for (int k = 0; k < GS; ++k)
                    if (xg + k < 32) {
                        t = f4add(t, ah[k]);
                        t = f4sub(t, bh[k]);
                        o[xg + k] = f4mul(t, scale);
                    }
            }
        } else {
            for (int x = 1; x < nout; ++x) {
                t = f4add(t, row[x + RR]);
                t = f4sub(t, row[x - RR - 1]);
                o[x] = f4mul(t, scale);
            }
        }
    }
    __syncthreads();
    const int j = threadIdx.x;
    if (j < TX && x0 + j < W) {
        const int nrow = H - y0 < 32 ? H - y0 : 32;
        const float4* col = xo + j;
        float4 t = z4;
        {
            float4 w[2 * RR + 1];
#pragma unroll
            for (int i = 0; i <= 2 * RR; ++i) w[i] = col[i * T::XP];
#pragma unroll
            for (int i = 0; i <= 2 * RR; ++i) t = f4add(t, w[i]);
        }
        sp[j] = f4mul(t, scale);
        if (nrow == 32) {
            constexpr int GS = 8;
#pragma unroll
            for (int yg = 1; yg < 32; yg += GS) {
                float4 ah[GS], bh[GS];
#pragma unroll
                for (int k = 0; k < GS; ++k)
                    if (yg + k < 32) {
                        ah[k] = col[(yg + k + 2 * RR) * T::XP];
                        bh[k] = col[(yg + k - 1) * T::XP];
                    }
#pragma unroll
                for (int k = 0; k < GS; ++k)
                    if (yg + k < 32) {
                        t = f4add(t, ah[k]);
                        t = f4sub(t, bh[k]);
                        sp[(yg + k) * T::SP + j] = f4mul(t, scale);
                    }
            }
        } else {
            for (int yy = 1; yy < nrow; ++yy) {
                t = f4add(t, col[(yy + 2 * RR) * T::XP]);
                t = f4sub(t, col[(yy - 1) * T::XP]);
                sp[yy * T::SP + j] = f4mul(t, scale);
            }
        }
    }
    __syncthreads();
}

// this workgroup's contiguous range [i0, i1) of the work items (G = gridDim.x, a multiple of 8;
// workgroup b runs on XCD b % 8, so each XCD gets one contiguous eighth of the list)
__device__ __forceinline__ void gf_range(int nitems, int& i0, int& i1) {
    const int b = blockIdx.x, G = gridDim.x;
    const int c = (b & 7) * (G >> 3) + (b >> 3);
    const int per = (nitems + G - 1) / G;
    i0 = c * per;
    i1 = i0 + per < nitems ? i0 + per : nitems;
}

// Both kernels loop over their range with the next item's tile loads in flight (registers) while the
// current one runs its box passes out of LDS; the per-tile operands of the epilogue (statistics,
// guide) are loaded once per tile -- items run a tile's slices back to back.
template <int RR, int TX>
__global__ __launch_bounds__(4 * TX) void k_gf_box1_ab(const float* __restrict__ cost, const uint32_t* __restrict__ bgrx,
                                                       const float* __restrict__ st, float4* __restrict__ ab, int W, int H,
                                                       size_t N, int S, int ntx, int nitems) {
    using T = GfTile<RR, TX>;
    __shared__ float4 sp[T::R * T::SP];
    __shared__ float4 xo[T::R * T::XP];
    int i0, i1;
    gf_range(nitems, i0, i1);
    if (i0 >= i1) return;
    const int tid = threadIdx.x;
    float pv[T::NPER];
    uint32_t gv[T::NPER];
    auto load = [&](int item) {
        const int s = item % S, tile = item / S;
        const int x0 = (tile % ntx) * TX, y0 = (tile / ntx) * 32;
        const float* p = cost + (size_t)s * N;
#pragma unroll
        for (int u = 0; u < T::NPER; ++u) {
            int idx = tid + u * T::NT;
            idx = idx < T::NS ? idx : T::NS - 1;
            const int rr = idx / T::C, cc = idx - rr * T::C;
            const int gy = y0 - RR + rr, gx = x0 - RR + cc;
            const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
            const size_t i = in ? (size_t)gy * W + gx : 0;
            const float a = p[i];
            const uint32_t g = bgrx[i];
            pv[u] = in ? a : 0.0f;
            gv[u] = in ? g : 0u;
        }
    };
    load(i0);
    int cur = -1;
    float sv[T::PU][9];
    for (int item = i0; item < i1; ++item) {
        const int s = item % S, tile = item / S;
        const int x0 = (tile % ntx) * TX, y0 = (tile / ntx) * 32;
#pragma unroll
        for (int u = 0; u < T::NPER; ++u) {
            const int idx = tid + u * T::NT;
            if (idx < T::NS) {
                const int rr = idx / T::C, cc = idx - rr * T::C;
                float r, g, b;
                guide_of(gv[u], r, g, b);  // k_gf_slice_in: p, r*p, g*p, b*p (outside: 0 * 0)
                sp[rr * T::SP + cc] = make_float4(pv[u], r * pv[u], g * pv[u], b * pv[u]);
            }
        }
        if (tile != cur) {
            cur = tile;
#pragma unroll
            for (int u = 0; u < T::PU; ++u) {
                const int idx = tid + u * T::NT;
                const int yy = idx / TX, jj = idx - yy * TX;
                const int gy = y0 + yy, gx = x0 + jj;
                const size_t i = gy < H && gx < W ? (size_t)gy * W + gx : 0;
#pragma unroll
                for (int k = 0; k < 9; ++k) sv[u][k] = st[k * N + i];
            }
        }
        __syncthreads();
        if (item + 1 < i1) load(item + 1);
        gf_box_tile<RR, TX>(sp, xo, x0, y0, W, H);
        // a, b per pixel (k_gf_ab's operations)
#pragma unroll
        for (int u = 0; u < T::PU; ++u) {
            const int idx = tid + u * T::NT;
            const int yy = idx / TX, jj = idx - yy * TX;
            const int gy = y0 + yy, gx = x0 + jj;
            if (gy >= H || gx >= W) continue;
            const float4 m = sp[yy * T::SP + jj];
            const float m_p = m.x;
            const float mr = sv[u][0], mg = sv[u][1], mb = sv[u][2];
            const float irr = sv[u][3], irg = sv[u][4], irb = sv[u][5];
            const float igg = sv[u][6], igb = sv[u][7], ibb = sv[u][8];
            const float cr = m.y - mr * m_p;
            const float cg = m.z - mg * m_p;
            const float cb = m.w - mb * m_p;
            const float ar = irr * cr + irg * cg + irb * cb;
            const float ag = irg * cr + igg * cg + igb * cb;
            const float ab_ = irb * cr + igb * cg + ibb * cb;
            const float bb = m_p - ar * mr - ag * mg - ab_ * mb;
            ab[(size_t)s * N + (size_t)gy * W + gx] = make_float4(bb, ar, ag, ab_);
        }
        __syncthreads();  // the epilogue's reads of sp before the next item's staging
    }
}

template <int RR, int TX>
__global__ __launch_bounds__(4 * TX) void k_gf_box2_q(const float4* __restrict__ ab, const uint32_t* __restrict__ bgrx,
                                                      float* __restrict__ q, int W, int H, size_t N, int S, int ntx,
                                                      int nitems) {
    using T = GfTile<RR, TX>;
    __shared__ float4 sp[T::R * T::SP];
    __shared__ float4 xo[T::R * T::XP];
    int i0, i1;
    gf_range(nitems, i0, i1);
    if (i0 >= i1) return;
    const int tid = threadIdx.x;
    float4 v[T::NPER];
    auto load = [&](int item) {
        const int s = item % S, tile = item / S;
        const int x0 = (tile % ntx) * TX, y0 = (tile / ntx) * 32;
        const float4* src = ab + (size_t)s * N;
#pragma unroll
        for (int u = 0; u < T::NPER; ++u) {
            int idx = tid + u * T::NT;
            idx = idx < T::NS ? idx : T::NS - 1;
            const int rr = idx / T::C, cc = idx - rr * T::C;
            const int gy = y0 - RR + rr, gx = x0 - RR + cc;
            const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
            const float4 a = src[in ? (size_t)gy * W + gx : 0];
            v[u] = in ? a : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
    };
    load(i0);
    int cur = -1;
    uint32_t gv[T::PU];
    for (int item = i0; item < i1; ++item) {
        const int s = item % S, tile = item / S;
        const int x0 = (tile % ntx) * TX, y0 = (tile / ntx) * 32;
#pragma unroll
        for (int u = 0; u < T::NPER; ++u) {
            const int idx = tid + u * T::NT;
            if (idx < T::NS) {
                const int rr = idx / T::C, cc = idx - rr * T::C;
                sp[rr * T::SP + cc] = v[u];
            }
        }
        if (tile != cur) {
            cur = tile;
#pragma unroll
            for (int u = 0; u < T::PU; ++u) {
                const int idx = tid + u * T::NT;
                const int yy = idx / TX, jj = idx - yy * TX;
                const int gy = y0 + yy, gx = x0 + jj;
                gv[u] = bgrx[gy < H && gx < W ? (size_t)gy * W + gx : 0];
            }
        }
        __syncthreads();
        if (item + 1 < i1) load(item + 1);
        gf_box_tile<RR, TX>(sp, xo, x0, y0, W, H);
#pragma unroll
        for (int u = 0; u < T::PU; ++u) {
            const int idx = tid + u * T::NT;
            const int yy = idx / TX, jj = idx - yy * TX;
            const int gy = y0 + yy, gx = x0 + jj;
            if (gy >= H || gx >= W) continue;
            float r, g, b;
            guide_of(gv[u], r, g, b);
            const float4 m = sp[yy * T::SP + jj];  // box(b), box(a_r), box(a_g), box(a_b)
            q[(size_t)s * N + (size_t)gy * W + gx] = m.x + m.y * r + m.z * g + m.w * b;
        }
        __syncthreads();
    }
}

// k_gf_q_wta's WTA over precomputed q
__global__ void k_gf_wta(const float* __restrict__ q, GfState st, size_t N, int S, int dloc0) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    float mn = st.mn[i], pre = st.pre[i], nxt = st.nxt[i], pq = st.prevq[i];
    int best = st.best[i];
    for (int s = 0; s < S; ++s) {
        const int d = dloc0 + s;
        const float qv = q[(size_t)s * N + i];
        if (best >= 0 && best == d - 1) nxt = qv;
        if (qv < mn) {
            mn = qv;
            best = d;
            pre = d == 0 ? 0.0f : pq;
            nxt = 0.0f;
        }
        pq = qv;
    }
    st.mn[i] = mn;
    st.best[i] = best;
    st.pre[i] = pre;
    st.nxt[i] = nxt;
    st.prevq[i] = pq;
}

static bool gf_fused(int r) {
    return r == 9 && getenv("SM_GF_UNFUSED") == nullptr;  // read per batch: tests toggle it
}

static hipError_t launch_gf_batch_fused(hipStream_t st, const float* cost, const uint32_t* bgrx, const float* stats, int W,
                                        int H, int S, int dloc0, float* pl, float* tmp, GfStateArgs sa) {
    constexpr int RR = 9, TX = 32;
    static_assert(GfTile<RR, TX>::LDS <= 81920, "two workgroups per CU");
    const size_t N = (size_t)W * H;
    const int nty = (H + 31) / 32, ntx = (W + TX - 1) / TX;
    const int n = ntx * nty * S;  // work items (tile, slice), slice fastest
    // two resident workgroups per CU (LDS), each looping over n / G items
    const char* e = getenv("SM_GF_WGS");
    int G = e ? atoi(e) : 512;
    G = std::max(8, std::min(G, (n + 7) & ~7)) & ~7;
    float4* ab = reinterpret_cast<float4*>(pl);  // [S][N] float4 in the 4S planes
    hipLaunchKernelGGL((k_gf_box1_ab<RR, TX>), dim3(G), dim3(4 * TX), 0, st, cost, bgrx, stats, ab, W, H, N, S, ntx, n);
    hipLaunchKernelGGL((k_gf_box2_q<RR, TX>), dim3(G), dim3(4 * TX), 0, st, ab, bgrx, tmp, W, H, N, S, ntx, n);
    const GfState gs{sa.mn, sa.best, sa.pre, sa.nxt, sa.prevq};
    hipLaunchKernelGGL(k_gf_wta, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, tmp, gs, N, S, dloc0);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
static dim3 pix_grid1(size_t N, int y = 1) { return dim3((unsigned)((N + 255) / 256), (unsigned)y); }

static void box(hipStream_t st, const float* in, float* tmp, float* out, int W, int H, int r, int planes) {
    const size_t N = (size_t)W * H;
    // x pass: the LDS kernel when two row tiles of at least one row fit in 64 KB (W <= 7943), else
    // the direct one (same arithmetic)
    const int nblk = (W + GF_BLOCK - 1) / GF_BLOCK;
    int rows = 256 / nblk;
    if (rows < 1) rows = 1;
    while (rows > 1 && (size_t)2 * rows * (W + nblk) * 4 > 65536) --rows;
    const size_t lds = (size_t)2 * rows * (W + nblk) * 4;
    if (lds <= 65536 && getenv("SM_GF_DIRECT_X") == nullptr)
        hipLaunchKernelGGL(k_gf_box_x_lds, dim3((H + rows - 1) / rows, planes), dim3(256), lds, st, in, tmp, W, H, r, N, rows);
    else
        hipLaunchKernelGGL(k_gf_box_x, dim3((H + 63) / 64, nblk, planes), dim3(64), 0, st, in, tmp, W, H, r, N);
    hipLaunchKernelGGL(k_gf_box_y, dim3((W + 255) / 256, (H + GF_BLOCK - 1) / GF_BLOCK, planes), dim3(256), 0, st, tmp, out, W,
                       H, r, N);
}

hipError_t launch_gf_guide(hipStream_t st, const uint32_t* bgrx, int W, int H, int r, float eps, float* planes, float* tmp,
                           float* means, float* stats) {
    const size_t N = (size_t)W * H;
    hipLaunchKernelGGL(k_gf_guide_in, pix_grid1(N), dim3(256), 0, st, bgrx, planes, N);
    box(st, planes, tmp, means, W, H, r, 9);
    hipLaunchKernelGGL(k_gf_stats, pix_grid1(N), dim3(256), 0, st, means, stats, N, eps);
    return hipGetLastError();
}

hipError_t launch_gf_batch(hipStream_t st, const float* cost, const uint32_t* bgrx, const float* stats, int W, int H, int r,
                           int S, int dloc0, float* pl, float* tmp, GfStateArgs sa) {
    if (gf_fused(r)) return launch_gf_batch_fused(st, cost, bgrx, stats, W, H, S, dloc0, pl, tmp, sa);
    const size_t N = (size_t)W * H;
    hipLaunchKernelGGL(k_gf_slice_in, pix_grid1(N, S), dim3(256), 0, st, cost, bgrx, pl, N, S);
    box(st, pl, tmp, pl, W, H, r, 4 * S);   // means of p, r*p, g*p, b*p
    hipLaunchKernelGGL(k_gf_ab, pix_grid1(N, S), dim3(256), 0, st, pl, stats, N, S);
    box(st, pl, tmp, pl, W, H, r, 4 * S);   // box(b), box(a_r), box(a_g), box(a_b)
    const GfState gs{sa.mn, sa.best, sa.pre, sa.nxt, sa.prevq};
    hipLaunchKernelGGL(k_gf_q_wta, pix_grid1(N), dim3(256), 0, st, pl, bgrx, gs, N, S, dloc0, 0);
    return hipGetLastError();
}

hipError_t launch_gf_init(hipStream_t st, GfStateArgs sa, size_t N) {
    const GfState gs{sa.mn, sa.best, sa.pre, sa.nxt, sa.prevq};
    hipLaunchKernelGGL(k_gf_init, pix_grid1(N), dim3(256), 0, st, gs, N);
    return hipGetLastError();
}

hipError_t launch_gf_out(hipStream_t st, GfStateArgs sa, size_t N, int dglob0, int dtot, int sub, int32_t* idx, double* minc,
                         float* disp) {
    const GfState gs{sa.mn, sa.best, sa.pre, sa.nxt, sa.prevq};
    hipLaunchKernelGGL(k_gf_out, pix_grid1(N), dim3(256), 0, st, gs, N, dglob0, dtot, sub, idx, minc, disp);
    return hipGetLastError();
}
