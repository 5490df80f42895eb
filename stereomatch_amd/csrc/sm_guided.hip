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
#include "sm_knob.h"

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
// row band layout of the fused path: rows in bands of 32, a band stored column by column, so the 32
// rows of one column are contiguous -- a wavefront whose lanes are consecutive rows reads one segment
__host__ __device__ __forceinline__ size_t gf_band(int gy, int gx, int W) { return ((size_t)(gy >> 5) * W + gx) * 32 + (gy & 31); }

// planes of stride NS: row-major (band = 0, NS = N) or in the row band layout (NS = 32 * ceil(H/32) * W)
__global__ void k_gf_stats(const float* __restrict__ m, float* __restrict__ st_, size_t N, float eps, int W, int band, size_t NS) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const size_t o = band ? gf_band((int)(i / W), (int)(i % W), W) : i;
    float* st = st_;
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
    st[o] = mr;
    st[NS + o] = mg;
    st[2 * NS + o] = mb;
    st[3 * NS + o] = irr / det;
    st[4 * NS + o] = irg / det;
    st[5 * NS + o] = irb / det;
    st[6 * NS + o] = igg / det;
    st[7 * NS + o] = igb / det;
    st[8 * NS + o] = ibb / det;
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
// through HBM ten times (slice_in, 2 x (box x, box y), ab, q) and runs a separate WTA pass; here two
// kernels, one workgroup (four wavefronts) per 32 x 32 tile, loop over the batch's slices:
//   k_gf_box1_ab    : cost slice + guide -> (p, r*p, g*p, b*p) -> x pass -> y pass -> (b, a_r, a_g,
//                     a_b) (colorGuidedFilterHelper3/2/4) -> HBM, [slice] float4 planes;
//   k_gf_box2_q_wta : (b, a_r, a_g, a_b) -> x pass -> y pass -> q (colorGuidedFilterHelper5) -> the
//                     running strict-< WTA, in registers.
// The tile is one 32-column block x one 32-row block, so the x pass runs the unfused kernels'
// per-32-column-block sliding sums and the y pass their per-32-row-block ones, with the same float
// operations in the same order: the staged tile (32 + 2r square) holds 0.0f outside the image
// exactly where the unfused kernels add 0.0f, and x-pass rows outside the image are 0.0f for the y
// pass likewise.  Each pass is one scalar chain per (row or column, plane) -- 4 x (32 + 2r) x-pass
// chains, 4 x 32 y-pass chains -- so every wavefront has chains to run; the next slice's tile is in
// flight in registers meanwhile, and the per-tile operands (guide, statistics, WTA state) are read
// once per batch.  Bit-identical to the unfused chain
// (tests/test_gpu_parity.py::test_guided_fused_tiles_match_unfused).
//
// Row band layout: the statistics and the (b, a) planes are stored in bands of 32 rows, a band
// column by column (gf_band), so the 32 rows of a column are contiguous: the epilogue (lanes on
// consecutive rows) and k_gf_box2_q_wta's staging read and write whole segments.
//
// Work order: tiles in raster order, dealt to the 8 XCDs in contiguous eighths (workgroup b runs on
// XCD b % 8), so neighbouring tiles' halos are re-read from that XCD's L2.

// the XCD-contiguous item of this workgroup (G = gridDim.x, a multiple of 8)
__device__ __forceinline__ int gf_item() {
    const int b = blockIdx.x, G = gridDim.x;
    return (b & 7) * (G >> 3) + (b >> 3);
}

constexpr int GF_XQ = 33;  // x-pass plane pitch (floats)

// x pass of staged row xr, plane xk of the tile at (x0, y0): sp = the staged float4 tile (pitch CP,
// column 0 = x0 - RR), o = the plane's x-pass row
template <int RR, int CP>
__device__ __forceinline__ void gf_xchain(const float4* sp, float* o, int xr, int xk, int x0, int y0, int W, int H) {
    const int nout = W - x0 < 32 ? W - x0 : 32;
    const int gy = y0 - RR + xr;
    if (gy < 0 || gy >= H) {
        for (int x = 0; x < nout; ++x) o[x] = 0.0f;
        return;
    }
    const float scale = 1.0f / (float)(2 * RR + 1);
    const float* row = reinterpret_cast<const float*>(sp + xr * CP + RR) + xk;  // staged column x0
    auto in = [&](int c) { return row[4 * c]; };
    float t = 0.0f;
    if (nout == 32) {  // whole block: each staged value read once, the chain unrolled
        float v[32 + 2 * RR];
#pragma unroll
        for (int i = 0; i < 32 + 2 * RR; ++i) v[i] = in(i - RR);
#pragma unroll
        for (int i = 0; i <= 2 * RR; ++i) t += v[i];
        o[0] = t * scale;
#pragma unroll
        for (int x = 1; x < 32; ++x) {
            t += v[x + 2 * RR];
            t -= v[x - 1];
            o[x] = t * scale;
        }
        return;
    }
    for (int i = -RR; i <= RR; ++i) t += in(i);
    o[0] = t * scale;
    for (int x = 1; x < nout; ++x) {
        t += in(x + RR);
        t -= in(x - RR - 1);
        o[x] = t * scale;
    }
}

// y pass of column j of one plane's x-pass rows (col = &plane[0][j]); the mean of tile row yy is
// written back in place into row yy, one step after that row's last read
template <int RR>
__device__ __forceinline__ void gf_ychain(float* col, int y0, int H) {
    const int nrow = H - y0 < 32 ? H - y0 : 32;
    const float scale = 1.0f / (float)(2 * RR + 1);
    float t = 0.0f;
#pragma unroll
    for (int i = 0; i <= 2 * RR; ++i) t += col[i * GF_XQ];
    float prev = t * scale;
    if (nrow == 32) {
#pragma unroll
        for (int yy = 1; yy < 32; ++yy) {
            const float a = col[(yy + 2 * RR) * GF_XQ], b = col[(yy - 1) * GF_XQ];
            t += a;
            t -= b;
            col[(yy - 1) * GF_XQ] = prev;
            prev = t * scale;
        }
    } else {
        for (int yy = 1; yy < nrow; ++yy) {
            const float a = col[(yy + 2 * RR) * GF_XQ], b = col[(yy - 1) * GF_XQ];
            t += a;
            t -= b;
            col[(yy - 1) * GF_XQ] = prev;
            prev = t * scale;
        }
    }
    col[(nrow - 1) * GF_XQ] = prev;
}

// k_gf_box1_ab: four wavefronts per tile, looping over the batch's slices: the tile's guide and its
// pixels' statistics are loaded once (registers), and the next slice's cost tile (32 + 2r square,
// coalesced row loads) is in flight in registers while the current one runs.  The staged tile holds
// the four products (p, r*p, g*p, b*p) per pixel; both box passes run one scalar chain per (row or
// column, plane) -- 4 x (32 + 2r) x-pass chains, 4 x 32 y-pass chains -- so all four wavefronts work
// in each pass.  Statistics in, (b, a_r, a_g, a_b) out, both in the row band layout (NS floats /
// float4 per plane), lanes on consecutive rows of a column.
template <int RR>
__global__ __launch_bounds__(256) void k_gf_box1_ab(const float* __restrict__ cost, const uint32_t* __restrict__ bgrx,
                                                    const float* __restrict__ stb, float4* __restrict__ ab, int W, int H,
                                                    size_t N, size_t NS, int S, int ntx, int ntiles, int dbg) {
    constexpr int R = 32 + 2 * RR, C = 32 + 2 * RR, CP = C | 1, NST = R * C, NPER = (NST + 255) / 256;
    constexpr int XQ = GF_XQ;
    __shared__ float4 sp[R * CP];
    __shared__ float xo[4 * R * XQ];
    const int tile = gf_item();
    if (tile >= ntiles) return;
    const int x0 = (tile % ntx) * 32, y0 = (tile / ntx) * 32;
    const int tid = threadIdx.x;
    auto stage_at = [&](int idx, size_t& i) {  // staged element idx -> pixel (false: outside)
        const int rr = idx / C, cc = idx - rr * C;
        const int gy = y0 - RR + rr, gx = x0 - RR + cc;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        i = in ? (size_t)gy * W + gx : 0;
        return in;
    };
    uint32_t gv[NPER];  // the guide of the thread's staged pixels, once
#pragma unroll
    for (int u = 0; u < NPER; ++u) {
        int idx = tid + u * 256;
        idx = idx < NST ? idx : NST - 1;
        size_t i;
        const bool in = stage_at(idx, i);
        const uint32_t g = bgrx[i];
        gv[u] = in ? g : 0u;
    }
    float sv[4][9];  // the statistics of the thread's 4 output pixels, once
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int gy = y0 + (tid & 31), gx = x0 + (tid >> 5) + 8 * u;
        const size_t i = gy < H && gx < W ? gf_band(gy, gx, W) : 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) sv[u][k] = stb[k * NS + i];
    }
    float pv[NPER];
    auto load = [&](int s) {
        const float* p = cost + (size_t)s * N;
#pragma unroll
        for (int u = 0; u < NPER; ++u) {
            int idx = tid + u * 256;
            idx = idx < NST ? idx : NST - 1;
            size_t i;
            const bool in = stage_at(idx, i);
            const float a = p[i];
            pv[u] = in ? a : 0.0f;
        }
    };
    load(0);
    // x-pass chain of this thread: staged row xr, plane xk (0: p, 1..3: r*p, g*p, b*p); plane fastest
    // across lanes, so a wavefront's scalar reads of the float4 tile hit 64 different banks
    const int xk = tid & 3, xr = tid >> 2;
    const bool xjob = xr < R;
    for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int u = 0; u < NPER; ++u) {
            const int idx = tid + u * 256;
            if (idx < NST) {
                float r, g, b;
                guide_of(gv[u], r, g, b);  // k_gf_slice_in: p, r*p, g*p, b*p (outside: 0 * 0)
                const float p = pv[u];
                sp[(idx / C) * CP + idx % C] = make_float4(p, r * p, g * p, b * p);
            }
        }
        __syncthreads();
        if (s + 1 < S) load(s + 1);
        if (xjob) gf_xchain<RR, CP>(sp, xo + (xk * R + xr) * XQ, xr, xk, x0, y0, W, H);
        __syncthreads();
        if (!(dbg & 2) && tid < 128 && x0 + (tid & 31) < W)  // y pass: (column, plane)
            gf_ychain<RR>(xo + (tid >> 5) * R * XQ + (tid & 31), y0, H);
        __syncthreads();
        if (!(dbg & 4)) {
            // a, b per pixel (k_gf_ab's operations)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int yy = tid & 31, jj = (tid >> 5) + 8 * u;
                const int gy = y0 + yy, gx = x0 + jj;
                if (gy >= H || gx >= W) continue;
                const float m_p = xo[yy * XQ + jj];
                const float mIr = xo[(R + yy) * XQ + jj];
                const float mIg = xo[(2 * R + yy) * XQ + jj];
                const float mIb = xo[(3 * R + yy) * XQ + jj];
                const float mr = sv[u][0], mg = sv[u][1], mb = sv[u][2];
                const float irr = sv[u][3], irg = sv[u][4], irb = sv[u][5];
                const float igg = sv[u][6], igb = sv[u][7], ibb = sv[u][8];
                const float cr = mIr - mr * m_p;
                const float cg = mIg - mg * m_p;
                const float cb = mIb - mb * m_p;
                const float ar = irr * cr + irg * cg + irb * cb;
                const float ag = irg * cr + igg * cg + igb * cb;
                const float ab_ = irb * cr + igb * cg + ibb * cb;
                const float bb = m_p - ar * mr - ag * mg - ab_ * mb;
                ab[(size_t)s * NS + gf_band(gy, gx, W)] = make_float4(bb, ar, ag, ab_);
            }
        }
        __syncthreads();  // xo / sp reads done before the next slice overwrites them
    }
}

// k_gf_box2_q_wta: four wavefronts per tile, looping over the batch's slices in ascending order
// like k_gf_box1_ab (the next slice's (b, a_r, a_g, a_b) tile in flight in registers, staged from the
// row band layout with lanes on consecutive rows), then q (colorGuidedFilterHelper5) and the running
// strict-< WTA of the thread's 4 pixels in registers (k_gf_q_wta's update; state in and out once per
// batch).
template <int RR>
__global__ __launch_bounds__(256) void k_gf_box2_q_wta(const float4* __restrict__ ab, const uint32_t* __restrict__ bgrx,
                                                       GfState wst, int W, int H, size_t NS, int S, int dloc0, int ntx,
                                                       int ntiles, int dbg) {
    constexpr int R = 32 + 2 * RR, C = 32 + 2 * RR, CP = C | 1, NST = R * C, NPER = (NST + 255) / 256;
    constexpr int XQ = GF_XQ;
    __shared__ float4 sp[R * CP];
    __shared__ float xo[4 * R * XQ];
    const int tile = gf_item();
    if (tile >= ntiles) return;
    const int x0 = (tile % ntx) * 32, y0 = (tile / ntx) * 32;
    const int tid = threadIdx.x;
    // staged element idx: row fastest (rr = idx % R), so a wavefront's loads are row band segments
    auto stage_at = [&](int idx, size_t& i) {
        const int cc = idx / R, rr = idx - cc * R;
        const int gy = y0 - RR + rr, gx = x0 - RR + cc;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        i = in ? gf_band(gy, gx, W) : 0;
        return in;
    };
    float4 pv[NPER];
    auto load = [&](int s) {
        const float4* src = ab + (size_t)s * NS;
#pragma unroll
        for (int u = 0; u < NPER; ++u) {
            int idx = tid + u * 256;
            idx = idx < NST ? idx : NST - 1;
            size_t i;
            const bool in = stage_at(idx, i);
            const float4 a = src[i];
            pv[u] = in ? a : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
    };
    load(0);
    // the thread's 4 pixels: guide and WTA state
    float gr[4], gg[4], gb[4], mn[4], pre[4], nxt[4], pq[4];
    int best[4];
    size_t pix[4];
    bool own[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int gy = y0 + (tid & 31), gx = x0 + (tid >> 5) + 8 * u;
        own[u] = gy < H && gx < W;
        pix[u] = own[u] ? (size_t)gy * W + gx : 0;
        guide_of(bgrx[pix[u]], gr[u], gg[u], gb[u]);
        mn[u] = wst.mn[pix[u]];
        best[u] = wst.best[pix[u]];
        pre[u] = wst.pre[pix[u]];
        nxt[u] = wst.nxt[pix[u]];
        pq[u] = wst.prevq[pix[u]];
    }
    const int xk = tid & 3, xr = tid >> 2;
    const bool xjob = xr < R;
    for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int u = 0; u < NPER; ++u) {
            const int idx = tid + u * 256;
            if (idx < NST) {
                const int cc = idx / R, rr = idx - cc * R;
                sp[rr * CP + cc] = pv[u];
            }
        }
        __syncthreads();
        if (s + 1 < S) load(s + 1);
        if (xjob) gf_xchain<RR, CP>(sp, xo + (xk * R + xr) * XQ, xr, xk, x0, y0, W, H);
        __syncthreads();
        if (!(dbg & 2) && tid < 128 && x0 + (tid & 31) < W)  // y pass: (column, plane)
            gf_ychain<RR>(xo + (tid >> 5) * R * XQ + (tid & 31), y0, H);
        __syncthreads();
        if (!(dbg & 4)) {
            const int d = dloc0 + s;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int yy = tid & 31, jj = (tid >> 5) + 8 * u;
                // box(b), box(a_r), box(a_g), box(a_b)
                const float q = xo[yy * XQ + jj] + xo[(R + yy) * XQ + jj] * gr[u] + xo[(2 * R + yy) * XQ + jj] * gg[u] +
                                xo[(3 * R + yy) * XQ + jj] * gb[u];
                if (best[u] >= 0 && best[u] == d - 1) nxt[u] = q;  // the winner's right neighbour
                if (q < mn[u]) {
                    mn[u] = q;
                    best[u] = d;
                    pre[u] = d == 0 ? 0.0f : pq[u];
                    nxt[u] = 0.0f;
                }
                pq[u] = q;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (own[u]) {
            wst.mn[pix[u]] = mn[u];
            wst.best[pix[u]] = best[u];
            wst.pre[pix[u]] = pre[u];
            wst.nxt[pix[u]] = nxt[u];
            wst.prevq[pix[u]] = pq[u];
        }
}

bool gf_fused(int r) { return r == 9 && sm_knob("SM_GF_UNFUSED") == nullptr; }  // read per call: tests toggle it

size_t gf_band_plane(int W, int H) { return (size_t)((H + 31) / 32) * 32 * W; }

static hipError_t launch_gf_batch_fused(hipStream_t st, const float* cost, const uint32_t* bgrx, const float* stats, int W,
                                        int H, int S, int dloc0, float* pl, float* tmp, GfStateArgs sa) {
    constexpr int RR = 9;
    const size_t N = (size_t)W * H;
    const int nty = (H + 31) / 32, ntx = (W + 31) / 32;
    const size_t NS = gf_band_plane(W, H);
    float4* ab = reinterpret_cast<float4*>(pl);  // [S][NS] float4, row band layout
    const char* e = sm_dev_knob("SM_GF_DBG");  // timing probes only (wrong results): 2 no y pass, 4 no epilogue
    const int dbg = e ? atoi(e) : 0;
    const int ntiles = ntx * nty;  // one workgroup per 32 x 32 tile, looping over the batch's slices
    hipLaunchKernelGGL((k_gf_box1_ab<RR>), dim3((ntiles + 7) & ~7), dim3(256), 0, st, cost, bgrx, stats, ab, W, H, N, NS, S,
                       ntx, ntiles, dbg);
    const GfState gs{sa.mn, sa.best, sa.pre, sa.nxt, sa.prevq};
    hipLaunchKernelGGL((k_gf_box2_q_wta<RR>), dim3((ntiles + 7) & ~7), dim3(256), 0, st, ab, bgrx, gs, W, H, NS, S, dloc0, ntx,
                       ntiles, dbg);
    (void)tmp;  // q never leaves the registers
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
    if (lds <= 65536 && sm_knob("SM_GF_DIRECT_X") == nullptr)
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
    // the fused path reads the statistics in the row band layout
    const bool band = gf_fused(r);
    hipLaunchKernelGGL(k_gf_stats, pix_grid1(N), dim3(256), 0, st, means, stats, N, eps, W, band ? 1 : 0,
                       band ? gf_band_plane(W, H) : N);
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
