// sm_post.hip -- the output step after the cross-rank WTA (sm_params.post bits, include/stereomst.h):
//
//   SM_POST_LABEL_TO_DISP  LabelToDisp's clamp to [0,1] of d/(Dmax-1) and the *= (Dmax-1) scaling of
//                          stereo3dmst (Stereo3DMST.cpp:189-201, 900-902), both maps, in float
//   SM_POST_LR_CHECK       leftRightConsistencyCheck (:632-662), left map
//   SM_POST_LR_FILL        ... with fill=true (:664-709): the per-row fill from the nearest valid pixels
//   SM_POST_OCCLUSION[_ZERO] handleOcclusionSharedMemory (PatchMatchStereoGPU.cu:1128-1288), both maps
//
// applied in that order to the float disparity maps (idx / minc untouched).  All are per-row or
// per-pixel, HBM-bound passes over 4-12 B per pixel (~10 us at 1920x1200); the row kernels run one
// 256-thread block per image row and replace the reference's sequential left-to-right searches by
// block-wide max-scans of "position of the nearest valid pixel" (same results, see each kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_launch.h"

// ---------------------------------------------------------------------------------------------
// LabelToDisp + scaling.  With the per-slice restatement the plane label of a pixel is (0, 0, d), so
// LabelToDisp (:197) computes MAX(0.0f, min(1.0f, (x*0 + y*0 + d)/(max_disp-1.0f))) = clamp of
// d/(Dmax-1.f) in float (x*0 + y*0 + d == d exactly), and :900-902 multiplies by (Dmax-1.f):
// cv::Mat *= s is convertTo(scale s) = one float multiply per element (32F->32F, shift 0).  In float
// d/(Dmax-1)*(Dmax-1) != d for some integers d (e.g. Dmax=100: d = 7, 14, 25, ...), and the L-R check
// then compares those values.  std::min(1.0f, q) = q < 1 ? q : 1; OpenCV's MAX(a, b) = a < b ? b : a.
// HIP float division is IEEE correctly rounded (clang's default for HIP), like the host's.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_label_to_disp(float* __restrict__ d0, float* __restrict__ d1, size_t N, float dm1) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    float* d = blockIdx.y ? d1 : d0;
    float q = d[i] / dm1;
    q = q < 1.0f ? q : 1.0f;
    q = 0.0f < q ? q : 0.0f;
    d[i] = q * dm1;
}

// ---------------------------------------------------------------------------------------------
// L-R check (:632-662): d = round(left) (std::round on a float = roundf, half away from zero); a
// pixel with x-d < 0, d < 0, d >= max_disp or |left - right(x-d)| > 1 becomes 0 and is marked.
// Each left pixel reads only right(x-d), so the in-place update is order-independent.  mask
// (optional, for the fill) gets 1 for marked pixels, 0 otherwise.
// ---------------------------------------------------------------------------------------------
__global__ void k_lr_check(float* __restrict__ left, const float* __restrict__ right, int W, int H, int max_disp,
                           uint8_t* __restrict__ mask) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const size_t idx = (size_t)y * W + x;
    const float df = left[idx];
    const int d = (int)roundf(df);
    bool bad = true;
    if (x - d >= 0 && d >= 0 && d < max_disp) bad = fabsf(df - right[idx - d]) > 1.0f;
    if (bad) left[idx] = 0.0f;
    if (mask) mask[idx] = bad ? 1 : 0;
}

// ---------------------------------------------------------------------------------------------
// block-wide scans over one image row, 256 threads = 4 waves
// ---------------------------------------------------------------------------------------------
#define ROW_T 256

// inclusive max-scan of v over the block, plus the carry from earlier tiles; returns the scan and
// updates carry (all threads) to the tile's maximum
__device__ __forceinline__ int block_scan_max(int v, int& carry, int* lds4) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o, 64);
        if (lane >= o) v = max(v, t);
    }
    if (lane == 63) lds4[wave] = v;
    __syncthreads();
    int pre = carry;
    for (int w = 0; w < wave; ++w) pre = max(pre, lds4[w]);
    v = max(v, pre);
    const int tile_max = max(max(max(lds4[0], lds4[1]), max(lds4[2], lds4[3])), carry);
    __syncthreads();  // lds4 is reused by the next tile
    carry = tile_max;
    return v;
}

// ---------------------------------------------------------------------------------------------
// L-R fill (:664-709, fill=true).  The reference walks each row left to right.  A marked pixel
// copies the nearest pixel to its left whose mask is 0 and clears its own mask; since every marked
// pixel with an unmarked pixel somewhere to its left gets cleared this way, the pixel it copies is
// the previous one, which already holds its final value.  It then takes the nearest unmarked pixel
// to its right (the right side is still unprocessed: original marks) if that value is smaller, or
// unconditionally when the left search failed (mask still 1).  By induction every pixel of a marked
// run with valid neighbours L (left) and R (right) ends as (R < L ? R : L); without L it takes R;
// without either it stays 0.  Two scans per row find L and R; marked pixels read only unmarked ones,
// so the update is in place.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(ROW_T) void k_lr_fill(float* __restrict__ left, const uint8_t* __restrict__ mask, int W,
                                                   int* __restrict__ lpos) {
    __shared__ int lds4[4];
    const int y = blockIdx.x;
    float* row = left + (size_t)y * W;
    const uint8_t* m = mask + (size_t)y * W;
    int* lp = lpos + (size_t)y * W;
    int carry = -1;
    for (int x0 = 0; x0 < W; x0 += ROW_T) {  // nearest unmarked position at or left of x
        const int x = x0 + threadIdx.x;
        const int v = (x < W && m[x] == 0) ? x : -1;
        const int s = block_scan_max(v, carry, lds4);
        if (x < W) lp[x] = s;
    }
    carry = -1;
    for (int x0 = 0; x0 < W; x0 += ROW_T) {  // mirrored: nearest unmarked position at or right of x
        const int x = W - 1 - (x0 + (int)threadIdx.x);
        const int v = (x >= 0 && m[x] == 0) ? (W - 1 - x) : -1;
        const int s = block_scan_max(v, carry, lds4);
        if (x >= 0 && m[x] != 0) {
            const int l = lp[x];
            const int r = s < 0 ? -1 : W - 1 - s;
            float out = 0.0f;
            if (l >= 0) {
                const float L = row[l];
                out = (r >= 0 && row[r] < L) ? row[r] : L;
            } else if (r >= 0) {
                out = row[r];
            }
            row[x] = out;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// handleOcclusionSharedMemory (PatchMatchStereoGPU.cu:1128-1288), one block per row, both maps.
//   mark:  left  x: rx = (int)(x - dL(x));  occluded iff rx < 0 or |dR(rx) - dL(x)| > thresh
//          right x: lx = (int)(x + dR(x));  occluded iff lx >= W or |dR(x) - dL(lx)| > thresh
//          (float arithmetic, truncation toward zero as the int conversions of :1150, :1158)
//   fill:  remove -> occluded pixels = min_disp; else an occluded pixel takes
//          fminf(nearest unoccluded to the left, nearest unoccluded to the right) of the ORIGINAL map,
//          a missing side counting 1e18f; both missing -> 255.
// The reference marks into shared memory and searches the marks without a barrier between the two
// phases (a race across warps); this kernel marks the whole row first, i.e. the race-free reading.
// W is not limited to the reference's one-thread-per-column 1024.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(ROW_T) void k_occlusion(float* __restrict__ L, float* __restrict__ R, int W, float thresh,
                                                     int remove, float min_disp, uint8_t* __restrict__ occ,
                                                     int* __restrict__ lpos) {
    __shared__ int lds4[4];
    const int y = blockIdx.x;
    float* lrow = L + (size_t)y * W;
    float* rrow = R + (size_t)y * W;
    uint8_t* o = occ + (size_t)y * W * 2;  // [0, W): left marks, [W, 2W): right marks
    int* lp = lpos + (size_t)y * W * 2;
    for (int x = threadIdx.x; x < W; x += ROW_T) {
        const float dl = lrow[x];
        const int rx = (int)((float)x - dl);
        o[x] = (rx < 0 || fabsf(rrow[rx] - dl) > thresh) ? 1 : 0;
        const float dr = rrow[x];
        const int lx = (int)((float)x + dr);
        o[W + x] = (lx >= W || fabsf(dr - lrow[lx]) > thresh) ? 1 : 0;
    }
    __syncthreads();
    if (remove) {
        for (int x = threadIdx.x; x < W; x += ROW_T) {
            if (o[x]) lrow[x] = min_disp;
            if (o[W + x]) rrow[x] = min_disp;
        }
        return;
    }
    for (int v = 0; v < 2; ++v) {
        float* row = v ? rrow : lrow;
        const uint8_t* m = o + v * W;
        int* l = lp + v * W;
        int carry = -1;
        for (int x0 = 0; x0 < W; x0 += ROW_T) {  // nearest unoccluded strictly left of x
            const int x = x0 + threadIdx.x;
            const int val = (x < W && m[x] == 0) ? x : -1;
            const int s = block_scan_max(val, carry, lds4);
            if (x < W) l[x] = s;
        }
        carry = -1;  // mirrored scan: nearest unoccluded strictly right of x (l[] consumed in place)
        for (int x0 = 0; x0 < W; x0 += ROW_T) {
            const int x = W - 1 - (x0 + (int)threadIdx.x);
            const int val = (x >= 0 && m[x] == 0) ? (W - 1 - x) : -1;
            const int s = block_scan_max(val, carry, lds4);
            if (x >= 0 && m[x] != 0) {
                const int lq = l[x];
                const int rq = s < 0 ? -1 : W - 1 - s;
                const float lv = lq >= 0 ? row[lq] : 1e18f;
                const float rv = rq >= 0 ? row[rq] : 1e18f;
                // stored after the scans of this map: occluded pixels are read by nobody
                l[x] = __float_as_int((lq < 0 && rq < 0) ? 255.f : fminf(lv, rv));
            }
        }
        __syncthreads();
        for (int x = threadIdx.x; x < W; x += ROW_T)
            if (m[x]) row[x] = __int_as_float(l[x]);
        __syncthreads();
    }
}

hipError_t launch_label_to_disp(hipStream_t st, float* d0, float* d1, size_t N, int dmax) {
    hipLaunchKernelGGL(k_label_to_disp, dim3((unsigned)((N + 255) / 256), 2), dim3(256), 0, st, d0, d1, N, (float)dmax - 1.f);
    return hipGetLastError();
}

hipError_t launch_lr_check(hipStream_t st, float* left, const float* right, int W, int H, int max_disp, uint8_t* mask) {
    hipLaunchKernelGGL(k_lr_check, dim3((W + 255) / 256, H), dim3(256), 0, st, left, right, W, H, max_disp, mask);
    return hipGetLastError();
}

hipError_t launch_lr_fill(hipStream_t st, float* left, const uint8_t* mask, int W, int H, int* scratch) {
    hipLaunchKernelGGL(k_lr_fill, dim3(H), dim3(ROW_T), 0, st, left, mask, W, scratch);
    return hipGetLastError();
}

hipError_t launch_occlusion(hipStream_t st, float* left, float* right, int W, int H, float thresh, int remove, float min_disp,
                            uint8_t* occ, int* scratch) {
    hipLaunchKernelGGL(k_occlusion, dim3(H), dim3(ROW_T), 0, st, left, right, W, thresh, remove, min_disp, occ, scratch);
    return hipGetLastError();
}
