// sm_reduce_rule.h -- the per-pixel rule of the cross-rank WTA exchange (sm_api.cpp stage_reduce), shared
// by the device kernels (sm_kernels.hip k_cand / k_finalize / k_cand64 / k_finalize64) and the host
// exports sm_reduce_candidates / sm_reduce_finalize (the CPU tests' gloo exchange calls those).
//
// After an all-reduce MIN of the fp64 minimum cost, a rank proposes its global index where its own
// minimum equals the global one (else the largest key); an all-reduce MIN of the candidates then
// picks the lowest index among the ranks that hold the minimum: the reference's strict-< first
// minimum over ascending d (Stereo3DMST.cpp:177, PatchMatchStereoGPU.cu:1700-1717) for contiguous
// ascending shards.  With subpixel disparities the candidate is (index << 32 | disparity bits).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__host__ __device__ inline int32_t sm_rule_cand32(double minc, double gmin, int32_t idx) {
    return minc == gmin ? idx : 0x7fffffff;
}

__host__ __device__ inline unsigned long long sm_rule_cand64(double minc, double gmin, int32_t idx, uint32_t disp_bits) {
    return minc == gmin ? ((unsigned long long)(uint32_t)idx << 32) | disp_bits : ~0ull;
}

// the global answer: minimum, index, and the float disparity (the index, or the winner's subpixel value)
__host__ __device__ inline void sm_rule_finalize32(double gmin, int32_t gidx, double& minc, int32_t& idx, float& disp) {
    minc = gmin;
    idx = gidx;
    disp = (float)gidx;
}

__host__ __device__ inline void sm_rule_finalize64(double gmin, unsigned long long key, double& minc, int32_t& idx,
                                                   uint32_t& disp_bits) {
    minc = gmin;
    idx = (int32_t)(key >> 32);
    disp_bits = (uint32_t)key;
}
