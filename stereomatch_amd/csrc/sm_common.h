// sm_common.h -- definitions shared by the HIP kernels and the C++ host side.
//
// Tree layout ("slot" space): every MST node gets a slot; slots are ordered by
// (light depth, heavy-first DFS preorder) so that
//   * each heavy path is a contiguous slot range [head, head+len), top first,
//   * each light-depth round is a contiguous slot range,
// and the aggregation buffers are [slot][Dpad] fp64 rows (Dpad = 64*SPL).  See DESIGN.md.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SM_NONE 0xFFFFFFFFu

// 32-byte per-slot record read by the walkers with one scalar load.
//   parent: the previous slot for a node on its parent's heavy path; SM_HEAD | (compact A row of the
//           parent) for a path head (the only reader of the parent's A row is the head); SM_NONE: root
//   cslot[3]: a node with a light child has at most 3 children (every node but the root has a parent,
//           and the root is the image's first pixel, a corner of its tree), so the fourth child word
//           holds the node's own compact A row: the down pass stores A only for light children's
//           parents, in a buffer of n_has_light rows instead of one row per slot (round 6)
struct alignas(32) SmMeta {
    uint32_t pix;        // pixel index y*W+x
    uint32_t parent;     // see above
    uint32_t lo;         // wp:10 | cw0:10 | cw1:10
    uint32_t hi;         // cw2:10 | cw3:10 | nch:3 | hidx:2 | has_light:1
    uint32_t cslot[4];   // child slots in DESCENDING (w,a,b) key order (the up-pass order); see above
};
#define SM_HEAD 0x80000000u  // parent word of a path head: SM_HEAD | compact A row of its parent
__host__ __device__ static inline uint32_t sm_arow(uint32_t parent_word) { return parent_word & ~SM_HEAD; }

// child ordering: the reference sums children in descending BFS id (Stereo3DMST.cpp:125),
// BFS ids of siblings follow ascending edge key (:436-446, :492-516), so the up pass folds
// children in descending key order.

__host__ __device__ static inline uint32_t sm_meta_wp(const SmMeta& m) { return m.lo & 1023u; }
__host__ __device__ static inline uint32_t sm_meta_cw(const SmMeta& m, int j) {
    return j == 0 ? (m.lo >> 10) & 1023u : j == 1 ? (m.lo >> 20) & 1023u : j == 2 ? m.hi & 1023u : (m.hi >> 10) & 1023u;
}
__host__ __device__ static inline uint32_t sm_meta_nch(const SmMeta& m) { return (m.hi >> 20) & 7u; }
__host__ __device__ static inline uint32_t sm_meta_hidx(const SmMeta& m) { return (m.hi >> 23) & 3u; }
__host__ __device__ static inline uint32_t sm_meta_has_light(const SmMeta& m) { return (m.hi >> 25) & 1u; }

__host__ __device__ static inline SmMeta sm_make_meta(uint32_t pix, uint32_t parent, uint32_t wp, const uint32_t cw[4], uint32_t nch,
                                  uint32_t hidx, uint32_t has_light, const uint32_t cslot[4]) {
    SmMeta m;
    m.pix = pix;
    m.parent = parent;
    m.lo = (wp & 1023u) | ((cw[0] & 1023u) << 10) | ((cw[1] & 1023u) << 20);
    m.hi = (cw[2] & 1023u) | ((cw[3] & 1023u) << 10) | ((nch & 7u) << 20) | ((hidx & 3u) << 23) | ((has_light & 1u) << 25);
    for (int i = 0; i < 4; ++i) m.cslot[i] = cslot[i];
    return m;
}

// A heavy path of one round: slots [head, head+len).
struct SmPath {
    uint32_t head;
    uint32_t len;
};

// Edge key preserving the reference's (w, a, b) order (include/segment-graph.h:34-42):
// b = a+1 (horizontal) or a+W (vertical), so (w, a, vertical) is order-isomorphic.
__host__ __device__ static inline uint64_t sm_edge_key(uint32_t w, uint32_t a, uint32_t vert) {
    return ((uint64_t)w << 33) | ((uint64_t)a << 1) | (uint64_t)vert;
}

#define SM_KEY_NONE 0xFFFFFFFFFFFFFFFFull
#define SM_MAX_W 765
#define SM_WEIGHT_NONE 0xFFFFu
