// sm_layout_gpu.h -- device buffers of the GPU tree layout (sm_layout_gpu.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_common.h"

#define SM_MAX_ROUNDS 32  // light depth <= log2(N) < 31
#define SM_NBUCKETS (2 * SM_MAX_ROUNDS)  // per round: [long paths | short paths]
#ifndef SM_LONG_PATH
#define SM_LONG_PATH 32   // paths of >= this many nodes go to the long-path chain engine (sm_chain.hip)
#endif
#define SM_PRE_SEG 32     // nodes per k_up_pre block (segment table granularity)
// A long path of >= 2P nodes is cut into len/P pieces of P nodes (the bottom piece takes the
// remainder, < 2P; -DSM_PIECE_EVEN balances the sizes instead: up chain 0.94 -> 1.01 ms at C2); the
// pieces' chains run concurrently from guessed inputs and are then repaired exactly (sm_chain.hip,
// "Pieces").  P = SM_PIECE by default (env SM_PIECE_LEN: a multiple of
// SM_PRE_SEG, >= 64; tests use short pieces to exercise the repair on small images).
// -DSM_PIECE_BALANCED (A/B): cut every path of > P nodes into ceil(len/P) balanced pieces.  Measured
// at C2 it is slower (up pre + chain 1.23 vs 1.12 ms): more cut paths need segment aggregates and
// repairs, and a round's time is set by the CUs' queues of work items, not by its longest piece.
#ifndef SM_PIECE
#define SM_PIECE 512
#endif
// Piece length of a long bucket of `nodes` nodes (one view).  P everywhere by default.  With
// -DSM_ADAPT_PIECES (A/B), a bucket too small to give every CU a work item (the root path's round:
// ~15k nodes per view) gets pieces of ~nodes/128 (two views share 256 CUs), not below 256 nodes.
// Measured at C2: the down chain gains 0.03 ms, the up chain loses 0.75 ms -- at 256 nodes the up
// pieces' repairs stop merging inside their pieces and take the serial slow path.
__host__ __device__ static inline uint32_t sm_bucket_piece_len(uint32_t nodes, uint32_t plen) {
#ifndef SM_ADAPT_PIECES
    (void)nodes;
    return plen;
#endif
    if (plen < SM_PIECE || nodes >= 128u * plen) return plen;
    uint32_t p = (nodes / 128u + SM_PRE_SEG - 1) / SM_PRE_SEG * SM_PRE_SEG;
    p = p < 256u ? 256u : p;
    return p < plen ? p : plen;
}
#ifndef SM_PIECE_BALANCED
__host__ __device__ static inline bool sm_piece_cut(uint32_t len, uint32_t plen) { return len >= 2 * plen; }
__host__ __device__ static inline uint32_t sm_piece_count(uint32_t len, uint32_t plen) {
    return len >= 2 * plen ? len / plen : 1u;
}
#ifndef SM_PIECE_EVEN  // P-node pieces, the bottom one takes the remainder (< 2P)
__host__ __device__ static inline uint32_t sm_piece_begin_p(uint32_t len, uint32_t M, uint32_t j, uint32_t plen) {
    return j >= M ? len : j * plen;
}
#else  // A/B: the same M pieces, balanced (boundaries on SM_PRE_SEG multiples): none longer than ~1.5P
__host__ __device__ static inline uint32_t sm_piece_begin_p(uint32_t len, uint32_t M, uint32_t j, uint32_t plen) {
    (void)plen;
    if (j >= M) return len;
    const uint32_t b = (uint32_t)(((uint64_t)len * j / M + SM_PRE_SEG / 2) / SM_PRE_SEG * SM_PRE_SEG);
    return b < len ? b : len;
}
#endif
#else
__host__ __device__ static inline bool sm_piece_cut(uint32_t len, uint32_t plen) { return len > plen; }
__host__ __device__ static inline uint32_t sm_piece_count(uint32_t len, uint32_t plen) {
    return len > plen ? (len + plen - 1) / plen : 1u;
}
// first node (from the path head) of piece j of M; j == M gives len
__host__ __device__ static inline uint32_t sm_piece_begin_p(uint32_t len, uint32_t M, uint32_t j, uint32_t plen) {
    (void)plen;
    if (j >= M) return len;
    const uint32_t b = (uint32_t)(((uint64_t)len * j / M + SM_PRE_SEG / 2) / SM_PRE_SEG * SM_PRE_SEG);
    return b < len ? b : len;
}
#endif

// Down pass: the same M pieces (same work items and status words), cut evenly.  The down pass
// has no segment table and its exact piece is the top one, so the floor rule would make the
// bottom piece -- the last to repair -- also the longest (up to 2P - 1 nodes).
// -DSM_DN_PIECE_FLOOR (A/B): the up pass's boundaries.
__host__ __device__ static inline uint32_t sm_piece_begin_dn(uint32_t len, uint32_t M, uint32_t i, uint32_t plen) {
#ifdef SM_DN_PIECE_FLOOR
    return sm_piece_begin_p(len, M, i, plen);
#else
    (void)plen;
    return i >= M ? len : (uint32_t)((uint64_t)len * i / M);
#endif
}

struct LayoutView {
    // inputs
    const uint8_t* mR;
    const uint8_t* mD;
    const uint16_t* wR;
    const uint16_t* wD;
    // per pixel
    uint8_t* adj;
    int8_t* pdir;       // direction to the parent (-1: root)
    int8_t* heavy;      // direction of the heavy child (-1: leaf)
    uint32_t* size;     // subtree size
    uint32_t* arcpix;   // per tour rank of a down arc: the child pixel it enters
    // per arc (4N)
    uint16_t* a_dist;
    uint32_t* a_cid;
    // per chain
    uint32_t* nchains;  // device counter
    uint32_t* c_last;
    uint32_t* c_len;
    uint64_t* cnw;      // per chain: successor chain (low 32 bits) | arcs to it (high 32 bits)
    // tour (2N-2); the scans' tile tickets (3, zeroed with the layout's other counters)
    uint32_t* tour;         // per tour rank: the arc's value (light << 27 | preorder offset, negated going up)
    // per heavy-first preorder position (layout-internal numbering)
    uint32_t* hk;        // (1 + head position) << 5 | light depth at a path head, 0 elsewhere;
                         // after the max-scan: the position's path head and its light depth
    uint32_t* pixpre;    // the pixel at the position
    // per slot
    SmMeta* meta;
    // paths
    SmPath* paths;           // {head slot, len}, bucket-major; slots of a bucket are contiguous
    uint32_t* pathpos;       // [preorder of a head] -> index of its path in paths[]
    uint32_t* plen;          // [path] -> len, inclusive-scanned into the path's end slot
    uint32_t* slotpix;       // [pixel] -> slot
    uint32_t* round_count;   // SM_NBUCKETS
    uint32_t* round_cursor;  // SM_NBUCKETS
    uint32_t* round_begin;   // SM_NBUCKETS + 1
    uint32_t* round_maxlen;  // SM_NBUCKETS: longest path per bucket
    uint32_t* round_nodes;   // SM_NBUCKETS: nodes per bucket
    uint32_t* seg_begin;     // SM_NBUCKETS + 1: first segment of each bucket in segtab
    uint2* segtab;           // cut long paths: {path index within its bucket, segment within the path}
    uint32_t* piece_begin;   // SM_NBUCKETS + 1: first piece of each bucket in pieces
    uint4* pieces_tmp;       // scratch of the items' longest-first reordering (k_long_segments)
    uint4* pieces;           // {path index within its bucket, j, M, first segment of the path
                             //  within the bucket}; piece j of M (0 = top), per path bottom first
    uint32_t* nrounds;
    uint32_t* n_has_light;   // nodes with at least one light child: the compact A rows (SmMeta::cslot[3])
    // compact A rows (round 6): a light children's parent's row is wrow's exclusive prefix at its
    // (tile, wave) of the layout's 32x32 pixel tiles plus its rank among that wave's (k_orient)
    uint8_t* lrank;          // [pixel] rank among the light children's parents of its tile wave (< 256)
    uint32_t* wrow;          // [4 * tile + wave]: their count, then (inclusive scan) the running total
};

// the layout scans' tile totals (sm_layout_gpu.hip k_scan_reduce), per view, one 64-bit slot per tile
struct ScanState {
    uint64_t* part[2];
    uint32_t* err;  // the call's device error word: bit 1, a layout index out of range
};
// tiles of the scans (at least 2048 elements each) over at most 2N elements
static inline size_t scan_tiles(size_t N) { return (2 * N + 2047) / 2048 + 1; }

struct LayoutPair {
    LayoutView v[2];
    const int* mst_ok;  // != 0 once the MST is complete (k_mst_done); every layout kernel checks it
    ScanState scan;
    int want_size;  // write the subtree sizes (V.size): only sm_build_tree reports them
};

hipError_t launch_layout(hipStream_t st, const LayoutPair& LP, int nviews, int W, int H, uint32_t max_chains,
                         uint32_t piece_len);
