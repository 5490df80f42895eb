// sm_segment.h -- host-side segment mode (sm_segment.cpp).  sm_segment_forest is exported with C
// linkage (library-internal, not part of include/stereomst.h) so the CPU tests can call it.
#pragma once
#include <stdint.h>

// weight code of the virtual edges that link the segment trees into one spanning tree:
// S_LUT[SM_VIRTUAL_W] = 0, S2_LUT[SM_VIRTUAL_W] = 1 (sm_tables.inc / sm_api.cpp)
#define SM_VIRTUAL_W 766

#ifdef __cplusplus
extern "C" {
#endif
// Felzenszwalb segmentation with threshold c and the min-size merge (segment-graph.h:54-89,
// Stereo3DMST.cpp:242-307) of the grid graph with right / down weights wR / wD (N = W*H each).
// Outputs per pixel: mR / mD = 1 where the right / down edge is a forest edge or one of the virtual
// edges that link each tree's root to an earlier tree; fwR / fwD = the weights with SM_VIRTUAL_W on
// the virtual edges.  Returns the number of trees.
int sm_segment_forest(const uint16_t* wR, const uint16_t* wD, int W, int H, float c, int min_size, uint8_t* mR,
                      uint8_t* mD, uint16_t* fwR, uint16_t* fwD);
#ifdef __cplusplus
}
#endif
