// ref_segment_probe.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
//
// Compiles the reference's own include/segment-graph.h + include/disjoint-set.h
// (from /root/reference, never copied into this repo) behind a C entry point so the
// golden-fixture script can run the REAL reference Kruskal/Felzenszwalb code on small
// images and pin the oracle's orc_segment() against it.  Built by oracle/Makefile into
// oracle/_ref/ (git-ignored); not part of the product and never shipped to users.
#include <cstring>
#include "segment-graph.h"

extern "C" int ref_segment_graph(int num_vertices, int num_edges, const int* a, const int* b,
                                 const double* w, float c, int* out_a, int* out_b, double* out_w,
                                 int* out_mask) {
    edge* edges = new edge[num_edges > 0 ? num_edges : 1];
    for (int i = 0; i < num_edges; ++i) { edges[i].a = a[i]; edges[i].b = b[i]; edges[i].w = w[i]; }
    std::memset(out_mask, 0, sizeof(int) * (size_t)num_edges);
    universe* u = segment_graph(num_vertices, num_edges, edges, out_mask, c);  // sorts in place
    for (int i = 0; i < num_edges; ++i) { out_a[i] = edges[i].a; out_b[i] = edges[i].b; out_w[i] = edges[i].w; }
    const int nsets = u->num_sets();
    delete u;
    delete[] edges;
    return nsets;
}
