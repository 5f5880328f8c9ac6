// sm_nl_tree.h — host-built minimum spanning tree + heavy paths for aggregation "NL" (sm_nl_tree.cpp).
#pragma once
#include <stdint.h>

#include <vector>

namespace sm {

struct NlTree {
    int n = 0;
    std::vector<int> parent;        // [n], parent[0] = 0 (root = pixel 0)
    std::vector<uint8_t> weight;    // [n] edge weight to the parent (0 for the root)
    std::vector<uint8_t> nchild;    // [n]
    std::vector<int> child;         // [n][4] in breadth-first discovery order, -1 unused
    std::vector<int8_t> heavy;      // [n] index j of the child continuing the node's path, -1 at leaves
    std::vector<int> chain_nodes;   // paths concatenated, each bottom -> top
    std::vector<int> chain_start, chain_len;
    std::vector<int> up_level, down_level;   // rounds of the filter's two passes
};

// ew: the pair's edge weights, H (W - 1) horizontal edges row by row, then (H - 1) W vertical
// edges column by column (qx_mst_compute_edges_4neighbor).
bool nl_build_tree(int H, int W, const uint8_t* ew, NlTree& t);

}  // namespace sm
