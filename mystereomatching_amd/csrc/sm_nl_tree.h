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
    std::vector<int> order;         // breadth-first order from the root
    // scratch kept with the tree so that repeated builds reuse their memory (no page faults)
    std::vector<int> s_order_e, s_uf, s_sz, s_nconn, s_conn, s_size, s_chain_of, s_path;
    std::vector<uint8_t> s_connw;
    std::vector<double> s_v;
};

// ew: the pair's edge weights, H (W - 1) horizontal edges row by row, then (H - 1) W vertical
// edges column by column (qx_mst_compute_edges_4neighbor).
bool nl_build_tree(int H, int W, const uint8_t* ew, NlTree& t);

// The tree's nodes as the filter kernels' records (NlArgs::rec), in path order: rec[4 k ..] =
// {node + base, meta, child weights, parent + base} for the k-th entry of t.chain_nodes.
void nl_pack_records(const NlTree& t, int W, int base, int32_t* rec);

// The filtered ones (the NL() weight sums, cpp:4899-4910) as floats: the tree filter of a constant
// 1 in double, with the GPU kernels' (and the reference's) arithmetic and order.  O(n) per pair.
void nl_weight_sums(NlTree& t, const double* table, float* wsum);

}  // namespace sm
