// sm_nl_tree.h — host-built minimum spanning tree + heavy paths for aggregation "NL" (sm_nl_tree.cpp).
#pragma once
#include <stdint.h>

#include <vector>

namespace sm {

// The tree is kept in breadth-first numbering: node i is the i-th pixel the walk from pixel 0
// reaches, so a node's parent precedes it and its children are consecutive (fc[i] ..
// fc[i] + nch[i] - 1, in discovery order); every pass over the tree is then a linear sweep.
struct NlTree {
    int n = 0;
    std::vector<int> pix;           // [n] pixel of node i (pix[0] = 0, the root)
    std::vector<int> par;           // [n] parent node (par[0] = 0)
    std::vector<int> fc;            // [n] first child node
    std::vector<uint8_t> nch;       // [n] number of children
    std::vector<uint8_t> wgt;       // [n] weight of the edge to the parent (0 for the root)
    std::vector<uint8_t> cdir;      // [n] the children's directions, 2 bits each in child order
                                    //     (0: +1, 1: -1, 2: +W, 3: -W, as q - pixel)
    std::vector<int8_t> heavy;      // [n] index j of the child continuing the node's path, -1 at leaves
    std::vector<int> slot;          // [n] record slot of node i (paths concatenated, each bottom -> top)
    std::vector<int> chain_start, chain_len;
    std::vector<int> up_level, down_level;   // rounds of the filter's two passes
    // scratch kept with the tree so that repeated builds reuse their memory (no page faults)
    std::vector<int> s_order_e, s_uf, s_size, s_hlen, s_ul, s_chain_of;
    std::vector<uint32_t> s_adj;
    std::vector<int32_t> s_rec;     // (sm_capi.cpp: the pair's neighbour lists, records and weight
    std::vector<float> s_wsum;      //  sums, page-locked for the copies; paths per round)
    std::vector<int> s_cu, s_cd;
    std::vector<uint8_t> s_pdir;
    std::vector<double> s_v;
};

// Neighbour lists of the pair's minimum spanning tree, one 32-bit word per pixel (the tree
// edges in Kruskal's acceptance order): count | direction j << (3 + 2 j), directions 0: +1, 1: -1,
// 2: +W, 3: -W (one column: 0 / 1), and the weights of the pixel's own right and down edges
// (tree edges or not) in bits 16-23 and 24-31.  The product path builds them on
// the GPU (sm_nl_mst.hip); nl_build_lists is the host's sequential Kruskal (tools, checks).
// ew: the pair's edge weights, H (W - 1) horizontal edges row by row, then (H - 1) W vertical
// edges column by column (qx_mst_compute_edges_4neighbor).  Lists land in t.s_adj.
bool nl_build_lists(int H, int W, const uint8_t* ew, NlTree& t);

// The breadth-first tree from pixel 0 over the lists, its heavy paths, rounds and record slots;
// false if the lists do not form a spanning tree.  With table, rec and wsum given, the records
// (as nl_pack_records with this base) and the weight sums (as nl_weight_sums) are written by the
// same two passes.
bool nl_tree_from_lists(int H, int W, const uint32_t* adj, NlTree& t, const double* table = nullptr, int base = 0,
                        int32_t* rec = nullptr, float* wsum = nullptr);

// nl_build_lists + nl_tree_from_lists
bool nl_build_tree(int H, int W, const uint8_t* ew, NlTree& t);

// The tree's nodes as the filter kernels' records (NlArgs::rec), in path order: rec[4 k ..] =
// {pixel + base, meta, child weights, parent pixel + base} for the node whose slot is k.
void nl_pack_records(const NlTree& t, int W, int base, int32_t* rec);

// The filtered ones (the NL() weight sums, cpp:4899-4910) as floats: the tree filter of a constant
// 1 in double, with the GPU kernels' (and the reference's) arithmetic and order.  O(n) per pair.
void nl_weight_sums(NlTree& t, const double* table, float* wsum);

}  // namespace sm
