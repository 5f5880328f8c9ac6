// sm_nl_tree.cpp — host side of aggregation "NL" (NL(), stereoMatching.cpp:4892-4917 ->
// NLCCA::aggreCV, NL/NLCCA.cpp:27-96): the minimum spanning tree of the left colour image and its
// breadth-first orientation (NL/qx_mst_kruskals_image.cpp:167-277), cut into heavy paths for the
// GPU tree filter (sm_nl.hip).
//
// The tree is the reference's, edge for edge: the GPU's edge weights (max channel difference of
// the 3x3-median-filtered image, horizontal edges row by row then vertical edges column by column)
// are sorted stably by weight (a counting sort, qx_sort_increase_using_histogram), Kruskal accepts
// an edge when its endpoints are in different components, and every accepted edge is appended to
// both endpoints' neighbour lists; the breadth-first walk from pixel 0 then makes every neighbour
// but the parent a child, in list order.  Kruskal's acceptance and the neighbour-list order depend
// only on the edge order, not on the union-find details.
//
// Heavy paths: every node continues the path of its largest child (the first of equal sizes), so
// any root path crosses at most log2(n) path boundaries.  The up pass of the filter runs the paths
// in rounds of "up level" (1 + the largest level of a path hanging off it, 0 for none), the down
// pass in rounds of depth in the path tree; each round is one launch in which a wave walks a whole
// path sequentially, the child on its own path arriving in a register and the others from memory.
// The per-node arithmetic and its order are the reference's (sm_nl.hip), so the rounds only
// schedule work.  This graph construction is O(n) host work per pair (pairs run on parallel host
// threads); the O(n D) filtering is on the GPU.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "sm_nl_tree.h"

namespace sm {

// Builds the tree of one pair (pixel ids 0 .. H W - 1) into t; returns false if the graph is
// not connected (cannot happen for a 4-neighbour grid with H W > 1).
bool nl_build_tree(int H, int W, const uint8_t* ew, NlTree& t) {
    const int n = H * W;
    const int neh = H * (W - 1), ne = neh + (H - 1) * W;
    t.n = n;
    // stable counting sort of the edges by weight; an edge is stored as its first endpoint u
    // and its direction (u << 1 | vertical), generated in edge-index order without divisions
    std::vector<int>& order_e = t.s_order_e;
    order_e.resize((size_t)std::max(ne, 1));
    int bstart[257];
    {
        int pos[257];
        memset(pos, 0, sizeof(pos));
        for (int e = 0; e < ne; e++) pos[ew[e] + 1]++;
        for (int v = 0; v < 256; v++) pos[v + 1] += pos[v];
        memcpy(bstart, pos, sizeof(pos));
        int e = 0;
        for (int y = 0; y < H; y++)            // horizontal: row by row, (y, x) - (y, x + 1)
            for (int x = 0; x < W - 1; x++, e++) order_e[pos[ew[e]]++] = (y * W + x) << 1;
        for (int x = 0; x < W; x++)            // vertical: column by column, (y, x) - (y + 1, x)
            for (int y = 0; y < H - 1; y++, e++) order_e[pos[ew[e]]++] = ((y * W + x) << 1) | 1;
    }
    // Kruskal: union-find with path halving and union by size (the accepted set is independent
    // of how the components are merged)
    std::vector<int>&uf = t.s_uf, &sz = t.s_sz, &nconn = t.s_nconn, &conn = t.s_conn;
    std::vector<uint8_t>& connw = t.s_connw;
    uf.resize(n);
    sz.assign(n, 1);
    nconn.assign(n, 0);
    conn.resize((size_t)n * 4);
    connw.resize((size_t)n * 4);
    for (int i = 0; i < n; i++) uf[i] = i;
    auto find = [&](int x) {
        while (uf[x] != x) {
            uf[x] = uf[uf[x]];
            x = uf[x];
        }
        return x;
    };
    int accepted = 0;
    for (int w = 0; w < 256 && accepted < n - 1; w++)   // weight buckets in order
    for (int j = bstart[w]; j < bstart[w + 1] && accepted < n - 1; j++) {
        const int pe = order_e[j];
        const int u = pe >> 1, v = u + ((pe & 1) ? W : 1);
        int ru = find(u), rv = find(v);
        if (ru == rv) continue;
        if (sz[ru] < sz[rv]) std::swap(ru, rv);
        uf[rv] = ru;
        sz[ru] += sz[rv];
        conn[(size_t)u * 4 + nconn[u]] = v;
        connw[(size_t)u * 4 + nconn[u]++] = (uint8_t)w;
        conn[(size_t)v * 4 + nconn[v]] = u;
        connw[(size_t)v * 4 + nconn[v]++] = (uint8_t)w;
        accepted++;
    }
    if (accepted != n - 1) return false;
    // breadth-first orientation from pixel 0 (build_tree)
    t.parent.assign(n, -1);
    t.weight.assign(n, 0);
    t.nchild.assign(n, 0);
    t.child.assign((size_t)n * 4, -1);
    std::vector<int>& bfs = t.order;
    bfs.resize(n);
    t.parent[0] = 0;
    bfs[0] = 0;
    int head = 0, len = 1;
    while (head < len) {
        const int p = bfs[head++];
        for (int i = 0; i < nconn[p]; i++) {
            const int q = conn[(size_t)p * 4 + i];
            if (t.parent[q] != -1) continue;
            t.parent[q] = p;
            t.weight[q] = connw[(size_t)p * 4 + i];
            t.child[(size_t)p * 4 + t.nchild[p]++] = q;
            bfs[len++] = q;
        }
    }
    if (len != n) return false;
    // Subtree sizes and heavy children in one reverse breadth-first pass (a node's children come
    // after it, so their sizes are final when it is reached): the heavy child is the first of
    // the largest children.
    std::vector<int>& size = t.s_size;
    size.assign(n, 1);
    t.heavy.resize(n);
    for (int i = n - 1; i >= 0; i--) {
        const int x = bfs[i];
        int best = -1, bs = 0;
        for (int j = 0; j < t.nchild[x]; j++) {
            const int cs = size[t.child[(size_t)x * 4 + j]];
            if (cs > bs) {
                bs = cs;
                best = j;
            }
        }
        t.heavy[x] = (int8_t)best;
        if (i > 0) size[t.parent[x]] += size[x];
    }
    // Heavy paths, numbered in breadth-first order of their tops (forward pass): a node continues
    // its parent's path when it is the parent's heavy child; pos = its depth below the path's top.
    // Down level = 1 + that of the path its top hangs off (0 for the root's path).
    std::vector<int>& chain_of = t.s_chain_of;
    std::vector<int>& pos = t.s_path;
    chain_of.resize(n);
    pos.resize(n);
    t.chain_len.clear();
    t.down_level.clear();
    for (int i = 0; i < n; i++) {
        const int x = bfs[i];
        const int p = t.parent[x];
        if (i > 0 && t.heavy[p] >= 0 && t.child[(size_t)p * 4 + t.heavy[p]] == x) {
            const int c = chain_of[p];
            chain_of[x] = c;
            pos[x] = pos[p] + 1;
            t.chain_len[c]++;
        } else {
            const int c = (int)t.chain_len.size();
            chain_of[x] = c;
            pos[x] = 0;
            t.chain_len.push_back(1);
            t.down_level.push_back(i == 0 ? 0 : t.down_level[chain_of[p]] + 1);
        }
    }
    const int nch = (int)t.chain_len.size();
    t.chain_start.resize(nch);
    for (int c = 0, o = 0; c < nch; c++) {
        t.chain_start[c] = o;
        o += t.chain_len[c];
    }
    // Nodes stored bottom -> top, and up levels (1 + the largest up level of a path hanging off
    // the path, 0 for none) in one reverse pass: the paths hanging off a node lie below it, so
    // their levels are final when it is reached.
    t.chain_nodes.resize(n);
    t.up_level.assign(nch, 0);
    for (int i = n - 1; i >= 0; i--) {
        const int x = bfs[i];
        const int c = chain_of[x];
        t.chain_nodes[t.chain_start[c] + t.chain_len[c] - 1 - pos[x]] = x;
        for (int j = 0; j < t.nchild[x]; j++)
            if (j != t.heavy[x]) t.up_level[c] = std::max(t.up_level[c], t.up_level[chain_of[t.child[(size_t)x * 4 + j]]] + 1);
    }
    return true;
}

void nl_pack_records(const NlTree& t, int W, int base, int32_t* rec) {
    for (int k = 0; k < t.n; k++) {
        const int x = t.chain_nodes[k];
        const int nc = t.nchild[x];
        int meta = nc | (t.heavy[x] + 1) << 3 | t.weight[x] << 16;
        uint32_t wp = 0;
        for (int j = 0; j < nc; j++) {
            const int q = t.child[(size_t)x * 4 + j], dq = q - x;
            const int code = dq == 1 ? 0 : dq == -1 ? 1 : dq == W ? 2 : 3;   // +1, -1, +W, -W
            meta |= code << (6 + 2 * j);
            wp |= (uint32_t)t.weight[q] << (8 * j);
        }
        int32_t* r = rec + (size_t)k * 4;
        r[0] = x + base;
        r[1] = meta;
        r[2] = (int32_t)wp;
        r[3] = t.parent[x] + base;
    }
}

void nl_weight_sums(NlTree& t, const double* table, float* wsum) {
    const int n = t.n;
    std::vector<double>& v = t.s_v;
    v.resize(n);
    for (int i = n - 1; i >= 0; i--) {     // up: children before parents
        const int x = t.order[i];
        double s = 1.0;
        for (int j = 0; j < t.nchild[x]; j++) {
            const int c = t.child[(size_t)x * 4 + j];
            const double m = v[c] * table[t.weight[c]];
            s = s + m;
        }
        v[x] = s;
    }
    for (int i = 1; i < n; i++) {          // down: parents before children (the root keeps its sum)
        const int x = t.order[i];
        const double w = table[t.weight[x]];
        const double m = w * v[x];
        const double q = v[t.parent[x]] - m;
        const double r = w * q;
        v[x] = r + v[x];
    }
    for (int x = 0; x < n; x++) wsum[x] = (float)v[x];
}

}  // namespace sm
