// sm_nl_tree.cpp — host side of aggregation "NL" (NL(), stereoMatching.cpp:4892-4917 ->
// NLCCA::aggreCV, NL/NLCCA.cpp:27-96): the breadth-first orientation of the left colour image's
// minimum spanning tree (NL/qx_mst_kruskals_image.cpp:167-277), cut into heavy paths for the GPU
// tree filter (sm_nl.hip).
//
// The tree is the reference's, edge for edge: over the edge weights (max channel difference of
// the 3x3-median-filtered image, horizontal edges row by row then vertical edges column by
// column), Kruskal visits the edges sorted stably by weight (a counting sort,
// qx_sort_increase_using_histogram), accepts an edge when its endpoints are in different
// components and appends it to both endpoints' neighbour lists; the breadth-first walk from pixel
// 0 then makes every neighbour but the parent a child, in list order.  The product path gets the
// neighbour lists from the GPU (sm_nl_mst.hip: Boruvka, the same tree and list order);
// nl_build_lists is the sequential Kruskal, kept for the host tools and checks.
//
// Heavy paths: every node continues the path of its largest child (the first of equal sizes), so
// any root path crosses at most log2(n) path boundaries.  The up pass of the filter runs the paths
// in rounds of "up level" (1 + the largest level of a path hanging off it, 0 for none), the down
// pass in rounds of depth in the path tree; each round is one launch in which a wave walks a whole
// path sequentially, the child on its own path arriving in a register and the others from memory.
// The per-node arithmetic and its order are the reference's (sm_nl.hip), so the rounds only
// schedule work.  The walk is O(n) host work per pair (pairs run on parallel host threads); the
// O(n D) filtering is on the GPU.
//
// Layout: the lists are one 32-bit word per pixel (2-bit directions + the pixel's right / down
// edge weights), the walk
// renumbers the nodes in breadth-first order, and every later pass (sizes, paths, levels, records,
// weight sums) is a linear sweep over that numbering: a node's children are consecutive and
// follow it, its parent precedes it.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "sm_nl_tree.h"

namespace sm {

bool nl_build_lists(int H, int W, const uint8_t* ew, NlTree& t) {
    const int n = H * W;
    const int neh = H * (W - 1), ne = neh + (H - 1) * W;
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
    // Kruskal with Rem's union-find (interleaved finds with splicing, a root is its own parent
    // and parents only grow towards the roots' larger index); the accepted set is independent of
    // how the components are merged.  A pixel's accepted edges, in acceptance order (the
    // reference's neighbour lists), as in sm_nl_tree.h: count | direction j << (3 + 2 j), and the
    // pixel's own right / down edge weights in bits 16-23 / 24-31.
    std::vector<int>& uf = t.s_uf;
    std::vector<uint32_t>& adj = t.s_adj;
    uf.resize(n);
    adj.resize(n);
    {
        int p = 0;
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++, p++) {
                const uint32_t wr = x < W - 1 ? ew[y * (W - 1) + x] : 0u;
                const uint32_t wd = y < H - 1 ? ew[neh + x * (H - 1) + y] : 0u;
                adj[p] = wr << 16 | wd << 24;
            }
    }
    int* P = uf.data();
    for (int i = 0; i < n; i++) P[i] = i;
    // true if x and y were in different components (which are then merged)
    auto unite = [P](int x, int y) {
        while (P[x] != P[y]) {
            if (P[x] < P[y]) {
                if (x == P[x]) {
                    P[x] = P[y];
                    return true;
                }
                const int z = P[x];
                P[x] = P[y];
                x = z;
            } else {
                if (y == P[y]) {
                    P[y] = P[x];
                    return true;
                }
                const int z = P[y];
                P[y] = P[x];
                y = z;
            }
        }
        return false;
    };
    auto link = [&](int p, uint32_t dir) {
        const uint32_t a = adj[p], k = a & 7u;
        adj[p] = (a + 1u) | dir << (3 + 2 * k);
    };
    int accepted = 0;
    for (int w = 0; w < 256 && accepted < n - 1; w++)   // weight buckets in order
    for (int j = bstart[w]; j < bstart[w + 1] && accepted < n - 1; j++) {
        const int pe = order_e[j];
        const uint32_t vert = (uint32_t)pe & 1u;
        const int u = pe >> 1, v = u + (vert ? W : 1);
        if (!unite(u, v)) continue;
        const uint32_t dc = W > 1 ? 2u * vert : 0u;   // (one column: +W is +1)
        link(u, dc);        // u -> v: +1 or +W
        link(v, dc + 1u);   // v -> u: -1 or -W
        accepted++;
    }
    return accepted == n - 1;
}

bool nl_build_tree(int H, int W, const uint8_t* ew, NlTree& t) {
    return nl_build_lists(H, W, ew, t) && nl_tree_from_lists(H, W, t.s_adj.data(), t);
}

bool nl_tree_from_lists(int H, int W, const uint32_t* adj, NlTree& t, const double* table, int base, int32_t* rec,
                        float* wsum) {
    const int n = H * W;
    const bool fused = table && rec && wsum;
    t.n = n;
    // A sequential check that every entry names a neighbour inside the image and that there are
    // 2 (n - 1) entries (a tree); it also brings the lists (fresh from a device copy) into the
    // cache before the walk reads them in breadth-first order.
    {
        uint64_t deg = 0;
        int p = 0;
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++, p++) {
                const uint32_t a = adj[p], cnt = a & 7u;
                if (cnt > 4) return false;
                for (uint32_t j = 0; j < cnt; j++) {
                    const uint32_t c = (a >> (3 + 2 * j)) & 3u;
                    const bool in = W > 1 ? (c == 0 ? x < W - 1 : c == 1 ? x > 0 : c == 2 ? y < H - 1 : y > 0)
                                          : (c == 0 ? y < H - 1 : c == 1 && y > 0);
                    if (!in) return false;
                }
                deg += cnt;
            }
        if (deg != 2 * (uint64_t)(n - 1)) return false;
    }
    // breadth-first walk from pixel 0 (build_tree): every neighbour but the parent is a child, in
    // list order; the nodes are numbered in the order the walk reaches them.  pdir = the
    // direction from a node to its parent (4 for the root), the entry skipped in its list.
    t.pix.resize(n);
    t.par.resize(n);
    t.fc.resize(n);
    t.nch.resize(n);
    t.wgt.resize(n);
    t.cdir.resize(n);
    std::vector<uint8_t>& pdir = t.s_pdir;
    pdir.resize(n);
    t.pix[0] = 0;
    t.par[0] = 0;
    t.wgt[0] = 0;
    pdir[0] = 4;
    const int delta[4] = {1, -1, W, -W};
    int len = 1;
    for (int i = 0; i < len; i++) {
        const int p = t.pix[i];
        const uint32_t a = adj[p];
        const uint32_t cnt = a & 7u, skip = pdir[i];
        t.fc[i] = len;
        uint32_t nc = 0, cd = 0;
        for (uint32_t j = 0; j < cnt; j++) {
            const uint32_t c = (a >> (3 + 2 * j)) & 3u;
            if (c == skip) continue;
            if (len == n) return false;   // not a tree (lists from elsewhere are not trusted)
            const int q = p + delta[c];
            // the edge's weight: the right / down field of its left / upper end (one column:
            // every edge is vertical)
            const uint32_t src = (c & 1u) ? adj[q] : a;
            t.pix[len] = q;
            t.par[len] = i;
            t.wgt[len] = (uint8_t)(((c & 2u) || W == 1) ? src >> 24 : src >> 16);
            pdir[len] = (uint8_t)(c ^ 1u);
            cd |= c << (2 * nc++);
            len++;
        }
        t.nch[i] = (uint8_t)nc;
        t.cdir[i] = (uint8_t)cd;
    }
    if (len != n) return false;
    // One reverse pass (a node's children follow it, so their values are final when it is
    // reached): subtree sizes; the heavy child = the first of the largest children; hlen = nodes
    // from the node down its path; ul = 1 + the largest ul of a light child anywhere on the path
    // below the node (0 for none), at a path's top the path's up level.  Fused: the up pass of
    // the weight sums (nl_weight_sums).
    std::vector<int>& size = t.s_size;
    std::vector<double>& v = t.s_v;
    if (fused) v.resize(n);
    std::vector<int>& hlen = t.s_hlen;
    std::vector<int>& ul = t.s_ul;
    size.assign(n, 1);
    hlen.resize(n);
    ul.resize(n);
    t.heavy.resize(n);
    for (int i = n - 1; i >= 0; i--) {
        const int f = t.fc[i], nc = t.nch[i];
        int best = -1, bs = 0;
        for (int j = 0; j < nc; j++) {
            const int cs = size[f + j];
            if (cs > bs) {
                bs = cs;
                best = j;
            }
        }
        int u = 0;
        for (int j = 0; j < nc; j++) u = std::max(u, j == best ? ul[f + j] : ul[f + j] + 1);
        t.heavy[i] = (int8_t)best;
        hlen[i] = best >= 0 ? hlen[f + best] + 1 : 1;
        ul[i] = u;
        if (i > 0) size[t.par[i]] += size[i];
        if (fused) {
            double sv = 1.0;
            for (int j = 0; j < nc; j++) {
                const double m = v[f + j] * table[t.wgt[f + j]];
                sv = sv + m;
            }
            v[i] = sv;
        }
    }
    // Heavy paths, numbered in breadth-first order of their tops, in one forward pass: a node
    // continues its parent's path when it is the parent's heavy child.  A path's records are
    // stored bottom -> top from its start, so a node's slot is start + hlen - 1.  Down level = 1 +
    // that of the path its top hangs off (0 for the root's path).  Fused: the down pass of the
    // weight sums and the records (nl_pack_records).
    std::vector<int>& chain_of = t.s_chain_of;
    chain_of.resize(n);
    t.slot.resize(n);
    t.chain_start.clear();
    t.chain_len.clear();
    t.up_level.clear();
    t.down_level.clear();
    int next = 0;
    for (int i = 0; i < n; i++) {
        const int p = t.par[i];
        int c;
        if (i > 0 && t.heavy[p] >= 0 && t.fc[p] + t.heavy[p] == i) {
            c = chain_of[p];
        } else {
            c = (int)t.chain_len.size();
            t.chain_start.push_back(next);
            t.chain_len.push_back(hlen[i]);
            t.up_level.push_back(ul[i]);
            t.down_level.push_back(i == 0 ? 0 : t.down_level[chain_of[p]] + 1);
            next += hlen[i];
        }
        chain_of[i] = c;
        const int sl = t.chain_start[c] + hlen[i] - 1;
        t.slot[i] = sl;
        if (fused) {
            if (i > 0) {
                const double w = table[t.wgt[i]];
                const double m = w * v[i];
                const double q = v[p] - m;
                const double r = w * q;
                v[i] = r + v[i];
            }
            wsum[t.pix[i]] = (float)v[i];
            const int nc = t.nch[i], f = t.fc[i];
            uint32_t wp = 0;
            for (int j = 0; j < nc; j++) wp |= (uint32_t)t.wgt[f + j] << (8 * j);
            int32_t* rr = rec + (size_t)sl * 4;
            rr[0] = t.pix[i] + base;
            rr[1] = nc | (t.heavy[i] + 1) << 3 | t.cdir[i] << 6 | t.wgt[i] << 16;
            rr[2] = (int32_t)wp;
            rr[3] = t.pix[p] + base;
        }
    }
    return true;
}

void nl_pack_records(const NlTree& t, int /*W*/, int base, int32_t* rec) {
    for (int i = 0; i < t.n; i++) {
        const int nc = t.nch[i], f = t.fc[i];
        uint32_t wp = 0;
        for (int j = 0; j < nc; j++) wp |= (uint32_t)t.wgt[f + j] << (8 * j);
        int32_t* r = rec + (size_t)t.slot[i] * 4;
        r[0] = t.pix[i] + base;
        r[1] = nc | (t.heavy[i] + 1) << 3 | t.cdir[i] << 6 | t.wgt[i] << 16;
        r[2] = (int32_t)wp;
        r[3] = t.pix[t.par[i]] + base;
    }
}

void nl_weight_sums(NlTree& t, const double* table, float* wsum) {
    const int n = t.n;
    std::vector<double>& v = t.s_v;
    v.resize(n);
    for (int i = n - 1; i >= 0; i--) {     // up: children before parents
        double s = 1.0;
        for (int j = 0; j < t.nch[i]; j++) {
            const int c = t.fc[i] + j;
            const double m = v[c] * table[t.wgt[c]];
            s = s + m;
        }
        v[i] = s;
    }
    for (int i = 1; i < n; i++) {          // down: parents before children (the root keeps its sum)
        const double w = table[t.wgt[i]];
        const double m = w * v[i];
        const double q = v[t.par[i]] - m;
        const double r = w * q;
        v[i] = r + v[i];
    }
    for (int i = 0; i < n; i++) wsum[t.pix[i]] = (float)v[i];
}

}  // namespace sm
