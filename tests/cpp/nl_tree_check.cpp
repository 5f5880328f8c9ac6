// nl_tree_check.cpp — host side of aggregation NL (mystereomatching_amd/csrc/sm_nl_tree.cpp)
// against the oracle's tree and filter (oracle/sm_oracle_agg.c, test infrastructure only).
// For random colour images of many shapes:
//  * the breadth-first tree walked from Kruskal's neighbour lists (nl_build_lists +
//    nl_tree_from_lists) equals smo_nl_tree node for node: order, parent, edge weight, children in
//    order;
//  * every pixel's list is its tree edges in increasing (weight, edge index) -- the order the
//    GPU lists (sm_nl_mst.hip) are sorted in;
//  * the fused records equal nl_pack_records, and the fused weight sums equal smo_nl_filter of
//    ones rounded to float, bit for bit;
//  * lists that are not a spanning tree are rejected.
// Prints "ok <cases>" and exits 0, or the first mismatch and exits 1.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "sm_nl_tree.h"
extern "C" {
#include "sm_oracle.h"
}

static int fail(const char* what, int cs) {
    printf("mismatch: %s (case %d)\n", what, cs);
    return 1;
}

int main() {
    srand(7);
    std::vector<double> table(256);
    smo_nl_table(0.1, table.data());
    int cases = 0;
    for (int cs = 0; cs < 80; cs++) {
        const int H = cs < 70 ? 1 + rand() % 33 : 60 + rand() % 40, W = cs < 70 ? 1 + rand() % 33 : 60 + rand() % 40;
        const int levels = cs % 3 == 0 ? 2 : (cs % 3 == 1 ? 256 : 12);
        const int n = H * W, ne = H * (W - 1) + (H - 1) * W;
        std::vector<uint8_t> bgr((size_t)n * 3), med((size_t)n * 3), ew(ne > 0 ? ne : 1);
        for (auto& v : bgr) v = (uint8_t)(rand() % levels * (255 / std::max(1, levels - 1)));
        smo_nl_median3(H, W, bgr.data(), med.data());
        int e = 0;
        auto wgt = [&](int u, int v) {
            int m = 0;
            for (int c = 0; c < 3; c++) m = std::max(m, abs((int)med[(size_t)v * 3 + c] - (int)med[(size_t)u * 3 + c]));
            return (uint8_t)m;
        };
        for (int y = 0; y < H; y++)
            for (int x = 0; x + 1 < W; x++) ew[e++] = wgt(y * W + x, y * W + x + 1);
        for (int x = 0; x < W; x++)
            for (int y = 0; y + 1 < H; y++) ew[e++] = wgt(y * W + x, (y + 1) * W + x);
        // oracle tree and weight sums
        std::vector<int> order(n), parent(n), nchild(n), child((size_t)n * 4);
        std::vector<uint8_t> weight(n);
        if (smo_nl_tree(H, W, bgr.data(), order.data(), parent.data(), weight.data(), nchild.data(), child.data()))
            return fail("oracle tree", cs);
        std::vector<double> ones(n, 1.0), backup(n);
        smo_nl_filter(n, 1, order.data(), parent.data(), weight.data(), nchild.data(), child.data(), table.data(),
                      ones.data(), backup.data());
        // host lists + walk (fused records / weight sums)
        sm::NlTree t;
        if (!sm::nl_build_lists(H, W, ew.data(), t)) return fail("lists", cs);
        const std::vector<uint32_t> adj = t.s_adj;
        std::vector<int32_t> rec((size_t)n * 4), rec2((size_t)n * 4);
        std::vector<float> wsum(n);
        if (!sm::nl_tree_from_lists(H, W, adj.data(), t, table.data(), 5, rec.data(), wsum.data())) return fail("walk", cs);
        for (int i = 0; i < n; i++) {
            const int p = t.pix[i];
            if (order[i] != p) return fail("breadth-first order", cs);
            if (parent[p] != t.pix[t.par[i]] || weight[p] != t.wgt[i] || nchild[p] != t.nch[i]) return fail("parent", cs);
            for (int j = 0; j < t.nch[i]; j++)
                if (child[(size_t)p * 4 + j] != t.pix[t.fc[i] + j]) return fail("child order", cs);
            uint32_t f;
            const float g = (float)ones[p];
            memcpy(&f, &wsum[p], 4);
            uint32_t gb;
            memcpy(&gb, &g, 4);
            if (f != gb) return fail("weight sums", cs);
        }
        sm::nl_pack_records(t, W, 5, rec2.data());
        if (rec != rec2) return fail("records", cs);
        // lists are in increasing (weight, edge index)
        for (int p = 0; p < n; p++) {
            const int y = p / W, x = p % W, cnt = (int)(adj[p] & 7);
            uint64_t prev = 0;
            for (int j = 0; j < cnt; j++) {
                const int d = (int)(adj[p] >> (3 + 2 * j)) & 3;
                const int q = W == 1 ? (d == 0 ? p + 1 : p - 1) : (d == 0 ? p + 1 : d == 1 ? p - 1 : d == 2 ? p + W : p - W);
                const uint32_t src = (d & 1) ? adj[q] : adj[p];
                const int ww = (int)(((d & 2) || W == 1) ? src >> 24 : (src >> 16) & 255);
                int idx;
                if (W == 1) idx = H * (W - 1) + x * (H - 1) + (d == 0 ? y : y - 1);
                else if (d == 0) idx = y * (W - 1) + x;
                else if (d == 1) idx = y * (W - 1) + x - 1;
                else if (d == 2) idx = H * (W - 1) + x * (H - 1) + y;
                else idx = H * (W - 1) + x * (H - 1) + y - 1;
                const uint64_t key = (uint64_t)ww << 32 | (uint32_t)idx;
                if (j > 0 && key <= prev) return fail("list order", cs);
                prev = key;
            }
        }
        // corrupted lists: one entry too many (degree sum off); a neighbour outside the image
        if (n >= 4 && W >= 2 && H >= 2) {
            std::vector<uint32_t> bad = adj;
            bad[0] = (bad[0] & ~7u) | ((bad[0] & 7) + 1);
            sm::NlTree t2;
            if (sm::nl_tree_from_lists(H, W, bad.data(), t2)) return fail("corrupt lists accepted", cs);
            bad = adj;   // an entry pointing out of the image (pixel 0 has no left neighbour)
            bad[0] = (bad[0] & ~(3u << 3)) | (1u << 3);
            if (sm::nl_tree_from_lists(H, W, bad.data(), t2)) return fail("out-of-image entry accepted", cs);
        }
        cases++;
    }
    printf("ok %d\n", cases);
    return 0;
}
