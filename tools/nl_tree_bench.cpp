// nl_tree_bench.cpp — host timing of the NL tree build phases (sm_nl_tree.cpp) on synthetic
// image-like edge weights (tools/Makefile builds it as tools/build/nl_tree_bench).
// usage: nl_tree_bench [H W reps]
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <vector>

#include "sm_nl_tree.h"

int main(int argc, char** argv) {
    const int H = argc > 1 ? atoi(argv[1]) : 375, W = argc > 2 ? atoi(argv[2]) : 450;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    // a smooth colour field with texture and a few edges, as max channel differences
    std::vector<uint8_t> img((size_t)H * W * 3);
    uint32_t s = 12345;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
            for (int c = 0; c < 3; c++) {
                s = s * 1664525u + 1013904223u;
                const double v = 128 + 60 * sin(0.03 * x + c) * cos(0.02 * y) + ((x / 37 + y / 29) % 3) * 20 + (s >> 28);
                img[((size_t)y * W + x) * 3 + c] = (uint8_t)std::min(255.0, std::max(0.0, v));
            }
    const int ne = H * (W - 1) + (H - 1) * W;
    std::vector<uint8_t> ew(ne);
    auto d = [&](int a, int b) {
        int m = 0;
        for (int c = 0; c < 3; c++) m = std::max(m, abs(img[(size_t)a * 3 + c] - img[(size_t)b * 3 + c]));
        return (uint8_t)m;
    };
    int e = 0;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W - 1; x++) ew[e++] = d(y * W + x, y * W + x + 1);
    for (int x = 0; x < W; x++)
        for (int y = 0; y < H - 1; y++) ew[e++] = d(y * W + x, (y + 1) * W + x);
    std::vector<double> table(256);
    for (int i = 0; i < 256; i++) table[i] = exp(-i / 25.5);
    sm::NlTree t;
    std::vector<int32_t> rec((size_t)H * W * 4);
    std::vector<float> wsum((size_t)H * W);
    using clk = std::chrono::steady_clock;
    double tb = 1e9, tp = 1e9, tw = 1e9;
    for (int r = 0; r < reps; r++) {
        auto t0 = clk::now();
        if (!sm::nl_build_tree(H, W, ew.data(), t)) return 1;
        auto t1 = clk::now();
        sm::nl_pack_records(t, W, 0, rec.data());
        auto t2 = clk::now();
        sm::nl_weight_sums(t, table.data(), wsum.data());
        auto t3 = clk::now();
        tb = std::min(tb, std::chrono::duration<double, std::milli>(t1 - t0).count());
        tp = std::min(tp, std::chrono::duration<double, std::milli>(t2 - t1).count());
        tw = std::min(tw, std::chrono::duration<double, std::milli>(t3 - t2).count());
    }
    long h = 0;
    for (int i = 0; i < H * W; i++) h = h * 31 + t.pix[t.par[i]];
    printf("H=%d W=%d build %.2f ms  pack %.2f ms  wsum %.2f ms  paths %zu  hash %ld\n", H, W, tb, tp, tw,
           t.chain_len.size(), h);
    return 0;
}
