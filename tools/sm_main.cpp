// sm_main.cpp — the reference driver's call sequence (main_.cpp:21-195) over the C++ facade.
// Reads a left/right pair as binary PPM (P6, RGB) files, converts to BGR + gray the way
// cv::imread(.., 1) / cv::imread(.., 0) would for PNG (libpng rgb->gray formula), runs
// costCalculate -> SolveAll(1, 0.3) -> dispOptimize, and writes DP[0] as a 16-bit PGM.
// Usage: sm_main left.ppm right.ppm max_disp out.pgm [device]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "../include/stereo_matching.hpp"

static bool read_ppm(const char* path, int& w, int& h, std::vector<uint8_t>& rgb) {
    std::ifstream f(path, std::ios::binary);
    std::string magic;
    int maxv;
    if (!(f >> magic >> w >> h >> maxv) || magic != "P6" || maxv != 255) return false;
    f.get();
    rgb.resize((size_t)w * h * 3);
    f.read((char*)rgb.data(), rgb.size());
    return (bool)f;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s left.ppm right.ppm max_disp out.pgm [device] [refine]\n", argv[0]);
        return 2;
    }
    int w, h, w2, h2;
    std::vector<uint8_t> l, r;
    if (!read_ppm(argv[1], w, h, l) || !read_ppm(argv[2], w2, h2, r) || w != w2 || h != h2) {
        std::fprintf(stderr, "can't read original img\n");  // main_.cpp:110
        return -1;
    }
    const int maxDisp = std::atoi(argv[3]);
    const int dev = argc > 5 ? std::atoi(argv[5]) : 0;
    smamd::StereoMatching::Do_refine = argc > 6 && std::atoi(argv[6]) != 0;
    std::vector<uint8_t> lb(l.size()), rb(r.size()), lg((size_t)w * h), rg((size_t)w * h);
    for (size_t i = 0; i < (size_t)w * h; i++) {
        for (int c = 0; c < 3; c++) {
            lb[i * 3 + c] = l[i * 3 + 2 - c];
            rb[i * 3 + c] = r[i * 3 + 2 - c];
        }
        lg[i] = (uint8_t)((l[i * 3] * 9798 + l[i * 3 + 1] * 19235 + l[i * 3 + 2] * 3735 + 16384) >> 15);
        rg[i] = (uint8_t)((r[i * 3] * 9798 + r[i * 3 + 1] * 19235 + r[i * 3 + 2] * 3735 + 16384) >> 15);
    }
    using smamd::Mat;
    Mat I1_c{h, w, 3, (size_t)w * 3, lb.data()}, I2_c{h, w, 3, (size_t)w * 3, rb.data()};
    Mat I1{h, w, 1, (size_t)w, lg.data()}, I2{h, w, 1, (size_t)w, rg.data()};
    std::printf("method: %s\n", (smamd::StereoMatching::costcalculation + smamd::StereoMatching::aggregation +
                                 smamd::StereoMatching::optimization).c_str());
    try {
        auto t0 = std::chrono::steady_clock::now();
        smamd::StereoMatching::Parameters param(maxDisp, h, w, 13, 1, 2, 109, 10, "", 1);
        auto* sm = new smamd::StereoMatching(I1_c, I2_c, I1, I2, param, dev);
        sm->costCalculate();
        smamd::SolveAll(&sm, 1, 0.3f);
        sm->dispOptimize();
        if (smamd::StereoMatching::Do_refine) sm->refine();  // main_.cpp:165-166
        auto t1 = std::chrono::steady_clock::now();
        std::printf("all Time: %.3f ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count());
        std::ofstream o(argv[4], std::ios::binary);
        o << "P5\n" << w << " " << h << "\n65535\n";
        for (int16_t d : sm->DP[0]) {
            uint16_t v = d < 0 ? 0 : (uint16_t)d;
            o.put((char)(v >> 8));
            o.put((char)(v & 0xff));
        }
        delete sm;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
