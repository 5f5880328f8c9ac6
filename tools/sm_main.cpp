// sm_main.cpp — the reference driver's call sequence (main_.cpp:21-195) over the C++ facade.
// Reads a left/right pair as binary PPM (P6, RGB) files with smamd::imread (BGR + gray the way
// cv::imread(.., 1) / cv::imread(.., 0) would for PNG: libpng rgb->gray formula), runs
// costCalculate -> SolveAll(1, 0.3) -> dispOptimize, and writes DP[0] as a 16-bit PGM.
// Usage: sm_main left.ppm right.ppm max_disp out.pgm [device]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "../include/stereo_matching.hpp"

using smamd::Mat;
using smamd::StereoMatching;

std::string StereoMatching::costcalculation = "censusGrad";   // main_.cpp:15-19
std::string StereoMatching::aggregation = "CBCA";
std::string StereoMatching::optimization = "sgm";
std::string StereoMatching::object = "";
const std::string StereoMatching::root = "";

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s left.ppm right.ppm max_disp out.pgm [device] [refine]\n", argv[0]);
        return 2;
    }
    Mat I1_c = smamd::imread(argv[1], 1), I2_c = smamd::imread(argv[2], 1);
    Mat I1 = smamd::imread(argv[1], 0), I2 = smamd::imread(argv[2], 0);
    if (I1_c.empty() || I2_c.empty() || I1_c.rows != I2_c.rows || I1_c.cols != I2_c.cols) {
        std::fprintf(stderr, "can't read original img\n");  // main_.cpp:110
        return -1;
    }
    const int w = I1_c.cols, h = I1_c.rows;
    const int maxDisp = std::atoi(argv[3]);
    const int dev = argc > 5 ? std::atoi(argv[5]) : 0;
    StereoMatching::Do_refine = argc > 6 && std::atoi(argv[6]) != 0;
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
        const int16_t* dp = sm->DP[0].ptr<int16_t>();
        for (size_t i = 0; i < (size_t)w * h; i++) {
            const int16_t d = dp[i];
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
