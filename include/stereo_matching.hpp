// stereo_matching.hpp — header-only C++ facade with the reference's class API over sm_capi.h.
//
// A user of the reference replaces `#include "stereoMatching.h"` by this header and keeps the
// main_.cpp call sequence (main_.cpp:138-172):
//
//   smamd::StereoMatching::Parameters param(maxDisp, rows, cols, lamCen, lamG, M, lamc, ts, csv, disSc);
//   auto* sm = new smamd::StereoMatching(I1_c, I2_c, I1, I2, param);
//   sm->costCalculate();                       // stereoMatching.cpp:945-1021
//   smamd::SolveAll(&sm, 1, 0.3f);             // stereoMatching.cpp:2142-2208
//   sm->dispOptimize();                        // stereoMatching.cpp:1046-1136
//   const int16_t* disparity = sm->DP[0].data();
//
// Images are plain views (smamd::Mat: rows, cols, channels, step, data) instead of cv::Mat so
// the facade needs no OpenCV; with OpenCV available, wrap a cv::Mat as {m.rows, m.cols,
// m.channels(), m.step, m.data}.  Non-OK statuses become std::runtime_error (the reference threw
// cv::Exception from CV_Assert).
#pragma once
#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "sm_capi.h"

namespace smamd {

struct Mat {
    int rows = 0, cols = 0, channels = 1;
    size_t step = 0;          // bytes per row
    const uint8_t* data = nullptr;
};

class StereoMatching {
   public:
    // static selectors (stereoMatching.h:51-53)
    inline static std::string costcalculation = "censusGrad";
    inline static std::string aggregation = "CBCA";
    inline static std::string optimization = "sgm";
    // h:70-80 are static const in the reference (compile-time); here they are read at construction
    inline static bool Do_refine = false;      // h:70
    static constexpr bool Do_LRConsis = true;  // h:72
    inline static bool Do_regionVote = true;   // h:75
    inline static bool Do_properIpol = true;   // h:76
    inline static bool Do_lastMedianBlur = true;  // h:80

    struct Parameters {  // StereoMatching::Parameters (h:85-351), the fields the hot path reads
        int numDisparities, rows, cols;
        int lamCen, lamG, disSc;
        int censusFunc = 3;
        int cbca_iterationNum = 2, cbca_minArmL = 1;
        int cbca_crossL0 = 17, cbca_crossL_out0 = 34, cbca_cTresh0 = 20, cbca_cTresh_out0 = 6;
        int sgm_scanNum = 4, sgm_corDifThres = 15, sgm_reduCoeffi1 = 4;
        int errorThreshold = 1;
        float LRmaxDiff = 0;                  // h:212
        int DISP_OCC = -2 * 16;               // h:216
        int region_vote_nums = 2;             // h:306
        Parameters(int maxDisp, int h, int w, int lamCen_ = 13, int lamG_ = 1, int /*M*/ = 2, int /*lamc*/ = 109,
                   int /*ts*/ = 10, const std::string& /*errCsvName*/ = "", int disSc_ = 1)
            : numDisparities(maxDisp + 1), rows(h), cols(w), lamCen(lamCen_), lamG(lamG_), disSc(disSc_) {}
    };

    StereoMatching(const Mat& I1_c, const Mat& I2_c, const Mat& I1_g, const Mat& I2_g, const Parameters& param,
                   int hip_device = 0)
        : h_(I1_c.rows), w_(I1_c.cols), d_(param.numDisparities) {
        sm_params p;
        sm_params_default(&p, param.numDisparities - 1, I1_c.rows, I1_c.cols);
        p.cost_method = costcalculation == "censusGrad" ? SM_COST_CENSUS_GRAD
                        : costcalculation == "Census"   ? SM_COST_CENSUS
                        : costcalculation == "ADCensus" ? SM_COST_AD_CENSUS
                        : costcalculation == "AD"       ? SM_COST_AD
                                                        : -1;
        if (p.cost_method < 0) throw std::invalid_argument("unsupported costcalculation: " + costcalculation);
        if (aggregation != "CBCA" && !aggregation.empty()) throw std::invalid_argument("unsupported aggregation: " + aggregation);
        if (optimization != "sgm" && optimization != "so" && !optimization.empty())
            throw std::invalid_argument("unsupported optimization: " + optimization);
        p.aggregation = aggregation == "CBCA" ? SM_AGG_CBCA : SM_AGG_NONE;
        p.optimization = optimization == "sgm" ? SM_OPT_SGM : (optimization == "so" ? SM_OPT_SO : SM_OPT_WTA);
        p.census_ring = param.censusFunc == 3;
        p.lam_cen = (float)param.lamCen;
        p.lam_g = (float)param.lamG;
        const int sc = param.disSc > 1 ? param.disSc : 1;   // calArms: L / scale (cpp:5367-5371)
        p.arm_l = param.cbca_crossL0 / sc;
        p.arm_l_out = param.cbca_crossL_out0 / sc;
        p.arm_c_thresh = param.cbca_cTresh0;
        p.arm_c_thresh_out = param.cbca_cTresh_out0;
        p.arm_min_l = param.cbca_minArmL;
        p.cbca_iterations = param.cbca_iterationNum;
        p.sgm_paths = param.sgm_scanNum;
        p.sgm_cor_dif_thres = param.sgm_corDifThres;
        p.sgm_redu_coeff = param.sgm_reduCoeffi1;
        p.do_refine = Do_refine ? 1 : 0;
        p.lr_max_diff = param.LRmaxDiff;
        p.disp_occ = param.DISP_OCC;
        p.region_vote_nums = param.region_vote_nums;
        p.do_region_vote = Do_regionVote ? 1 : 0;
        p.do_proper_ipol = Do_properIpol ? 1 : 0;
        p.do_last_median_blur = Do_lastMedianBlur ? 1 : 0;
        check(sm_create(&ctx_, &p, hip_device), "sm_create");
        if (I1_c.channels != 3 || I2_c.channels != 3 || I1_g.channels != 1 || I2_g.channels != 1)
            throw std::invalid_argument("expected BGR colour and single-channel gray images");
        check(sm_set_images(ctx_, I1_c.data, I2_c.data, I1_c.step, I1_g.data, I2_g.data, I1_g.step), "sm_set_images");
    }
    ~StereoMatching() { sm_destroy(ctx_); }
    StereoMatching(const StereoMatching&) = delete;
    StereoMatching& operator=(const StereoMatching&) = delete;

    void costCalculate() { check(sm_cost_calculate(ctx_), "costCalculate"); }
    void dispOptimize() {  // DP[0] (and DP[1] when Do_refine), cpp:1046-1136
        DP[0].resize((size_t)h_ * w_);
        check(sm_disp_optimize(ctx_, DP[0].data()), "dispOptimize");
        if (Do_refine) {
            DP[1].resize((size_t)h_ * w_);
            check(sm_get_disp(ctx_, 1, DP[1].data()), "DP[1]");
        }
    }
    void refine() {  // cpp:1138-1511; needs Do_refine at construction
        DP[0].resize((size_t)h_ * w_);
        check(sm_refine(ctx_, DP[0].data()), "refine");
    }
    std::vector<float> volume(int view = 0) {
        std::vector<float> v((size_t)h_ * w_ * d_);
        check(sm_get_volume(ctx_, view, v.data()), "vm");
        return v;
    }

    std::vector<int16_t> DP[2];  // DP[0]: int16 H x W disparity, -1 = invalid (h:2724)
    int h_, w_, d_;
    sm_ctx* ctx_ = nullptr;

   private:
    void check(sm_status s, const char* what) {
        if (s != SM_OK) throw std::runtime_error(std::string(what) + ": " + sm_last_error(ctx_));
    }
    friend void SolveAll(StereoMatching** smPyr, int PY_LVL, float REG_LAMBDA);
};

// SolveAll (cpp:2142-2208): PY_LVL = 1 scales vm[0]; PY_LVL in [2, 3] combines the levels
// smPyr[0..PY_LVL-1] of main_.cpp:134-156's pyramid into smPyr[0].
inline void SolveAll(StereoMatching** smPyr, int PY_LVL, float REG_LAMBDA) {
    if (PY_LVL == 1) {
        smPyr[0]->check(sm_solve_all(smPyr[0]->ctx_, PY_LVL, REG_LAMBDA), "SolveAll");
        return;
    }
    std::vector<sm_ctx*> lv;
    for (int i = 0; i < PY_LVL; i++) lv.push_back(smPyr[i]->ctx_);
    smPyr[0]->check(sm_solve_all_pyr(lv.data(), PY_LVL, REG_LAMBDA), "SolveAll");
}

// cv::pyrDown for u8 images (main_.cpp:145-148) on the GPU; returns the (rows+1)/2 x (cols+1)/2 image.
inline std::vector<uint8_t> pyrDown(const Mat& src, int hip_device = 0) {
    std::vector<uint8_t> in((size_t)src.rows * src.cols * src.channels);
    for (int r = 0; r < src.rows; r++)
        std::copy(src.data + (size_t)r * src.step, src.data + (size_t)r * src.step + (size_t)src.cols * src.channels,
                  in.begin() + (size_t)r * src.cols * src.channels);
    std::vector<uint8_t> out((size_t)((src.rows + 1) / 2) * ((src.cols + 1) / 2) * src.channels);
    if (sm_pyr_down(hip_device, in.data(), src.rows, src.cols, src.channels, out.data()) != SM_OK)
        throw std::runtime_error("pyrDown failed");
    return out;
}

}  // namespace smamd
