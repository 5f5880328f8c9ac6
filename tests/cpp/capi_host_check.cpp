// capi_host_check.cpp — the host side of the C-ABI (mystereomatching_amd/csrc/sm_capi.cpp) under
// -fsanitize=address,undefined on a machine without a GPU (tests/test_sanitizers.py): parameter
// validation for every field that sm_create checks before touching a device, the struct_size
// guard, null and out-of-range arguments of every entry point, sm_run_batch_multi's argument
// checks, the calErr evaluator (h:1748-1825) on random maps and masks, and the host expf.
// Prints "ok <checks>" and exits 0; a failed expectation prints it and exits 1; a sanitizer
// finding aborts.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "sm_capi.h"

static int checks = 0;
static bool expect(bool ok, const std::string& what) {
    checks++;
    if (!ok) std::printf("FAILED: %s\n", what.c_str());
    return ok;
}

// sm_create with one field changed must fail with SM_EINVAL and a message naming it
static bool rejects(const char* name, const std::function<void(sm_params&)>& set, const char* msg, int max_disp = 63) {
    sm_params p;
    sm_params_default(&p, max_disp, 32, 32);
    set(p);
    sm_ctx* c = nullptr;
    const sm_status st = sm_create(&c, &p, 0);
    const std::string err = sm_last_error(c);
    sm_destroy(c);
    return expect(st == SM_EINVAL && err.find(msg) != std::string::npos,
                  std::string("validation of ") + name + ": status " + std::to_string(st) + " '" + err + "'");
}

int main() {
    bool ok = true;
    // defaults and the struct guard
    for (int md : {0, 1, 15, 63, 255, 1023})
        for (int r : {2, 3, 375, 2000}) {
            sm_params p;
            sm_params_default(&p, md, r, r + 1);
            ok &= expect(p.struct_size == sizeof(sm_params) && p.num_disparities == md + 1 && p.rows == r &&
                             p.lr_consis == 1 && p.fuse_norm_scan == -1,
                         "sm_params_default");
        }
    ok &= rejects("struct_size", [](sm_params& p) { p.struct_size = 4; }, "struct_size");
    ok &= rejects("rows", [](sm_params& p) { p.rows = 1; }, "rows");
    ok &= rejects("cols", [](sm_params& p) { p.cols = -5; }, "rows and cols");
    ok &= rejects("rows*cols", [](sm_params& p) { p.rows = 65535; p.cols = 1 << 16; }, "too large");
    ok &= rejects("num_disparities 0", [](sm_params& p) { p.num_disparities = 0; }, "num_disparities");
    ok &= rejects("num_disparities 2000", [](sm_params& p) { p.num_disparities = 2000; }, "num_disparities");
    ok &= rejects("cost_method", [](sm_params& p) { p.cost_method = 7; }, "cost_method");
    ok &= rejects("cost_method -1", [](sm_params& p) { p.cost_method = -1; }, "cost_method");
    ok &= rejects("aggregation", [](sm_params& p) { p.aggregation = 4; }, "aggregation");
    ok &= rejects("census_rv", [](sm_params& p) { p.census_rv = 7; }, "census");
    ok &= rejects("arm_l_out", [](sm_params& p) { p.arm_l_out = 200; }, "arm");
    ok &= rejects("sgm_paths", [](sm_params& p) { p.sgm_paths = 9; }, "sgm_paths");
    ok &= rejects("batch_capacity", [](sm_params& p) { p.batch_capacity = 0; }, "batch");
    ok &= rejects("lam_cen", [](sm_params& p) { p.lam_cen = 0.0f; }, "lambda");
    ok &= rejects("lam_g", [](sm_params& p) { p.lam_g = -1.0f; }, "lambda");
    ok &= rejects("lam_g NaN", [](sm_params& p) { p.lam_g = NAN; }, "lambda");
    ok &= rejects("grad_trunc", [](sm_params& p) { p.grad_trunc = -0.0f; }, "truncation");
    ok &= rejects("ad_trunc_ad", [](sm_params& p) { p.ad_trunc_ad = -0.0f; }, "truncation");
    ok &= rejects("sgm_p1", [](sm_params& p) { p.sgm_p1 = -0.0f; }, "penalties");
    ok &= rejects("sgm_p2", [](sm_params& p) { p.sgm_p2 = -1.0f; }, "penalties");
    ok &= rejects("sgm_redu_coeff", [](sm_params& p) { p.sgm_redu_coeff = -4; }, "penalties");
    ok &= rejects("num_streams", [](sm_params& p) { p.num_streams = 5; }, "num_streams");
    ok &= rejects("sub_batch", [](sm_params& p) { p.sub_batch = -1; }, "sub_batch");
    ok &= rejects("rv_ratio", [](sm_params& p) { p.do_refine = 1; p.rv_ratio = 0.0f; }, "rv_ratio");
    ok &= rejects("region_vote_nums", [](sm_params& p) { p.do_refine = 1; p.region_vote_nums = -1; }, "region_vote_nums");
    ok &= rejects("GF rows", [](sm_params& p) { p.aggregation = 2; p.rows = 8; }, "GF", 15);
    ok &= rejects("GF MY_GUIDE rows", [](sm_params& p) { p.aggregation = 2; p.gf_mode = 1; p.rows = 18; }, "GF", 15);
    ok &= rejects("GF eps", [](sm_params& p) { p.aggregation = 2; p.gf_eps = 0.0f; }, "gf_eps", 15);
    ok &= rejects("GF mode", [](sm_params& p) { p.aggregation = 2; p.gf_mode = 2; }, "gf_mode", 15);
    ok &= rejects("NL rows", [](sm_params& p) { p.aggregation = 3; p.rows = 2; }, "NL", 15);
    ok &= rejects("NL sigma", [](sm_params& p) { p.aggregation = 3; p.nl_sigma = 0.0; }, "nl_sigma", 15);
    ok &= rejects("NL size", [](sm_params& p) { p.aggregation = 3; p.rows = 8192; p.cols = 8192; p.batch_capacity = 8; },
                  "2^29", 15);
    {   // a valid struct passes validation and fails only at the device (no GPU here)
        sm_params p;
        sm_params_default(&p, 63, 32, 32);
        sm_ctx* c = nullptr;
        const sm_status st = sm_create(&c, &p, 0);
        ok &= expect(st != SM_EINVAL || std::string(sm_last_error(c)).find("device") != std::string::npos,
                     std::string("valid params: ") + sm_last_error(c));
        sm_destroy(c);
    }
    // null contexts and pointers
    ok &= expect(sm_create(nullptr, nullptr, 0) == SM_EINVAL, "sm_create(null)");
    ok &= expect(sm_destroy(nullptr) == SM_OK, "sm_destroy(null)");
    ok &= expect(std::string(sm_last_error(nullptr)) == "null context", "sm_last_error(null)");
    ok &= expect(sm_cost_calculate(nullptr) == SM_EINVAL && sm_solve_all(nullptr, 1, 0.3f) == SM_EINVAL &&
                     sm_disp_optimize(nullptr, nullptr) == SM_EINVAL && sm_refine(nullptr, nullptr) == SM_EINVAL &&
                     sm_get_disp(nullptr, 0, nullptr) == SM_EINVAL && sm_set_disp(nullptr, 0, nullptr) == SM_EINVAL &&
                     sm_get_volume(nullptr, 0, nullptr) == SM_EINVAL && sm_get_arms(nullptr, 0, nullptr) == SM_EINVAL &&
                     sm_upload_batch(nullptr, 1, nullptr, nullptr, nullptr, nullptr) == SM_EINVAL &&
                     sm_run(nullptr, 1, 0.3f, nullptr) == SM_EINVAL && sm_download_disp(nullptr, 1, nullptr) == SM_EINVAL &&
                     sm_download_disp_async(nullptr, 1, nullptr) == SM_EINVAL && sm_synchronize(nullptr) == SM_EINVAL &&
                     sm_profile_enable(nullptr, 1) == SM_EINVAL && sm_profile_reset(nullptr) == SM_EINVAL &&
                     sm_set_images(nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0) == SM_EINVAL &&
                     sm_get_census(nullptr, 0, nullptr) == SM_EINVAL && sm_solve_all_pyr(nullptr, 2, 0.3f) == SM_EINVAL,
                 "null context");
    for (int s = 0; s <= 5; s++) ok &= expect(sm_status_string((sm_status)s) != nullptr, "sm_status_string");
    ok &= expect(std::string(sm_status_string((sm_status)7)) == "unknown status", "sm_status_string(7)");
    {
        std::vector<uint8_t> b(64);
        std::vector<int16_t> out(64);
        sm_ctx* none[1] = {nullptr};
        ok &= expect(sm_run_batch_multi(nullptr, 1, 1, b.data(), b.data(), b.data(), b.data(), 0.3f, out.data()) == SM_EINVAL &&
                         sm_run_batch_multi(none, 1, 1, b.data(), b.data(), b.data(), b.data(), 0.3f, out.data()) == SM_EINVAL &&
                         sm_run_batch_multi(none, 0, 1, b.data(), b.data(), b.data(), b.data(), 0.3f, out.data()) == SM_EINVAL &&
                         sm_run_batch_multi(none, 1, 0, b.data(), b.data(), b.data(), b.data(), 0.3f, out.data()) == SM_EINVAL,
                     "sm_run_batch_multi arguments");
        ok &= expect(sm_pyr_down(0, nullptr, 4, 4, 1, nullptr) != SM_OK && sm_pyr_down_f32(0, nullptr, 4, 4, nullptr) != SM_OK,
                     "sm_pyr_down null");
    }
    // calErr (h:1748-1825) against a direct evaluation in the reference's order
    {
        std::mt19937 g(7);
        for (int t = 0; t < 40; t++) {
            const int H = 1 + (int)(g() % 40), W = 1 + (int)(g() % 50);
            std::vector<int16_t> d(H * W);
            std::vector<float> gt(H * W);
            std::vector<uint8_t> m(H * W);
            for (int i = 0; i < H * W; i++) {
                d[i] = (int16_t)((int)(g() % 80) - 8);
                gt[i] = (float)(g() % 700) / 10.0f;
                m[i] = (g() % 3) ? 255 : (uint8_t)(g() % 255);
            }
            const float thres = (float)(g() % 4);
            float pbm = -1, rms = -1;
            const sm_status st = sm_cal_err(d.data(), gt.data(), m.data(), H, W, thres, &pbm, &rms);
            int cnt = 0, err = 0;
            float sum = 0.f;
            for (int i = 0; i < H * W; i++) {
                if (m[i] != 255) continue;
                cnt++;
                if (d[i] < 0) {
                    err++;
                    sum += 2;
                } else {
                    const float dif = std::fabs(gt[i] - (float)d[i]);
                    if (dif > thres) err++;
                    sum += (float)std::pow(dif, 2);
                }
            }
            if (cnt == 0) {
                ok &= expect(st != SM_OK || (pbm >= 0 && rms >= 0), "calErr empty mask");
                continue;
            }
            ok &= expect(st == SM_OK && pbm == (float)err / (float)cnt, "calErr pbm " + std::to_string(t));
            ok &= expect(std::isfinite(rms), "calErr rms " + std::to_string(t));
        }
        float pbm, rms;
        ok &= expect(sm_cal_err(nullptr, nullptr, nullptr, 4, 4, 1.0f, &pbm, &rms) == SM_EINVAL, "calErr null");
    }
    // the host expf on the edges of its domain
    for (float x : {0.0f, -0.0f, -1e-30f, -1.0f, -17.5f, -87.3f, -103.9f, -104.0f, -1e30f}) {
        const float y = sm_expf_host(x);
        ok &= expect(y >= 0.0f && y <= 1.0f, "expf_host range");
    }
    std::printf("ok %d\n", checks);
    return ok ? 0 : 1;
}
