// sm_capi.cpp — C-ABI of libsm_hip.so: context, HBM buffers, stage drivers, profiling.
// The entry points mirror the reference's StereoMatching call sequence (see include/sm_capi.h
// for the file:line of each reference interface).  No exceptions cross the ABI.
#include "../../include/sm_capi.h"

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cfloat>
#include <array>
#include <chrono>
#include <cmath>
#include <map>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "sm_kernels.h"


namespace {

struct ProfRec {
    int kernel;
    hipEvent_t start, stop;
};

struct ProfStat {
    int64_t launches = 0;
    double total_ms = 0;
    double bytes = 0;  // algorithmic bytes per launch (last seen)
};

}  // namespace

struct sm_ctx {
    sm_params p{};
    int device = 0;
    hipStream_t st = nullptr;
    std::string err;
    int cap = 1;
    size_t npix = 0, nvol = 0;
    size_t vtail = 0;           // floats of tail pad after each volume's cap * nvol
    uint8_t* bgr = nullptr;     // [cap][2][npix][3]
    uint8_t* gray = nullptr;    // [cap][2][npix]
    ulonglong2* code = nullptr; // [cap][2][npix]
    uint8_t* arms = nullptr;    // [cap][2 views][2 planes][npix] u32: (L | R<<16), (U | D<<16)
    uint8_t* arms_alloc = nullptr;  // arms - front pad of 2 * lag rows (CBCA V sweeps read there)
    size_t arms_bytes = 0;
    float* vm0 = nullptr;       // [cap][npix][D]
    float* vm1 = nullptr;       // [cap][npix][D] (right view, optional)
    float* acc = nullptr;       // [cap][npix][D]
    float* ck = nullptr;        // [cap][ck_pair]: checkpointed SGM path pairs (k_sgm_ck)
    size_t ck_pair = 0;         // floats per pair: lines x segments x D of the longer direction
    float* lx = nullptr;        // [cap][npix][D]: L5 between the diagonal pair (8 paths, sgm_ck_diag_ok)
    int16_t* disp = nullptr;    // [cap][npix] DP[0]
    int16_t* disp1 = nullptr;   // [cap][npix] DP[1] (do_refine)
    int16_t* disp_tmp = nullptr;// [cap][npix] refine ping-pong (do_refine)
    float* dummy = nullptr;     // 64 floats written by lanes past D
    uint8_t* flags = nullptr;   // [cap][npix] SGM colour-difference penalty bits, left image
    uint8_t* flags1 = nullptr;  // [cap][npix] same for the right image (do_refine)
    uint8_t* so_trace = nullptr;   // [cap][npix][D] "so" choice codes
    uint16_t* so_cidx = nullptr;   // [cap][npix] "so" row-minimum indices
    uint32_t* px = nullptr;     // [cap][2][npix] packed BGR, then the pxh and pxv arm-walk planes (same shape)
    // aggregation "GF": three scratch volumes (the SGM sum is the fourth), image planes, per-pixel terms
    float* gf_s = nullptr;      // [3 (+1 without acc)][cap][nvol]
    float* gf_planes = nullptr; // [cap][10][npix]
    sm::GfPix* gf_pix = nullptr;// [cap][npix]
    // aggregation "GF", ximgproc form: row sums (4 double volumes), alpha / beta (4 float volumes),
    // image-plane row sums [cap][9][npix] doubles and per-pixel terms [cap][9][npix] floats
    double* gfc_rs = nullptr;
    float* gfc_ab = nullptr;
    double* gfc_img = nullptr;
    float* gfc_pix = nullptr;
    // aggregation "NL": median image, edge weights, spanning trees, the tree walk, filter values
    uint8_t* nl_med = nullptr;  // [cap][npix][3]
    uint8_t* nl_ew = nullptr;   // [cap][ne]
    int* nl_ints = nullptr;     // two sets of: chain_start, chain_len, order_up, order_down [cap][npix] each
    int* nl_rec = nullptr;      // two sets of path-node records (4 ints) [cap][npix], zero padding on both sides
    int* nl_par = nullptr;      // spanning-tree union-find parents [cap][npix] (sm_nl_mst.hip)
    unsigned long long* nl_best = nullptr;  // lightest edge key offered to each component [cap][npix]
    uint8_t* nl_mst = nullptr;              // spanning-tree work space (sm::nl_mst_scratch_bytes)
    uint32_t* nl_adj = nullptr;             // tree neighbour lists [cap][npix]
    uint8_t* nl_walk = nullptr;             // tree-walk work space (sm::nl_walk_scratch_bytes)
    int* nl_offs = nullptr;                 // round offsets + error flags (device)
    int* nl_offs_h = nullptr;               // the same, page-locked host copy
    int nl_set = 0;                         // record / table set of the next call (double-buffered)
    int nl_opt_set = 0;                     // pipelined NL: the set the current call's optimiser reads
    hipStream_t nl_st = nullptr;        // NL front (median, edge weights, spanning trees, tree walk)
    hipEvent_t nl_ev_set[2] = {nullptr, nullptr};   // the last filter reading each record / table set (on c->st)
    // pipelined NL front (sm_run with NL + SGM, one view): the call's prep and cost volume also run
    // on nl_st, into a cost volume and penalty flags of the call's set, so they overlap the
    // previous call's filter and SGM on c->st
    bool nl_pipe = false;
    float* nl_vc = nullptr;                 // [2][cap][nvol] cost volumes (filter input)
    uint8_t* nl_fl = nullptr;               // [2][cap][npix] SGM penalty flags
    hipEvent_t nl_ev_opt[2] = {nullptr, nullptr};   // the last optimiser reading each set (on c->st)
    double* nl_table = nullptr; // [256]
    double* nl_val = nullptr;   // [cap][nvol]
    double* nl_oup = nullptr;   // [cap][npix] the ones channel: up sums
    double* nl_ofin = nullptr;  // [cap][npix] final sums
    int n_loaded = 0;
    int stage = 0;              // 0 none, 1 images, 2 cost+agg, 3 solve_all, 4 optimized, 5 refined
    float lut_a[1024], lut_b[1024];
    float* luts = nullptr;      // device copy of lut_a | lut_b (per context: contexts on one device may differ)
    float ad_oor_exp = 0;
    bool fuse_norm_scan = false;
    int num_cu = 256;           // compute units of the device
    int sub_batch = 0;          // sm_params.sub_batch: run sm_run in groups of k pairs (0 = all)
    int nstreams = 1;           // sm_params.num_streams: groups alternate over s streams (see sm_run)
    bool auto_groups = false;   // num_streams = 0 chose two streams: sm_run splits n pairs into two groups
    bool pipelined = false;     // auto_groups with CBCA + SGM: the two groups run as a pipeline across calls
    bool pipe_live = false;     // the side stream still runs the second group of the last sm_run (not joined)
    int pipe_g = 0;             // pairs in the first group of the last pipelined sm_run
    hipEvent_t ev_copy2 = nullptr;   // async copy of a pipelined run's second group done (cst)
    bool copy_split = false;    // the pending async copy is two copies (ev_copy: group 0, ev_copy2: group 1)
    int copy_g = 0;             // with copy_split: pairs [0, copy_g) are ev_copy's, ev_copy2 covers all n
    hipEvent_t ev_dl[2] = {};   // the last two async downloads' copies done (cst), for sm_download_wait
    int dl_slot = 0;            // ev_dl slot of the next async download
    int dl_count = 0;
    hipEvent_t ev_up[2] = {};   // an async upload's copies done: main stream, side stream
    hipEvent_t ev_in[2] = {};   // a pipelined run's group k has read its input images (after the cost volume)
    // (an early async upload goes on the null stream: the runtime spreads streams round-robin over
    // GPU_MAX_HW_QUEUES (4) in-order hardware queues, and a fifth stream of the context shared one
    // with a group or the map copies, whose kernels / copies the upload then waited behind; the
    // null stream's queue carries nothing else on the hot path, and the context's streams are
    // non-blocking, so it implies no synchronisation with them)
    bool up_split = false;      // the async upload's second group went on the side stream
    hipStream_t xst[3] = {nullptr, nullptr, nullptr};  // extra streams when nstreams > 1
    hipStream_t cst = nullptr;  // copy stream of sm_download_disp_async
    hipEvent_t ev_run = nullptr, ev_copy = nullptr;     // run done (c->st) / async copy done (cst)
    bool copy_pending = false;  // an async copy may still read the maps
    int place_trials = 0;       // > 1: the first sm_run chooses among that many volume sets (place_volumes)
    std::vector<double> place_ms;   // the trials' pipeline times (sm_placement_trials_ms)
    int place_best = -1;
    std::vector<hipEvent_t> xev;                        // stagger / join events
    hipEvent_t stagger_ev = nullptr;                    // SM_STAGGER_STAGE 1: recorded after the first CBCA sweep
    // profiling
    bool prof = false;
    std::vector<ProfRec> recs;
    std::vector<hipEvent_t> free_events;
    std::vector<std::string> knames;
    std::map<std::string, int> kidx;
    std::vector<ProfStat> kstat;
};

namespace {

sm_status fail(sm_ctx* c, sm_status s, const std::string& msg) {
    if (c) c->err = msg;
    return s;
}

sm_status hip_fail(sm_ctx* c, hipError_t e, const char* where) {
    return fail(c, SM_EHIP, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(c, expr)                                      \
    do {                                                      \
        hipError_t e_ = (expr);                               \
        if (e_ != hipSuccess) return hip_fail((c), e_, #expr); \
    } while (0)

hipEvent_t get_event(sm_ctx* c) {
    if (!c->free_events.empty()) {
        hipEvent_t e = c->free_events.back();
        c->free_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int kernel_id(sm_ctx* c, const char* name, double bytes) {
    auto it = c->kidx.find(name);
    int id;
    if (it == c->kidx.end()) {
        id = (int)c->knames.size();
        c->kidx[name] = id;
        c->knames.push_back(name);
        c->kstat.emplace_back();
    } else {
        id = it->second;
    }
    c->kstat[id].bytes = bytes;
    return id;
}

// Brackets one launch with events when profiling is on.
template <typename F>
sm_status timed(sm_ctx* c, const char* name, double bytes, F&& launch) {
    ProfRec r{-1, nullptr, nullptr};
    if (c->prof) {
        r.kernel = kernel_id(c, name, bytes);
        r.start = get_event(c);
        r.stop = get_event(c);
        if (r.start) hipEventRecord(r.start, c->st);
    }
    launch();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(c, e, name);
    if (c->prof && r.start && r.stop) {
        hipEventRecord(r.stop, c->st);
        c->recs.push_back(r);
    }
    return SM_OK;
}

int census_len(const sm_params& p) { return (2 * p.census_rv + 1) * (2 * p.census_ru + 1) + (p.census_ring ? 8 : 0); }

bool needs_census(const sm_params& p) { return p.cost_method != SM_COST_AD; }
bool needs_arms(const sm_params& p) {
    return p.cost_method == SM_COST_CENSUS_GRAD || p.aggregation == SM_AGG_CBCA || p.do_refine;  // + regionVote (cpp:1393-1396)
}
// "so" runs on both views when Do_LRConsis (num = Do_LRConsis ? 2 : 1, cpp:1093, Do_LRConsis = 1,
// h:72; imgNum = Do_LRConsis ? 2 : 1 in costCalculate, cpp:952), so DP[1] = so(vm[1]) needs the
// right cost volume even without Do_refine
bool so_views2(const sm_params& p) { return p.optimization == SM_OPT_SO && p.lr_consis; }
bool right_view(const sm_params& p) { return p.compute_right_view || p.do_refine || so_views2(p); }
int n_views(const sm_params& p) { return p.do_refine ? 2 : 1; }   // imgNum = Do_refine && Do_LRConsis ? 2 : 1
// views dispOptimize runs on: sgm / WTA num = Do_refine && Do_LRConsis ? 2 : 1 (cpp:1054, 1110);
// so num = Do_LRConsis ? 2 : 1 (cpp:1093) -- on vm[1] as costCalculate left it (CBCA and
// SolveAll touch vm[1] only with Do_refine, cpp:5592, 2178)
int opt_views(const sm_params& p) { return p.optimization == SM_OPT_SO ? (p.lr_consis ? 2 : 1) : n_views(p); }

int cbca_lag(const sm_params& p) { return p.arm_l_out > p.arm_min_l ? p.arm_l_out : p.arm_min_l; }

// Every dividend of iteration k's normalisation (genfinalVm_cbca, cpp:3969-3992) is 0 or
// >= 2^-110, so the area division needs no check for tiny dividends (sm_device.h div_area)?
// Costs are 0 or >= 2^f0: censusGrad / ADCensus fl(fl(2 - e0) - e1) with e0, e1 in [0, 1] is 0
// or >= 2^-24 (fl(2 - e0) = 1 gives 1 - e1 >= 2^-24 unless e1 = 1, else >= 1 + 2^-23 - 1);
// Census costs are integers; AD costs are 0 or >= min(1/3, trunc).  A prefix sum of values 0 or
// >= 2^f is 0 or >= 2^f, and a difference of two such sums is 0, the larger sum, or >= ulp(2^f)
// = 2^(f - 23); so iteration k's scan outputs are 0 or >= 2^(f_k - 23), its normalisation's
// dividends 0 or >= 2^(f_k - 46), and its quotients (areas < 2^15) 0 or >= 2^(f_k - 61) = f_{k+1}.
bool cbca_div_safe(const sm_params& p, int k) {
    int f0;
    if (p.cost_method == SM_COST_CENSUS_GRAD || p.cost_method == SM_COST_AD_CENSUS) {
        f0 = -24;
    } else if (p.cost_method == SM_COST_CENSUS) {
        f0 = 0;
    } else if (p.cost_method == SM_COST_AD) {   // AD: min(s / 3, trunc)
        if (p.ad_trunc_ad == 0.0f) return true;   // every cost is 0
        const float m = std::min(1.0f / 3.0f, p.ad_trunc_ad);
        f0 = std::ilogb(m);
    } else {
        return false;   // a cost method without a proof keeps the IEEE fallback
    }
    return f0 - 61 * k - 46 >= -110;
}

bool nonneg(float x) { return x >= 0 && !std::signbit(x); }   // >= +0 (rejects NaN and -0.0)

sm_status validate(const sm_params& p, std::string& why) {
    auto bad = [&](const char* m) { why = m; return SM_EINVAL; };
    if (p.rows < 2 || p.cols < 2) return bad("rows and cols must be >= 2 (calGrad reads I[1] and I[w-2])");
    if ((long long)p.rows * p.cols > (1LL << 30)) return bad("rows*cols too large");
    if (p.rows > 65535) return bad("rows must be <= 65535");
    if (p.num_disparities < 1 || p.num_disparities > 1024) return bad("num_disparities must be in [1, 1024]");
    if (p.cost_method < 0 || p.cost_method > 3) return bad("unknown cost_method");
    if (p.aggregation < 0 || p.aggregation > 3) return bad("unknown aggregation");
    if (p.aggregation == SM_AGG_GF) {
        if (p.gf_mode != SM_GF_XIMGPROC && p.gf_mode != SM_GF_MY_GUIDE)
            return bad("gf_mode must be 0 (ximgproc::guidedFilter) or 1 (MY_GUIDE)");
        // MY_GUIDE: BoxFilter's windows need 2 r + 1 = 19 rows and columns (cpp:5156 asserts only
        // >= r, and reads outside the image below 2 r + 1); ximgproc: the reflected border of a
        // radius-9 box needs >= 9 (one reflection)
        if (p.gf_mode == SM_GF_MY_GUIDE && (p.rows < 19 || p.cols < 19))
            return bad("aggregation GF (MY_GUIDE) needs rows, cols >= 19 (box radius 9)");
        if (p.gf_mode == SM_GF_XIMGPROC && (p.rows < 9 || p.cols < 9))
            return bad("aggregation GF (ximgproc) needs rows, cols >= 9 (box radius 9, reflected border)");
        // the "so" optimiser's minima assume costs >= 0
        if (p.optimization == SM_OPT_SO) return bad("aggregation GF (costs may be negative) supports optimization sgm or WTA");
        if (!(p.gf_eps > 0)) return bad("gf_eps must be > 0");
    }
    if (p.aggregation == SM_AGG_NL) {
        if (!(p.nl_sigma > 0)) return bad("nl_sigma must be > 0");
        // ctmf's 3x3 median asserts width >= 3 and height >= 3 (NL/ctmf.c:211-212)
        if (p.rows < 3 || p.cols < 3) return bad("aggregation NL needs rows, cols >= 3 (ctmf median)");
        // the GPU tree walk indexes the batch's tour arcs (4 per pixel) with 32-bit ints
        if (4.0 * (double)p.rows * (double)p.cols * (double)(p.batch_capacity > 0 ? p.batch_capacity : 1) >= 2147483647.0)
            return bad("aggregation NL: rows * cols * batch_capacity must stay below 2^29");
    }
    if (p.optimization < 0 || p.optimization > 2) return bad("unknown optimization");
    if (p.census_rv < 0 || p.census_ru < 0 || census_len(p) > 128) return bad("census code longer than 128 bits");
    if (p.arm_l_out < 0 || p.arm_l_out > 84 || p.arm_min_l < 0 || p.arm_min_l > 84 || p.arm_l < 0)
        return bad("arm lengths must be in [0, 84]");
    if (p.cbca_iterations < 0 || p.cbca_iterations > 64) return bad("cbca_iterations must be in [0, 64]");
    if (p.sgm_paths < 1 || p.sgm_paths > 8) return bad("sgm_paths must be in [1, 8]");
    if (p.sgm_redu_coeff == 0) return bad("sgm_redu_coeff must be non-zero");
    if (p.batch_capacity < 1) return bad("batch_capacity must be >= 1");
    if (p.sub_batch < 0 || p.num_streams < 0 || p.num_streams > 4) return bad("sub_batch >= 0 and num_streams in [0, 4] required");
    if (p.fuse_norm_scan < -1 || p.fuse_norm_scan > 1) return bad("fuse_norm_scan must be -1 (auto), 0 or 1");
    if (p.placement_trials < -1 || p.placement_trials > 8) return bad("placement_trials must be in [-1, 8]");
    // The kernels rely on every cost and path cost being >= +0 (SGM and WTA minima compare float
    // bit patterns as unsigned integers, sm_device.h), which these constants guarantee: fusion
    // terms 2 - exp(-C / lam) - exp(-G / lam) with C, G >= 0, truncations >= 0, P1, P2 >= 0.
    if (!(p.lam_cen > 0) || !(p.lam_g > 0) || !(p.lam_ad > 0) || !(p.lam_cen_adc > 0))
        return bad("fusion lambdas must be > 0");
    // -0.0 passes `>= 0` but its bit pattern 0x80000000 ranks above every positive cost in those
    // unsigned minima (the reference's std::min would treat it as 0), so it is rejected as well
    if (!nonneg(p.grad_trunc) || !nonneg(p.ad_trunc_adc) || !nonneg(p.ad_trunc_ad)) return bad("truncations must be >= +0");
    if (!nonneg(p.sgm_p1) || !nonneg(p.sgm_p2) || p.sgm_redu_coeff < 0) return bad("SGM penalties must be >= +0");
    if (p.do_refine) {
        if (!(p.rv_ratio > 0)) return bad("rv_ratio must be > 0");
        if (p.disp_occ == -32768) return bad("disp_occ = -32768 is reserved (properIpol's outside-the-image mark)");
        if (p.region_vote_nums < 0 || p.region_vote_nums > 64) return bad("region_vote_nums must be in [0, 64]");
    }
    return SM_OK;
}

void build_luts(sm_ctx* c) {
    const sm_params& p = c->p;
    for (int i = 0; i < 1024; i++) {
        c->lut_a[i] = 0;
        c->lut_b[i] = 0;
    }
    if (p.cost_method == SM_COST_CENSUS_GRAD) {
        for (int i = 0; i < 1024; i++) c->lut_a[i] = expf(-(float)i / p.lam_cen);    // cpp:3585, ARU0 = lamCen
    } else if (p.cost_method == SM_COST_AD_CENSUS) {
        for (int i = 0; i < 1024; i++) c->lut_a[i] = expf(-(float)i / p.lam_cen_adc); // census term, ARU1 = 30
        for (int s = 0; s < 1024; s++) {
            float ad = (float)s / 3;  // sum / channels (cpp:2504)
            if (p.ad_trunc_adc < ad) ad = p.ad_trunc_adc;
            c->lut_b[s] = expf(-ad / p.lam_ad);                                        // AD term, ARU0 = 10
        }
        c->ad_oor_exp = expf(-p.ad_trunc_adc / p.lam_ad);
    }
}

// sm_params.num_streams / sub_batch -> the schedule sm_run follows (sm_create, sm_set_schedule).
// num_streams 0 (auto): two streams with CBCA at volumes >= 256 MiB per pair, where the next
// group's prep, cost and H scan share the CUs with this group's LDS-bound NORM_SCAN sweep
// (full resolution 37.8 -> 36.0 ms, 1080p x8 53.0 -> 50.3 ms, profiles/r4j; since the groups are
// pipelined across calls, round 5: KITTI x4 8.22 -> 7.58 ms, profiles/r5_final_wl; with the
// two-wave V sweep full resolution is as fast on one stream, 36.04 vs 35.99 ms, and KITTI still
// gains, 8.09 -> 7.58 ms, so the rule stays); and for batches of >= 8 smaller pairs with 4-path
// SGM and no refinement (Teddy x16 in two groups of 8: 2.48 -> 2.37 ms, profiles/r5_final3).
// Side streams are created on first use and kept.
sm_status apply_schedule(sm_ctx* c, int num_streams, int sub_batch) {
    const sm_params& p = c->p;
    if (sub_batch < 0 || num_streams < 0 || num_streams > 4)
        return fail(c, SM_EINVAL, "sub_batch >= 0 and num_streams in [0, 4] required");
    c->sub_batch = sub_batch;
    c->auto_groups = num_streams == 0 && p.aggregation == SM_AGG_CBCA && p.cbca_iterations > 0 &&
                     (c->nvol * 4 >= ((size_t)1 << 28) ||
                      (c->cap >= 8 && p.optimization == SM_OPT_SGM && p.sgm_paths == 4 && !p.do_refine));
    c->nstreams = c->auto_groups ? 2 : (num_streams < 1 ? 1 : num_streams);
    // the pipelined form of the two groups (sm_run): CBCA + SGM without refinement, where the
    // groups touch only their own pairs' buffers
    c->pipelined = c->auto_groups && p.optimization == SM_OPT_SGM && !p.do_refine;
    for (int i = 0; i + 1 < c->nstreams; i++)
        if (!c->xst[i]) HIP_TRY(c, hipStreamCreateWithFlags(&c->xst[i], hipStreamNonBlocking));
    return SM_OK;
}

template <typename T>
sm_status dalloc(sm_ctx* c, T** ptr, size_t count) {
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)ptr, count * sizeof(T));
    if (e != hipSuccess) {
        *ptr = nullptr;
        return fail(c, SM_ENOMEM, std::string("hipMalloc(") + std::to_string(count * sizeof(T)) + " B) failed: " + hipGetErrorString(e));
    }
    return SM_OK;
}

void free_all(sm_ctx* c) {
    void* ptrs[] = {c->bgr, c->gray, c->code, c->arms_alloc, c->vm0, c->vm1, c->acc, c->ck, c->lx, c->disp,
                    c->disp1, c->disp_tmp, c->dummy, c->flags, c->flags1, c->px, c->so_trace, c->so_cidx,
                    c->gf_s, c->gf_planes, c->gf_pix, c->gfc_rs, c->gfc_ab, c->gfc_img, c->gfc_pix, c->nl_med, c->nl_ew, c->nl_ints, c->nl_rec,
                    c->nl_table, c->nl_val, c->nl_oup, c->nl_ofin, c->nl_par, c->nl_best, c->nl_mst, c->nl_adj, c->nl_walk,
                    c->nl_offs, c->luts, c->nl_vc, c->nl_fl};
    for (void* q : ptrs)
        if (q) hipFree(q);
    if (c->nl_st) {
        hipStreamSynchronize(c->nl_st);
        hipStreamDestroy(c->nl_st);
        c->nl_st = nullptr;
    }
    for (hipEvent_t* ev : {c->nl_ev_set, c->nl_ev_opt})
        for (int i = 0; i < 2; i++)
            if (ev[i]) {
                hipEventSynchronize(ev[i]);
                hipEventDestroy(ev[i]);
                ev[i] = nullptr;
            }
    if (c->nl_offs_h) {
        hipHostFree(c->nl_offs_h);
        c->nl_offs_h = nullptr;
    }
    for (auto& r : c->recs) {
        if (r.start) hipEventDestroy(r.start);
        if (r.stop) hipEventDestroy(r.stop);
    }
    for (auto e : c->free_events) hipEventDestroy(e);
    for (auto e : c->xev) hipEventDestroy(e);
    c->xev.clear();
    if (c->cst) {
        hipStreamSynchronize(c->cst);
        hipStreamDestroy(c->cst);
        c->cst = nullptr;
    }
    for (hipEvent_t* ev : {&c->ev_dl[0], &c->ev_dl[1], &c->ev_up[0], &c->ev_up[1], &c->ev_in[0], &c->ev_in[1]})
        if (*ev) {
            hipEventDestroy(*ev);
            *ev = nullptr;
        }
    if (c->ev_run) hipEventDestroy(c->ev_run);
    if (c->ev_copy) hipEventDestroy(c->ev_copy);
    if (c->ev_copy2) hipEventDestroy(c->ev_copy2);
    c->ev_run = c->ev_copy = c->ev_copy2 = nullptr;
    for (auto& x : c->xst)
        if (x) {
            hipStreamDestroy(x);
            x = nullptr;
        }
    c->recs.clear();
    c->free_events.clear();
    if (c->st) hipStreamDestroy(c->st);
}

// ---- stage drivers (all asynchronous on c->st) -------------------------------------------

// Device pointers of pair `off` onward (the kernels index pairs from their base pointers).
struct Bufs {
    uint8_t* bgr;
    uint8_t* gray;
    ulonglong2* code;
    uint8_t* arms;
    float* vm0;
    float* vm1;
    float* acc;
    float* ck;
    float* lx;
    int16_t* disp;
    int16_t* disp1;
    int16_t* disp_tmp;
    uint8_t* flags;
    uint8_t* flags1;
    uint32_t* px;
    uint32_t* pxh;
    uint32_t* pxv;
};

Bufs at(const sm_ctx* c, int off) {
    const size_t o = (size_t)off, np = c->npix, nv = c->nvol;
    Bufs b;
    b.bgr = c->bgr + o * 2 * np * 3;
    b.gray = c->gray + o * 2 * np;
    b.code = c->code + o * 2 * np;
    b.arms = c->arms + o * 2 * 2 * np * 4;
    b.vm0 = c->vm0 + o * nv;
    b.vm1 = c->vm1 ? c->vm1 + o * nv : nullptr;
    b.acc = c->acc ? c->acc + o * nv : nullptr;
    b.ck = c->ck ? c->ck + o * c->ck_pair : nullptr;
    b.lx = c->lx ? c->lx + o * nv : nullptr;
    b.disp = c->disp + o * np;
    b.disp1 = c->disp1 ? c->disp1 + o * np : nullptr;
    b.disp_tmp = c->disp_tmp ? c->disp_tmp + o * np : nullptr;
    b.flags = c->flags + o * np;
    b.flags1 = c->flags1 ? c->flags1 + o * np : nullptr;
    b.px = c->px + o * 2 * np;
    b.pxh = c->px + (c->cap + o) * 2 * np;
    b.pxv = c->px + (2 * c->cap + o) * 2 * np;
    return b;
}

sm_status run_prep(sm_ctx* c, int n, const Bufs& B) {
    const sm_params& p = c->p;
    const int H = p.rows, W = p.cols;
    const bool census = needs_census(p), arms = needs_arms(p);
    const bool flags = p.optimization == SM_OPT_SGM;
    {
        sm::PrepArgs a{};
        a.gray = B.gray;
        a.bgr = B.bgr;
        a.px = B.px;
        a.pxh = B.pxh;
        a.pxv = B.pxv;
        a.code = B.code;
        a.arms = B.arms;
        a.flags = B.flags;
        a.flags1 = flags && p.do_refine ? B.flags1 : nullptr;
        a.H = H;
        a.W = W;
        a.rv = p.census_rv;
        a.ru = p.census_ru;
        a.ring = p.census_ring;
        a.L = p.arm_l;
        a.L_out = p.arm_l_out;
        a.C_D = p.arm_c_thresh;
        a.C_D_out = p.arm_c_thresh_out;
        a.minL = p.arm_min_l;
        a.cor_thres = p.sgm_cor_dif_thres;
        a.do_census = census;
        a.do_arms = arms;
        a.do_flags = flags;
        // the packed BGR plane's later readers: the GF image planes, so, refine's properIpol
        a.pack_px = p.aggregation == SM_AGG_GF || p.optimization == SM_OPT_SO || p.do_refine;
        return timed(c, "prep", (double)n * 2 * c->npix * (1 + 3 + (census ? 16 : 0) + (arms ? 8 : 0)) +
                                    (flags ? (double)n * c->npix * n_views(p) : 0),
                     [&] { sm::launch_prep(a, n, c->st); });
    }
}

sm_status run_cost(sm_ctx* c, int n, int view, const Bufs& B) {
    const sm_params& p = c->p;
    sm::CostArgs a{};
    a.vm = view == 0 ? B.vm0 : B.vm1;
    a.code = B.code;
    a.gray = B.gray;
    a.arms = B.arms;
    a.bgr = B.bgr;
    a.H = p.rows;
    a.W = p.cols;
    a.D = p.num_disparities;
    a.view = view;
    a.nwords = (census_len(p) + 63) / 64;
    a.cwords = (census_len(p) + 31) / 32;
    a.census_default = (float)census_len(p) * 1.0f;
    a.grad_trunc = p.grad_trunc;
    a.grad_oor = (float)sqrt(pow((double)p.grad_trunc, 2) * 2);
    a.grad_adaptive = p.grad_adaptive;
    a.lam2 = p.lam_g;
    a.ad_trunc = p.ad_trunc_ad;
    a.ad_oor_exp = c->ad_oor_exp;
    a.lut = c->luts;
    const int m = p.cost_method == SM_COST_CENSUS_GRAD ? sm::SM_M_CENSUS_GRAD
                  : p.cost_method == SM_COST_CENSUS    ? sm::SM_M_CENSUS
                  : p.cost_method == SM_COST_AD_CENSUS ? sm::SM_M_AD_CENSUS
                                                       : sm::SM_M_AD;
    return timed(c, view == 0 ? "cost_volume" : "cost_volume_right", (double)n * c->nvol * 4.0,
                 [&] { sm::launch_cost(a, m, n, c->st); });
}

sm_status run_cbca(sm_ctx* c, int n, int view, bool fuse_scale, float w, const Bufs& B) {
    // cbca_core (cpp:5585-5666): iteration k runs H then V for even k, V then H for odd k.
    // The last pass of iteration k and the first pass of iteration k+1 share a direction and
    // are fused into one CB_NORM_SCAN sweep, so N iterations take N + 1 sweeps.
    const sm_params& p = c->p;
    const int N = p.cbca_iterations;
    if (N <= 0) return SM_OK;
    sm::CbcaArgs a{};
    a.vm = view == 0 ? B.vm0 : B.vm1;
    a.view = view;
    a.dummy = c->dummy;
    a.arms = (const uint32_t*)B.arms;
    a.H = p.rows;
    a.W = p.cols;
    a.D = p.num_disparities;
    a.lag = cbca_lag(p);
    a.vm_end = (view == 0 ? c->vm0 : c->vm1) + (size_t)c->cap * c->nvol + c->vtail;   // incl. the tail pad
    a.arms_end = (const uint32_t*)(c->arms + c->arms_bytes);
    a.scale = w;
    a.apply_scale = 0;
    a.num_cu = c->num_cu;
    a.arm_pad_rows = 2 * cbca_lag(p);
    const double bytes = (double)n * c->nvol * 8.0;
    // profile names: "cbca_h_scan" etc. for vm[0], "cbca_h_scan_r" etc. for vm[1]
    std::string sfx = view == 0 ? "" : "_r";
    auto nm = [&](const char* base) { static thread_local std::string t; t = std::string(base) + sfx; return t.c_str(); };
    sm_status s = timed(c, nm("cbca_h_scan"), bytes, [&] { sm::launch_cbca(a, true, sm::CB_SCAN, n, c->st); });
    if (s) return s;
    if (c->stagger_ev) {   // the next group may start: this group's next sweep is LDS- and issue-bound
        HIP_TRY(c, hipEventRecord(c->stagger_ev, c->st));
        c->stagger_ev = nullptr;
    }
    for (int k = 0; k < N; k++) {
        const bool dir_h = (k % 2 == 1);  // direction of iteration k's second pass
        a.div_safe = cbca_div_safe(p, k) ? 1 : 0;   // this step's normalisation is iteration k's
        if (k + 1 < N && c->fuse_norm_scan) {
            s = timed(c, nm(dir_h ? "cbca_h_norm_scan" : "cbca_v_norm_scan"), bytes,
                      [&] { sm::launch_cbca(a, dir_h, sm::CB_NORM_SCAN, n, c->st); });
        } else if (k + 1 < N) {
            s = timed(c, nm(dir_h ? "cbca_h_norm" : "cbca_v_norm"), bytes,
                      [&] { sm::launch_cbca(a, dir_h, sm::CB_NORM, n, c->st); });
            if (s) return s;
            s = timed(c, nm(dir_h ? "cbca_h_scan" : "cbca_v_scan"), bytes,
                      [&] { sm::launch_cbca(a, dir_h, sm::CB_SCAN, n, c->st); });
        } else {
            a.apply_scale = fuse_scale ? 1 : 0;
            s = timed(c, nm(dir_h ? "cbca_h_norm" : "cbca_v_norm"), bytes,
                      [&] { sm::launch_cbca(a, dir_h, sm::CB_NORM, n, c->st); });
        }
        if (s) return s;
    }
    return SM_OK;
}

sm_status run_scale(sm_ctx* c, int n, int view, float w, const Bufs& B) {
    return timed(c, view == 0 ? "solve_all_scale" : "solve_all_scale_r", (double)n * c->nvol * 8.0,
                 [&] { sm::launch_scale(view == 0 ? B.vm0 : B.vm1, (size_t)n * c->nvol, w, c->st); });
}

// dispOptimize (cpp:1046-1136) for one view: vm[0] with the left image's penalty flags
// (leftFirst = true) -> DP[0]; vm[1] with the right image's (leftFirst = false) -> DP[1].
// guideFilter(0, vm) on one view (cpp:4492-4516): ximgproc form (the shipped build, sm_gf_cv.hip)
// or the MY_GUIDE form (sm_gf.hip), by sm_params.gf_mode
sm_status run_gf(sm_ctx* c, int n, int view, const Bufs& B, bool solve_all, float w) {
    const size_t off = (size_t)(B.vm0 - c->vm0) / c->nvol, cap = c->cap, nv = c->nvol;
    if (c->p.gf_mode == SM_GF_XIMGPROC) {
        sm::GfCvArgs a{};
        a.vm = view == 0 ? B.vm0 : B.vm1;
        a.rs = c->gfc_rs + off * nv;
        a.ab = c->gfc_ab + off * nv;
        a.cap = c->cap;
        a.px = B.px + (size_t)view * c->npix;        // packed words of the view's image (run_prep)
        a.px_pair_stride = 2 * c->npix;
        a.img_rs = c->gfc_img + off * 9 * c->npix;
        a.pix = c->gfc_pix + off * 9 * c->npix;
        a.H = c->p.rows;
        a.W = c->p.cols;
        a.D = c->p.num_disparities;
        a.eps = c->p.gf_eps;
        a.solve_all = solve_all;
        a.scale = w;
        // R0: read p, write 4 doubles; C0: read 4 doubles, write 4 floats; R1: read 4 floats, write 4
        // doubles; C1: read 4 doubles, write q (the leaving rows / positions re-read from cache)
        const double bytes = (double)n * nv * (4 + 32 + 32 + 16 + 16 + 32 + 32 + 4);
        return timed(c, view == 0 ? "gf" : "gf_r", bytes, [&] { sm::launch_gf_cv(a, n, c->st); });
    }
    sm::GfArgs a{};
    a.vm = view == 0 ? B.vm0 : B.vm1;
    float* s0 = c->acc ? c->acc : c->gf_s + 3 * cap * nv;
    a.s0 = s0 + off * nv;
    a.s1 = c->gf_s + (0 * cap + off) * nv;
    a.s2 = c->gf_s + (1 * cap + off) * nv;
    a.s3 = c->gf_s + (2 * cap + off) * nv;
    a.bgr = B.bgr + (size_t)view * c->npix * 3;   // I_c[view] (cpp:4502)
    a.bgr_pair_stride = 2 * c->npix * 3;
    a.px = B.px + (size_t)view * c->npix;        // packed words of the same image (run_prep)
    a.px_pair_stride = 2 * c->npix;
    a.planes = c->gf_planes + off * 10 * c->npix;
    a.pix = c->gf_pix + off * c->npix;
    a.H = c->p.rows;
    a.W = c->p.cols;
    a.D = c->p.num_disparities;
    a.eps = c->p.gf_eps;
    a.solve_all = solve_all;
    a.scale = w;
    // four volume sweeps, each reading and writing four channels (V0: reads one)
    const double bytes = (double)n * nv * (4 + 16 + 32 + 32 + 16 + 4);
    return timed(c, view == 0 ? "gf" : "gf_r", bytes, [&] { sm::launch_gf(a, n, c->st); });
}

// NL() on vm[0] (cpp:4892-4917): edge weights, spanning trees, the tree walk and the tree filter,
#ifndef SM_NL_PIPE
#define SM_NL_PIPE 1   // sm_run: NL's prep and cost volume on the front stream (A/B switch)
#endif
// all on the GPU (sm_nl.hip, sm_nl_mst.hip, sm_nl_walk.hip)
sm_status run_nl(sm_ctx* c, int n, const Bufs& B, bool solve_all, float w, Bufs* pipe = nullptr) {
    const size_t off = (size_t)(B.vm0 - c->vm0) / c->nvol, np = c->npix;
    const int H = c->p.rows, W = c->p.cols, D = c->p.num_disparities;
    const size_t ne = (size_t)H * (W - 1) + (size_t)(H - 1) * W;
    const size_t slot = (size_t)c->cap * np;
    // The front (median, edge weights, spanning trees, the tree walk) runs on its own stream: it
    // reads only the colour images, which change only through upload() (which synchronises), so
    // it need not wait for the work still queued on c->st -- with inputs resident across calls,
    // this call's trees are built while the GPU finishes the previous call's filter and
    // optimisation.  Records and path tables are double-buffered across calls; the walk waits
    // only for the filter that last read the set it writes.
    if (!c->nl_st) {
        HIP_TRY(c, hipStreamCreateWithFlags(&c->nl_st, hipStreamNonBlocking));
        for (hipEvent_t* ev : {c->nl_ev_set, c->nl_ev_opt})
            for (int i = 0; i < 2; i++) {
                HIP_TRY(c, hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
                HIP_TRY(c, hipEventRecord(ev[i], c->st));
            }
    }
    const int set = c->nl_set;
    c->nl_set ^= 1;
    int* I = c->nl_ints + (size_t)set * 4 * slot;
    int* rec_d = c->nl_rec + ((size_t)set * (slot + 2 * sm::NL_REC_PAD) + sm::NL_REC_PAD) * 4;
    constexpr int NOFF = 2 * (sm::NL_LEVELS + 1) + 1;
    sm_status s;
    {
        struct Swap {   // the front's launches (and their profiling events) go to nl_st
            sm_ctx* c;
            hipStream_t keep;
            ~Swap() { c->st = keep; }
        } sw{c, c->st};
        c->st = c->nl_st;
        if (pipe) {
            // this call's prep and cost volume, into the set's flags and cost volume: the set was
            // last read by the optimiser two calls back (its filter read the cost volume before)
            *pipe = B;
            pipe->vm0 = c->nl_vc + ((size_t)set * c->cap + off) * c->nvol;
            pipe->flags = c->nl_fl + ((size_t)set * c->cap + off) * np;
            HIP_TRY(c, hipStreamWaitEvent(c->st, c->nl_ev_opt[set], 0));
            if ((s = run_prep(c, n, *pipe))) return s;
            if ((s = run_cost(c, n, 0, *pipe))) return s;
        }
        s = timed(c, "nl_edges", (double)n * np * 4, [&] {
            sm::launch_nl_edges(B.bgr, 2 * np * 3, c->nl_med + off * np * 3, c->nl_ew + off * ne, H, W, n, c->st);
        });
        if (s) return s;
        // the spanning trees' neighbour lists (Boruvka on the GPU, sm_nl_mst.hip); bytes = the edge
        // weights read once
        s = timed(c, "nl_mst", (double)n * ne, [&] {
            sm::launch_nl_mst(c->nl_ew + off * ne, H, W, n, c->nl_par + off * np, c->nl_best + off * np,
                              c->nl_mst, c->nl_adj + off * np, c->st);
        });
        if (s) return s;
        HIP_TRY(c, hipStreamWaitEvent(c->st, c->nl_ev_set[set], 0));
        // the tree walk (sm_nl_walk.hip); bytes = the records and path tables written
        s = timed(c, "nl_walk", (double)n * np * 32, [&] {
            sm::launch_nl_walk(c->nl_adj + off * np, H, W, n, c->nl_walk, (int4*)rec_d, I, I + slot, I + 2 * slot,
                               I + 3 * slot, c->nl_offs, c->st);
        });
        if (s) return s;
        HIP_TRY(c, hipMemcpyAsync(c->nl_offs_h, c->nl_offs, NOFF * sizeof(int), hipMemcpyDeviceToHost, c->st));
    }
    HIP_TRY(c, hipStreamSynchronize(c->nl_st));   // the round offsets (the records are then in place)
    const int* up_off = c->nl_offs_h;
    const int* dn_off = c->nl_offs_h + sm::NL_LEVELS + 1;
    if (c->nl_offs_h[NOFF - 1] != 0)
        return fail(c, SM_EINVAL, "NL: spanning tree walk failed (flags " + std::to_string(c->nl_offs_h[NOFF - 1]) + ")");
    sm::NlArgs a{};
    a.chain_start = I;
    a.chain_len = I + slot;
    a.order_up = I + 2 * slot;
    a.order_down = I + 3 * slot;
    a.rec = (const int4*)rec_d;
    a.table = c->nl_table;
    a.val = c->nl_val;
    a.vm = B.vm0;
    a.vc = pipe ? pipe->vm0 : B.vm0;
    a.oup = c->nl_oup;
    a.ofin = c->nl_ofin;
    a.nodes = (long)n * (long)np;
    a.W = W;
    a.solve_all = solve_all;
    a.scale = w;
    // the cost volume and the ones: up rounds, then down rounds; per voxel: cost in, up sum out;
    // up sum in, final out, float out (+ the light children's sums, about one per node)
    const double bytes = (double)n * c->nvol * (4 + 8 + 8 + 8 + 8 + 4);
    s = timed(c, "nl_filter", bytes, [&] {
        for (int r = 0; r < sm::NL_LEVELS; r++) sm::launch_nl_round(a, true, up_off[r], up_off[r + 1], D, c->st);
        for (int r = 0; r < sm::NL_LEVELS; r++) sm::launch_nl_round(a, false, dn_off[r], dn_off[r + 1], D, c->st);
    });
    if (s) return s;
    HIP_TRY(c, hipEventRecord(c->nl_ev_set[set], c->st));
    if (pipe) {   // the optimiser reads the final volume (vm[0]) and this set's flags
        pipe->vm0 = B.vm0;
        c->nl_opt_set = set;
    }
    return SM_OK;
}

#ifndef SM_FUSE_SOLVE_ALL
#define SM_FUSE_SOLVE_ALL 1   // sm_run: SolveAll's scaling in the GF / NL output stores (tuning switch)
#endif

// aggregation other than CBCA: GF on every view (num = Do_refine ? 2 : 1, cpp:4499), NL on vm[0]
sm_status run_other_agg(sm_ctx* c, int n, const Bufs& B, bool solve_all = false, float w = 1.f) {
    sm_status s = SM_OK;
    if (c->p.aggregation == SM_AGG_GF)
        for (int v = 0; v < n_views(c->p) && !s; v++) s = run_gf(c, n, v, B, solve_all, w);
    if (c->p.aggregation == SM_AGG_NL) s = run_nl(c, n, B, solve_all, w);
    return s;
}

sm_status run_optimize(sm_ctx* c, int n, int view, const Bufs& B) {
    const sm_params& p = c->p;
    float* vm = view == 0 ? B.vm0 : B.vm1;
    int16_t* disp = view == 0 ? B.disp : B.disp1;
    const char* sfx = view == 0 ? "" : "_r";
    if (p.optimization == SM_OPT_SGM) {
        static const int RV[8] = {+1, -1, 0, 0, +1, +1, -1, -1};  // cpp:6207
        static const int RU[8] = {0, 0, +1, -1, -1, +1, +1, -1};  // cpp:6208
        static const char* NAMES[8] = {"sgm_path0", "sgm_path1", "sgm_path2", "sgm_path3",
                                       "sgm_path4", "sgm_path5", "sgm_path6", "sgm_path7"};
        sm::SgmArgs a{};
        a.flags = view == 0 ? B.flags : B.flags1;
        a.dummy = c->dummy;
        a.vm = vm;
        a.acc = B.acc;
        a.bgr = B.bgr;
        a.disp = disp;
        a.H = p.rows;
        a.W = p.cols;
        a.D = p.num_disparities;
        a.p1 = p.sgm_p1;
        a.p2 = p.sgm_p2;
        a.cor_thres = p.sgm_cor_dif_thres;
        a.redu = p.sgm_redu_coeff;
        a.keep_final = p.keep_final_volume;
        a.signed_costs = p.aggregation == SM_AGG_GF;   // the guided filter's output can be < 0
        int first = 0;   // first path left to the plain sweeps
        if (B.ck) {
            // checkpointed pairs (0, 1) and (2, 3): 4 + 8 + 4 + 8 B per element (+ 4 / S for
            // the checkpoints each way) instead of 8 + 12 + 12 + 8; with 8 paths the second
            // pair adds into the running sum (12 B) and paths 4 .. 7 follow as sweeps
            a.ck = B.ck;
            const double ckb = 4.0 / sm::sgm_ck_seg(p.num_disparities);
            const double nv = (double)n * c->nvol;
            const bool four = p.sgm_paths == 4;
            struct Pass { int path, mode; const char* name; double per; };
            const Pass passes[4] = {
                {0, sm::CK_A, "sgm_ck_a01", 4.0 + ckb},
                {0, sm::CK_B, "sgm_ck_b01", 8.0 + ckb},
                {2, sm::CK_A, "sgm_ck_a23", 4.0 + ckb},
                four ? Pass{2, sm::CK_B | sm::SGM_LAST, "sgm_last_wta", 8.0 + ckb + (p.keep_final_volume ? 4.0 : 0)}
                     : Pass{2, sm::CK_B | sm::CK_MID, "sgm_ck_b23", 12.0 + ckb}};
            for (const Pass& ps : passes) {
                a.rv = RV[ps.path];
                a.ru = RU[ps.path];
                a.dir = ps.path;
                a.dir2 = ps.path + 1;
                const double bytes = nv * ps.per + ((ps.mode & sm::SGM_LAST) ? (double)n * c->npix * 2 : 0);
                const std::string name = std::string(ps.name) + sfx;
                sm_status s = timed(c, name.c_str(), bytes, [&] { sm::launch_sgm_ck(a, ps.mode, n, c->st); });
                if (s) return s;
            }
            first = 4;
            if (B.lx) {
                // 8 paths: the diagonal pair (4, 6) with L5 between them (sm_sgm.hip): pass A of
                // path 4, path 5 as an SGM_FIRST sweep storing L5, pass B of path 6 reading acc and
                // L5 (acc = ((acc + L4) + L5) + L6); path 7 follows as the last sweep
                const double ckd = 4.0 / sm::sgm_ck_diag_seg();
                a.rv = RV[4];
                a.ru = RU[4];
                a.dir = 4;
                a.dir2 = 6;
                sm_status s = timed(c, (std::string("sgm_ck_a46") + sfx).c_str(), nv * (4.0 + ckd),
                                    [&] { sm::launch_sgm_ck(a, sm::CK_A, n, c->st); });
                if (s) return s;
                sm::SgmArgs a5 = a;
                a5.rv = RV[5];
                a5.ru = RU[5];
                a5.dir = 5;
                a5.acc = B.lx;   // SGM_FIRST stores 0 + L5 == L5 (path costs are never -0)
                s = timed(c, (std::string("sgm_l5") + sfx).c_str(), nv * 8.0,
                          [&] { sm::launch_sgm_path(a5, sm::SGM_FIRST, n, c->st); });
                if (s) return s;
                a.lx = B.lx;
                s = timed(c, (std::string("sgm_ck_b46") + sfx).c_str(), nv * (16.0 + ckd),
                          [&] { sm::launch_sgm_ck(a, sm::CK_B | sm::CK_MID | sm::CK_X, n, c->st); });
                if (s) return s;
                first = 7;
            }
        }
        for (int i = first; i < p.sgm_paths; i++) {
            a.rv = RV[i];
            a.ru = RU[i];
            a.dir = i;
            int mode = (i == 0 ? sm::SGM_FIRST : 0) | (i == p.sgm_paths - 1 ? sm::SGM_LAST : 0);
            // algorithmic bytes per element: read C (+ read acc) (+ write acc | write final)
            double per = 4.0 + ((mode & sm::SGM_FIRST) ? 0 : 4.0) + ((mode & sm::SGM_LAST) ? (p.keep_final_volume ? 4.0 : 0) : 4.0);
            double bytes = (double)n * c->nvol * per + ((mode & sm::SGM_LAST) ? (double)n * c->npix * 2 : 0);
            const std::string name = std::string((mode & sm::SGM_LAST) ? "sgm_last_wta" : NAMES[i]) + sfx;
            sm_status s = timed(c, name.c_str(), bytes, [&] { sm::launch_sgm_path(a, mode, n, c->st); });
            if (s) return s;
        }
    } else if (p.optimization == SM_OPT_SO) {
        // so(vm[i], DP[i], I_c) reads I[0] — the left colours — for both views (cpp:1098, 6284)
        sm::SoArgs a{};
        a.vm = vm;
        a.trace = c->so_trace + (size_t)(B.disp - c->disp) * p.num_disparities;
        a.cidx = c->so_cidx + (B.disp - c->disp);
        a.px = B.px;
        a.disp = disp;
        a.H = p.rows;
        a.W = p.cols;
        a.D = p.num_disparities;
        a.n = n;
        a.keep_final = p.keep_final_volume;
        const std::string name = std::string("so") + sfx;
        sm_status s = timed(c, name.c_str(), (double)n * c->nvol * (4.0 + 1.0 + (p.keep_final_volume ? 4.0 : 0)),
                            [&] { sm::launch_so(a, c->st); });
        if (s) return s;
    } else {
        const std::string name = std::string("wta") + sfx;
        sm_status s = timed(c, name.c_str(), (double)n * c->nvol * 4.0 + (double)n * c->npix * 2,
                            [&] { sm::launch_wta(vm, disp, n, p.rows, p.cols, p.num_disparities, c->st); });
        if (s) return s;
    }
    return SM_OK;
}

// refine(), non-USE_RECONCV branch (cpp:1347-1510), on DP[0] of n pairs: LR check (in place),
// region votes and proper interpolations (Jacobi, ping-pong with disp_tmp), 3x3 median.
sm_status run_refine(sm_ctx* c, int n, const Bufs& B) {
    const sm_params& p = c->p;
    const int H = p.rows, W = p.cols;
    const double map = (double)n * c->npix * 2;
    sm_status s = timed(c, "refine_lr_check", 3 * map,
                        [&] { sm::launch_lr_check(B.disp, B.disp1, n, H, W, p.lr_max_diff, c->st); });
    if (s) return s;
    int16_t* cur = B.disp;
    int16_t* nxt = B.disp_tmp;
    const uint32_t* arms = (const uint32_t*)B.arms;
    if (p.do_region_vote)
        for (int i = 0; i < p.region_vote_nums; i++) {
            if ((s = timed(c, "refine_region_vote", 2 * map,
                           [&] { sm::launch_region_vote(cur, nxt, arms, n, H, W, p.rv_s, p.rv_ratio, c->st); })))
                return s;
            std::swap(cur, nxt);
        }
    if (p.do_proper_ipol)
        for (int i = 0; i < p.region_vote_nums; i++) {
            if ((s = timed(c, "refine_proper_ipol", 2 * map,
                           [&] { sm::launch_proper_ipol(cur, nxt, B.px, n, H, W, p.disp_occ, c->st); })))
                return s;
            std::swap(cur, nxt);
        }
    if (p.do_last_median_blur) {
        if ((s = timed(c, "refine_median3", 2 * map, [&] { sm::launch_median3(cur, nxt, n, H, W, c->st); }))) return s;
        std::swap(cur, nxt);
    }
    if (cur != B.disp) HIP_TRY(c, hipMemcpyAsync(B.disp, cur, (size_t)map, hipMemcpyDeviceToDevice, c->st));
    return SM_OK;
}

sm_status upload(sm_ctx* c, int n, const uint8_t* lbgr, const uint8_t* rbgr, size_t cstride, const uint8_t* lgray,
                 const uint8_t* rgray, size_t gstride) {
    const sm_params& p = c->p;
    const size_t H = p.rows, W = p.cols;
    // dst rows: pair-major, view-interleaved; src: n stacked images of H rows each
    const size_t crow = W * 3;
    for (int view = 0; view < 2; view++) {
        const uint8_t* src = view == 0 ? lbgr : rbgr;
        const uint8_t* gsrc = view == 0 ? lgray : rgray;
        for (int b = 0; b < n; b++) {
            uint8_t* dst = c->bgr + ((size_t)b * 2 + view) * c->npix * 3;
            HIP_TRY(c, hipMemcpy2DAsync(dst, crow, src + (size_t)b * H * cstride, cstride, crow, H, hipMemcpyDefault, c->st));
            uint8_t* gdst = c->gray + ((size_t)b * 2 + view) * c->npix;
            HIP_TRY(c, hipMemcpy2DAsync(gdst, W, gsrc + (size_t)b * H * gstride, gstride, W, H, hipMemcpyDefault, c->st));
        }
    }
    HIP_TRY(c, hipStreamSynchronize(c->st));
    c->n_loaded = n;
    c->stage = 1;
    return SM_OK;
}

// the maps are about to be written: an asynchronous copy of the previous maps must be done
sm_status wait_copy(sm_ctx* c) {
    if (c->copy_pending) HIP_TRY(c, hipStreamWaitEvent(c->st, c->ev_copy, 0));
    if (c->copy_pending && c->copy_split) HIP_TRY(c, hipStreamWaitEvent(c->st, c->ev_copy2, 0));
    return SM_OK;
}

sm_status check_nojoin(sm_ctx* c) {
    if (!c) return SM_EINVAL;
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return hip_fail(c, e, "hipSetDevice");
    return SM_OK;
}

// A pipelined sm_run leaves its second group running on the side stream; every other entry point
// first orders the main stream after it (one event), so that it sees (and may overwrite) the state
// of the whole call.
sm_status join_all(sm_ctx* c) {
    if (!c->pipe_live) return SM_OK;
    c->pipe_live = false;
    hipError_t e = hipEventRecord(c->xev[9], c->xst[0]);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->st, c->xev[9], 0);
    if (e != hipSuccess) {
        hipStreamSynchronize(c->xst[0]);   // a failed join: drain on the host
        return hip_fail(c, e, "stream join");
    }
    return SM_OK;
}

sm_status check(sm_ctx* c) {
    sm_status s = check_nojoin(c);
    if (s) return s;
    return join_all(c);
}

}  // namespace

extern "C" {

void sm_params_default(sm_params* p, int32_t max_disp, int32_t rows, int32_t cols) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->struct_size = (uint32_t)sizeof(sm_params);
    p->rows = rows;
    p->cols = cols;
    p->num_disparities = max_disp + 1;  // h:209
    p->cost_method = SM_COST_CENSUS_GRAD;
    p->aggregation = SM_AGG_CBCA;
    p->optimization = SM_OPT_SGM;
    p->census_rv = 3;   // cpp:815
    p->census_ru = 4;
    p->census_ring = 1; // censusFunc = 3 (h:244)
    p->lam_cen = 13.0f;
    p->lam_g = 1.0f;
    p->grad_trunc = 500.0f;
    p->grad_adaptive = 1;
    p->lam_ad = 10.0f;
    p->lam_cen_adc = 30.0f;
    p->ad_trunc_adc = 1000.0f;
    p->ad_trunc_ad = 20.0f;
    p->arm_l = 17;
    p->arm_l_out = 34;
    p->arm_c_thresh = 20;
    p->arm_c_thresh_out = 6;
    p->arm_min_l = 1;
    p->cbca_iterations = 2;
    p->sgm_paths = 4;
    p->sgm_p1 = 1.0f;
    p->sgm_p2 = 3.0f;
    p->sgm_cor_dif_thres = 15;
    p->sgm_redu_coeff = 4;
    p->compute_right_view = 0;
    p->keep_final_volume = 0;
    p->batch_capacity = 1;
    p->do_refine = 0;           // h:70
    p->lr_max_diff = 0.0f;      // h:212
    p->do_region_vote = 1;      // h:75
    p->region_vote_nums = 2;    // h:306
    p->rv_ratio = 0.4f;         // cpp:1400
    p->rv_s = 20;               // cpp:1401
    p->do_proper_ipol = 1;      // h:76
    p->disp_occ = -2 * 16;      // h:216
    p->do_last_median_blur = 1; // h:80
    p->sub_batch = 0;
    p->num_streams = 0;        // auto (see sm_capi.h)
    p->fuse_norm_scan = -1;   // auto: fused where the lag-34 sweep applies or for volumes >= 256 MiB per pair
    p->gf_eps = 0.0001f;        // gf_eps[0] = 1e-4 (h:298; guidedFilter / guideFilterCore_matlab, cpp:4509-4513)
    p->gf_mode = SM_GF_XIMGPROC;  // `//#define MY_GUIDE` (h:38): the shipped build calls ximgproc::guidedFilter
    p->nl_sigma = 0.1;          // NLCCA::aggreCV (NL/NLCCA.cpp:33)
    p->lr_consis = 1;           // Do_LRConsis (h:72)
    p->placement_trials = -1;   // auto (see sm_capi.h)
}

const char* sm_status_string(sm_status s) {
    // (a C caller may pass any int: read the bits, never an out-of-range enum value)
    int32_t v;
    static_assert(sizeof(v) == sizeof(s), "sm_status is an int");
    memcpy(&v, &s, sizeof v);
    switch (v) {
        case SM_OK: return "ok";
        case SM_EINVAL: return "invalid argument";
        case SM_ENOMEM: return "out of memory";
        case SM_EHIP: return "HIP runtime error";
        case SM_ESTATE: return "call out of order";
    }
    return "unknown status";
}

sm_status sm_create(sm_ctx** out, const sm_params* p, int32_t hip_device) {
    if (!out || !p) return SM_EINVAL;
    *out = nullptr;
    sm_ctx* c = new (std::nothrow) sm_ctx();
    if (!c) return SM_ENOMEM;
    *out = c;  // returned even on failure so sm_last_error works; caller must sm_destroy
    // a struct from another version of sm_capi.h (or not filled by sm_params_default) is refused
    // before any field past struct_size is read
    if (p->struct_size != (uint32_t)sizeof(sm_params))
        return fail(c, SM_EINVAL, "sm_params.struct_size != sizeof(sm_params): initialise the struct with sm_params_default "
                                  "from this library's sm_capi.h");
    c->p = *p;
    c->device = hip_device;
    if (hipDeviceGetAttribute(&c->num_cu, hipDeviceAttributeMultiprocessorCount, hip_device) != hipSuccess || c->num_cu < 1)
        c->num_cu = 256;
    std::string why;
    if (validate(c->p, why) != SM_OK) return fail(c, SM_EINVAL, why);
    int ndev = 0;
    HIP_TRY(c, hipGetDeviceCount(&ndev));
    if (hip_device < 0 || hip_device >= ndev) return fail(c, SM_EINVAL, "hip_device out of range");
    HIP_TRY(c, hipSetDevice(hip_device));
    HIP_TRY(c, hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    c->cap = p->batch_capacity;
    c->npix = (size_t)p->rows * p->cols;
    c->nvol = c->npix * (size_t)p->num_disparities;
    const size_t cap = c->cap;
    sm_status s;
    if ((s = dalloc(c, &c->bgr, cap * 2 * c->npix * 3 + 16))) return s;   // tail pad: prep's dword quads (load_quad_bgr)
    if ((s = dalloc(c, &c->gray, cap * 2 * c->npix))) return s;
    if ((s = dalloc(c, &c->code, cap * 2 * c->npix))) return s;
    {
        // front pad: V sweeps read rows i - lag >= -2 lag; tail pad: the fast V sweep's arm loads
        // run up to lag + T rows past the last plane's end (sm_cbca.hip NsV clamps later tiles)
        const size_t pad = ((size_t)2 * cbca_lag(*p) * p->cols * 4 + 255) / 256 * 256;
        const size_t tail = (size_t)(2 * cbca_lag(*p) + 64) * p->cols * 4;
        c->arms_bytes = cap * 2 * 2 * c->npix * 4;
        if ((s = dalloc(c, &c->arms_alloc, pad + c->arms_bytes + tail))) return s;
        c->arms = c->arms_alloc + pad;
        // the pads hold zero arms (never written later): rows the sweeps read outside the planes
        // then give zero-length windows, so every window slot stays inside the rings
        HIP_TRY(c, hipMemset(c->arms_alloc, 0, pad));
        HIP_TRY(c, hipMemset(c->arms + c->arms_bytes, 0, tail));
    }
    // volumes carry a tail: vectorised SGM lanes past D read (never write) into it, and the fast V
    // sweep's tiles that straddle the last rows read up to CBCA_VM_TAIL_ROWS rows past them
    const size_t vpad = 1024 + (size_t)sm::CBCA_VM_TAIL_ROWS * p->cols * p->num_disparities;
    c->vtail = vpad;
    if ((s = dalloc(c, &c->vm0, cap * c->nvol + vpad))) return s;
    if (right_view(*p))
        if ((s = dalloc(c, &c->vm1, cap * c->nvol + vpad))) return s;
    if (p->optimization == SM_OPT_SGM && p->sgm_paths > 1)
        if ((s = dalloc(c, &c->acc, cap * c->nvol + vpad))) return s;
    if (p->optimization == SM_OPT_SGM && sm::sgm_ck_ok(p->num_disparities, p->sgm_paths)) {
        const size_t S = (size_t)sm::sgm_ck_seg(p->num_disparities), H = (size_t)p->rows, W = (size_t)p->cols;
        size_t lines_x_segs = std::max(H * ((W + S - 1) / S), W * ((H + S - 1) / S));
        const bool diag = sm::sgm_ck_diag_ok(p->num_disparities, p->sgm_paths);
        if (diag) {   // the diagonal pair: W + H - 1 lines, slots strided by the longest diagonal
            const size_t SD = (size_t)sm::sgm_ck_diag_seg();
            lines_x_segs = std::max(lines_x_segs, (W + H - 1) * ((std::min(H, W) + SD - 1) / SD));
        }
        c->ck_pair = lines_x_segs * (size_t)p->num_disparities;
        if ((s = dalloc(c, &c->ck, cap * c->ck_pair))) return s;
        if (diag && (s = dalloc(c, &c->lx, cap * c->nvol + vpad))) return s;
    }
    if ((s = dalloc(c, &c->disp, cap * c->npix))) return s;
    if ((s = dalloc(c, &c->dummy, 64))) return s;
    if ((s = dalloc(c, &c->flags, cap * c->npix))) return s;
    if (p->optimization == SM_OPT_SO) {
        if ((s = dalloc(c, &c->so_trace, cap * c->nvol))) return s;
        if ((s = dalloc(c, &c->so_cidx, cap * c->npix))) return s;
    }
    if (p->do_refine || p->optimization == SM_OPT_SO)
        if ((s = dalloc(c, &c->disp1, cap * c->npix))) return s;
    if (p->do_refine) {
        if ((s = dalloc(c, &c->flags1, cap * c->npix))) return s;
        if ((s = dalloc(c, &c->disp_tmp, cap * c->npix))) return s;
    }
    if ((s = dalloc(c, &c->px, 3 * cap * 2 * c->npix))) return s;
    if (p->aggregation == SM_AGG_GF && p->gf_mode == SM_GF_XIMGPROC) {
        if ((s = dalloc(c, &c->gfc_rs, 4 * cap * c->nvol))) return s;
        if ((s = dalloc(c, &c->gfc_ab, 4 * cap * c->nvol))) return s;
        if ((s = dalloc(c, &c->gfc_img, cap * 9 * c->npix))) return s;
        if ((s = dalloc(c, &c->gfc_pix, cap * 9 * c->npix))) return s;
    } else if (p->aggregation == SM_AGG_GF) {
        if ((s = dalloc(c, &c->gf_s, (c->acc ? 3 : 4) * cap * c->nvol))) return s;
        if ((s = dalloc(c, &c->gf_planes, cap * 10 * c->npix))) return s;
        if ((s = dalloc(c, &c->gf_pix, cap * c->npix))) return s;
    }
    if (p->aggregation == SM_AGG_NL) {
        const size_t ne = (size_t)p->rows * (p->cols - 1) + (size_t)(p->rows - 1) * p->cols;
        if ((s = dalloc(c, &c->nl_med, cap * c->npix * 3))) return s;
        if ((s = dalloc(c, &c->nl_ew, cap * ne))) return s;
        if ((s = dalloc(c, &c->nl_ints, 2 * cap * c->npix * 4))) return s;
        if ((s = dalloc(c, &c->nl_rec, 2 * (cap * c->npix + 2 * sm::NL_REC_PAD) * 4))) return s;
        HIP_TRY(c, hipMemset(c->nl_rec, 0, 2 * (cap * c->npix + 2 * sm::NL_REC_PAD) * 16));
        if ((s = dalloc(c, &c->nl_table, 256))) return s;
        if ((s = dalloc(c, &c->nl_val, cap * c->nvol))) return s;
        if ((s = dalloc(c, &c->nl_oup, cap * c->npix))) return s;
        if ((s = dalloc(c, &c->nl_ofin, cap * c->npix))) return s;
        if ((s = dalloc(c, &c->nl_walk, sm::nl_walk_scratch_bytes(p->rows, p->cols, cap)))) return s;
        if ((s = dalloc(c, &c->nl_offs, 2 * (sm::NL_LEVELS + 1) + 1))) return s;
        HIP_TRY(c, hipHostMalloc((void**)&c->nl_offs_h, (2 * (sm::NL_LEVELS + 1) + 1) * sizeof(int), hipHostMallocDefault));
        if ((s = dalloc(c, &c->nl_par, cap * c->npix))) return s;
        if ((s = dalloc(c, &c->nl_best, cap * c->npix))) return s;
        if ((s = dalloc(c, &c->nl_mst, sm::nl_mst_scratch_bytes(p->rows, p->cols, cap)))) return s;
        if ((s = dalloc(c, &c->nl_adj, cap * c->npix))) return s;
        // sm_run's pipelined front (one view, SGM): two sets of cost volume and penalty flags
        c->nl_pipe = SM_NL_PIPE && p->optimization == SM_OPT_SGM && !right_view(*p);
        if (c->nl_pipe) {
            if ((s = dalloc(c, &c->nl_vc, 2 * cap * c->nvol + vpad))) return s;
            if ((s = dalloc(c, &c->nl_fl, 2 * cap * c->npix))) return s;
        }
        double table[256];
        const double sg = p->nl_sigma < 0.01 ? 0.01 : p->nl_sigma;   // update_table (qx_tree_filter.cpp:23-24)
        for (int i = 0; i < 256; i++) table[i] = exp(-(double)i / (255 * sg));
        HIP_TRY(c, hipMemcpy(c->nl_table, table, 256 * sizeof(double), hipMemcpyHostToDevice));
    }
    {
        const bool plain = p->aggregation == SM_AGG_CBCA && p->cbca_iterations > 0 && p->optimization == SM_OPT_SGM;
        c->place_trials = p->placement_trials >= 0 ? p->placement_trials
                                                   : (plain && c->nvol * 4 >= ((size_t)1 << 28) ? 3 : 0);
        if (!(p->aggregation == SM_AGG_CBCA || p->aggregation == SM_AGG_NONE)) c->place_trials = 0;   // (GF / NL scratch not moved)
    }
    if (getenv("SM_TRACE_ALLOC"))   // diagnostics: where the large buffers landed
        fprintf(stderr, "[alloc] vm0 %p vm1 %p acc %p arms %p code %p px %p\n", (void*)c->vm0, (void*)c->vm1,
                (void*)c->acc, (void*)c->arms, (void*)c->code, (void*)c->px);
    build_luts(c);
    {
        // auto: the generic fused sweep wins where a pair's volume is large (full resolution:
        // v_norm + v_scan 12.2 -> 11.3 ms; 1080p 16.2 -> 16.0 ms) and loses at Teddy size (0.79 ->
        // 0.82 ms); the dedicated sweep at the reference's lag (NsV, D % 64 == 0) wins at every
        // size (Teddy x16: 0.765 -> 0.692 ms, profiles/r4b/ab_teddy.txt)
        const bool nsv = cbca_lag(*p) == 34 && p->num_disparities % 64 == 0;
        c->fuse_norm_scan = p->fuse_norm_scan == 1 || (p->fuse_norm_scan == -1 && (nsv || c->nvol * 4 >= ((size_t)1 << 28)));
        if ((s = apply_schedule(c, p->num_streams, p->sub_batch))) return s;
        for (int i = 0; i < 16; i++) {
            hipEvent_t e;
            HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->xev.push_back(e);
        }
    }
    if ((s = dalloc(c, &c->luts, 2048))) return s;
    HIP_TRY(c, hipMemcpyAsync(c->luts, c->lut_a, sizeof(c->lut_a), hipMemcpyHostToDevice, c->st));
    HIP_TRY(c, hipMemcpyAsync(c->luts + 1024, c->lut_b, sizeof(c->lut_b), hipMemcpyHostToDevice, c->st));
    HIP_TRY(c, hipStreamSynchronize(c->st));
    return SM_OK;
}

sm_status sm_destroy(sm_ctx* c) {
    if (!c) return SM_OK;
    hipSetDevice(c->device);
    if (c->pipe_live) join_all(c);
    if (c->st) hipStreamSynchronize(c->st);
    free_all(c);
    delete c;
    return SM_OK;
}

const char* sm_last_error(const sm_ctx* c) { return c ? c->err.c_str() : "null context"; }

sm_status sm_set_images(sm_ctx* c, const uint8_t* lbgr, const uint8_t* rbgr, size_t cstride, const uint8_t* lgray,
                        const uint8_t* rgray, size_t gstride) {
    sm_status s = check(c);
    if (s) return s;
    if (!lbgr || !rbgr || !lgray || !rgray) return fail(c, SM_EINVAL, "null image pointer");
    if (cstride < (size_t)c->p.cols * 3 || gstride < (size_t)c->p.cols) return fail(c, SM_EINVAL, "row stride too small");
    return upload(c, 1, lbgr, rbgr, cstride, lgray, rgray, gstride);
}

sm_status sm_cost_calculate(sm_ctx* c) {
    sm_status s = check(c);
    if (s) return s;
    if (c->stage < 1) return fail(c, SM_ESTATE, "sm_cost_calculate before sm_set_images");
    const int n = c->n_loaded;
    const Bufs B = at(c, 0);
    if ((s = run_prep(c, n, B))) return s;
    if ((s = run_cost(c, n, 0, B))) return s;
    if (right_view(c->p) && (s = run_cost(c, n, 1, B))) return s;
    if (c->p.aggregation == SM_AGG_CBCA)
        for (int v = 0; v < n_views(c->p); v++)
            if ((s = run_cbca(c, n, v, false, 1.0f, B))) return s;
    if ((s = run_other_agg(c, n, B))) return s;
    c->stage = 2;
    return SM_OK;
}

sm_status sm_solve_all(sm_ctx* c, int32_t py_lev, float reg_lambda) {
    sm_status s = check(c);
    if (s) return s;
    if (c->stage != 2) return fail(c, SM_ESTATE, "sm_solve_all must follow sm_cost_calculate");
    if (py_lev != 1) return fail(c, SM_EINVAL, "PY_LVL > 1 needs every level's context: use sm_solve_all_pyr");
    const float m = 1 + reg_lambda;
    const float w = (float)(1. / (double)m);  // Mat::inv of the 1x1 regMat (cpp:2164)
    for (int v = 0; v < n_views(c->p); v++)   // img_n = Do_refine ? 2 : 1 (cpp:2178)
        if ((s = run_scale(c, c->n_loaded, v, w, at(c, 0)))) return s;
    c->stage = 3;
    return SM_OK;
}

// invWgt = row 0 of regMat.inv() (cpp:2147-2168): OpenCV's invert for a CV_32F matrix of order
// n <= 3 evaluates the adjugate over the determinant in double and rounds each entry to float;
// for n > 3 Mat::inv (DECOMP_LU) runs LUImpl<float> on a copy with the identity as right-hand
// side (lu_inv_row0; OpenCV's scalar loops, each product and sum rounded, pivot failure below
// 10 * FLT_EPSILON).
static bool lu_inv_row0(int L, float (*M)[sm::kMaxPyr], float* w) {
    float B[sm::kMaxPyr][sm::kMaxPyr];
    for (int i = 0; i < L; i++)
        for (int j = 0; j < L; j++) B[i][j] = i == j ? 1.f : 0.f;
    for (int i = 0; i < L; i++) {
        int k = i;
        for (int j = i + 1; j < L; j++)
            if (std::fabs(M[j][i]) > std::fabs(M[k][i])) k = j;
        if (std::fabs(M[k][i]) < FLT_EPSILON * 10) return false;
        if (k != i) {
            for (int j = i; j < L; j++) std::swap(M[i][j], M[k][j]);
            for (int j = 0; j < L; j++) std::swap(B[i][j], B[k][j]);
        }
        const float d = -1 / M[i][i];
        for (int j = i + 1; j < L; j++) {
            const float alpha = M[j][i] * d;
            for (int q = i + 1; q < L; q++) M[j][q] += alpha * M[i][q];
            for (int q = 0; q < L; q++) B[j][q] += alpha * B[i][q];
        }
    }
    for (int i = L - 1; i >= 0; i--)
        for (int j = 0; j < L; j++) {
            float s = B[i][j];
            for (int q = i + 1; q < L; q++) s -= M[i][q] * B[q][j];
            B[i][j] = s / M[i][i];
        }
    for (int j = 0; j < L; j++) w[j] = B[0][j];
    return true;
}

static bool pyr_weights(int L, float lam, float* w) {
    float M[sm::kMaxPyr][sm::kMaxPyr] = {};
    for (int s = 0; s < L; s++) {
        if (s == 0) {
            M[s][s] = 1 + lam;
            if (L > 1) M[s][s + 1] = -lam;
        } else if (s == L - 1) {
            M[s][s] = 1 + lam;
            M[s][s - 1] = -lam;
        } else {
            M[s][s] = 1 + 2 * lam;
            M[s][s - 1] = -lam;
            M[s][s + 1] = -lam;
        }
    }
    if (L > 3) return lu_inv_row0(L, M, w);
    if (L == 1) {
        w[0] = (float)(1. / (double)M[0][0]);
        return true;
    }
    if (L == 2) {
        double d = (double)M[0][0] * M[1][1] - (double)M[0][1] * M[1][0];
        if (d == 0.) return false;
        d = 1. / d;
        w[0] = (float)(M[1][1] * d);
        w[1] = (float)(-M[0][1] * d);
        return true;
    }
    double d = M[0][0] * ((double)M[1][1] * M[2][2] - (double)M[1][2] * M[2][1]) -
               M[0][1] * ((double)M[1][0] * M[2][2] - (double)M[1][2] * M[2][0]) +
               M[0][2] * ((double)M[1][0] * M[2][1] - (double)M[1][1] * M[2][0]);
    if (d == 0.) return false;
    d = 1. / d;
    w[0] = (float)(((double)M[1][1] * M[2][2] - (double)M[1][2] * M[2][1]) * d);
    w[1] = (float)(((double)M[0][2] * M[2][1] - (double)M[0][1] * M[2][2]) * d);
    w[2] = (float)(((double)M[0][1] * M[1][2] - (double)M[0][2] * M[1][1]) * d);
    return true;
}

sm_status sm_solve_all_pyr(sm_ctx* const* levels, int32_t py_lvl, float reg_lambda) {
    if (!levels || !levels[0]) return SM_EINVAL;
    sm_ctx* c = levels[0];
    sm_status s = check(c);
    if (s) return s;
    if (py_lvl < 1 || py_lvl > sm::kMaxPyr) return fail(c, SM_EINVAL, "PY_LVL must be in [1, 8]");
    if (py_lvl == 1) return sm_solve_all(c, 1, reg_lambda);
    sm::PyrArgs a{};
    a.levels = py_lvl;
    a.n = c->n_loaded;
    for (int l = 0; l < py_lvl; l++) {
        sm_ctx* q = levels[l];
        if (!q) return fail(c, SM_EINVAL, "null level context");
        if (q->device != c->device) return fail(c, SM_EINVAL, "pyramid levels must share one device");
        if (q->stage != 2) return fail(c, SM_ESTATE, "every level needs sm_cost_calculate (and no SolveAll yet)");
        if (q->n_loaded != c->n_loaded) return fail(c, SM_EINVAL, "pyramid levels must hold the same number of pairs");
        if (n_views(q->p) < n_views(c->p)) return fail(c, SM_EINVAL, "coarser levels need do_refine like level 0");
        if (l > 0) {
            const sm_params& pp = levels[l - 1]->p;
            if (q->p.rows != (pp.rows + 1) / 2 || q->p.cols != (pp.cols + 1) / 2)
                return fail(c, SM_EINVAL, "level sizes must follow pyrDown: ((rows + 1) / 2, (cols + 1) / 2)");
            if (q->p.num_disparities < pp.num_disparities / 2 + 1)
                return fail(c, SM_EINVAL, "level num_disparities too small for curD = (curD + 1) / 2");
        }
        a.H[l] = q->p.rows;
        a.W[l] = q->p.cols;
        a.D[l] = q->p.num_disparities;
        if (l > 0) HIP_TRY(c, hipStreamSynchronize(q->st));   // coarse volumes complete
    }
    if (!pyr_weights(py_lvl, reg_lambda, a.w)) return fail(c, SM_EINVAL, "singular regularisation matrix");
    for (int v = 0; v < n_views(c->p); v++) {
        for (int l = 0; l < py_lvl; l++) a.vm[l] = v == 0 ? levels[l]->vm0 : levels[l]->vm1;
        const double bytes = (double)a.n * c->nvol * 8.0;
        if ((s = timed(c, v == 0 ? "solve_all_pyr" : "solve_all_pyr_r", bytes, [&] { sm::launch_solve_all_pyr(a, c->st); })))
            return s;
    }
    c->stage = 3;
    for (int l = 1; l < py_lvl; l++) levels[l]->stage = 3;
    return SM_OK;
}

sm_status sm_pyr_down(int32_t dev, const uint8_t* src, int32_t rows, int32_t cols, int32_t ch, uint8_t* dst) {
    if (!src || !dst || rows < 1 || cols < 1 || (ch != 1 && ch != 3)) return SM_EINVAL;
    if (hipSetDevice(dev) != hipSuccess) return SM_EHIP;
    const size_t in = (size_t)rows * cols * ch, out = (size_t)((rows + 1) / 2) * ((cols + 1) / 2) * ch;
    uint8_t *dsrc = nullptr, *ddst = nullptr;
    hipError_t e = hipMalloc((void**)&dsrc, in);
    if (e == hipSuccess) e = hipMalloc((void**)&ddst, out);
    if (e == hipSuccess) e = hipMemcpy(dsrc, src, in, hipMemcpyDefault);
    if (e == hipSuccess) {
        sm::launch_pyr_down(dsrc, ddst, rows, cols, ch, nullptr);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(dst, ddst, out, hipMemcpyDefault);
    if (dsrc) hipFree(dsrc);
    if (ddst) hipFree(ddst);
    return e == hipSuccess ? SM_OK : SM_EHIP;
}

sm_status sm_pyr_down_f32(int32_t dev, const float* src, int32_t rows, int32_t cols, float* dst) {
    if (!src || !dst || rows < 1 || cols < 1) return SM_EINVAL;
    if (hipSetDevice(dev) != hipSuccess) return SM_EHIP;
    const size_t in = (size_t)rows * cols * 4, out = (size_t)((rows + 1) / 2) * ((cols + 1) / 2) * 4;
    float *dsrc = nullptr, *ddst = nullptr;
    hipError_t e = hipMalloc((void**)&dsrc, in);
    if (e == hipSuccess) e = hipMalloc((void**)&ddst, out);
    if (e == hipSuccess) e = hipMemcpy(dsrc, src, in, hipMemcpyDefault);
    if (e == hipSuccess) {
        sm::launch_pyr_down_f32(dsrc, ddst, rows, cols, nullptr);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(dst, ddst, out, hipMemcpyDefault);
    if (dsrc) hipFree(dsrc);
    if (ddst) hipFree(ddst);
    return e == hipSuccess ? SM_OK : SM_EHIP;
}

sm_status sm_disp_optimize(sm_ctx* c, int16_t* disp_out) {
    sm_status s = check(c);
    if (s) return s;
    if (c->stage < 2 || c->stage > 3) return fail(c, SM_ESTATE, "sm_disp_optimize must follow sm_cost_calculate / sm_solve_all");
    if ((s = wait_copy(c))) return s;
    for (int v = 0; v < opt_views(c->p); v++)   // num (cpp:1054, 1093, 1110)
        if ((s = run_optimize(c, c->n_loaded, v, at(c, 0)))) return s;
    c->stage = 4;
    if (disp_out) return sm_download_disp(c, 1, disp_out);
    return SM_OK;
}

sm_status sm_refine(sm_ctx* c, int16_t* disp_out) {
    sm_status s = check(c);
    if (s) return s;
    if (!c->p.do_refine) return fail(c, SM_ESTATE, "sm_refine needs do_refine = 1 at sm_create (DP[1] is not computed otherwise)");
    if (c->stage != 4) return fail(c, SM_ESTATE, "sm_refine must follow sm_disp_optimize");
    if ((s = wait_copy(c))) return s;
    if ((s = run_refine(c, c->n_loaded, at(c, 0)))) return s;
    c->stage = 5;
    if (disp_out) return sm_download_disp(c, 1, disp_out);
    return SM_OK;
}

sm_status sm_get_disp(sm_ctx* c, int32_t view, int16_t* dst) {
    sm_status s = check(c);
    if (s) return s;
    if (!dst || view < 0 || view > 1) return fail(c, SM_EINVAL, "bad arguments");
    if (c->stage < 4) return fail(c, SM_ESTATE, "no disparity map yet");
    const int16_t* src = view == 0 ? c->disp : c->disp1;
    if (!src) return fail(c, SM_EINVAL, "DP[1] is only computed with do_refine = 1 or optimization so");
    HIP_TRY(c, hipMemcpyAsync(dst, src, c->npix * 2, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(c, hipStreamSynchronize(c->st));
    return SM_OK;
}

sm_status sm_set_disp(sm_ctx* c, int32_t view, const int16_t* src) {
    sm_status s = check(c);
    if (s) return s;
    if (!src || view < 0 || view > 1) return fail(c, SM_EINVAL, "bad arguments");
    if (c->stage < 4) return fail(c, SM_ESTATE, "sm_set_disp must follow sm_disp_optimize");
    if ((s = wait_copy(c))) return s;
    int16_t* dst = view == 0 ? c->disp : c->disp1;
    if (!dst) return fail(c, SM_EINVAL, "DP[1] is only allocated with do_refine = 1 or optimization so");
    HIP_TRY(c, hipMemcpyAsync(dst, src, c->npix * 2, hipMemcpyHostToDevice, c->st));
    HIP_TRY(c, hipStreamSynchronize(c->st));
    c->stage = 4;   // refine() may run (again) on the new maps
    return SM_OK;
}

sm_status sm_get_volume(sm_ctx* c, int32_t view, float* dst) {
    sm_status s = check(c);
    if (s) return s;
    if (!dst) return fail(c, SM_EINVAL, "null dst");
    if (c->stage < 2) return fail(c, SM_ESTATE, "no volume yet");
    float* src = view == 0 ? c->vm0 : (view == 1 ? c->vm1 : nullptr);
    if (!src) return fail(c, SM_EINVAL, view == 1 ? "right view not computed (compute_right_view = 0)" : "bad view");
    if (c->stage >= 4 && !c->p.keep_final_volume && c->p.optimization == SM_OPT_SGM)
        return fail(c, SM_ESTATE, "vm[view] after SGM is only kept with keep_final_volume = 1");
    HIP_TRY(c, hipMemcpyAsync(dst, src, c->nvol * 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(c, hipStreamSynchronize(c->st));
    return SM_OK;
}

sm_status sm_get_arms(sm_ctx* c, int32_t view, uint16_t* dst) {
    sm_status s = check(c);
    if (s) return s;
    if (!dst || view < 0 || view > 1) return fail(c, SM_EINVAL, "bad arguments");
    if (c->stage < 2 || !needs_arms(c->p)) return fail(c, SM_ESTATE, "arms not computed");
    std::vector<uint32_t> tmp(c->npix * 2);
    HIP_TRY(c, hipMemcpyAsync(tmp.data(), c->arms + (size_t)view * 2 * c->npix * 4, c->npix * 8, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(c, hipStreamSynchronize(c->st));
    for (size_t i = 0; i < c->npix; i++) {
        dst[i * 4 + 0] = tmp[i] & 0xffff;
        dst[i * 4 + 1] = tmp[i] >> 16;
        dst[i * 4 + 2] = tmp[c->npix + i] & 0xffff;
        dst[i * 4 + 3] = tmp[c->npix + i] >> 16;
    }
    return SM_OK;
}

sm_status sm_get_census(sm_ctx* c, int32_t view, uint64_t* dst) {
    sm_status s = check(c);
    if (s) return s;
    if (!dst || view < 0 || view > 1) return fail(c, SM_EINVAL, "bad arguments");
    if (c->stage < 2 || !needs_census(c->p)) return fail(c, SM_ESTATE, "census not computed");
    HIP_TRY(c, hipMemcpyAsync(dst, c->code + (size_t)view * c->npix, c->npix * 16, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(c, hipStreamSynchronize(c->st));
    return SM_OK;
}

sm_status sm_upload_batch(sm_ctx* c, int32_t n, const uint8_t* lbgr, const uint8_t* rbgr, const uint8_t* lgray,
                          const uint8_t* rgray) {
    sm_status s = check(c);
    if (s) return s;
    if (n < 1 || n > c->cap) return fail(c, SM_EINVAL, "n must be in [1, batch_capacity]");
    if (!lbgr || !rbgr || !lgray || !rgray) return fail(c, SM_EINVAL, "null image pointer");
    return upload(c, n, lbgr, rbgr, (size_t)c->p.cols * 3, lgray, rgray, (size_t)c->p.cols);
}

#ifndef SM_STAGGER_STAGE
#define SM_STAGGER_STAGE 1   // 0: CBCA groups also start after the previous group's whole CBCA (A/B)
#endif
#ifndef SM_UP_EARLY
#define SM_UP_EARLY 1   // async uploads into a pipelined context wait for the inputs' last reader, not the group's end
#endif
static sm_status place_volumes(sm_ctx* c, int k, int n, float reg_lambda);

sm_status sm_run(sm_ctx* c, int32_t n, float reg_lambda, int16_t* disp_out) {
    sm_status s = check_nojoin(c);   // (a pipelined run continues from the previous one's streams)
    if (s) return s;
    if (c->stage < 1) return fail(c, SM_ESTATE, "sm_run before images were uploaded");
    if (n < 1 || n > c->n_loaded) return fail(c, SM_EINVAL, "n must be in [1, pairs uploaded]");
    if (c->place_trials > 1) {   // the first run: choose the volume placement (place_volumes)
        const int k = c->place_trials;
        c->place_trials = 0;
        if ((s = join_all(c)) || (s = place_volumes(c, k, n, reg_lambda))) return s;
    }
    const float m = 1 + reg_lambda;
    const float w = (float)(1. / (double)m);
    // Sub-batches: all stages of a group of pairs run back to back so that one pass's output is
    // still in the 256 MB Infinity Cache when the next pass reads it.  With SM_STREAMS = s > 1 the
    // groups alternate over s streams and group k + 1 starts once group k has finished its CBCA,
    // so the LDS-bound aggregation sweeps of one group share the CUs with the SGM paths of the
    // previous one; the main stream joins every stream at the end.
    const int g = c->sub_batch > 0 ? c->sub_batch : (c->auto_groups ? (n + 1) / 2 : n);
    const int ns = c->nstreams;
    // where group k + 1 starts: with CBCA after group k's first CBCA sweep (the next group's
    // prep, cost and first sweep then share the CUs with this group's LDS-bound NORM_SCAN
    // sweep: profiles/r4j, 1.5-5 % faster than starting after the whole CBCA), else after group
    // k's aggregation
    //
    // Pipelined (num_streams 0 with CBCA + SGM, two groups): group 0 on the main stream, group 1 on
    // the side stream, and the call returns WITHOUT joining them: the next call's group 0 follows
    // this call's group 0 on the main stream and its group 1 this call's group 1 on the side
    // stream, so group 1 keeps running about half a call behind group 0 -- its LDS- and
    // issue-bound CBCA sweeps (NsV: three waves per CU, one SIMD idle, 3 TB/s) beside group 0's SGM
    // passes, which use no LDS and stream HBM.  Two single-pair pipelines offset by half a call:
    // 36.1 -> 35.2 ms per two full-resolution pairs in the bench (profiles/r5l); the placement of an
    // instance's allocations moves both by up to 2 ms (tools/overlap_probe2.py).  Only
    // a pipeline start staggers group 1 (after group 0's CBCA); every other entry point joins
    // first (check -> join_all), and the asynchronous map copy waits for both groups.
    const bool piped = c->pipelined && ns == 2 && n >= 2 && (n + g - 1) / g == 2;
    const bool early = !piped && SM_STAGGER_STAGE == 1 && c->p.aggregation == SM_AGG_CBCA && c->p.cbca_iterations > 0;
    // (a different split of the pairs would let the groups of two calls share a pair: join first)
    if ((!piped || g != c->pipe_g) && (s = join_all(c))) return s;
    const bool start = !(piped && c->pipe_live);   // groups start from a joined state
    hipStream_t main_st = c->st;
    int k = 0;
    sm_status s_out = SM_OK;
    if (ns > 1 && start) {   // the side streams start after everything queued so far on the main stream
        HIP_TRY(c, hipEventRecord(c->xev[0], main_st));
        for (int i = 0; i + 1 < ns; i++) HIP_TRY(c, hipStreamWaitEvent(c->xst[i], c->xev[0], 0));
    }
    for (int off = 0; off < n; off += g, k++) {
        const int m2 = n - off < g ? n - off : g;
        const Bufs B = at(c, off);
        c->st = (ns > 1 && k % ns) ? c->xst[k % ns - 1] : main_st;
        hipError_t e = hipSuccess;
        if (ns > 1 && k > 0 && start && (e = hipStreamWaitEvent(c->st, c->xev[1 + (k - 1) % 8], 0)) != hipSuccess) {
            s_out = hip_fail(c, e, "hipStreamWaitEvent (group stagger)");
            break;
        }
        Bufs Bo = B;   // what the optimiser reads
        const bool pipe = c->nl_pipe && m2 == n && ns == 1 && SM_FUSE_SOLVE_ALL;
        if (pipe) {   // prep, cost volume and trees on the NL front stream (run_nl)
            if ((s_out = run_nl(c, m2, B, true, w, &Bo))) break;
        } else {
            if ((s_out = run_prep(c, m2, B))) break;
            if ((s_out = run_cost(c, m2, 0, B))) break;
            if (right_view(c->p) && (s_out = run_cost(c, m2, 1, B))) break;
            if ((s_out = run_other_agg(c, m2, B, SM_FUSE_SOLVE_ALL, w))) break;   // SolveAll fused into GF / NL
        }
        // the group's input images are read by prep and the cost volume only (CBCA + SGM, no
        // refinement: the pipelined form): the next call's async upload may overwrite them now
        if (piped && SM_UP_EARLY) {
            if (!c->ev_in[k] && (e = hipEventCreateWithFlags(&c->ev_in[k], hipEventDisableTiming)) != hipSuccess) {
                s_out = hip_fail(c, e, "hipEventCreate (inputs read)");
                break;
            }
            if ((e = hipEventRecord(c->ev_in[k], c->st)) != hipSuccess) {
                s_out = hip_fail(c, e, "hipEventRecord (inputs read)");
                break;
            }
        }
        if (ns > 1 && early) c->stagger_ev = c->xev[1 + k % 8];
        for (int v = 0; v < n_views(c->p) && !s_out && !pipe; v++) {
            if (c->p.aggregation == SM_AGG_CBCA && c->p.cbca_iterations > 0)
                s_out = run_cbca(c, m2, v, true, w, B);   // SolveAll fused into the last pass
            else if (!SM_FUSE_SOLVE_ALL || !(c->p.aggregation == SM_AGG_GF || (c->p.aggregation == SM_AGG_NL && v == 0)))
                s_out = run_scale(c, m2, v, w, B);      // (GF and NL's vm[0]: fused above)
        }
        if (s_out) break;
        // the maps are written from here on: an asynchronous copy of the previous run's maps
        // (sm_download_disp_async) must be done reading them
        // (a split copy: ev_copy covers pairs [0, copy_g) only; a group reaching past them -- the
        // second group, or any group of a different split or schedule -- waits for ev_copy2,
        // recorded after both copies)
        const bool past = c->copy_split && off + m2 > c->copy_g;
        if (c->copy_pending && (e = hipStreamWaitEvent(c->st, past ? c->ev_copy2 : c->ev_copy, 0)) != hipSuccess) {
            s_out = hip_fail(c, e, "hipStreamWaitEvent (async map copy)");
            break;
        }
        c->stagger_ev = nullptr;
        if (ns > 1 && !early && (e = hipEventRecord(c->xev[1 + k % 8], c->st)) != hipSuccess) {
            s_out = hip_fail(c, e, "hipEventRecord (group CBCA done)");
            break;
        }
        for (int v = 0; v < opt_views(c->p) && !s_out; v++) s_out = run_optimize(c, m2, v, Bo);
        if (s_out) break;
        if (pipe && (e = hipEventRecord(c->nl_ev_opt[c->nl_opt_set], c->st)) != hipSuccess) {
            s_out = hip_fail(c, e, "hipEventRecord (NL set released)");
            break;
        }
        if (c->p.do_refine && (s_out = run_refine(c, m2, B))) break;
    }
    c->st = main_st;
    c->stagger_ev = nullptr;
    if (piped && !s_out) {
        c->pipe_live = true;   // group 1 stays on the side stream (joined by the next other call)
        c->pipe_g = g;
    } else if (ns > 1) {   // the join runs on the error path too: nothing stays queued behind the main stream
        for (int i = 0; i + 1 < ns; i++) {
            hipError_t e = hipEventRecord(c->xev[9 + i], c->xst[i]);
            if (e == hipSuccess) e = hipStreamWaitEvent(main_st, c->xev[9 + i], 0);
            if (e != hipSuccess) {
                // a failed join: drain the side stream on the host so its groups cannot race later work
                hipStreamSynchronize(c->xst[i]);
                if (!s_out) s_out = hip_fail(c, e, "stream join");
            }
        }
    }
    if (s_out) return s_out;
    c->stage = c->p.do_refine ? 5 : 4;
    if (disp_out) return sm_download_disp(c, n, disp_out);
    return SM_OK;
}

// Volume placement trials (sm_params.placement_trials).  One library, one process: the
// same kernels on different device allocations of the volumes run 5-8 % apart, stably per
// allocation -- with identical request counts (TCC_EA0_RDREQ / WRREQ) and no more translation
// misses (TCP_UTCL1_TRANSLATION_MISS ~1e3 of 4e8 requests), but more DRAM credit stalls
// (TCC_EA0_RDREQ_DRAM_CREDIT_STALL, TCC_TAG_STALL), i.e. the physical pages' spread over the HBM
// channels (profiles/r6g).  No allocation flag selects that, so the first sm_run holds k candidate
// sets of the large volumes at once (distinct pages), times the call's own pipeline on each (one
// warm-up, then the best of two) and keeps the fastest; the others are freed.  The maps are the
// same on every set; the trial runs' maps are overwritten by the real run that follows.
static sm_status place_volumes(sm_ctx* c, int k, int n, float reg_lambda) {
    float** slot[4] = {&c->vm0, &c->vm1, &c->acc, &c->ck};
    const size_t vol = (c->cap * c->nvol + c->vtail) * sizeof(float);
    const size_t bytes[4] = {vol, vol, vol, c->cap * c->ck_pair * sizeof(float)};
    std::vector<std::array<float*, 4>> sets(1);
    for (int i = 0; i < 4; i++) sets[0][i] = *slot[i];
    for (int t = 1; t < k; t++) {
        std::array<float*, 4> v{};
        bool ok = true;
        for (int i = 0; i < 4 && ok; i++)
            if (sets[0][i] && hipMalloc((void**)&v[i], bytes[i]) != hipSuccess) {
                v[i] = nullptr;
                ok = false;
            }
        if (!ok) {   // (no room for another set: try the ones held)
            for (float* q : v)
                if (q) hipFree(q);
            (void)hipGetLastError();
            break;
        }
        sets.push_back(v);
    }
    if (sets.size() < 2) return SM_OK;
    const bool prof = c->prof;
    c->prof = false;
    sm_status s = SM_OK;
    size_t best = 0;
    double best_t = 1e30;
    c->place_ms.clear();
    for (size_t i = 0; i < sets.size() && !s; i++) {
        for (int j = 0; j < 4; j++) *slot[j] = sets[i][j];
        double tmin = 1e30;
        for (int r = 0; r < 3 && !s; r++) {   // (r = 0 touches the set's pages first)
            const auto t0 = std::chrono::steady_clock::now();
            s = sm_run(c, n, reg_lambda, nullptr);
            if (!s) s = sm_synchronize(c);
            const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (r > 0) tmin = std::min(tmin, t);
        }
        c->place_ms.push_back(tmin * 1e3);
        if (tmin < best_t) {
            best_t = tmin;
            best = i;
        }
    }
    c->prof = prof;
    for (size_t i = 0; i < sets.size(); i++)
        if (i != best)
            for (float* q : sets[i])
                if (q) hipFree(q);
    for (int j = 0; j < 4; j++) *slot[j] = sets[best][j];
    c->place_best = (int)best;
    if (getenv("SM_TRACE_ALLOC")) {
        fprintf(stderr, "[place] %zu volume sets, kept %zu:", sets.size(), best);
        for (double t : c->place_ms) fprintf(stderr, " %.3f", t);
        fprintf(stderr, " ms\n");
    }
    return s;
}

sm_status sm_download_disp(sm_ctx* c, int32_t n, int16_t* disp_out) {
    sm_status s = check(c);
    if (s) return s;
    if (!disp_out || n < 1 || n > c->cap) return fail(c, SM_EINVAL, "bad arguments");
    if (c->stage < 4) return fail(c, SM_ESTATE, "no disparity map yet");
    HIP_TRY(c, hipMemcpyAsync(disp_out, c->disp, (size_t)n * c->npix * 2, hipMemcpyDefault, c->st));
    HIP_TRY(c, hipStreamSynchronize(c->st));
    return SM_OK;
}

sm_status sm_download_disp_async(sm_ctx* c, int32_t n, int16_t* disp_out) {
    sm_status s = check_nojoin(c);   // (keeps a pipelined run's groups apart)
    if (s) return s;
    if (!disp_out || n < 1 || n > c->cap) return fail(c, SM_EINVAL, "bad arguments");
    if (c->stage < 4) return fail(c, SM_ESTATE, "no disparity map yet");
    if (!c->cst) HIP_TRY(c, hipStreamCreateWithFlags(&c->cst, hipStreamNonBlocking));
    if (!c->ev_run) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_run, hipEventDisableTiming));
    if (!c->ev_copy) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_copy, hipEventDisableTiming));
    if (!c->ev_copy2) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_copy2, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(c->ev_run, c->st));
    HIP_TRY(c, hipStreamWaitEvent(c->cst, c->ev_run, 0));
    c->copy_split = c->pipe_live && n > c->pipe_g;
    c->copy_g = c->pipe_g;
    if (c->copy_split) {
        // a pipelined run: the first group's maps once the main stream is there, the second's once
        // the side stream is (waited for, not joined), so that the next run's group k waits for
        // its own maps' copy only
        const size_t g = (size_t)c->pipe_g;
        HIP_TRY(c, hipMemcpyAsync(disp_out, c->disp, g * c->npix * 2, hipMemcpyDefault, c->cst));
        HIP_TRY(c, hipEventRecord(c->ev_copy, c->cst));
        HIP_TRY(c, hipEventRecord(c->xev[10], c->xst[0]));
        HIP_TRY(c, hipStreamWaitEvent(c->cst, c->xev[10], 0));
        HIP_TRY(c, hipMemcpyAsync(disp_out + g * c->npix, c->disp + g * c->npix, ((size_t)n - g) * c->npix * 2,
                                  hipMemcpyDefault, c->cst));
        HIP_TRY(c, hipEventRecord(c->ev_copy2, c->cst));
    } else {
        if (c->pipe_live) {   // (n within the first group: its maps only)
            HIP_TRY(c, hipEventRecord(c->xev[10], c->xst[0]));
            HIP_TRY(c, hipStreamWaitEvent(c->cst, c->xev[10], 0));
        }
        HIP_TRY(c, hipMemcpyAsync(disp_out, c->disp, (size_t)n * c->npix * 2, hipMemcpyDefault, c->cst));
        HIP_TRY(c, hipEventRecord(c->ev_copy, c->cst));
    }
    c->copy_pending = true;
    // (one event after both copies on the copy stream: sm_download_wait's per-call marker)
    if (!c->ev_dl[c->dl_slot]) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_dl[c->dl_slot], hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(c->ev_dl[c->dl_slot], c->cst));
    c->dl_slot ^= 1;
    c->dl_count++;
    return SM_OK;
}

sm_status sm_download_wait(sm_ctx* c, int32_t back) {
    sm_status s = check_nojoin(c);   // (the pipeline stays live)
    if (s) return s;
    if (back < 0 || back > 1) return fail(c, SM_EINVAL, "back must be 0 (the last async download) or 1 (the one before)");
    if (c->dl_count <= back) return SM_OK;   // (no such download: nothing to wait for)
    hipEvent_t e = c->ev_dl[(c->dl_slot + 1 + back) & 1];
    if (e) HIP_TRY(c, hipEventSynchronize(e));
    return SM_OK;
}

// Asynchronous upload for a pipelined stream of calls (DistributedBatchRunner over hip_compute_fn):
// the copies are queued without joining a live pipeline or waiting on the host -- the next call's
// first group's pairs on the main stream (after that group's previous call), the second group's on
// the side stream (after the previous call's second group) -- so a call's inputs arrive while the
// previous call still runs.  The sources must stay unchanged until sm_upload_wait returns.
sm_status sm_upload_batch_async(sm_ctx* c, int32_t n, const uint8_t* lbgr, const uint8_t* rbgr, const uint8_t* lgray,
                                const uint8_t* rgray) {
    sm_status s = check_nojoin(c);
    if (s) return s;
    if (n < 1 || n > c->cap) return fail(c, SM_EINVAL, "n must be in [1, batch_capacity]");
    if (!lbgr || !rbgr || !lgray || !rgray) return fail(c, SM_EINVAL, "null image pointer");
    // the split the next run will keep (sm_run: g = (n + 1) / 2 under the auto schedule); any
    // other shape joins first, as a synchronous upload does
    const int g = c->sub_batch > 0 ? c->sub_batch : (c->auto_groups ? (n + 1) / 2 : n);
    const bool split = c->pipe_live && c->pipelined && g == c->pipe_g && (n + g - 1) / g == 2;
    if (!split && (s = join_all(c))) return s;
    for (int i = 0; i < 2; i++)
        if (!c->ev_up[i]) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_up[i], hipEventDisableTiming));
    const sm_params& p = c->p;
    const size_t H = p.rows, W = p.cols, crow = W * 3;
    // early: the copies go on their own stream as soon as each group's previous inputs are read
    // (ev_in, recorded after its cost volume), so they overlap that group's CBCA and SGM; the
    // group's next kernels wait for its copies (ev_up)
    const bool early = split && SM_UP_EARLY && c->ev_in[0] && c->ev_in[1];
    const hipStream_t ust = nullptr;
    for (int grp = 0; grp < (early ? 2 : 1); grp++) {
        if (early) HIP_TRY(c, hipStreamWaitEvent(ust, c->ev_in[grp], 0));
        const int b0 = early ? grp * g : 0, b1 = early ? std::min(n, (grp + 1) * g) : n;
    for (int view = 0; view < 2; view++) {
        const uint8_t* src = view == 0 ? lbgr : rbgr;
        const uint8_t* gsrc = view == 0 ? lgray : rgray;
        for (int b = b0; b < b1; b++) {
            hipStream_t st = early ? ust : (split && b >= g) ? c->xst[0] : c->st;
            uint8_t* dst = c->bgr + ((size_t)b * 2 + view) * c->npix * 3;
            HIP_TRY(c, hipMemcpy2DAsync(dst, crow, src + (size_t)b * H * crow, crow, crow, H, hipMemcpyDefault, st));
            uint8_t* gdst = c->gray + ((size_t)b * 2 + view) * c->npix;
            HIP_TRY(c, hipMemcpy2DAsync(gdst, W, gsrc + (size_t)b * H * W, W, W, H, hipMemcpyDefault, st));
        }
    }
        if (early) {
            HIP_TRY(c, hipEventRecord(c->ev_up[grp], ust));
            HIP_TRY(c, hipStreamWaitEvent(grp == 0 ? c->st : c->xst[0], c->ev_up[grp], 0));
        }
    }
    if (!early) {
        HIP_TRY(c, hipEventRecord(c->ev_up[0], c->st));
        if (split) HIP_TRY(c, hipEventRecord(c->ev_up[1], c->xst[0]));
    }
    c->up_split = split;
    c->n_loaded = n;
    c->stage = 1;
    return SM_OK;
}

sm_status sm_upload_wait(sm_ctx* c) {
    sm_status s = check_nojoin(c);
    if (s) return s;
    if (c->ev_up[0]) HIP_TRY(c, hipEventSynchronize(c->ev_up[0]));
    if (c->up_split && c->ev_up[1]) HIP_TRY(c, hipEventSynchronize(c->ev_up[1]));
    return SM_OK;
}

sm_status sm_run_batch(sm_ctx* c, int32_t n, const uint8_t* lbgr, const uint8_t* rbgr, const uint8_t* lgray,
                       const uint8_t* rgray, float reg_lambda, int16_t* disp_out) {
    sm_status s = sm_upload_batch(c, n, lbgr, rbgr, lgray, rgray);
    if (s) return s;
    return sm_run(c, n, reg_lambda, disp_out);
}

sm_status sm_run_batch_multi(sm_ctx* const* ctxs, int32_t nctx, int32_t n, const uint8_t* lbgr, const uint8_t* rbgr,
                             const uint8_t* lgray, const uint8_t* rgray, float reg_lambda, int16_t* disp_out) {
    if (!ctxs || nctx < 1 || n < 1 || !lbgr || !rbgr || !lgray || !rgray || !disp_out) return SM_EINVAL;
    for (int i = 0; i < nctx; i++) {
        if (!ctxs[i]) return SM_EINVAL;
        for (int j = 0; j < i; j++)
            if (ctxs[j] == ctxs[i]) return fail(ctxs[i], SM_EINVAL, "sm_run_batch_multi: a context appears twice");
        const sm_params& a = ctxs[i]->p;
        const sm_params& b = ctxs[0]->p;
        if (a.rows != b.rows || a.cols != b.cols || a.num_disparities != b.num_disparities)
            return fail(ctxs[i], SM_EINVAL, "sm_run_batch_multi: contexts of different shapes");
    }
    // contiguous blocks of ceil(n / nctx) pairs: context i owns pairs [i * per, min(n, (i + 1) * per))
    const int per = (n + nctx - 1) / nctx;
    const size_t npix = (size_t)ctxs[0]->p.rows * ctxs[0]->p.cols;
    for (int i = 0; i < nctx; i++) {
        const int lo = std::min(n, i * per), cnt = std::min(n, lo + per) - lo;
        if (cnt > ctxs[i]->cap) return fail(ctxs[i], SM_EINVAL, "sm_run_batch_multi: block larger than batch_capacity");
    }
    std::vector<sm_status> st(nctx, SM_OK);
    auto work = [&](int i) {
        const int lo = std::min(n, i * per), cnt = std::min(n, lo + per) - lo;
        if (cnt <= 0) return;
        st[i] = sm_run_batch(ctxs[i], cnt, lbgr + lo * npix * 3, rbgr + lo * npix * 3, lgray + lo * npix,
                             rgray + lo * npix, reg_lambda, disp_out + lo * npix);
    };
    // one host thread per context (each context is used by one thread only, the C-ABI's rule)
    std::vector<std::thread> th;
    for (int i = 1; i < nctx; i++) th.emplace_back(work, i);
    work(0);
    for (auto& t : th) t.join();
    for (int i = 0; i < nctx; i++)
        if (st[i] != SM_OK) return st[i];
    return SM_OK;
}

int32_t sm_placement_trials_ms(sm_ctx* c, double* ms, int32_t max) {
    if (!c) return -1;
    const int32_t nt = (int32_t)c->place_ms.size();
    for (int32_t i = 0; ms && i < nt && i < max; i++) ms[i] = c->place_ms[i];
    return nt;
}

int32_t sm_placement_kept(const sm_ctx* c) { return c ? c->place_best : -1; }

sm_status sm_set_schedule(sm_ctx* c, int32_t num_streams, int32_t sub_batch) {
    sm_status s = check(c);
    if (s) return s;
    // (the previous sm_run joined its side streams into the main stream, so the next run's
    // groups are ordered after it whichever streams they use)
    if ((s = apply_schedule(c, num_streams, sub_batch))) return s;
    c->p.num_streams = num_streams;
    c->p.sub_batch = sub_batch;
    return SM_OK;
}

sm_status sm_synchronize(sm_ctx* c) {
    sm_status s = check(c);
    if (s) return s;
    HIP_TRY(c, hipStreamSynchronize(c->st));
    if (c->cst) {
        HIP_TRY(c, hipStreamSynchronize(c->cst));
        c->copy_pending = false;
    }
    return SM_OK;
}

// (a pipelined sm_run leaves its second group on a side stream: the main stream is made to wait
// for it first, so work ordered after the returned stream sees the whole call)
void* sm_stream(sm_ctx* c) {
    if (!c || check(c) != SM_OK) return nullptr;
    return (void*)c->st;
}

sm_status sm_profile_enable(sm_ctx* c, int32_t on) {
    if (!c) return SM_EINVAL;
    c->prof = on != 0;
    return SM_OK;
}

static sm_status drain_profile(sm_ctx* c) {
    if (c->recs.empty()) return SM_OK;
    HIP_TRY(c, hipStreamSynchronize(c->st));
    for (auto& r : c->recs) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, r.start, r.stop) == hipSuccess) {
            c->kstat[r.kernel].launches++;
            c->kstat[r.kernel].total_ms += ms;
        }
        c->free_events.push_back(r.start);
        c->free_events.push_back(r.stop);
    }
    c->recs.clear();
    return SM_OK;
}

sm_status sm_profile_read(sm_ctx* c, int32_t max, char* names, int64_t* launches, double* total_ms,
                          double* bytes_per_launch, int32_t* count) {
    sm_status s = check(c);
    if (s) return s;
    if ((s = drain_profile(c))) return s;
    const int k = (int)c->knames.size();
    if (count) *count = k;
    for (int i = 0; i < k && i < max; i++) {
        if (names) {
            strncpy(names + (size_t)i * 48, c->knames[i].c_str(), 47);
            names[(size_t)i * 48 + 47] = 0;
        }
        if (launches) launches[i] = c->kstat[i].launches;
        if (total_ms) total_ms[i] = c->kstat[i].total_ms;
        if (bytes_per_launch) bytes_per_launch[i] = c->kstat[i].bytes;
    }
    return SM_OK;
}

sm_status sm_profile_reset(sm_ctx* c) {
    sm_status s = check(c);
    if (s) return s;
    if ((s = drain_profile(c))) return s;
    for (auto& st : c->kstat) st = ProfStat();
    return SM_OK;
}

sm_status sm_cal_err(const int16_t* DP, const float* DT, const uint8_t* mask, int32_t rows, int32_t cols, float thres,
                     float* pbm, float* rms) {
    if (!DP || !DT || !mask || !pbm || !rms || rows < 1 || cols < 1) return SM_EINVAL;
    int sumNum = 0, errorNumer = 0;
    float errorValueSum = 0;
    for (size_t i = 0; i < (size_t)rows * cols; i++) {
        if (mask[i] != 255) continue;
        sumNum++;
        if (DP[i] >= 0) {
            const float dif = fabsf(DT[i] - (float)DP[i]);
            errorValueSum = (float)((double)errorValueSum + pow((double)dif, 2));   // float += pow(float, int)
            if (dif > thres) errorNumer++;
        } else {
            errorNumer++;
            errorValueSum += 2;
        }
    }
    if (sumNum == 0) {   // the reference divides 0 / 0 here; report 0 instead of NaN
        *pbm = 0;
        *rms = 0;
        return SM_OK;
    }
    *pbm = (float)errorNumer / sumNum;
    *rms = sqrtf(errorValueSum / sumNum);
    return SM_OK;
}

float sm_expf_host(float x) { return sm::expf_host(x); }

sm_status sm_expf_device_range(sm_ctx* c, uint32_t first_bits, uint32_t n, float* out) {
    sm_status s = check(c);
    if (s) return s;
    if (!out) return fail(c, SM_EINVAL, "null out");
    float* dbuf = nullptr;
    if ((s = dalloc(c, &dbuf, n))) return s;
    sm::launch_expf_range(first_bits, n, dbuf, c->st);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out, dbuf, (size_t)n * 4, hipMemcpyDeviceToHost, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);
    hipFree(dbuf);
    if (e != hipSuccess) return hip_fail(c, e, "sm_expf_device_range");
    return SM_OK;
}

sm_status sm_copy_ceiling(sm_ctx* c, uint64_t bytes, int32_t reps, double* best_gbs, double* median_gbs) {
    sm_status s = check(c);
    if (s) return s;
    if (!best_gbs || !median_gbs || reps < 1 || reps > 1000 || bytes < 16384) return fail(c, SM_EINVAL, "bad arguments");
    bytes = bytes / 16384 * 16384;
    char *src = nullptr, *dst = nullptr;
    if ((s = dalloc(c, &src, bytes))) return s;
    if ((s = dalloc(c, &dst, bytes))) {
        hipFree(src);
        return s;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    std::vector<double> gbs;
    hipError_t e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMemsetAsync(src, 1, bytes, c->st);
    // grid sizes bracketing the volume sweeps' launch shapes; every (grid, repetition) is one sample
    for (int grid : {4096, 16384, 65536}) {
        for (int r = 0; r < reps + 1 && e == hipSuccess; r++) {
            if ((e = hipEventRecord(e0, c->st)) != hipSuccess) break;
            sm::launch_copy_x4(src, dst, bytes, grid, c->st);
            if ((e = hipGetLastError()) != hipSuccess) break;
            if ((e = hipEventRecord(e1, c->st)) != hipSuccess) break;
            if ((e = hipEventSynchronize(e1)) != hipSuccess) break;
            float ms = 0.f;
            if ((e = hipEventElapsedTime(&ms, e0, e1)) != hipSuccess) break;
            if (r > 0 && ms > 0.f) gbs.push_back(2.0 * (double)bytes / (ms * 1e-3) / 1e9);   // read + write
        }
    }
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    hipFree(src);
    hipFree(dst);
    if (e != hipSuccess) return hip_fail(c, e, "sm_copy_ceiling");
    if (gbs.empty()) return fail(c, SM_EHIP, "sm_copy_ceiling: no timing samples");
    std::sort(gbs.begin(), gbs.end());
    *best_gbs = gbs.back();
    *median_gbs = gbs[gbs.size() / 2];
    return SM_OK;
}

sm_status sm_div_area_check(sm_ctx* c, int32_t exp2, int32_t bmax, uint64_t* mismatches) {
    sm_status s = check(c);
    if (s) return s;
    if (!mismatches || bmax < 1 || bmax > 65535 || exp2 < -126 || exp2 > 126) return fail(c, SM_EINVAL, "bad arguments");
    unsigned long long* dbad = nullptr;
    if ((s = dalloc(c, &dbad, 1))) return s;
    hipError_t e = hipMemsetAsync(dbad, 0, sizeof(*dbad), c->st);
    if (e == hipSuccess) {
        sm::launch_div_check(exp2, bmax, dbad, c->st);
        e = hipGetLastError();
    }
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, dbad, sizeof(h), hipMemcpyDeviceToHost, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);
    hipFree(dbad);
    if (e != hipSuccess) return hip_fail(c, e, "sm_div_area_check");
    *mismatches = h;
    return SM_OK;
}

}  // extern "C"
