/*
 * sm_capi.h — C-ABI of the MI355X stereo-matching back end (libsm_hip.so).
 *
 * This is the drop-in boundary for the reference's hot path: the calls that
 * main_.cpp makes on class StereoMatching (reference main_.cpp:138-172) map one-to-one onto the
 * entry points below.  Plain pointers and sizes only; no exceptions, no exit(), no globals:
 * every call returns an sm_status and sm_last_error(ctx) holds the message.
 *
 * Reference interface each entry point replaces (paths relative to the reference root):
 *   sm_params_default  <- StereoMatching::Parameters::Parameters     stereoMatching.h:204-350
 *   sm_create          <- StereoMatching::StereoMatching (ctor)      stereoMatching.cpp:2058-2110
 *   sm_set_images      <- ctor image arguments I1_c,I2_c,I1_g,I2_g   stereoMatching.cpp:2063-2071
 *   sm_cost_calculate  <- StereoMatching::costCalculate              stereoMatching.cpp:945-1021
 *   sm_solve_all       <- SolveAll(StereoMatching**&, PY_LVL, REG_LAMBDA)  stereoMatching.cpp:2142-2208
 *   sm_solve_all_pyr   <- the same with PY_LVL > 1 (one ctx per level)     stereoMatching.cpp:2142-2208
 *   sm_pyr_down        <- cv::pyrDown on the inputs                     main_.cpp:145-148
 *   sm_cal_err         <- StereoMatching::calErr (one region)          stereoMatching.h:1748-1825
 *   sm_disp_optimize   <- StereoMatching::dispOptimize + DP[0]       stereoMatching.cpp:1046-1136, h:2724
 *   sm_refine          <- StereoMatching::refine (Do_refine)         stereoMatching.cpp:1138-1511, main_.cpp:165-166
 *   sm_get_disp / sm_set_disp <- public member DP[view]              stereoMatching.h:2724
 *   sm_get_volume      <- public member vm[view]                     stereoMatching.h:2720
 *   sm_get_arms        <- public member HVL[view]                    stereoMatching.h:2717
 *   sm_destroy         <- delete smPsy[p]                            main_.cpp:173-178
 *   sm_run / sm_run_batch  <- the whole main_.cpp:139-163 sequence for n independent pairs
 *   sm_run_batch_multi     <- the same over several contexts / GPUs (one host thread each)
 * Threading: one sm_ctx per host thread; each ctx owns one HIP stream on its device.
 */
#ifndef SM_CAPI_H
#define SM_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define SM_API __attribute__((visibility("default")))
#else
#define SM_API
#endif

typedef enum sm_status {
    SM_OK = 0,
    SM_EINVAL = 1,   /* bad argument / unsupported parameter combination */
    SM_ENOMEM = 2,   /* device or host allocation failed */
    SM_EHIP = 3,     /* HIP runtime error (launch, copy, sync) */
    SM_ESTATE = 4,   /* call out of order (e.g. optimize before cost) */
} sm_status;

/* static std::string costcalculation / aggregation / optimization selectors (h:51-53). */
typedef enum sm_cost_method {
    SM_COST_CENSUS_GRAD = 0, /* "censusGrad" (main:15; cpp:25-48) — default */
    SM_COST_CENSUS = 1,      /* "Census"     (cpp:975-976) */
    SM_COST_AD_CENSUS = 2,   /* "ADCensus"   (cpp:894-915, 5250-5277) */
    SM_COST_AD = 3,          /* "AD"         (cpp:954-955) */
} sm_cost_method;

typedef enum sm_aggregation {
    SM_AGG_NONE = 0,
    SM_AGG_CBCA = 1,         /* "CBCA" (main:16; cpp:1002-1003) — default */
    SM_AGG_GF = 2,           /* "GF"  guideFilter (cpp:4492-4516), form chosen by gf_mode; sgm / WTA only */
    SM_AGG_NL = 3,           /* "NL"  non-local MST tree filter (cpp:4892-4917, NL/NLCCA.cpp:27-96) */
} sm_aggregation;

/* guideFilter's two builds (stereoMatching.h:38 `//#define MY_GUIDE`): */
typedef enum sm_gf_mode {
    SM_GF_XIMGPROC = 0,      /* cv::ximgproc::guidedFilter(I, vm, vm, 9, 1e-4) (cpp:4513) — the shipped build */
    SM_GF_MY_GUIDE = 1,      /* guideFilterCore_matlab (cpp:4509, 4975-5104) — the MY_GUIDE build */
} sm_gf_mode;

typedef enum sm_optimization {
    SM_OPT_WTA = 0,          /* "" : WTA only (cpp:1104-1128) */
    SM_OPT_SGM = 1,          /* "sgm" (main:17; cpp:1051-1060) — default */
    SM_OPT_SO = 2,           /* "so" scan-line DP + backtrack (cpp:1091-1105, 6272-6394) */
} sm_optimization;

/* The subset of StereoMatching::Parameters (h:85-351) that the hot path reads, plus the
 * static selectors.  Field defaults come from sm_params_default (= the reference ctor). */
typedef struct sm_params {
    uint32_t struct_size;        /* = sizeof(sm_params), set by sm_params_default; sm_create refuses others */
    int32_t rows, cols;          /* h_, w_ */
    int32_t num_disparities;     /* numDisparities = maxDisp + 1 (h:209) */
    int32_t cost_method;         /* sm_cost_method */
    int32_t aggregation;         /* sm_aggregation */
    int32_t optimization;        /* sm_optimization */
    int32_t census_rv, census_ru;/* census window radii {3, 4} (cpp:815) */
    int32_t census_ring;         /* censusFunc == 3 -> 8 ring bits (h:244) */
    float lam_cen, lam_g;        /* lamCen = 13, lamG = 1 (main:56-57) */
    float grad_trunc;            /* 500 (cpp:34) */
    int32_t grad_adaptive;       /* gradFuse_adpWgt = 1 (h:245) */
    float lam_ad, lam_cen_adc;   /* ADCensus fusion constants 10, 30 (cpp:5270) */
    float ad_trunc_adc;          /* 1000 (cpp:905) */
    float ad_trunc_ad;           /* 20 (cpp:955) */
    int32_t arm_l, arm_l_out;    /* cbca_crossL[0] = 17, cbca_crossL_out[0] = 34 (h:263, 266) */
    int32_t arm_c_thresh, arm_c_thresh_out; /* cbca_cTresh[0] = 20, cbca_cTresh_out[0] = 6 */
    int32_t arm_min_l;           /* cbca_minArmL = 1 (h:259) */
    int32_t cbca_iterations;     /* cbca_iterationNum = 2 (h:260) */
    int32_t sgm_paths;           /* 4 (cpp:6214) or 8 (full table cpp:6207-6208) */
    float sgm_p1, sgm_p2;        /* 1.0, 3.0 (h:2234-2235) */
    int32_t sgm_cor_dif_thres;   /* 15 (h:239) */
    int32_t sgm_redu_coeff;      /* 4 (h:240) */
    int32_t compute_right_view;  /* build vm[1] too (Do_LRConsis, h:72); 0 = skip (unused downstream) */
    int32_t keep_final_volume;   /* write the SGM path-sum back into vm[0] (reference does); 0 = fuse into WTA */
    int32_t batch_capacity;      /* max pairs per sm_run call (device buffers sized for it) */
    /* refinement: Do_refine (h:70) = 1 runs vm[1] through CBCA / SolveAll / SGM / WTA as well
     * (cbca_core cpp:5592, SolveAll cpp:2178, dispOptimize cpp:1054) and refine() afterwards
     * (sm_refine; sm_run does both).  Stage switches and constants as in the reference. */
    int32_t do_refine;           /* Do_refine = 0 (h:70) */
    float lr_max_diff;           /* LRmaxDiff = 0 (h:212) */
    int32_t do_region_vote;      /* Do_regionVote = 1 (h:75) */
    int32_t region_vote_nums;    /* region_vote_nums = 2 (h:306): rounds of region vote and of properIpol */
    float rv_ratio;              /* rv_ratio[i] = 0.4 (cpp:1400); must be > 0 */
    int32_t rv_s;                /* rv_s[i] = 20 (cpp:1401) */
    int32_t do_proper_ipol;      /* Do_properIpol = 1 (h:76) */
    int32_t disp_occ;            /* DISP_OCC = -2 * 16 (h:216) */
    int32_t do_last_median_blur; /* Do_lastMedianBlur = 1 (h:80) */
    /* scheduling of sm_run (results are identical for every setting): */
    int32_t sub_batch;           /* run the n pairs in groups of k (0 = one group), stages back to back */
    int32_t num_streams;         /* 0 (default): auto -- with CBCA and a volume >= 256 MiB per pair (or
                                  * batch_capacity >= 8 with 4-path SGM and no refinement), two
                                  * streams and (sub_batch 0) two groups of n / 2 pairs; with SGM
                                  * and no refinement the groups are pipelined ACROSS calls: sm_run
                                  * returns with the second group still queued on the side stream
                                  * (about half a call behind the first), the next sm_run's groups
                                  * follow on their own streams, sm_download_disp_async copies each
                                  * group's maps after that group, and every other call first waits
                                  * for both; else one stream; 1: one stream; 2-4: groups alternate
                                  * over that many streams (group k + 1 starts after group k's first
                                  * CBCA sweep, or its aggregation without CBCA), joined per call */
    int32_t fuse_norm_scan;      /* CBCA: iteration k's normalising sweep fused with iteration k+1's
                                  * scan (one sweep, 8 B per element less): 1 = always, 0 = never,
                                  * -1 (default) = when the dedicated sweep for the reference's lag
                                  * applies (arm length 34, D % 64 == 0) or a pair's volume is
                                  * >= 256 MiB (measured faster there; the generic fused sweep is
                                  * slower at Teddy size) */
    /* alternative aggregators */
    float gf_eps;                /* gf_eps[0] = 0.0001 (h:298; radius gf_r[0] = 9, h:297) */
    int32_t gf_mode;             /* sm_gf_mode: SM_GF_XIMGPROC (default, the shipped build) or SM_GF_MY_GUIDE */
    double nl_sigma;             /* NLCCA sigma = 0.1 (NL/NLCCA.cpp:33): weights exp(-c / (255 sigma)) */
    int32_t lr_consis;           /* Do_LRConsis = 1 (h:72): "so" optimises both views, DP[1] = so(vm[1])
                                  * (num = Do_LRConsis ? 2 : 1, cpp:1093); 0: "so" builds and optimises
                                  * the left view only */
    int32_t placement_trials;    /* volume placement (results are identical for every setting): the
                                  * same kernels run 5-8 % apart on different device allocations of
                                  * the volumes -- same request counts, more DRAM credit stalls
                                  * (TCC_EA0_RDREQ_DRAM_CREDIT_STALL) -- so the first
                                  * sm_run of a context may time its own pipeline on k candidate
                                  * volume sets held at once and keep the fastest (k - 1 extra sets
                                  * of memory during that call only; fewer if they do not fit).
                                  * -1 (default) = 3 with CBCA + SGM and a volume >= 256 MiB per
                                  * pair, else off; 0 / 1 = off; 2-8 = k */
} sm_params;

typedef struct sm_ctx sm_ctx;

SM_API void sm_params_default(sm_params* p, int32_t max_disp, int32_t rows, int32_t cols);
SM_API sm_status sm_create(sm_ctx** out, const sm_params* p, int32_t hip_device);
SM_API sm_status sm_destroy(sm_ctx* ctx);
SM_API const char* sm_last_error(const sm_ctx* ctx);
SM_API const char* sm_status_string(sm_status s);

/* Single-pair, reference-ordered API (pair slot 0).  Host buffers: BGR u8 rows of
 * `cstride` bytes, gray u8 rows of `gstride` bytes; copied to the device. */
SM_API sm_status sm_set_images(sm_ctx* ctx, const uint8_t* lbgr, const uint8_t* rbgr, size_t cstride,
                               const uint8_t* lgray, const uint8_t* rgray, size_t gstride);
SM_API sm_status sm_cost_calculate(sm_ctx* ctx);
SM_API sm_status sm_solve_all(sm_ctx* ctx, int32_t py_lev, float reg_lambda);
SM_API sm_status sm_disp_optimize(sm_ctx* ctx, int16_t* disp_out);
/* SolveAll(smPyr, PY_LVL, REG_LAMBDA) over PY_LVL in [1, 8] contexts, one per pyramid level
 * (main_.cpp:131-158): level s has rows (rows_{s-1} + 1) / 2, cols likewise, num_disparities
 * >= num_disparities_{s-1} / 2 + 1, the same pair count and device, and sm_cost_calculate done.
 * levels[0]'s volume(s) receive the cross-scale sum; the coarser levels are only read. */
SM_API sm_status sm_solve_all_pyr(sm_ctx* const* levels, int32_t py_lvl, float reg_lambda);
/* cv::pyrDown (u8, 1 or 3 channels, BORDER_REFLECT_101) on `hip_device`; src rows x cols, dst
 * ((rows + 1) / 2) x ((cols + 1) / 2); host or device pointers, synchronous.  (main_.cpp:145-148) */
SM_API sm_status sm_pyr_down(int32_t hip_device, const uint8_t* src, int32_t rows, int32_t cols, int32_t channels,
                             uint8_t* dst);
/* cv::pyrDown of a 1-channel f32 image (the ground truth DT, main_.cpp:149), same contract. */
SM_API sm_status sm_pyr_down_f32(int32_t hip_device, const float* src, int32_t rows, int32_t cols, float* dst);
/* refine() on DP[0] (needs do_refine = 1 at sm_create and a preceding sm_disp_optimize). */
SM_API sm_status sm_refine(sm_ctx* ctx, int16_t* disp_out);
SM_API sm_status sm_get_disp(sm_ctx* ctx, int32_t view, int16_t* dst);  /* DP[view], H*W int16; DP[1] exists
                                                                        * with do_refine or optimization "so"
                                                                        * (so runs on both views, cpp:1093) */
/* Overwrite DP[view] (the reference's DP is a public member, h:2724); after sm_disp_optimize. */
SM_API sm_status sm_set_disp(sm_ctx* ctx, int32_t view, const int16_t* src);
SM_API sm_status sm_get_volume(sm_ctx* ctx, int32_t view, float* dst);   /* H*W*D floats */
SM_API sm_status sm_get_arms(sm_ctx* ctx, int32_t view, uint16_t* dst);  /* H*W*4 (L,R,U,D) */

/* Batched, device-resident API.  Inputs are packed [n][H][W][3] (BGR) and [n][H][W] (gray) and may
 * be host or device pointers (unified addressing: e.g. a torch tensor already in HBM is copied
 * device-to-device).  A device source must be complete before the call (its stream synchronized). */
SM_API sm_status sm_upload_batch(sm_ctx* ctx, int32_t n, const uint8_t* lbgr, const uint8_t* rbgr,
                                 const uint8_t* lgray, const uint8_t* rgray);
/* Run cost -> CBCA -> SolveAll(py_lev=1, reg_lambda) -> SGM -> WTA [-> refine] on the n uploaded pairs.
 * Asynchronous on the ctx stream.  disp_out: host or device [n][H][W] int16 (synchronous copy) or
 * NULL to leave the maps on the device (read them with sm_download_disp). */
SM_API sm_status sm_run(sm_ctx* ctx, int32_t n, float reg_lambda, int16_t* disp_out);
SM_API sm_status sm_download_disp(sm_ctx* ctx, int32_t n, int16_t* disp_out);
/* The same copy, enqueued on the ctx's copy stream behind the work queued so far, returning at
 * once: the next sm_run's disparity-writing kernels wait for it, so the copy overlaps the next
 * run's cost / aggregation work.  disp_out must be page-locked host memory (or device memory) and
 * stays in flight until sm_synchronize. */
SM_API sm_status sm_download_disp_async(sm_ctx* ctx, int32_t n, int16_t* disp_out);
/* A pipelined stream of calls without host waits in between (the batch runner's product path):
 * sm_upload_batch_async queues the copies of the next call's inputs behind the groups of the
 * previous call that read the same pairs (no join, no host wait; the sources must stay unchanged
 * until sm_upload_wait returns); sm_download_wait(ctx, back) waits on the host for the copies of
 * the last (back = 0) or the previous (back = 1) sm_download_disp_async -- neither joins the
 * pipeline. */
SM_API sm_status sm_upload_batch_async(sm_ctx* ctx, int32_t n, const uint8_t* lbgr, const uint8_t* rbgr,
                                       const uint8_t* lgray, const uint8_t* rgray);
SM_API sm_status sm_upload_wait(sm_ctx* ctx);
SM_API sm_status sm_download_wait(sm_ctx* ctx, int32_t back);
SM_API sm_status sm_run_batch(sm_ctx* ctx, int32_t n, const uint8_t* lbgr, const uint8_t* rbgr,
                              const uint8_t* lgray, const uint8_t* rgray, float reg_lambda,
                              int16_t* disp_out);
/* Multi-device batch (SURVEY §8b/§8e without torch.distributed): the n packed host pairs are split
 * into contiguous blocks of ceil(n / nctx), block i runs on ctxs[i] (each context on its own
 * device, or several on one), one host thread per context; disp_out receives all n maps in order.
 * Contexts must share rows / cols / num_disparities and hold batch_capacity >= the block size.
 * Returns the first failing context's status (its sm_last_error has the message). */
SM_API sm_status sm_run_batch_multi(sm_ctx* const* ctxs, int32_t nctx, int32_t n, const uint8_t* lbgr,
                                    const uint8_t* rbgr, const uint8_t* lgray, const uint8_t* rgray,
                                    float reg_lambda, int16_t* disp_out);
/* Change sm_params.num_streams / sub_batch of an existing context (same meaning and ranges as at
 * sm_create); applies from the next sm_run.  Results are identical for every schedule; this lets
 * one context (one set of device allocations) time schedules against each other. */
SM_API sm_status sm_set_schedule(sm_ctx* ctx, int32_t num_streams, int32_t sub_batch);
/* placement trials of the first sm_run (sm_params.placement_trials): the number of volume sets
 * timed (0: none ran), their pipeline times in ms (up to max), and the index of the set kept */
SM_API int32_t sm_placement_trials_ms(sm_ctx* ctx, double* ms, int32_t max);
SM_API int32_t sm_placement_kept(const sm_ctx* ctx);
SM_API sm_status sm_synchronize(sm_ctx* ctx);
SM_API void* sm_stream(sm_ctx* ctx);      /* the ctx's main hipStream_t, joined first: after a
                                             pipelined sm_run (num_streams 0, the default) the
                                             call's second group runs on a side stream until the
                                             next entry point joins it; sm_stream joins it, so work
                                             ordered after the returned stream sees the whole call.
                                             NULL on error (sm_last_error) */

/* Per-kernel timing with HIP events on the ctx stream. */
SM_API sm_status sm_profile_enable(sm_ctx* ctx, int32_t on);
/* Fills up to max entries: name (NUL-terminated, 48 chars max), launches, total ms,
 * algorithmic bytes per launch.  Returns the number of distinct kernels in *count. */
SM_API sm_status sm_profile_read(sm_ctx* ctx, int32_t max, char* names /* max*48 */, int64_t* launches,
                                 double* total_ms, double* bytes_per_launch, int32_t* count);
SM_API sm_status sm_profile_reset(sm_ctx* ctx);

/* calErr (stereoMatching.h:1748-1825) for one region mask: over pixels with mask == 255, an error
 * is DP < 0 or |DT - DP| > thres; *pbm = errors / count, *rms = sqrt(sum / count) where the float
 * sum adds pow(dif, 2) per valid pixel and 2 per invalid one, in raster order (host code, exact
 * reference arithmetic).  Host pointers; rows x cols, packed. */
SM_API sm_status sm_cal_err(const int16_t* disp, const float* gt, const uint8_t* mask, int32_t rows, int32_t cols,
                            float thres, float* pbm, float* rms);

/* Diagnostics used by the parity tests. */
SM_API float sm_expf_host(float x);   /* the device expf algorithm, evaluated on the host */
/* Device expf over the float bit patterns [first_bits, first_bits + n) into host out[n]. */
SM_API sm_status sm_expf_device_range(sm_ctx* ctx, uint32_t first_bits, uint32_t n, float* out);
SM_API sm_status sm_get_census(sm_ctx* ctx, int32_t view, uint64_t* dst); /* H*W*2 words */
/* CBCA's area division (div_area, sm_device.h) against IEEE division on the device: every
 * dividend mantissa at binary exponent `exp2` (a in [2^exp2, 2^(exp2+1))) for every divisor
 * 1 <= b <= bmax; *mismatches receives the number of differing results. */
SM_API sm_status sm_div_area_check(sm_ctx* ctx, int32_t exp2, int32_t bmax, uint64_t* mismatches);
/* Measured HBM ceiling: a dwordx4 copy between two fresh device buffers of `bytes`
 * each (rounded down to 16 KiB) on the ctx's device and stream, at three grid sizes, `reps` timed
 * launches each; GB/s counts read + write bytes.  Best and median over the samples. */
SM_API sm_status sm_copy_ceiling(sm_ctx* ctx, uint64_t bytes, int32_t reps, double* best_gbs, double* median_gbs);

#ifdef __cplusplus
}
#endif
#endif /* SM_CAPI_H */
