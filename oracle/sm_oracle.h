/*
 * sm_oracle.h — CPU restatement of the reference's census/CBCA/SGM/WTA hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (mystereomatching_amd/, include/)
 * links, loads or calls this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg do, and only as the checker / the CPU baseline.
 *
 * PARITY UNPINNED: the reference (xinge456/myStereoMatching, mounted at /root/reference)
 * cannot be built here (needs OpenCV + opencv_contrib/ximgproc + a missing util.h + MSVC-only
 * constructs) and it ships no tests, fixtures or golden vectors.
 * This restatement follows the reference source line by line (citations per function in
 * sm_oracle.c) and is cross-checked against an independent pure-Python restatement
 * (tests/pyref.py) on small inputs; it is not pinned to outputs of the reference binary.
 *
 * Every function is single-threaded, compiled -O2 -ffp-contract=off -fno-fast-math so that
 * each float operation rounds exactly as the reference's scalar C++ does.
 */
#ifndef SM_ORACLE_H
#define SM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { SMO_COST_CENSUS_GRAD = 0, SMO_COST_CENSUS = 1, SMO_COST_AD_CENSUS = 2, SMO_COST_AD = 3 };

typedef struct smo_config {
    int H, W, D;                 /* D = numDisparities = maxdisp + 1 (h:209) */
    int cost_method;             /* SMO_COST_*; default censusGrad (main:15) */
    int census_rv, census_ru;    /* census window radii {3,4} (cpp:815) */
    int census_ring;             /* censusFunc == 3: 8 ring bits (h:244, h:910-928) */
    float lam_cen, lam_g;        /* 13, 1 (main:56-57, cpp:38-39) */
    float grad_trunc;            /* 500 (cpp:34) */
    int grad_adaptive;           /* gradFuse_adpWgt = 1 (h:245) */
    float lam_ad, lam_cen_adc;   /* ADCensus fusion 10, 30 (cpp:5270) */
    float ad_trunc_adc;          /* ADCensus AD trunc 1000 (cpp:905) */
    float ad_trunc_ad;           /* "AD" cost trunc 20 (cpp:955) */
    int arm_L, arm_L_out;        /* cbca_crossL[0]=17, cbca_crossL_out[0]=34 (h:263,266) */
    int arm_cT, arm_cT_out;      /* cbca_cTresh[0]=20, cbca_cTresh_out[0]=6 (h:269,272) */
    int arm_minL;                /* cbca_minArmL = 1 (h:259) */
    int aggregation;             /* 0 none, 1 CBCA (main:16), 2 GF (MY_GUIDE form), 3 NL */
    int cbca_iters;              /* cbca_iterationNum = 2 (h:260) */
    int solve_all;               /* apply SolveAll(PY_LEV=1) (main:158) */
    float reg_lambda;            /* REG_LAMBDA = 0.3 (main:157) */
    int optimization;            /* 0 WTA only, 1 SGM (main:17), 2 "so" scan-line DP (cpp:1091-1105) */
    int sgm_paths;               /* 4 (cpp:6214); 8 = full direction table (cpp:6207-6208) */
    float sgm_p1, sgm_p2;        /* 1.0, 3.0 hard-coded in updateCost (h:2234-2235) */
    int sgm_cor_thres;           /* sgm_corDifThres = 15 (h:239) */
    int sgm_redu;                /* sgm_reduCoeffi1 = 4 (h:240) */
    /* refinement (refine(), cpp:1138-1511, non-USE_RECONCV branch cpp:1347-1510) */
    int do_refine;               /* Do_refine (h:70; default 0): both views through CBCA/SGM + refine() */
    float lr_max_diff;           /* LRmaxDiff = 0 (h:212) */
    int do_region_vote;          /* Do_regionVote = 1 (h:75) */
    int region_vote_nums;        /* region_vote_nums = 2 (h:306) */
    float rv_ratio;              /* rv_ratio[i] = 0.4 (cpp:1400) */
    int rv_s;                    /* rv_s[i] = 20 (cpp:1401) */
    int do_proper_ipol;          /* Do_properIpol = 1 (h:76) */
    int disp_occ;                /* DISP_OCC = -2 * 16 (h:216) */
    int do_last_median;          /* Do_lastMedianBlur = 1 (h:80) */
    /* alternative aggregators (sm_oracle_agg.c): aggregation 2 = "GF", 3 = "NL" */
    int gf_r;                    /* gf_r[0] = 9 (h:297) */
    float gf_eps;                /* gf_eps[0] = 0.0001 (h:298) */
    double nl_sigma;             /* NLCCA::aggreCV sigma = 0.1 (NL/NLCCA.cpp:33) */
    int gf_mode;                 /* 0: ximgproc::guidedFilter (cpp:4513, the shipped build), 1: MY_GUIDE (cpp:4509) */
} smo_config;

void smo_default_config(smo_config* c, int maxdisp, int H, int W);

/* sm_oracle_agg.c */
void smo_box_filter(int H, int W, int r, const float* src, float* dst, float* tmp);
int smo_guided_filter(const smo_config* c, float* vm, const uint8_t* bgr);   /* dispatches on gf_mode */
int smo_guided_filter_my(const smo_config* c, float* vm, const uint8_t* bgr);
int smo_guided_filter_cv(const smo_config* c, float* vm, const uint8_t* bgr);
/* OpenCV boxFilter(src, dst, CV_32F, (2r+1)^2, normalize, BORDER_REFLECT) of a float image (ximgproc's
 * meanFilter): RowSum<float, double> then ColumnSum<double, float>.  rs: H*W doubles of scratch. */
void smo_box_filter_cv(int H, int W, int r, const float* src, float* dst, double* rs);
/* OpenCV borderInterpolate(BORDER_REFLECT). */
int smo_reflect(int p, int len);
void smo_nl_median3(int H, int W, const uint8_t* src, uint8_t* dst);
int smo_nl_tree(int H, int W, const uint8_t* bgr, int* order, int* parent, uint8_t* weight, int* nchild, int* child);
void smo_nl_table(double sigma, double* table);
void smo_nl_filter(int n, int P, const int* order, const int* parent, const uint8_t* weight, const int* nchild,
                   const int* child, const double* table, double* cost, double* backup);
int smo_nl_aggregate(const smo_config* c, float* vm, const uint8_t* bgrL);

/* OpenCV borderInterpolate(BORDER_REFLECT_101). */
int smo_reflect101(int p, int len);

int smo_census_nwords(const smo_config* c);
void smo_census(const smo_config* c, const uint8_t* gray, uint64_t* codes);
void smo_grad_x(int H, int W, const uint8_t* gray, float* g);
void smo_grad_y(int H, int W, const uint8_t* gray, float* g);
void smo_arms(const smo_config* c, const uint8_t* bgr, uint16_t* arms /* H*W*4 */);

/* Cost volume for one view (0 = left reference, 1 = right), H*W*D floats. */
void smo_cost_volume(const smo_config* c, const uint8_t* bgrL, const uint8_t* bgrR,
                     const uint8_t* grayL, const uint8_t* grayR, int view, float* vm);
/* view 0: intersection min(armsL(u), armsR(u-d)); view 1: min(armsL(u+d), armsR(u)) (cpp:2794-2845) */
void smo_cbca(const smo_config* c, float* vm, const uint16_t* armsL, const uint16_t* armsR);
void smo_cbca_view(const smo_config* c, float* vm, const uint16_t* armsL, const uint16_t* armsR, int view);
float smo_solve_all_weight(float reg_lambda);
void smo_solve_all(const smo_config* c, float* vm);
void smo_sgm(const smo_config* c, float* vm, const uint8_t* bgrL);
void smo_wta(const smo_config* c, const float* vm, int16_t* disp);
/* so (cpp:6272-6394): per-row left-to-right DP with trace, then backtracking; vm is updated in
 * place (accumulated), DP written directly.  Ic is I[0] = the LEFT colour image for both views
 * (dispOptimize passes I_c and so() reads I[0] only, cpp:1098, 6284). */
void smo_so(const smo_config* c, float* vm, int16_t* disp, const uint8_t* Ic);

/* refine() stages (cpp:1364-1506); all act in place on an H*W int16 map. */
void smo_lr_check(const smo_config* c, int16_t* disp0, const int16_t* disp1);          /* cpp:2262-2282 */
void smo_region_vote(const smo_config* c, int16_t* disp, const uint16_t* armsL,
                     float rv_ratio, int rv_s);                                      /* cpp:7219-7277 */
void smo_proper_ipol(const smo_config* c, int16_t* disp, const uint8_t* bgrL);        /* cpp:7395-7490 */
void smo_median3(int H, int W, int16_t* disp);                                        /* cv::medianBlur(.,.,3) */
void smo_refine(const smo_config* c, int16_t* disp0, const int16_t* disp1, const uint16_t* armsL,
                const uint8_t* bgrL);                                                  /* cpp:1347-1510 */

/* Optional intermediate outputs of smo_run_ex (any may be NULL). */
typedef struct smo_dumps {
    float* vol_cost;             /* vm[0] after the cost stage */
    float* vol_agg;              /* vm[0] after CBCA */
    float* vol_final;            /* vm[0] after the SGM path sum */
    float* vol_right;            /* vm[1] cost volume */
    float* vol_agg_right;        /* vm[1] after CBCA (do_refine) */
    int16_t* disp_left_raw;      /* DP[0] after WTA, before refine() (do_refine) */
    int16_t* disp_right;         /* DP[1] after WTA (do_refine) */
    double* stage_ms;            /* [7]: cost, cbca, solveall, sgm, wta, refine, total */
} smo_dumps;
int smo_run_ex(const smo_config* c, const uint8_t* bgrL, const uint8_t* bgrR,
               const uint8_t* grayL, const uint8_t* grayR, int16_t* disp, const smo_dumps* d);

/* Cross-scale pyramid (main:131-158, SolveAll cpp:2142-2208 with PY_LVL > 1).
 * cv::pyrDown for u8 images (BORDER_REFLECT_101): dst is ((rows+1)/2) x ((cols+1)/2),
 * dst = (sum_ij k_i k_j src(2y+i-2, 2x+j-2) + 128) >> 8 with k = {1, 4, 6, 4, 1}. */
void smo_pyr_down_u8(const uint8_t* src, int rows, int cols, int channels, uint8_t* dst);
#define SMO_MAX_PYR 8
/* invWgt[s] = regInv(0, s) of SolveAll's regularisation matrix (cpp:2147-2167), OpenCV's float
 * Mat::inv: the small-matrix path (n <= 3), LUImpl<float> above.  Returns 0, or -1 for PY_LVL
 * outside [1, SMO_MAX_PYR] or a singular matrix. */
int smo_pyr_weights(int py_lvl, float reg_lambda, float* w);
/* SolveAll's cross-scale sum for one view: vms[s] is level s's volume (cfgs[s] its shape);
 * vms[0] receives sum_s invWgt[s] * vm_s(y >> s, x >> s, d_s) with d_s = (d_{s-1} + 1) / 2. */
int smo_solve_all_pyr(const smo_config* cfgs, float* const* vms, int py_lvl, float reg_lambda);
/* main:131-166 with PY_LEV levels: per-level images by pyrDown, per-level Parameters
 * (maxdisp_{p+1} = maxdisp_p / 2 + 1, disSc = 2^p: arm lengths L / disSc, L_out / disSc,
 * cpp:5369-5371), costCalculate per level, SolveAll(PY_LEV), dispOptimize [+ refine] at level 0. */
int smo_run_pyr(const smo_config* c0, int py_lvl, const uint8_t* bgrL, const uint8_t* bgrR,
                const uint8_t* grayL, const uint8_t* grayR, int16_t* disp);

/* Whole default pipeline for one pair (main:138-163 call order).  Optional dumps may be NULL:
 * vol_cost = vm[0] after the cost stage, vol_agg = after CBCA, vol_final = after SGM sum,
 * vol_right = vm[1] cost volume.  stage_ms[6] (optional): cost, cbca, solveall, sgm, wta, total.
 * Returns 0 on success, -1 on bad config / allocation failure. */
int smo_run(const smo_config* c, const uint8_t* bgrL, const uint8_t* bgrR,
            const uint8_t* grayL, const uint8_t* grayR, int16_t* disp,
            float* vol_cost, float* vol_agg, float* vol_final, float* vol_right,
            double* stage_ms);

/* bad-t evaluator (h:1748-1825): returns PBM; rms_out optional. */
float smo_bad_ratio(int H, int W, const int16_t* disp, const float* gt, const uint8_t* mask,
                    float thres, float* rms_out);

/* libm expf over float bit patterns [first, first+n). */
void smo_expf_range(uint32_t first, uint32_t n, float* out);

#ifdef __cplusplus
}
#endif
#endif
