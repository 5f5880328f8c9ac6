/*
 * sm_oracle.c — CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * PARITY UNPINNED — see sm_oracle.h.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product never does.
 *
 * Each function cites the reference lines (relative to /root/reference/) it restates.
 * "h" = stereoMatching.h, "cpp" = stereoMatching.cpp, "main" = main_.cpp.
 * Memory-lean but op-order-identical: the h×w×D×5 arm-intersection tensor of
 * genTrueHorVerArms (cpp:2794-2845) is evaluated on the fly (it is a pure min of two
 * arm records), and SGM path volumes are accumulated in path order as gen_sgm_vm does.
 */
#include "sm_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* std::min(a, b) == (b < a) ? b : a */
static inline float fminstd(float a, float b) { return (b < a) ? b : a; }
static inline int imin(int a, int b) { return b < a ? b : a; }
static inline int imax(int a, int b) { return a < b ? b : a; }

void smo_default_config(smo_config* c, int maxdisp, int H, int W) {
    memset(c, 0, sizeof(*c));
    c->H = H;
    c->W = W;
    c->D = maxdisp + 1;          /* Parameters: numDisparities = maxDisp + 1 (h:209) */
    c->cost_method = SMO_COST_CENSUS_GRAD;
    c->census_rv = 3;            /* census_W[0] = {3, 4} (cpp:815) */
    c->census_ru = 4;
    c->census_ring = 1;          /* censusFunc = 3 (h:244) */
    c->lam_cen = 13.0f;          /* lamCen (main:57) */
    c->lam_g = 1.0f;             /* lamG (main:56) */
    c->grad_trunc = 500.0f;      /* grad(gradVm, 500) (cpp:34) */
    c->grad_adaptive = 1;        /* gradFuse_adpWgt (h:245) */
    c->lam_ad = 10.0f;           /* gen_vm_from2vm_exp(..., 10, 30) (cpp:5270) */
    c->lam_cen_adc = 30.0f;
    c->ad_trunc_adc = 1000.0f;   /* asdCal(vm_asd, "AD", imgNum, 1000) (cpp:905) */
    c->ad_trunc_ad = 20.0f;      /* asdCal(vm, costcalculation, imgNum, 20) (cpp:955) */
    c->arm_L = 17;               /* cbca_crossL[0] (h:263) */
    c->arm_L_out = 34;           /* cbca_crossL_out[0] (h:266) */
    c->arm_cT = 20;              /* cbca_cTresh[0] (h:269) */
    c->arm_cT_out = 6;           /* cbca_cTresh_out[0] (h:272) */
    c->arm_minL = 1;             /* cbca_minArmL (h:259) */
    c->aggregation = 1;          /* "CBCA" (main:16) */
    c->cbca_iters = 2;           /* cbca_iterationNum (h:260) */
    c->solve_all = 1;            /* SolveAll(smPsy, 1, 0.3f) (main:157-158) */
    c->reg_lambda = 0.3f;
    c->optimization = 1;         /* "sgm" (main:17) */
    c->sgm_paths = 4;            /* numOfDirec = 4 (cpp:6214) */
    c->sgm_p1 = 1.0f;            /* updateCost P1 (h:2234) */
    c->sgm_p2 = 3.0f;            /* updateCost P2 (h:2235) */
    c->sgm_cor_thres = 15;       /* sgm_corDifThres (h:239) */
    c->sgm_redu = 4;             /* sgm_reduCoeffi1 (h:240) */
    c->do_refine = 0;            /* Do_refine (h:70) */
    c->lr_max_diff = 0.0f;       /* LRmaxDiff (h:212) */
    c->do_region_vote = 1;       /* Do_regionVote (h:75) */
    c->region_vote_nums = 2;     /* region_vote_nums (h:306) */
    c->rv_ratio = 0.4f;          /* rv_ratio[] (cpp:1400) */
    c->rv_s = 20;                /* rv_s[] (cpp:1401) */
    c->do_proper_ipol = 1;       /* Do_properIpol (h:76) */
    c->disp_occ = -2 * 16;       /* DISP_OCC (h:216) */
    c->do_last_median = 1;       /* Do_lastMedianBlur (h:80) */
    c->gf_r = 9;                 /* gf_r[0] = 9, gf_eps[0] = 0.0001 (h:297-298) */
    c->gf_eps = 0.0001f;
    c->gf_mode = 0;              /* `//#define MY_GUIDE` (h:38): the shipped build calls ximgproc::guidedFilter */
    c->nl_sigma = 0.1;           /* NLCCA::aggreCV (NL/NLCCA.cpp:33) */
}

/* OpenCV borderInterpolate, BORDER_REFLECT_101 (used by copyMakeBorder, h:870-871). */
int smo_reflect101(int p, int len) {
    if (len == 1) return 0;
    do {
        if (p < 0)
            p = -p;
        else
            p = 2 * len - p - 2;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

int smo_census_nwords(const smo_config* c) {
    /* codeLength (cpp:829-831), varNum = ceil(codeLength / 64.) (cpp:832) */
    int len = (2 * c->census_rv + 1) * (2 * c->census_ru + 1) + (c->census_ring ? 8 : 0);
    return (len + 63) / 64;
}

static int census_length(const smo_config* c) {
    return (2 * c->census_rv + 1) * (2 * c->census_ru + 1) + (c->census_ring ? 8 : 0);
}

/* genCensusCode_NC_Sur (h:867-934) on one gray image; censusFunc == 0 (genCensusCode,
 * h:634-688) is the same loop without the ring bits.  Bits are shifted in MSB-first; a word
 * is flushed when `step > 63` before the next bit (h:895-901, 916-922). */
void smo_census(const smo_config* c, const uint8_t* I, uint64_t* codes) {
    const int H = c->H, W = c->W, RV = c->census_rv, RU = c->census_ru;
    const int nw = smo_census_nwords(c);
    static const int dv_sur[9] = {-1, -1, -1, 0, 1, 1, 1, 0, -1};  /* h:873 */
    static const int du_sur[9] = {-1, 0, 1, 1, 1, 0, -1, -1, -1};  /* h:874 */
    for (int v = 0; v < H; v++) {
        for (int u = 0; u < W; u++) {
            uint64_t* censP = codes + ((size_t)v * W + u) * nw;
            for (int k = 0; k < nw; k++) censP[k] = 0;
            int center = I[(size_t)v * W + u];
            uint64_t cs = 0;
            int step = 0, dep = 0;
            for (int dv = -RV; dv <= RV; dv++) {
                int vv = smo_reflect101(v + dv, H);
                for (int du = -RU; du <= RU; du++) {
                    int uu = smo_reflect101(u + du, W);
                    if (step > 63) {
                        censP[dep] = cs;
                        cs = 0;
                        step = 0;
                        dep++;
                    }
                    cs <<= 1;
                    if (center - (int)I[(size_t)vv * W + uu] < 0) cs++;  /* h:903 */
                    step++;
                }
            }
            if (c->census_ring) {
                for (int i = 0; i < 8; i++) {
                    int pv = smo_reflect101(v + dv_sur[i], H), pu = smo_reflect101(u + du_sur[i], W);
                    int av = smo_reflect101(v + dv_sur[i + 1], H), au = smo_reflect101(u + du_sur[i + 1], W);
                    if (step > 63) {
                        censP[dep] = cs;
                        cs = 0;
                        step = 0;
                        dep++;
                    }
                    cs <<= 1;
                    if ((int)I[(size_t)pv * W + pu] - (int)I[(size_t)av * W + au] < 0) cs++;  /* h:924 */
                    step++;
                }
            }
            if (step > 0) censP[dep] = cs;
        }
    }
}

/* calGrad, single-channel branch (cpp:271-287): gx = 0.5*(I[u+1]-I[u-1]); edges full diff. */
void smo_grad_x(int H, int W, const uint8_t* I, float* g) {
    for (int v = 0; v < H; v++) {
        const uint8_t* iP = I + (size_t)v * W;
        float* gP = g + (size_t)v * W;
        for (int u = 1; u < W - 1; u++) gP[u] = (float)(0.5 * (iP[u + 1] - iP[u - 1]));
        gP[0] = (float)(iP[1] - iP[0]);
        gP[W - 1] = (float)(iP[W - 1] - iP[W - 2]);
    }
}

/* calGrad_y, single-channel branch (cpp:320-350). */
void smo_grad_y(int H, int W, const uint8_t* I, float* g) {
    for (int v = 1; v < H - 1; v++)
        for (int u = 0; u < W; u++)
            g[(size_t)v * W + u] = (float)(0.5 * (I[(size_t)(v + 1) * W + u] - I[(size_t)(v - 1) * W + u]));
    for (int u = 0; u < W; u++) g[u] = (float)(I[(size_t)W + u] - I[u]);
    for (int u = 0; u < W; u++)
        g[(size_t)(H - 1) * W + u] = (float)(I[(size_t)(H - 1) * W + u] - I[(size_t)(H - 2) * W + u]);
}

/* judgeColorDif (cpp:2847-2856) on 3-channel u8 pixels. */
static inline int color_ok(const uint8_t* a, const uint8_t* b, int thres) {
    for (int ch = 0; ch < 3; ch++)
        if (abs((int)a[ch] - (int)b[ch]) > thres) return 0;
    return 1;
}

/* calHorVerDis, 7-argument overload (cpp:2959-3050) with the arguments calArms passes
 * (cpp:5371: L, L_out, cTresh, cTresh_out, minL).  Direction order L, R, U, D (cpp:2978-2998). */
void smo_arms(const smo_config* c, const uint8_t* I, uint16_t* arms) {
    const int h = c->H, w = c->W;
    const int L = c->arm_L, L_out = c->arm_L_out, C_D = c->arm_cT, C_D_out = c->arm_cT_out;
    const int minL = c->arm_minL;
    const int dus[4] = {-1, 1, 0, 0}, dvs[4] = {0, 0, -1, 1};
    for (int direc = 0; direc < 4; direc++) {
        const int du = dus[direc], dv = dvs[direc];
        for (int v = 0; v < h; v++) {
            for (int u = 0; u < w; u++) {
                const uint8_t* IPtr = I + ((size_t)v * w + u) * 3;
                int arm = 1;
                for (; arm <= L_out; arm++) {
                    int v_arm = v + arm * dv, u_arm = u + arm * du;
                    if (v_arm < 0 || v_arm >= h || u_arm < 0 || u_arm >= w) break;
                    const uint8_t* armPtr = I + ((size_t)v_arm * w + u_arm) * 3;
                    const uint8_t* armPrePtr = I + ((size_t)(v + (arm - 1) * dv) * w + (u + (arm - 1) * du)) * 3;
                    int nb = color_ok(armPtr, armPrePtr, C_D);
                    int ip = arm <= L ? color_ok(IPtr, armPtr, C_D) : color_ok(IPtr, armPtr, C_D_out);
                    if (!nb || !ip) break;
                }
                uint16_t out = 0;
                if (--arm >= minL)
                    out = (uint16_t)arm;
                else {
                    for (int len = minL; len >= 0; len--) {
                        if (u + len * du >= 0 && u + len * du <= w - 1 && v + len * dv >= 0 && v + len * dv <= h - 1) {
                            out = (uint16_t)len;
                            break;
                        }
                    }
                }
                arms[((size_t)v * w + u) * 4 + direc] = out;
            }
        }
    }
}

/* gen_cenVM_XOR (h:936-981) for one view: lp = u + d*left, rp = u - d*right. */
static void census_volume(const smo_config* c, const uint64_t* codeL, const uint64_t* codeR, int view, float* vm) {
    const int H = c->H, W = c->W, D = c->D, nw = smo_census_nwords(c);
    const float DEFAULT = (float)census_length(c) * 1.0f;  /* codeLength * truncRat (h:938) */
    const int lc = view == 1 ? 1 : 0, rc = view == 1 ? 0 : 1;
    for (int v = 0; v < H; v++)
        for (int u = 0; u < W; u++) {
            float* cP = vm + ((size_t)v * W + u) * D;
            for (int d = 0; d < D; d++) {
                int lp = u + d * lc, rp = u - d * rc;
                if (lp >= W || rp < 0)
                    cP[d] = DEFAULT;
                else {
                    float cost = 0;
                    for (int k = 0; k < nw; k++)
                        cost += (float)__builtin_popcountll(codeL[((size_t)v * W + lp) * nw + k] ^ codeR[((size_t)v * W + rp) * nw + k]);
                    cP[d] = fminstd(cost, DEFAULT);
                }
            }
        }
}

/* calgradvm (cpp:388-455) for one view, arms = HVL[view]. */
static void grad_volume(const smo_config* c, const float* gx0, const float* gx1, const float* gy0, const float* gy1,
                        const uint16_t* arms, int view, float* vm) {
    const int H = c->H, W = c->W, n = c->D;
    const float Trunc = c->grad_trunc;
    const int leftCoe = view == 1 ? 1 : 0, rightCoe = view == 1 ? 0 : -1;
    const float oor = (float)sqrt(pow((double)Trunc, 2) * 2);  /* sqrt(pow(Trunc, 2) * 2) (cpp:440) */
    for (int v = 0; v < H; v++)
        for (int u = 0; u < W; u++) {
            const uint16_t* arm = arms + ((size_t)v * W + u) * 4;
            float shortestH = 10000, shortestV = 10000;
            for (int dir = 0; dir < 2; dir++)
                if (arm[dir] < shortestH) shortestH = arm[dir];
            for (int dir = 2; dir < 4; dir++)
                if (arm[dir] < shortestV) shortestV = arm[dir];
            if (shortestH == 0) shortestH++;
            if (shortestV == 0) shortestV++;
            float a = shortestH / (shortestH + shortestV);
            float* vP = vm + ((size_t)v * W + u) * n;
            const float* g0 = gx0 + (size_t)v * W;
            const float* g1 = gx1 + (size_t)v * W;
            const float* y0 = gy0 + (size_t)v * W;
            const float* y1 = gy1 + (size_t)v * W;
            for (int d = 0; d < n; d++) {
                int u0 = u + leftCoe * d, u1 = u + rightCoe * d;
                if (u0 >= W || u1 < 0)
                    vP[d] = oor;
                else if (c->grad_adaptive) {
                    float t1 = a * fminstd(fabsf(g0[u0] - g1[u1]), Trunc);
                    float t2 = (1 - a) * fminstd(fabsf(y0[u0] - y1[u1]), Trunc);
                    vP[d] = t1 + t2;
                } else {
                    vP[d] = fminstd(fabsf(g0[u0] - g1[u1]), Trunc) + fminstd(fabsf(y0[u0] - y1[u1]), Trunc);
                }
            }
        }
}

/* gen_ad_sd_vm, AD branch with 3 colour channels (cpp:2468-2509). */
static void ad_volume(const smo_config* c, const uint8_t* I0, const uint8_t* I1, int view, float trunc, float* vm) {
    const int H = c->H, W = c->W, n = c->D;
    const int lc = view == 1 ? 1 : 0, rc = view == 1 ? 0 : -1;
    for (int v = 0; v < H; v++)
        for (int u = 0; u < W; u++) {
            float* vP = vm + ((size_t)v * W + u) * n;
            for (int d = 0; d < n; d++) {
                int uL = u + d * lc, uR = u + d * rc;
                if (uL >= W || uR < 0)
                    vP[d] = trunc;
                else {
                    const uint8_t* l = I0 + ((size_t)v * W + uL) * 3;
                    const uint8_t* r = I1 + ((size_t)v * W + uR) * 3;
                    float sum = 0;
                    for (int ch = 0; ch < 3; ch++) sum = (float)((double)sum + pow(fabsf((float)l[ch] - (float)r[ch]), 1));
                    vP[d] = fminstd(sum / 3, trunc);
                }
            }
        }
}

/* gen_vm_from2vm_exp (cpp:3566-3590): out = 2 - exp(-vm0/ARU0) - exp(-vm1/ARU1). */
static void fuse_exp(size_t n, const float* vm0, const float* vm1, float aru0, float aru1, float* out) {
    for (size_t i = 0; i < n; i++) out[i] = 2 - expf(-vm0[i] / aru0) - expf(-vm1[i] / aru1);
}

void smo_cost_volume(const smo_config* c, const uint8_t* bgrL, const uint8_t* bgrR,
                     const uint8_t* grayL, const uint8_t* grayR, int view, float* vm) {
    const int H = c->H, W = c->W;
    const size_t npix = (size_t)H * W, nvol = npix * c->D;
    if (c->cost_method == SMO_COST_AD) {           /* asdCal "AD" (cpp:954-955) */
        ad_volume(c, bgrL, bgrR, view, c->ad_trunc_ad, vm);
        return;
    }
    const int nw = smo_census_nwords(c);
    uint64_t* cL = (uint64_t*)malloc(npix * nw * 8);
    uint64_t* cR = (uint64_t*)malloc(npix * nw * 8);
    smo_census(c, grayL, cL);                      /* censusCal (cpp:856-872) */
    smo_census(c, grayR, cR);
    if (c->cost_method == SMO_COST_CENSUS) {       /* costcalculation "Census" (cpp:975-976) */
        census_volume(c, cL, cR, view, vm);
    } else if (c->cost_method == SMO_COST_AD_CENSUS) {  /* ADCensusCal (cpp:894-915) */
        float* ad = (float*)malloc(nvol * 4);
        float* cen = (float*)malloc(nvol * 4);
        ad_volume(c, bgrL, bgrR, view, c->ad_trunc_adc, ad);
        census_volume(c, cL, cR, view, cen);
        fuse_exp(nvol, ad, cen, c->lam_ad, c->lam_cen_adc, vm);   /* adCensus (cpp:5270) */
        free(ad);
        free(cen);
    } else {                                       /* censusGrad (cpp:25-48) */
        float* gx0 = (float*)malloc(npix * 4);
        float* gx1 = (float*)malloc(npix * 4);
        float* gy0 = (float*)malloc(npix * 4);
        float* gy1 = (float*)malloc(npix * 4);
        uint16_t* arms = (uint16_t*)malloc(npix * 8);
        smo_grad_x(H, W, grayL, gx0);
        smo_grad_x(H, W, grayR, gx1);
        smo_grad_y(H, W, grayL, gy0);
        smo_grad_y(H, W, grayR, gy1);
        smo_arms(c, view == 1 ? bgrR : bgrL, arms);  /* HVL[num] of that view (cpp:403) */
        float* gv = (float*)malloc(nvol * 4);
        float* cv = (float*)malloc(nvol * 4);
        grad_volume(c, gx0, gx1, gy0, gy1, arms, view, gv);
        census_volume(c, cL, cR, view, cv);
        fuse_exp(nvol, cv, gv, c->lam_cen, c->lam_g, vm);        /* cpp:40-43 */
        free(gv);
        free(cv);
        free(gx0);
        free(gx1);
        free(gy0);
        free(gy1);
        free(arms);
    }
    free(cL);
    free(cR);
}

/* HVL_INTERSECTION[num] element k at (v,u,d) — genTrueHorVerArms (cpp:2794-2845):
 * num 0 (left view):  u_l = u,     u_r = u - d;
 * num 1 (right view): u_l = u + d, u_r = u;
 * value min(HVL[0](v,u_l)[k], HVL[1](v,u_r)[k]); zero (memset, cpp:2799-2800) once u_r < 0 or
 * u_l >= w (the d loop breaks, cpp:2821-2822). */
static inline int isect(const uint16_t* aL, const uint16_t* aR, int W, int v, int u, int d, int k, int view) {
    const int ul = view ? u + d : u, ur = view ? u : u - d;
    if (ur < 0 || ul >= W) return 0;
    int a = aL[((size_t)v * W + ul) * 4 + k], b = aR[((size_t)v * W + ur) * 4 + k];
    return imin(a, b);
}

/* gen1DCumu (cpp:3896-3926) with cbca_intersect = 1. */
static void cumu(const smo_config* c, float* vm, int32_t* area, int dv, int du) {
    const int H = c->H, W = c->W, n = c->D;
    for (int v = 0; v < H; v++)
        for (int u = 0; u < W; u++) {
            int vPre = v + dv, uPre = u + du;
            int inner = (vPre >= 0 && vPre < H && uPre >= 0 && uPre < W);
            if (!inner) continue;
            float* p = vm + ((size_t)v * W + u) * n;
            const float* q = vm + ((size_t)vPre * W + uPre) * n;
            int32_t* a = area + ((size_t)v * W + u) * n;
            const int32_t* b = area + ((size_t)vPre * W + uPre) * n;
            for (int d = 0; d < n; d++) {
                p[d] += q[d];
                a[d] += b[d];
            }
        }
}

/* cal1DCost (h:1643-1715) with cbca_intersect = 1; writes temps then copies back. */
static void cost1d(const smo_config* c, float* vm, int32_t* area, float* vmT, int32_t* areaT,
                   const uint16_t* aL, const uint16_t* aR, int dv, int du, int direc, int view) {
    const int H = c->H, W = c->W, n = c->D;
    const int head_num = direc * 2 + 1, tail_num = direc * 2;
    for (int v = 0; v < H; v++)
        for (int u = 0; u < W; u++) {
            float* vT = vmT + ((size_t)v * W + u) * n;
            int32_t* aT = areaT + ((size_t)v * W + u) * n;
            for (int d = 0; d < n; d++) {
                int tailL = isect(aL, aR, W, v, u, d, tail_num, view), headL = isect(aL, aR, W, v, u, d, head_num, view);
                int tail_u = u + du * tailL, tail_v = v + dv * tailL;
                int head_u = u - du * headL, head_v = v - dv * headL;
                int pre_tailU = tail_u + du, pre_tailV = tail_v + dv;
                int inner = (pre_tailU >= 0 && pre_tailU < W && pre_tailV >= 0 && pre_tailV < H);
                size_t hi = ((size_t)head_v * W + head_u) * n + d;
                size_t ti = ((size_t)pre_tailV * W + pre_tailU) * n + d;
                if (inner) {
                    aT[d] = area[hi] - area[ti];
                    vT[d] = vm[hi] - vm[ti];
                } else {
                    aT[d] = area[hi];
                    vT[d] = vm[hi];
                }
            }
        }
    memcpy(vm, vmT, (size_t)H * W * n * 4);
    memcpy(area, areaT, (size_t)H * W * n * 4);
}

/* cbca_core (cpp:5585-5666) for one LOR (imgNum = Do_refine && Do_LRConsis ? 2 : 1). */
void smo_cbca(const smo_config* c, float* vm, const uint16_t* aL, const uint16_t* aR) { smo_cbca_view(c, vm, aL, aR, 0); }

void smo_cbca_view(const smo_config* c, float* vm, const uint16_t* aL, const uint16_t* aR, int view) {
    const size_t nvol = (size_t)c->H * c->W * c->D;
    const int du[2] = {-1, 0}, dv[2] = {0, -1};
    int32_t* area = (int32_t*)malloc(nvol * 4);
    int32_t* areaT = (int32_t*)malloc(nvol * 4);
    float* vmT = (float*)malloc(nvol * 4);
    for (int it = 0; it < c->cbca_iters; it++) {
        for (size_t i = 0; i < nvol; i++) area[i] = 1;  /* Scalar::all(1) (cpp:5604) */
        if (it % 2 == 0) {
            cumu(c, vm, area, dv[0], du[0]);
            cost1d(c, vm, area, vmT, areaT, aL, aR, dv[0], du[0], 0, view);
            cumu(c, vm, area, dv[1], du[1]);
            cost1d(c, vm, area, vmT, areaT, aL, aR, dv[1], du[1], 1, view);
        } else {
            cumu(c, vm, area, dv[1], du[1]);
            cost1d(c, vm, area, vmT, areaT, aL, aR, dv[1], du[1], 1, view);
            cumu(c, vm, area, dv[0], du[0]);
            cost1d(c, vm, area, vmT, areaT, aL, aR, dv[0], du[0], 0, view);
        }
        for (size_t i = 0; i < nvol; i++) vm[i] /= area[i];  /* genfinalVm_cbca (cpp:3969-3992) */
    }
    free(area);
    free(areaT);
    free(vmT);
}

/* SolveAll (cpp:2142-2208) with PY_LVL = 1: regMat = [1 + REG_LAMBDA]; OpenCV's 1×1 float
 * invert computes (float)(1. / (double)m). */
float smo_solve_all_weight(float reg_lambda) {
    float m = 1 + reg_lambda;
    return (float)(1. / (double)m);
}

void smo_solve_all(const smo_config* c, float* vm) {
    const size_t nvol = (size_t)c->H * c->W * c->D;
    const float w = smo_solve_all_weight(c->reg_lambda);
    for (size_t i = 0; i < nvol; i++) {
        float sum = 0;
        sum += w * vm[i];
        vm[i] = sum;
    }
}

/* updateCost<float> (h:2206-2280) for one pixel.  D1 compares I_c[0] when leftFirst, I_c[1]
 * otherwise (h:2219-2224): the caller passes that view's colour image.  D2 is computed there but
 * never used, so it is omitted. */
static void update_cost(const smo_config* c, float* Lr, const float* vm, const uint8_t* Ic, int v, int u,
                        int rv, int ru, int preIsInner) {
    const int W = c->W, n = c->D;
    const float* vmPtr = vm + ((size_t)v * W + u) * n;
    float* out = Lr + ((size_t)v * W + u) * n;
    if (!preIsInner) {
        for (int d = 0; d < n; d++) out[d] = vmPtr[d];
        return;
    }
    int D1 = 0;
    for (int ch = 0; ch < 3; ch++)
        D1 = imax(D1, abs((int)Ic[((size_t)v * W + u) * 3 + ch] - (int)Ic[((size_t)(v + rv) * W + (u + ru)) * 3 + ch]));
    const float* fore = Lr + ((size_t)(v + rv) * W + (u + ru)) * n;
    float minC = FLT_MAX;
    for (int d = 0; d < n; d++) minC = fminstd(fore[d], minC);
    for (int d = 0; d < n; d++) {
        float P1 = c->sgm_p1, P2 = c->sgm_p2;
        if (D1 > c->sgm_cor_thres) {
            P1 /= c->sgm_redu;
            P2 /= c->sgm_redu;
        }
        P1 -= minC;
        float cost = vmPtr[d];
        float S1 = fore[d] - minC;
        float S2 = d - 1 >= 0 ? fore[d - 1] + P1 : FLT_MAX;
        float S3 = d + 1 < n ? fore[d + 1] + P1 : FLT_MAX;
        float S4 = P2;
        out[d] = cost + fminstd(fminstd(S1, S2), fminstd(S3, S4));  /* min4 (h:2200-2203) */
    }
}

/* sgm (cpp:6204-6224) + costScan (cpp:1983-2029) + gen_sgm_vm (cpp:2031-2056).  Ic = I_c[0] for
 * vm[0] (leftFirst = true), I_c[1] for vm[1] (dispOptimize, cpp:1057-1059). */
void smo_sgm(const smo_config* c, float* vm, const uint8_t* Ic) {
    static const int RV[8] = {+1, -1, 0, 0, +1, +1, -1, -1};  /* cpp:6207 */
    static const int RU[8] = {0, 0, +1, -1, -1, +1, +1, -1};  /* cpp:6208 */
    const int h = c->H, w = c->W;
    const size_t nvol = (size_t)h * w * c->D;
    float* Lr = (float*)malloc(nvol * 4);
    float* acc = (float*)malloc(nvol * 4);
    for (size_t i = 0; i < nvol; i++) acc[i] = 0;
    for (int i = 0; i < c->sgm_paths; i++) {
        int rv = RV[i], ru = RU[i];
        int v0 = 0, v1 = h, u0 = 0, u1 = w, dv = +1, du = +1;
        if ((rv > 0) || (rv == 0 && ru > 0)) {
            v0 = h - 1; v1 = -1; u0 = w - 1; u1 = -1; dv = -1; du = -1;
        }
        for (int v = v0; v != v1; v += dv)
            for (int u = u0; u != u1; u += du) {
                int pre = !(v + rv > h - 1 || v + rv < 0 || u + ru > w - 1 || u + ru < 0);
                update_cost(c, Lr, vm, Ic, v, u, rv, ru, pre);
            }
        for (size_t k = 0; k < nvol; k++) acc[k] += Lr[k];  /* sum += Lr[num] in path order */
    }
    memcpy(vm, acc, nvol * 4);
    free(Lr);
    free(acc);
}

/* gen_dispFromVm (cpp:3928-3967), ChooseSmall = true. */
void smo_wta(const smo_config* c, const float* vm, int16_t* disp) {
    const int n = c->D;
    for (size_t p = 0; p < (size_t)c->H * c->W; p++) {
        float minC = FLT_MAX;
        int d_best = -1;
        const float* vP = vm + p * n;
        for (int d = 0; d < n; d++)
            if (minC > vP[d]) {
                minC = vP[d];
                d_best = d;
            }
        disp[p] = (int16_t)d_best;
    }
}

/* so (cpp:6272-6394). */
void smo_so(const smo_config* c, float* vm, int16_t* DP, const uint8_t* Ic) {
    const int h = c->H, w = c->W, D = c->D;
    int32_t* trace = (int32_t*)malloc((size_t)h * w * D * sizeof(int32_t));
    for (int v = 0; v < h; v++)
        for (int u = 1; u < w; u++) {
            const uint8_t* IP = Ic + ((size_t)v * w + u) * 3;
            const uint8_t* IPp = Ic + ((size_t)v * w + u - 1) * 3;
            float sum = 0;
            int L_isDisc = 0;
            for (int ch = 0; ch < 3; ch++) sum += abs((int)IP[ch] - (int)IPp[ch]);
            sum /= 3;
            if (sum > 15) L_isDisc = 1;
            float* vmP = vm + ((size_t)v * w + u) * D;
            const float* vmPre = vm + ((size_t)v * w + u - 1) * D;
            int32_t* traP = trace + ((size_t)v * w + u) * D;
            for (int d = 0; d < D; d++) {
                float Pn2 = 1.2f, Pn3 = 3.6f;   /* float Pn2 = 1.2; float Pn3 = 3.6; (cpp:6303-6304) */
                if (L_isDisc) {
                    Pn2 /= 2;
                    Pn3 /= 2;
                }
                float c_min = vmPre[0];
                float d_cMin = 0;
                for (int dl = 1; dl < D; dl++)
                    if (vmPre[dl] < c_min) {
                        c_min = vmPre[dl];
                        d_cMin = (float)dl;
                    }
                float c_minus = d > 0 ? vmPre[d - 1] + Pn2 : FLT_MAX;
                float c_plus = d < D - 1 ? vmPre[d + 1] + Pn2 : FLT_MAX;
                c_min += Pn3;
                int d_min = d;
                float cost_min = vmPre[d];
                if (c_minus < cost_min) {
                    d_min = d - 1;
                    cost_min = c_minus;
                }
                if (c_plus < cost_min) {
                    d_min = d + 1;
                    cost_min = c_plus;
                }
                if (c_min < cost_min) {
                    d_min = (int)d_cMin;
                    cost_min = c_min;
                }
                vmP[d] += cost_min;
                traP[d] = d_min;
            }
        }
    for (int v = 0; v < h; v++) {
        int16_t* disp = DP + (size_t)v * w;
        const float* cP = vm + ((size_t)v * w + w - 1) * D;
        float c_min = cP[0];
        int d_min = 0;
        for (int d = 1; d < D; d++)
            if (cP[d] < c_min) {
                c_min = cP[d];
                d_min = d;
            }
        disp[w - 1] = (int16_t)d_min;
        for (int u = w - 1; u > 0; u--) {
            const int d_pre = trace[((size_t)v * w + u) * D + d_min];
            disp[u - 1] = (int16_t)d_pre;
            d_min = d_pre;
        }
    }
    free(trace);
}

/* LRConsistencyCheck_normal (cpp:2262-2282), LOR = 0: a left disparity survives only if the
 * right map at u - d agrees within LRmaxDiff; otherwise -1. */
void smo_lr_check(const smo_config* c, int16_t* disp0, const int16_t* disp1) {
    const int H = c->H, W = c->W;
    for (int v = 0; v < H; v++) {
        int16_t* D1 = disp0 + (size_t)v * W;
        const int16_t* D2 = disp1 + (size_t)v * W;
        for (int u = 0; u < W; u++) {
            const int16_t d = D1[u];
            /* abs(int) > float: the int difference converts to float (exact for |x| < 2^24) */
            if (d < 0 || u - d < 0 || (float)abs(d - D2[u - d]) > c->lr_max_diff) D1[u] = -1;
        }
    }
}

/* regionVote_my (cpp:7219-7277): every invalid pixel collects the valid disparities of its
 * cross region (rows v-U..v+D of its own column, each row spanning that row's L/R arms at the
 * column, HVL[0]); with more than rv_s of them the most frequent one (first maximum) replaces it
 * when hist[most] / validNum >= rv_ratio — an INTEGER division (cpp:7270).  Reads Dp, writes a
 * copy (dp_res). */
void smo_region_vote(const smo_config* c, int16_t* disp, const uint16_t* armsL, float rv_ratio, int rv_s) {
    const int H = c->H, W = c->W, n = c->D;
    int16_t* res = (int16_t*)malloc((size_t)H * W * 2);
    int* hist = (int*)malloc((size_t)n * sizeof(int));
    memcpy(res, disp, (size_t)H * W * 2);
    for (int v = 0; v < H; v++)
        for (int u = 0; u < W; u++) {
            if (disp[(size_t)v * W + u] >= 0) continue;
            for (int d = 0; d < n; d++) hist[d] = 0;
            int validNum = 0;
            const uint16_t* a = armsL + ((size_t)v * W + u) * 4;
            const int v_begin = v - a[2], v_end = v + a[3];
            for (int vn = v_begin; vn <= v_end; vn++) {
                const uint16_t* an = armsL + ((size_t)vn * W + u) * 4;
                const int u_begin = u - an[0], u_end = u + an[1];
                const int16_t* dp = disp + (size_t)vn * W;
                for (int un = u_begin; un <= u_end; un++)
                    if (dp[un] >= 0) {
                        validNum++;
                        hist[dp[un]]++;
                    }
            }
            if (validNum <= rv_s) continue;
            int most = 0;
            for (int d = 1; d < n; d++)
                if (hist[d] > hist[most]) most = d;
            if ((float)(hist[most] / validNum) >= rv_ratio) res[(size_t)v * W + u] = (int16_t)most;
        }
    memcpy(disp, res, (size_t)H * W * 2);
    free(res);
    free(hist);
}

/* properIpol (cpp:7395-7490): each invalid pixel searches 16 directions up to 20 steps for the
 * first valid disparity (steps alternate pw/2 and pw - pw/2, C truncating division); DISP_OCC
 * pixels take the smallest found disparity, others the one whose colour (max channel |diff| of
 * I_c[0]) is closest, first strict minimum below 255.  Reads Dp, writes a copy. */
void smo_proper_ipol(const smo_config* c, int16_t* disp, const uint8_t* bgrL) {
    static const int DW[16] = {0, 2, 2, 2, 0, -2, -2, -2, 1, 2, 2, 1, -1, -2, -2, -1};
    static const int DH[16] = {2, 2, 0, -2, -2, -2, 0, 2, 2, 1, -1, -2, -2, -1, 1, 2};
    const int h = c->H, w = c->W, searchDepth = 20;
    int16_t* cp = (int16_t*)malloc((size_t)h * w * 2);
    for (int v = 0; v < h; v++)
        for (int u = 0; u < w; u++) {
            const int16_t dv = disp[(size_t)v * w + u];
            if (dv >= 0) {
                cp[(size_t)v * w + u] = dv;
                continue;
            }
            int dDisp[16], dDiff[16];
            for (int k = 0; k < 16; k++) {
                dDisp[k] = -1;
                dDiff[k] = -1;
                const int ph = DH[k], pw = DW[k];
                int posw = u, posh = v;
                for (int dep = 0; dep < searchDepth; dep++) {
                    if (dep % 2 == 0) {
                        posw += pw / 2;
                        posh += ph / 2;
                    } else {
                        posw += pw - pw / 2;
                        posh += ph - ph / 2;
                    }
                    if (!(posw >= 0 && posw < w && posh >= 0 && posh < h)) break;
                    const int16_t q = disp[(size_t)posh * w + posw];
                    if (q >= 0) {
                        dDisp[k] = q;
                        int cd = 0;
                        for (int ch = 0; ch < 3; ch++) {
                            int x = abs((int)bgrL[((size_t)v * w + u) * 3 + ch] - (int)bgrL[((size_t)posh * w + posw) * 3 + ch]);
                            if (x > cd) cd = x;
                        }
                        dDiff[k] = cd;
                        break;
                    }
                }
            }
            if (dv == c->disp_occ) {
                int minDisp = 2147483647;
                for (int k = 0; k < 16; k++)
                    if (dDisp[k] >= 0 && minDisp > dDisp[k]) minDisp = dDisp[k];
                cp[(size_t)v * w + u] = minDisp != 2147483647 ? (int16_t)minDisp : dv;
            } else {
                int minDif = 255, best = -1;
                for (int k = 0; k < 16; k++)
                    if (dDiff[k] >= 0 && minDif > dDiff[k]) {
                        minDif = dDiff[k];
                        best = dDisp[k];
                    }
                cp[(size_t)v * w + u] = best >= 0 ? (int16_t)best : dv;
            }
        }
    memcpy(disp, cp, (size_t)h * w * 2);
    free(cp);
}

/* cv::medianBlur(DP[0], DP[0], 3) (cpp:1497-1505) on CV_16S: the 3x3 sorting-network path, rows
 * and columns clamped at the border (replicate); in place means the source is copied first. */
static int16_t med3(int16_t a, int16_t b, int16_t c) {
    int16_t t;
    if (a > b) { t = a; a = b; b = t; }
    if (b > c) { t = b; b = c; c = t; }
    if (a > b) { t = a; a = b; b = t; }
    return b;
}
void smo_median3(int H, int W, int16_t* disp) {
    int16_t* src = (int16_t*)malloc((size_t)H * W * 2);
    memcpy(src, disp, (size_t)H * W * 2);
    if (H == 1 || W == 1) {
        const int len = H * W;
        for (int i = 0; i < len; i++)
            disp[i] = med3(src[i > 0 ? i - 1 : 0], src[i], src[i < len - 1 ? i + 1 : len - 1]);
    } else {
        int16_t p[9];
        for (int v = 0; v < H; v++)
            for (int u = 0; u < W; u++) {
                int k = 0;
                for (int dv = -1; dv <= 1; dv++)
                    for (int du = -1; du <= 1; du++) {
                        int vv = imin(imax(v + dv, 0), H - 1), uu = imin(imax(u + du, 0), W - 1);
                        p[k++] = src[(size_t)vv * W + uu];
                    }
                for (int i = 1; i < 9; i++)  /* insertion sort; the median of 9 is unique */
                    for (int j = i; j > 0 && p[j - 1] > p[j]; j--) {
                        int16_t t = p[j];
                        p[j] = p[j - 1];
                        p[j - 1] = t;
                    }
                disp[(size_t)v * W + u] = p[4];
            }
    }
    free(src);
}

/* refine(), non-USE_RECONCV branch (cpp:1347-1510) with the default stage switches (h:72-81):
 * LR check, region_vote_nums x regionVote_my(0.4, 20), region_vote_nums x properIpol, 3x3 median. */
void smo_refine(const smo_config* c, int16_t* disp0, const int16_t* disp1, const uint16_t* armsL, const uint8_t* bgrL) {
    smo_lr_check(c, disp0, disp1);                                     /* Do_LRConsis (cpp:1364-1375) */
    if (c->do_region_vote)
        for (int i = 0; i < c->region_vote_nums; i++) smo_region_vote(c, disp0, armsL, c->rv_ratio, c->rv_s);  /* cpp:1390-1422 */
    if (c->do_proper_ipol)
        for (int i = 0; i < c->region_vote_nums; i++) smo_proper_ipol(c, disp0, bgrL);   /* cpp:1437-1451 */
    if (c->do_last_median) smo_median3(c->H, c->W, disp0);                              /* cpp:1497-1505 */
}

/* main:138-166 for one pair: costCalculate, SolveAll(PY_LVL = 1), dispOptimize, [refine]. */
int smo_run_ex(const smo_config* c, const uint8_t* bgrL, const uint8_t* bgrR, const uint8_t* grayL,
               const uint8_t* grayR, int16_t* disp, const smo_dumps* dd) {
    if (c->H < 2 || c->W < 2 || c->D < 1) return -1;
    smo_dumps none;
    memset(&none, 0, sizeof(none));
    const smo_dumps* d = dd ? dd : &none;
    const int refine = c->do_refine;
    const int views = refine ? 2 : 1;
    /* "so" runs on both views whenever Do_LRConsis (= 1, h:72): num = Do_LRConsis ? 2 : 1
     * (cpp:1093), so DP[1] = so(vm[1]) also without Do_refine -- on the raw right cost volume,
     * since CBCA (cpp:5592) and SolveAll (cpp:2178) touch vm[1] only with Do_refine */
    const int so_views = c->optimization == 2 ? 2 : views;
    const int right = refine || so_views == 2;
    const size_t npix = (size_t)c->H * c->W, nvol = npix * c->D;
    double t0 = now_ms(), t;
    double ms[7] = {0, 0, 0, 0, 0, 0, 0};
    float* vm[2] = {NULL, NULL};
    int16_t* dp1 = NULL;
    uint16_t *aL = NULL, *aR = NULL;
    int rc = -1;
    vm[0] = (float*)malloc(nvol * 4);
    if (!vm[0]) goto done;
    if (right && !(vm[1] = (float*)malloc(nvol * 4))) goto done;
    smo_cost_volume(c, bgrL, bgrR, grayL, grayR, 0, vm[0]);
    if (right) smo_cost_volume(c, bgrL, bgrR, grayL, grayR, 1, vm[1]);
    else if (d->vol_right) smo_cost_volume(c, bgrL, bgrR, grayL, grayR, 1, d->vol_right);
    if (right && d->vol_right) memcpy(d->vol_right, vm[1], nvol * 4);
    if (d->vol_cost) memcpy(d->vol_cost, vm[0], nvol * 4);
    t = now_ms(); ms[0] = t - t0; t0 = t;
    if (c->aggregation == 1 || refine) {
        aL = (uint16_t*)malloc(npix * 8);
        aR = (uint16_t*)malloc(npix * 8);
        if (!aL || !aR) goto done;
        smo_arms(c, bgrL, aL);                   /* calArms for both images (cpp:5358-5385) */
        smo_arms(c, bgrR, aR);
    }
    if (c->aggregation == 1)
        for (int i = 0; i < views; i++) smo_cbca_view(c, vm[i], aL, aR, i);   /* cbca_core LOR loop (cpp:5598) */
    if (c->aggregation == 2)   /* GF: guideFilter(0, vm), num = Do_refine ? 2 : 1 (cpp:4499-4516) */
        for (int i = 0; i < views; i++)
            if (smo_guided_filter(c, vm[i], i == 0 ? bgrL : bgrR)) goto done;
    if (c->aggregation == 3 && smo_nl_aggregate(c, vm[0], bgrL)) goto done;   /* NL(): vm[0] only (cpp:4898) */
    if (d->vol_agg) memcpy(d->vol_agg, vm[0], nvol * 4);
    if (refine && d->vol_agg_right) memcpy(d->vol_agg_right, vm[1], nvol * 4);
    t = now_ms(); ms[1] = t - t0; t0 = t;
    if (c->solve_all)
        for (int i = 0; i < views; i++) smo_solve_all(c, vm[i]);               /* img_n (cpp:2178) */
    t = now_ms(); ms[2] = t - t0; t0 = t;
    if (right && !(dp1 = (int16_t*)malloc(npix * 2))) goto done;
    if (c->optimization == 1)
        for (int i = 0; i < views; i++) smo_sgm(c, vm[i], i == 0 ? bgrL : bgrR);  /* cpp:1053-1060 */
    if (c->optimization == 2)   /* "so": DP directly, I_c[0] for both views (cpp:1091-1105) */
        for (int i = 0; i < so_views; i++) smo_so(c, vm[i], i == 0 ? disp : dp1, bgrL);
    if (d->vol_final) memcpy(d->vol_final, vm[0], nvol * 4);
    t = now_ms(); ms[3] = t - t0; t0 = t;
    if (c->optimization != 2) smo_wta(c, vm[0], disp);
    if (refine && c->optimization != 2) smo_wta(c, vm[1], dp1);               /* cpp:1110-1127 */
    if (dp1) {
        if (d->disp_left_raw) memcpy(d->disp_left_raw, disp, npix * 2);
        if (d->disp_right) memcpy(d->disp_right, dp1, npix * 2);
    }
    t = now_ms(); ms[4] = t - t0; t0 = t;
    if (refine) smo_refine(c, disp, dp1, aL, bgrL);                           /* main:165-166 */
    t = now_ms(); ms[5] = t - t0;
    ms[6] = ms[0] + ms[1] + ms[2] + ms[3] + ms[4] + ms[5];
    if (d->stage_ms) memcpy(d->stage_ms, ms, sizeof(ms));
    rc = 0;
done:
    free(vm[0]);
    free(vm[1]);
    free(dp1);
    free(aL);
    free(aR);
    return rc;
}

int smo_run(const smo_config* c, const uint8_t* bgrL, const uint8_t* bgrR,
            const uint8_t* grayL, const uint8_t* grayR, int16_t* disp,
            float* vol_cost, float* vol_agg, float* vol_final, float* vol_right, double* stage_ms) {
    double ms[7];
    smo_dumps d;
    memset(&d, 0, sizeof(d));
    d.vol_cost = vol_cost;
    d.vol_agg = vol_agg;
    d.vol_final = vol_final;
    d.vol_right = vol_right;
    d.stage_ms = ms;
    int rc = smo_run_ex(c, bgrL, bgrR, grayL, grayR, disp, &d);
    if (rc == 0 && stage_ms) {   /* legacy layout: cost, cbca, solveall, sgm, wta (+refine), total */
        memcpy(stage_ms, ms, 4 * sizeof(double));
        stage_ms[4] = ms[4] + ms[5];
        stage_ms[5] = ms[6];
    }
    return rc;
}

/* cv::pyrDown, 8-bit, BORDER_DEFAULT = BORDER_REFLECT_101: the separable 1-4-6-4-1 integer
 * filter, (sum + 128) >> 8 (FixPtCast<uchar, 8>); intermediate row sums are exact ints. */
void smo_pyr_down_u8(const uint8_t* src, int rows, int cols, int ch, uint8_t* dst) {
    static const int k[5] = {1, 4, 6, 4, 1};
    const int dr = (rows + 1) / 2, dc = (cols + 1) / 2;
    for (int y = 0; y < dr; y++)
        for (int x = 0; x < dc; x++)
            for (int c = 0; c < ch; c++) {
                int sum = 0;
                for (int i = 0; i < 5; i++) {
                    const int sy = smo_reflect101(2 * y + i - 2, rows);
                    int row = 0;
                    for (int j = 0; j < 5; j++) row += k[j] * src[((size_t)sy * cols + smo_reflect101(2 * x + j - 2, cols)) * ch + c];
                    sum += k[i] * row;
                }
                dst[((size_t)y * dc + x) * ch + c] = (uint8_t)((sum + 128) >> 8);
            }
}

/* SolveAll's regMat (cpp:2147-2163) and regInv = regMat.inv() (cpp:2164): OpenCV's invert for
 * CV_32F with n <= 3 evaluates the adjugate / determinant in double and rounds each entry to
 * float (n = 1: (float)(1. / a); n = 2: d = 1 / det2, Df(0,j) = (float)(+-S * d); n = 3: the
 * t[0..2] cofactor row times 1 / det3).  For n > 3 Mat::inv (DECOMP_LU) copies regMat, sets the
 * destination to the identity and runs hal::LU32f on it: OpenCV's LUImpl<float> (core
 * matrix_decomp.cpp; OpenCV is not vendored in the reference) — per column the partial pivot
 * (first row of largest |a|, failure below 10 * FLT_EPSILON), d = -1 / a_ii, every later row
 * a_jk += (a_ji * d) * a_ik and b_jk += (a_ji * d) * b_ik, then back substitution
 * b_ij = (b_ij - sum_k a_ik * b_kj) / a_ii; all in float, each product and sum rounded (the
 * scalar loops; an OpenCV build whose SIMD rows fuse the multiply-add could differ in the last
 * bit: parity unpinned beyond n = 3).  invWgt[s] = regInv(0, s) (cpp:2165-2168). */
static int lu_inv_row0(int L, float M[SMO_MAX_PYR][SMO_MAX_PYR], float* w) {
    float B[SMO_MAX_PYR][SMO_MAX_PYR];
    for (int i = 0; i < L; i++)
        for (int j = 0; j < L; j++) B[i][j] = i == j ? 1.f : 0.f;
    for (int i = 0; i < L; i++) {
        int k = i;
        for (int j = i + 1; j < L; j++)
            if (fabsf(M[j][i]) > fabsf(M[k][i])) k = j;
        if (fabsf(M[k][i]) < FLT_EPSILON * 10) return -1;
        if (k != i) {
            for (int j = i; j < L; j++) { float t = M[i][j]; M[i][j] = M[k][j]; M[k][j] = t; }
            for (int j = 0; j < L; j++) { float t = B[i][j]; B[i][j] = B[k][j]; B[k][j] = t; }
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
    return 0;
}

int smo_pyr_weights(int L, float lam, float* w) {
    if (L < 1 || L > SMO_MAX_PYR) return -1;
    float M[SMO_MAX_PYR][SMO_MAX_PYR] = {{0}};
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
    } else if (L == 2) {
        double d = (double)M[0][0] * M[1][1] - (double)M[0][1] * M[1][0];
        if (d == 0.) return -1;
        d = 1. / d;
        w[0] = (float)(M[1][1] * d);
        w[1] = (float)(-M[0][1] * d);
    } else {
        double d = M[0][0] * ((double)M[1][1] * M[2][2] - (double)M[1][2] * M[2][1]) -
                   M[0][1] * ((double)M[1][0] * M[2][2] - (double)M[1][2] * M[2][0]) +
                   M[0][2] * ((double)M[1][0] * M[2][1] - (double)M[1][1] * M[2][0]);
        if (d == 0.) return -1;
        d = 1. / d;
        w[0] = (float)(((double)M[1][1] * M[2][2] - (double)M[1][2] * M[2][1]) * d);
        w[1] = (float)(((double)M[0][2] * M[2][1] - (double)M[0][1] * M[2][2]) * d);
        w[2] = (float)(((double)M[0][1] * M[1][2] - (double)M[0][2] * M[1][1]) * d);
    }
    return 0;
}

/* SolveAll (cpp:2169-2205) for PY_LVL levels, one view: sum += invWgt[s] * vm_s[curY][curX][curD]
 * in level order, then curY /= 2, curX /= 2, curD = (curD + 1) / 2. */
int smo_solve_all_pyr(const smo_config* cfgs, float* const* vms, int L, float lam) {
    float w[SMO_MAX_PYR];
    if (smo_pyr_weights(L, lam, w)) return -1;
    const smo_config* c0 = &cfgs[0];
    for (int y = 0; y < c0->H; y++)
        for (int x = 0; x < c0->W; x++)
            for (int d = 0; d < c0->D; d++) {
                int cy = y, cx = x, cd = d;
                float sum = 0;
                for (int s = 0; s < L; s++) {
                    const smo_config* c = &cfgs[s];
                    if (cy >= c->H || cx >= c->W || cd >= c->D) return -1;
                    const float cur = vms[s][((size_t)cy * c->W + cx) * c->D + cd];
                    sum += w[s] * cur;
                    cy /= 2;
                    cx /= 2;
                    cd = (cd + 1) / 2;
                }
                vms[0][((size_t)y * c0->W + x) * c0->D + d] = sum;
            }
    return 0;
}

int smo_run_pyr(const smo_config* c0, int L, const uint8_t* bgrL, const uint8_t* bgrR, const uint8_t* grayL,
                const uint8_t* grayR, int16_t* disp) {
    if (L < 1 || L > SMO_MAX_PYR || c0->H < 2 || c0->W < 2) return -1;
    smo_config cfg[SMO_MAX_PYR];
    uint8_t* img[SMO_MAX_PYR][4] = {{NULL}};  /* per level: bgrL, bgrR, grayL, grayR */
    float* vm[SMO_MAX_PYR][2] = {{NULL}};
    uint16_t* arms[SMO_MAX_PYR][2] = {{NULL}};
    const int views = c0->do_refine ? 2 : 1;
    int rc = -1, maxdisp = c0->D - 1, disSc = 1;
    for (int p = 0; p < L; p++) {
        smo_config* c = &cfg[p];
        *c = *c0;
        if (p > 0) {
            c->H = (cfg[p - 1].H + 1) / 2;
            c->W = (cfg[p - 1].W + 1) / 2;
            if (c->H < 2 || c->W < 2) goto done;
            const size_t np = (size_t)c->H * c->W;
            for (int k = 0; k < 4; k++) {
                const int ch = k < 2 ? 3 : 1;
                img[p][k] = (uint8_t*)malloc(np * ch);
                if (!img[p][k]) goto done;
                const uint8_t* src = p == 1 ? (k == 0 ? bgrL : k == 1 ? bgrR : k == 2 ? grayL : grayR) : img[p - 1][k];
                smo_pyr_down_u8(src, cfg[p - 1].H, cfg[p - 1].W, ch, img[p][k]);   /* main:145-148 */
            }
        }
        c->D = maxdisp + 1;
        c->arm_L = c0->arm_L / disSc;          /* calArms: L / scale (cpp:5369-5371) */
        c->arm_L_out = c0->arm_L_out / disSc;
        const uint8_t* bL = p ? img[p][0] : bgrL;
        const uint8_t* bR = p ? img[p][1] : bgrR;
        const uint8_t* gL = p ? img[p][2] : grayL;
        const uint8_t* gR = p ? img[p][3] : grayR;
        const size_t np = (size_t)c->H * c->W, nv = np * c->D;
        for (int v = 0; v < views; v++) {
            vm[p][v] = (float*)malloc(nv * 4);
            if (!vm[p][v]) goto done;
            smo_cost_volume(c, bL, bR, gL, gR, v, vm[p][v]);
        }
        for (int k = 0; k < 2; k++) {
            arms[p][k] = (uint16_t*)malloc(np * 8);
            if (!arms[p][k]) goto done;
            smo_arms(c, k ? bR : bL, arms[p][k]);
        }
        if (c->aggregation == 1)
            for (int v = 0; v < views; v++) smo_cbca_view(c, vm[p][v], arms[p][0], arms[p][1], v);
        maxdisp = maxdisp / 2 + 1;             /* main:143 */
        disSc *= 2;
    }
    for (int v = 0; v < views; v++) {          /* SolveAll(smPsy, PY_LEV, REG_LAMBDA) (main:158) */
        float* vv[SMO_MAX_PYR];
        for (int p = 0; p < L; p++) vv[p] = vm[p][v];
        if (c0->solve_all && smo_solve_all_pyr(cfg, vv, L, c0->reg_lambda)) goto done;
    }
    {
        const smo_config* c = &cfg[0];
        if (c->optimization == 1)
            for (int v = 0; v < views; v++) smo_sgm(c, vm[0][v], v == 0 ? bgrL : bgrR);
        if (c->optimization == 2)
            smo_so(c, vm[0][0], disp, bgrL);
        else
            smo_wta(c, vm[0][0], disp);
        if (c->do_refine) {
            int16_t* d1 = (int16_t*)malloc((size_t)c->H * c->W * 2);
            if (!d1) goto done;
            if (c->optimization == 2)
                smo_so(c, vm[0][1], d1, bgrL);
            else
                smo_wta(c, vm[0][1], d1);
            smo_refine(c, disp, d1, arms[0][0], bgrL);
            free(d1);
        }
    }
    rc = 0;
done:
    for (int p = 0; p < SMO_MAX_PYR; p++) {
        for (int k = 0; k < 4; k++) free(img[p][k]);
        for (int v = 0; v < 2; v++) free(vm[p][v]);
        for (int k = 0; k < 2; k++) free(arms[p][k]);
    }
    return rc;
}

/* calErr (h:1748-1825): bad pixel ratio over mask == 255 with threshold `thres`. */
float smo_bad_ratio(int H, int W, const int16_t* DP, const float* DT, const uint8_t* mask, float thres, float* rms_out) {
    int sumNum = 0, errorNumer = 0;
    float errorValueSum = 0;
    for (size_t p = 0; p < (size_t)H * W; p++) {
        if (mask[p] != 255) continue;
        sumNum++;
        if (DP[p] >= 0) {
            float dif = fabsf(DT[p] - DP[p]);
            errorValueSum = (float)(errorValueSum + pow(dif, 2));
            if (dif > thres) errorNumer++;
        } else {
            errorNumer++;
            errorValueSum += 2;
        }
    }
    if (sumNum == 0) {
        if (rms_out) *rms_out = 0;
        return 0;
    }
    if (rms_out) *rms_out = sqrtf(errorValueSum / sumNum);
    return (float)errorNumer / sumNum;
}

/* libm expf over the float bit patterns [first, first + n) — the checker for the device expf. */
void smo_expf_range(uint32_t first, uint32_t n, float* out) {
    for (uint32_t i = 0; i < n; i++) {
        uint32_t b = first + i;
        float x;
        memcpy(&x, &b, 4);
        out[i] = expf(x);
    }
}
