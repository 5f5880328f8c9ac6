/*
 * sm_oracle_agg.c — CPU restatement of the reference's alternative aggregators.
 * TEST INFRASTRUCTURE ONLY (see sm_oracle.h); PARITY UNPINNED.
 *
 *  "GF"  guideFilter (stereoMatching.cpp:4492-4516), r = gf_r[0] = 9, eps = gf_eps[0] = 1e-4
 *        (h:297-298), guide = the view's BGR image as float (gf_channel_isColor, h:301), in two forms:
 *        gf_mode 0 — the shipped build (`//#define MY_GUIDE`, h:38): opencv_contrib's
 *          cv::ximgproc::guidedFilter(I, vm, vm, 9, 1e-4) (cpp:4513).  opencv_contrib is a
 *          third-party dependency absent from /root/reference (version unpinned: the reference has
 *          no build files).  Restated from its published algorithm (He et al., "Guided Image
 *          Filtering", colour guide) in the structure of ximgproc's GuidedFilterImpl
 *          (modules/ximgproc/src/guided_filter.cpp): every mean is meanFilter =
 *          boxFilter(CV_32F, (2r+1)^2, normalize, BORDER_REFLECT), i.e. OpenCV's generic
 *          RowSum<float, double> running row sums then ColumnSum<double, float> running column sums
 *          scaled by 1 / (2r+1)^2; the guide covariance Sigma + eps (float, eps added to the
 *          diagonal) is inverted per pixel by cofactors / det in float; per source channel
 *          alpha = Sigma^-1 cov(I, p) and beta = mean_p - alpha . mean_I with separate float products
 *          and sums (the scalar add_mul / sub_mul row helpers), q = mean_beta + mean_alpha . I.
 *          Assumptions that nothing here can pin (PARITY UNPINNED): the non-IPP, non-SIMD code path
 *          (IPP's box filter and FMA-based add_mul of SIMD builds round differently), the
 *          double casts inside RowSum's running update (OpenCV 4.x), the cofactor order.
 *        gf_mode 1 — the MY_GUIDE build: per disparity slice guideFilterCore_matlab (cpp:4975-5104),
 *          the same filter with the reference's own O(1) BoxFilter / CumSum (cpp:5107-5202).
 *  "NL"  NL() (cpp:4892-4917) -> NLCCA::aggreCV (NL/NLCCA.cpp:27-96): Qingxiong Yang's non-local
 *        aggregation on a minimum spanning tree of the left colour image (NL/qx_mst_kruskals_image
 *        .cpp: 3x3 ctmf median, 4-neighbour edges weighted by the max channel difference, counting
 *        sort, Kruskal, breadth-first tree from pixel 0) and the two-pass tree filter
 *        (NL/qx_tree_filter.cpp:61-117) in double, run once on the cost volume and once on a
 *        volume of ones; vm[0] = filtered cost / filtered ones (cpp:4898-4910).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sm_oracle.h"

/* ---------------------------------------------------------------------------------------------
 * Guided filter (MY_GUIDE)
 * ------------------------------------------------------------------------------------------- */

/* BoxFilter(imSrc, r) (cpp:5151-5202) with CumSum (cpp:5107-5144): cumulative sum down each
 * column, windowed differences, then the same along each row.  Needs H, W >= 2 r + 1. */
void smo_box_filter(int H, int W, int r, const float* src, float* dst, float* tmp) {
    /* CumSum(src, 1): row 0 is 0 + src (dest starts zeroed and preData aliases the row itself) */
    for (int x = 0; x < W; x++) tmp[x] = 0.0f + src[x];
    for (int y = 1; y < H; y++)
        for (int x = 0; x < W; x++) tmp[(size_t)y * W + x] = tmp[(size_t)(y - 1) * W + x] + src[(size_t)y * W + x];
    for (int y = 0; y < H; y++) {
        float* o = dst + (size_t)y * W;
        const float* plus = tmp + (size_t)(y < H - r ? y + r : H - 1) * W;
        if (y < r + 1) {
            for (int x = 0; x < W; x++) o[x] = plus[x];
        } else {
            const float* minus = tmp + (size_t)(y - r - 1) * W;
            for (int x = 0; x < W; x++) o[x] = plus[x] - minus[x];
        }
    }
    /* CumSum(imDst, 2): x = 0 copies (no 0 + here), then running sums along the row */
    for (int y = 0; y < H; y++) {
        float* c = tmp + (size_t)y * W;
        const float* s = dst + (size_t)y * W;
        c[0] = s[0];
        for (int x = 1; x < W; x++) c[x] = c[x - 1] + s[x];
        float* o = dst + (size_t)y * W;
        for (int x = 0; x < W; x++) {
            const float plus = c[x < W - r ? x + r : W - 1];
            o[x] = (x < r + 1) ? plus : plus - c[x - r - 1];
        }
    }
}

/* guideFilterCore_matlab(I, p, r, eps) (cpp:4975-5104) for every slice d of vm (in place),
 * I = the view's colour image as float, channels in BGR order (split of I_c, cpp:4977-4978). */
int smo_guided_filter_my(const smo_config* c, float* vm, const uint8_t* bgr) {
    const int H = c->H, W = c->W, D = c->D, r = c->gf_r;
    const float eps = c->gf_eps;
    if (H < 2 * r + 1 || W < 2 * r + 1) return -1;
    const size_t n = (size_t)H * W;
    float* buf = (float*)malloc(n * 4 * 32);
    double* cof = (double*)malloc(n * 8 * 10);
    if (!buf || !cof) {
        free(buf);
        free(cof);
        return -1;
    }
    float* tmp = buf;
    float* N = buf + n;
    float* Ich[3] = {buf + 2 * n, buf + 3 * n, buf + 4 * n};
    float* meanI[3] = {buf + 5 * n, buf + 6 * n, buf + 7 * n};
    float* var[6] = {buf + 8 * n, buf + 9 * n, buf + 10 * n, buf + 11 * n, buf + 12 * n, buf + 13 * n};
    float* p = buf + 14 * n;
    float* t = buf + 15 * n;
    float* mean_p = buf + 16 * n;
    float* cov[3] = {buf + 17 * n, buf + 18 * n, buf + 19 * n};
    float* a[3] = {buf + 20 * n, buf + 21 * n, buf + 22 * n};
    float* b = buf + 23 * n;
    float* q = buf + 24 * n;
    float* mt = buf + 25 * n;
    for (size_t i = 0; i < n; i++) {
        t[i] = 1.0f;
        for (int ch = 0; ch < 3; ch++) Ich[ch][i] = (float)bgr[i * 3 + ch];
    }
    smo_box_filter(H, W, r, t, N, tmp);                              /* N = BoxFilter(ones) */
    for (int ch = 0; ch < 3; ch++) {
        smo_box_filter(H, W, r, Ich[ch], meanI[ch], tmp);
        for (size_t i = 0; i < n; i++) meanI[ch][i] = meanI[ch][i] / N[i];
    }
    int vi = 0;
    for (int c0 = 0; c0 < 3; c0++)
        for (int c1 = c0; c1 < 3; c1++, vi++) {                      /* var_I (cpp:5003-5016) */
            for (size_t i = 0; i < n; i++) t[i] = Ich[c0][i] * Ich[c1][i];
            smo_box_filter(H, W, r, t, var[vi], tmp);
            for (size_t i = 0; i < n; i++) {
                var[vi][i] = var[vi][i] / N[i];
                var[vi][i] -= meanI[c0][i] * meanI[c1][i];
            }
        }
    /* the p-independent part of the 3x3 inverse (cpp:5048-5078), per pixel in double:
     * cof[0..8] = the nine cofactor expressions as written, cof[9] = 1 / DET */
    for (size_t i = 0; i < n; i++) {
        const double a11 = var[0][i] + eps, a12 = var[1][i], a13 = var[2][i];
        const double a21 = var[1][i], a22 = var[3][i] + eps, a23 = var[4][i];
        const double a31 = var[2][i], a32 = var[4][i], a33 = var[5][i] + eps;
        double* k = cof + i * 10;
        double DET = a11 * (a33 * a22 - a32 * a23) - a21 * (a33 * a12 - a32 * a13) + a31 * (a23 * a12 - a22 * a13);
        k[0] = a33 * a22 - a32 * a23;
        k[1] = a31 * a23 - a33 * a21;
        k[2] = a32 * a21 - a31 * a22;
        k[3] = a32 * a13 - a33 * a12;
        k[4] = a33 * a11 - a31 * a13;
        k[5] = a31 * a12 - a32 * a11;
        k[6] = a23 * a12 - a22 * a13;
        k[7] = a21 * a13 - a23 * a11;
        k[8] = a22 * a11 - a21 * a12;
        k[9] = 1 / DET;
    }
    for (int d = 0; d < D; d++) {
        for (size_t i = 0; i < n; i++) p[i] = vm[i * D + d];
        smo_box_filter(H, W, r, p, mean_p, tmp);
        for (size_t i = 0; i < n; i++) mean_p[i] = mean_p[i] / N[i];
        for (int ch = 0; ch < 3; ch++) {                              /* cpp:4988-4997 */
            for (size_t i = 0; i < n; i++) t[i] = Ich[ch][i] * p[i];
            smo_box_filter(H, W, r, t, cov[ch], tmp);
            for (size_t i = 0; i < n; i++) {
                const float mIp = cov[ch][i] / N[i];
                const float m = meanI[ch][i] * mean_p[i];
                cov[ch][i] = mIp - m;
            }
        }
        for (size_t i = 0; i < n; i++) {
            const double* k = cof + i * 10;
            const double c0 = cov[0][i], c1 = cov[1][i], c2 = cov[2][i];
            a[0][i] = (float)(k[9] * (c0 * k[0] + c1 * k[1] + c2 * k[2]));
            a[1][i] = (float)(k[9] * (c0 * k[3] + c1 * k[4] + c2 * k[5]));
            a[2][i] = (float)(k[9] * (c0 * k[6] + c1 * k[7] + c2 * k[8]));
            float bb = mean_p[i];                                       /* cpp:5083-5088 */
            for (int ch = 0; ch < 3; ch++) {
                const float m = a[ch][i] * meanI[ch][i];
                bb -= m;
            }
            b[i] = bb;
        }
        smo_box_filter(H, W, r, b, q, tmp);                              /* mean_b (cpp:5095) */
        for (size_t i = 0; i < n; i++) q[i] = q[i] / N[i];
        for (int ch = 0; ch < 3; ch++) {                                  /* q += mean_a[c] * I_c */
            smo_box_filter(H, W, r, a[ch], mt, tmp);
            for (size_t i = 0; i < n; i++) {
                const float ma = mt[i] / N[i];
                const float m = ma * Ich[ch][i];
                q[i] += m;
            }
        }
        for (size_t i = 0; i < n; i++) vm[i * D + d] = q[i];
    }
    free(buf);
    free(cof);
    return 0;
}

/* OpenCV borderInterpolate(p, len, BORDER_REFLECT): fedcba|abcdefgh|hgfedcb */
int smo_reflect(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p - 1 : 2 * len - 1 - p;
    return p;
}

/* ximgproc's meanFilter: boxFilter(src, dst, CV_32F, Size(k, k), Point(-1, -1), true,
 * BORDER_REFLECT), k = 2 r + 1, on a 1-channel float image.  OpenCV's FilterEngine runs
 * RowSum<float, double> on every border-extended row (running sum: s = sum of the first k,
 * then s += (double)S[i + k] - (double)S[i]), then ColumnSum<double, float> down the rows (SUM =
 * sum of the first k - 1 row sums; per output row s0 = SUM + Sp, out = (float)(s0 * scale),
 * SUM = s0 - Sm), scale = 1.0 / (k * k). */
void smo_box_filter_cv(int H, int W, int r, const float* src, float* dst, double* rs) {
    const int k = 2 * r + 1;
    const double scale = 1. / (k * k);
    for (int y = 0; y < H; y++) {
        const float* S = src + (size_t)y * W;
        double* D = rs + (size_t)y * W;
        double s = 0;
        for (int i = 0; i < k; i++) s += (double)S[smo_reflect(i - r, W)];
        D[0] = s;
        for (int i = 0; i < W - 1; i++) {
            s += (double)S[smo_reflect(i + k - r, W)] - (double)S[smo_reflect(i - r, W)];
            D[i + 1] = s;
        }
    }
    for (int x = 0; x < W; x++) {
        double SUM = 0;
        for (int i = 0; i < k - 1; i++) SUM += rs[(size_t)smo_reflect(i - r, H) * W + x];
        for (int y = 0; y < H; y++) {
            const double s0 = SUM + rs[(size_t)smo_reflect(y + r, H) * W + x];
            dst[(size_t)y * W + x] = (float)(s0 * scale);
            SUM = s0 - rs[(size_t)smo_reflect(y - r, H) * W + x];
        }
    }
}

/* cv::ximgproc::guidedFilter(I, vm, vm, r, eps) (cpp:4513) for every channel d of vm (in place),
 * I = the view's colour image as float, channels B, G, R.  See the file header for the source of
 * each step. */
int smo_guided_filter_cv(const smo_config* c, float* vm, const uint8_t* bgr) {
    const int H = c->H, W = c->W, D = c->D, r = c->gf_r;
    const float eps = c->gf_eps;
    if (H < 1 || W < 1 || r < 0) return -1;
    const size_t n = (size_t)H * W;
    float* buf = (float*)malloc(n * 4 * 32);
    double* rs = (double*)malloc(n * 8);
    if (!buf || !rs) {
        free(buf);
        free(rs);
        return -1;
    }
    float* I[3] = {buf, buf + n, buf + 2 * n};
    float* mI[3] = {buf + 3 * n, buf + 4 * n, buf + 5 * n};
    float* inv[6] = {buf + 6 * n, buf + 7 * n, buf + 8 * n, buf + 9 * n, buf + 10 * n, buf + 11 * n};  /* 00 01 02 11 12 22 */
    float* t = buf + 12 * n;
    float* p = buf + 13 * n;
    float* mP = buf + 14 * n;
    float* cov[3] = {buf + 15 * n, buf + 16 * n, buf + 17 * n};
    float* al[3] = {buf + 18 * n, buf + 19 * n, buf + 20 * n};
    float* be = buf + 21 * n;
    float* sg[6] = {buf + 22 * n, buf + 23 * n, buf + 24 * n, buf + 25 * n, buf + 26 * n, buf + 27 * n};
    for (size_t i = 0; i < n; i++)
        for (int ch = 0; ch < 3; ch++) I[ch][i] = (float)bgr[i * 3 + ch];   /* convertTo(CV_32F) */
    /* init: guideCnMean = meanFilter(guideCn); covars(i, j) = meanFilter(I_i I_j) - m_i m_j,
     * + eps on the diagonal; covarsInv = cofactors / det */
    for (int ch = 0; ch < 3; ch++) smo_box_filter_cv(H, W, r, I[ch], mI[ch], rs);
    int vi = 0;
    for (int c0 = 0; c0 < 3; c0++)
        for (int c1 = c0; c1 < 3; c1++, vi++) {
            for (size_t i = 0; i < n; i++) t[i] = I[c0][i] * I[c1][i];
            smo_box_filter_cv(H, W, r, t, sg[vi], rs);
            for (size_t i = 0; i < n; i++) {
                const float m = mI[c0][i] * mI[c1][i];
                sg[vi][i] = sg[vi][i] - m;
                if (c0 == c1) sg[vi][i] = sg[vi][i] + eps;
            }
        }
    for (size_t i = 0; i < n; i++) {
        const float a00 = sg[0][i], a01 = sg[1][i], a02 = sg[2][i], a11 = sg[3][i], a12 = sg[4][i], a22 = sg[5][i];
        float b00 = a11 * a22, b01 = a02 * a12, b02 = a01 * a12, b11 = a00 * a22, b12 = a01 * a02, b22 = a00 * a11;
        float m;
        m = a12 * a12; b00 = b00 - m;
        m = a01 * a22; b01 = b01 - m;
        m = a02 * a11; b02 = b02 - m;
        m = a02 * a02; b11 = b11 - m;
        m = a00 * a12; b12 = b12 - m;
        m = a01 * a01; b22 = b22 - m;
        float det = a00 * b00;
        m = a01 * b01; det = det + m;
        m = a02 * b02; det = det + m;
        inv[0][i] = b00 / det;
        inv[1][i] = b01 / det;
        inv[2][i] = b02 / det;
        inv[3][i] = b11 / det;
        inv[4][i] = b12 / det;
        inv[5][i] = b22 / det;
    }
    static const int IX[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
    for (int d = 0; d < D; d++) {
        for (size_t i = 0; i < n; i++) p[i] = vm[i * D + d];
        smo_box_filter_cv(H, W, r, p, mP, rs);                               /* srcCnMean */
        for (int ch = 0; ch < 3; ch++) {                                     /* computeCovGuideAndSrc */
            for (size_t i = 0; i < n; i++) t[i] = p[i] * I[ch][i];
            smo_box_filter_cv(H, W, r, t, cov[ch], rs);
            for (size_t i = 0; i < n; i++) {
                const float m = mP[i] * mI[ch][i];
                cov[ch][i] = cov[ch][i] - m;
            }
        }
        for (size_t i = 0; i < n; i++) {
            for (int gi = 0; gi < 3; gi++) {                                 /* alpha = Sigma^-1 cov */
                float y = inv[IX[gi][0]][i] * cov[0][i];
                for (int k = 1; k < 3; k++) {
                    const float m = inv[IX[gi][k]][i] * cov[k][i];
                    y = y + m;
                }
                al[gi][i] = y;
            }
            float b = mP[i];                                                 /* beta = mean_p - alpha . mean_I */
            for (int gi = 0; gi < 3; gi++) {
                const float m = al[gi][i] * mI[gi][i];
                b = b - m;
            }
            be[i] = b;
        }
        smo_box_filter_cv(H, W, r, be, t, rs);                              /* mean beta -> t */
        for (int gi = 0; gi < 3; gi++) {
            smo_box_filter_cv(H, W, r, al[gi], cov[gi], rs);                /* mean alpha -> cov */
        }
        for (size_t i = 0; i < n; i++) {                                     /* q = mean_beta + mean_alpha . I */
            float q = t[i];
            for (int gi = 0; gi < 3; gi++) {
                const float m = cov[gi][i] * I[gi][i];
                q = q + m;
            }
            vm[i * D + d] = q;
        }
    }
    free(buf);
    free(rs);
    return 0;
}

int smo_guided_filter(const smo_config* c, float* vm, const uint8_t* bgr) {
    return c->gf_mode == 1 ? smo_guided_filter_my(c, vm, bgr) : smo_guided_filter_cv(c, vm, bgr);
}

/* ---------------------------------------------------------------------------------------------
 * Non-local aggregation (NL): minimum spanning tree + tree filter
 * ------------------------------------------------------------------------------------------- */

/* ctmf(src, dst, w, h, ..., r = 1, cn = 3) as qx_mst_kruskals_image::mst calls it (NL/
 * qx_mst_kruskals_image.cpp:174): per channel, the 5th smallest of the 3x3 window with rows and
 * columns clamped at the image border (ctmf.c:227-258 replicate the first / last row into the
 * column histograms; pad_left / MIN(j + r, n - 1) replicate the columns). */
void smo_nl_median3(int H, int W, const uint8_t* src, uint8_t* dst) {
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
            for (int ch = 0; ch < 3; ch++) {
                int hist[256];
                memset(hist, 0, sizeof(hist));
                for (int dy = -1; dy <= 1; dy++)
                    for (int dx = -1; dx <= 1; dx++) {
                        const int yy = y + dy < 0 ? 0 : (y + dy >= H ? H - 1 : y + dy);
                        const int xx = x + dx < 0 ? 0 : (x + dx >= W ? W - 1 : x + dx);
                        hist[src[((size_t)yy * W + xx) * 3 + ch]]++;
                    }
                int v = 0, acc = 0;
                while (acc + hist[v] <= 4) acc += hist[v++];   /* first value whose count passes 2r^2 + 2r */
                dst[((size_t)y * W + x) * 3 + ch] = (uint8_t)v;
            }
}

/* The tree of NLCCA (qx_mst_kruskals_image::mst + build_tree, cpp:167-277):
 *   edges: horizontal (y, x)-(y, x+1) row by row, then vertical (y, x)-(y+1, x) column by
 *          column (qx_mst_compute_edges_4neighbor), weight = max channel |difference| of the
 *          median-filtered image;
 *   order: counting sort by weight, ties in edge order (qx_sort_increase_using_histogram);
 *   Kruskal with union-find (path compression, parent[root(u)] = root(v)); every accepted edge
 *          is appended to both endpoints' neighbour lists;
 *   tree:  breadth-first from pixel 0, children in neighbour-list order.
 * Outputs: order[n] (BFS order), parent[n] (parent[0] = 0), weight[n] (edge weight to the
 * parent, 0 for the root), nchild[n], child[n * 4]. */
int smo_nl_tree(int H, int W, const uint8_t* bgr, int* order, int* parent, uint8_t* weight, int* nchild, int* child) {
    const int n = H * W;
    if (H < 1 || W < 1) return -1;
    const int ne = (H - 1) * W + (W - 1) * H;
    uint8_t* med = (uint8_t*)malloc((size_t)n * 3);
    int* eu = (int*)malloc(sizeof(int) * (size_t)(ne > 0 ? ne : 1));
    int* ev = (int*)malloc(sizeof(int) * (size_t)(ne > 0 ? ne : 1));
    uint8_t* ew = (uint8_t*)malloc((size_t)(ne > 0 ? ne : 1));
    int* sorted = (int*)malloc(sizeof(int) * (size_t)(ne > 0 ? ne : 1));
    int* uf = (int*)malloc(sizeof(int) * (size_t)n);
    int* nconn = (int*)calloc((size_t)n, sizeof(int));
    int* conn = (int*)malloc(sizeof(int) * (size_t)n * 4);
    uint8_t* connw = (uint8_t*)malloc((size_t)n * 4);
    int rc = -1;
    if (!med || !eu || !ev || !ew || !sorted || !uf || !nconn || !conn || !connw) goto out;
    smo_nl_median3(H, W, bgr, med);
    {
        int k = 0;
        for (int y = 0; y < H; y++)
            for (int x = 0; x + 1 < W; x++, k++) {
                eu[k] = y * W + x;
                ev[k] = y * W + x + 1;
            }
        for (int x = 0; x < W; x++)
            for (int y = 0; y + 1 < H; y++, k++) {
                eu[k] = y * W + x;
                ev[k] = (y + 1) * W + x;
            }
        for (int e = 0; e < ne; e++) {
            int m = 0;
            for (int ch = 0; ch < 3; ch++) {
                const int dv = abs((int)med[(size_t)ev[e] * 3 + ch] - (int)med[(size_t)eu[e] * 3 + ch]);
                if (dv > m) m = dv;
            }
            ew[e] = (uint8_t)m;
        }
    }
    {   /* stable counting sort by weight */
        int start[257];
        memset(start, 0, sizeof(start));
        for (int e = 0; e < ne; e++) start[ew[e] + 1]++;
        for (int v = 0; v < 256; v++) start[v + 1] += start[v];
        for (int e = 0; e < ne; e++) sorted[start[ew[e]]++] = e;
    }
    for (int i = 0; i < n; i++) uf[i] = i;
    for (int j = 0; j < ne; j++) {
        const int e = sorted[j], u = eu[e], v = ev[e];
        int pu = u, pv = v;
        while (uf[pu] != pu) pu = uf[pu];
        while (uf[pv] != pv) pv = uf[pv];
        for (int x = u; uf[x] != pu;) {   /* path compression (the recursion's effect) */
            const int nx = uf[x];
            uf[x] = pu;
            x = nx;
        }
        for (int x = v; uf[x] != pv;) {
            const int nx = uf[x];
            uf[x] = pv;
            x = nx;
        }
        if (pu != pv) {
            conn[(size_t)u * 4 + nconn[u]] = v;
            connw[(size_t)u * 4 + nconn[u]++] = ew[e];
            conn[(size_t)v * 4 + nconn[v]] = u;
            connw[(size_t)v * 4 + nconn[v]++] = ew[e];
            uf[pu] = pv;
        }
    }
    for (int i = 0; i < n; i++) {
        parent[i] = -1;
        nchild[i] = 0;
    }
    parent[0] = 0;
    weight[0] = 0;
    order[0] = 0;
    {
        int head = 0, len = 1;
        while (head < len) {
            const int p = order[head++];
            for (int i = 0; i < nconn[p]; i++) {
                const int q = conn[(size_t)p * 4 + i];
                if (parent[q] == -1) {
                    parent[q] = p;
                    weight[q] = connw[(size_t)p * 4 + i];
                    child[(size_t)p * 4 + nchild[p]++] = q;
                    order[len++] = q;
                }
            }
        }
        rc = len == n ? 0 : -1;
    }
out:
    free(med);
    free(eu);
    free(ev);
    free(ew);
    free(sorted);
    free(uf);
    free(nconn);
    free(conn);
    free(connw);
    return rc;
}

/* exp(-i / (255 * sigma)) for the 256 edge weights (qx_tree_filter::update_table, sigma >= 0.01) */
void smo_nl_table(double sigma, double* table) {
    if (sigma < 0.01) sigma = 0.01;
    for (int i = 0; i <= 255; i++) table[i] = exp(-(double)i / (255 * sigma));
}

/* qx_tree_filter::filter (NL/qx_tree_filter.cpp:61-117) on P planes of doubles per node. */
void smo_nl_filter(int n, int P, const int* order, const int* parent, const uint8_t* weight, const int* nchild,
                   const int* child, const double* table, double* cost, double* backup) {
    memcpy(backup, cost, sizeof(double) * (size_t)n * P);
    for (int i = n - 1; i >= 0; i--) {   /* children before parents */
        const int id = order[i];
        double* s = backup + (size_t)id * P;
        for (int j = 0; j < nchild[id]; j++) {
            const int ch = child[(size_t)id * 4 + j];
            const double w = table[weight[ch]];
            const double* vc = backup + (size_t)ch * P;
            for (int k = 0; k < P; k++) s[k] += vc[k] * w;
        }
    }
    memcpy(cost + (size_t)order[0] * P, backup + (size_t)order[0] * P, sizeof(double) * P);
    for (int i = 1; i < n; i++) {
        const int id = order[i];
        const double w = table[weight[id]];
        const double* vp = cost + (size_t)parent[id] * P;
        const double* vc = backup + (size_t)id * P;
        double* o = cost + (size_t)id * P;
        for (int k = 0; k < P; k++) o[k] = w * (vp[k] - w * vc[k]) + vc[k];
    }
}

/* NL() (cpp:4892-4910): vm = aggreCV(vm) / aggreCV(ones), tree of the left colour image. */
int smo_nl_aggregate(const smo_config* c, float* vm, const uint8_t* bgrL) {
    const int H = c->H, W = c->W, D = c->D, n = H * W;
    int* order = (int*)malloc(sizeof(int) * (size_t)n);
    int* parent = (int*)malloc(sizeof(int) * (size_t)n);
    uint8_t* weight = (uint8_t*)malloc((size_t)n);
    int* nchild = (int*)malloc(sizeof(int) * (size_t)n);
    int* child = (int*)malloc(sizeof(int) * (size_t)n * 4);
    double* cost = (double*)malloc(sizeof(double) * (size_t)n * D);
    double* backup = (double*)malloc(sizeof(double) * (size_t)n * D);
    double* ones = (double*)malloc(sizeof(double) * (size_t)n);
    double* ones_b = (double*)malloc(sizeof(double) * (size_t)n);
    double table[256];
    int rc = -1;
    if (!order || !parent || !weight || !nchild || !child || !cost || !backup || !ones || !ones_b) goto out;
    if (smo_nl_tree(H, W, bgrL, order, parent, weight, nchild, child)) goto out;
    smo_nl_table(c->nl_sigma, table);
    for (size_t i = 0; i < (size_t)n * D; i++) cost[i] = (double)vm[i];
    smo_nl_filter(n, D, order, parent, weight, nchild, child, table, cost, backup);
    /* the ones volume: every plane is the same single-plane filter (aggreCV of wetNL) */
    for (int i = 0; i < n; i++) ones[i] = 1.0;
    smo_nl_filter(n, 1, order, parent, weight, nchild, child, table, ones, ones_b);
    for (int i = 0; i < n; i++) {
        const float wsum = (float)ones[i];
        for (int d = 0; d < D; d++) vm[(size_t)i * D + d] = (float)cost[(size_t)i * D + d] / wsum;
    }
    rc = 0;
out:
    free(order);
    free(parent);
    free(weight);
    free(nchild);
    free(child);
    free(cost);
    free(backup);
    free(ones);
    free(ones_b);
    return rc;
}
