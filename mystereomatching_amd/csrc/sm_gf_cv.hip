// sm_gf_cv.hip — aggregation "GF" in the form the reference's shipped build runs:
// cv::ximgproc::guidedFilter(I_c[i] as float, vm[i], vm[i], gf_r[0] = 9, gf_eps[0] = 1e-4)
// (stereoMatching.cpp:4513, `//#define MY_GUIDE` at h:38; constants h:297-298).  The restated
// algorithm (oracle/sm_oracle_agg.c, smo_guided_filter_cv) is He et al.'s colour guided filter in
// the structure of ximgproc's GuidedFilterImpl, every mean an OpenCV normalised box filter with
// BORDER_REFLECT whose row and column sums run in double:
//
//   box(x)(y, u) = (float)(s0 * 1/361),  s0 = SUM_y + RS(y + r),  SUM_{y+1} = s0 - RS(y - r)
//   RS(y, u)     = running row sum: the first 19 reflected values, then += (double)x[u + 10 + ...]
//   Sigma        = box(I_i I_j) - mean_I_i mean_I_j (+ eps on the diagonal), inverted by cofactors
//   alpha_c      = sum_k Sigma^-1(c, k) (box(p I_k) - mean_p mean_I_k),  beta = mean_p - alpha . mean_I
//   q            = box(beta) + sum_c box(alpha_c) I_c
//
// gfx950 mapping.  The p-independent terms (mean_I and Sigma^-1 per pixel, 9 floats) come from
// nine image planes, row-summed by one thread per row (k_gfcv_img_rows), column-summed by one
// thread per plane and column (k_gfcv_img_cols), Sigma inverted per pixel (k_gfcv_pix).  The volume work is four line
// sweeps over [H][W][D] with lane = disparity and one wave per (line, 64-disparity chunk), each
// carrying four channels:
//   R0: row sums of (p, p B, p G, p R)          -> RS (four double volumes)
//   C0: column sums -> mean_p, cov, alpha, beta -> AB (four float volumes)
//   R1: row sums of (alpha_0..2, beta)           -> RS
//   C1: column sums -> q                         -> vm  [+ SolveAll's 0 + w q]
// The double intermediates are what OpenCV's FilterEngine keeps between its row and column
// filters; a row chain (RowSum's running update) can only run sequentially along the whole row,
// so the row sums round-trip HBM.  Every operation is the restatement's, in its order
// (-ffp-contract=off: no fused multiply-adds), so the volume is bit-exact to the oracle.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

namespace sm {

namespace {

constexpr int GC_R = 9;              // gf_r[0] (h:297)
constexpr int GC_K = 2 * GC_R + 1;   // box size
#ifndef SM_GFCV_RING
#define SM_GFCV_RING 1   // column sweeps keep the window's row sums in a register ring (k_gfcv_cols)
#endif
#ifndef SM_GFCV_PF
#define SM_GFCV_PF 3     // rows of row sums prefetched ahead by the ring form (divides 18)
#endif

// OpenCV borderInterpolate(BORDER_REFLECT) for len >= GC_R (one reflection suffices)
__device__ __forceinline__ int refl(int p, int len) { return p < 0 ? -p - 1 : (p >= len ? 2 * len - 1 - p : p); }

// image planes 0..8: B, G, R, BB, BG, BR, GG, GR, RR (float products of the float guide)
__device__ __forceinline__ float gc_plane(uint32_t w, int k) {
    const float b = (float)(w & 0xffu), g = (float)((w >> 8) & 0xffu), r = (float)((w >> 16) & 0xffu);
    switch (k) {
        case 0: return b;
        case 1: return g;
        case 2: return r;
        case 3: return b * b;
        case 4: return b * g;
        case 5: return b * r;
        case 6: return g * g;
        case 7: return g * r;
        default: return r * r;
    }
}

// one thread per (pair, plane, row): RowSum<float, double> over the reflected row into rs
__global__ __launch_bounds__(256) void k_gfcv_img_rows(const uint32_t* __restrict__ px, size_t px_pair_stride,
                                                       double* __restrict__ rs, int H, int W, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 9 * H) return;
    const int y = t % H, k = (t / H) % 9, b = t / (9 * H);
    const uint32_t* row = px + (size_t)b * px_pair_stride + (size_t)y * W;
    double* out = rs + (((size_t)b * 9 + k) * H + y) * W;
    double s = 0;
    for (int i = 0; i < GC_K; i++) s += (double)gc_plane(row[refl(i - GC_R, W)], k);
    out[0] = s;
    for (int i = 0; i < W - 1; i++) {
        s += (double)gc_plane(row[refl(i + GC_K - GC_R, W)], k) - (double)gc_plane(row[refl(i - GC_R, W)], k);
        out[i + 1] = s;
    }
}

// one thread per (pair, plane, column): ColumnSum<double, float> of the plane into pix[b][k]
// (the means; planes 3..8 are replaced by Sigma^-1 in k_gfcv_pix).  The next rows' sums are
// loaded while the current ones are added (a column walk is a chain of dependent adds).
__global__ __launch_bounds__(256) void k_gfcv_img_cols(const double* __restrict__ rs, float* __restrict__ pix, int H, int W,
                                                       int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 9 * W) return;
    const int x = t % W, k = (t / W) % 9, b = t / (9 * W);
    const size_t npix = (size_t)H * W;
    const double* base = rs + ((size_t)b * 9 + k) * npix + x;
    float* out = pix + ((size_t)b * 9 + k) * npix + x;
    const double scale = 1. / (GC_K * GC_K);
    double SUM = 0;
    for (int i = 0; i < GC_K - 1; i++) SUM += base[(size_t)refl(i - GC_R, H) * W];
    constexpr int U = 4;
    double sp[U], sm[U], np[U], nm[U];
    auto fetch = [&](double (&p)[U], double (&m)[U], int y0) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int y = min(y0 + u, H - 1);
            p[u] = base[(size_t)refl(y + GC_R, H) * W];
            m[u] = base[(size_t)refl(y - GC_R, H) * W];
        }
    };
    fetch(np, nm, 0);
    for (int y0 = 0; y0 < H; y0 += U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            sp[u] = np[u];
            sm[u] = nm[u];
        }
        if (y0 + U < H) fetch(np, nm, y0 + U);
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (y0 + u >= H) break;
            const double s0 = SUM + sp[u];
            out[(size_t)(y0 + u) * W] = (float)(s0 * scale);
            SUM = s0 - sm[u];
        }
    }
}

// per pixel: Sigma = box(I_i I_j) - m_i m_j (+ eps on the diagonal) and its inverse by the
// restatement's float cofactors / det, written over the box(I_i I_j) planes 3..8 as the entries
// 00, 01, 02, 11, 12, 22 (planes 0..2 keep mean_I)
__global__ __launch_bounds__(256) void k_gfcv_pix(float* __restrict__ pix, int H, int W, int n, float eps) {
    const size_t npix = (size_t)H * W;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npix * n) return;
    const size_t b = t / npix, i = t - b * npix;
    float* pl = pix + b * 9 * npix + i;
    float m[9];
#pragma unroll
    for (int k = 0; k < 9; k++) m[k] = pl[k * npix];
    float a[6];
    {
        const int I0[6] = {0, 0, 0, 1, 1, 2}, I1[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
        for (int v = 0; v < 6; v++) {
            const float mm = m[I0[v]] * m[I1[v]];
            a[v] = m[3 + v] - mm;
            if (I0[v] == I1[v]) a[v] = a[v] + eps;
        }
    }
    const float a00 = a[0], a01 = a[1], a02 = a[2], a11 = a[3], a12 = a[4], a22 = a[5];
    float b00 = a11 * a22, b01 = a02 * a12, b02 = a01 * a12, b11 = a00 * a22, b12 = a01 * a02, b22 = a00 * a11;
    float mm;
    mm = a12 * a12; b00 = b00 - mm;
    mm = a01 * a22; b01 = b01 - mm;
    mm = a02 * a11; b02 = b02 - mm;
    mm = a02 * a02; b11 = b11 - mm;
    mm = a00 * a12; b12 = b12 - mm;
    mm = a01 * a01; b22 = b22 - mm;
    float det = a00 * b00;
    mm = a01 * b01; det = det + mm;
    mm = a02 * b02; det = det + mm;
    pl[3 * npix] = b00 / det;
    pl[4 * npix] = b01 / det;
    pl[5 * npix] = b02 / det;
    pl[6 * npix] = b11 / det;
    pl[7 * npix] = b12 / det;
    pl[8 * npix] = b22 / det;
}

#ifndef SM_GFCV_T
#define SM_GFCV_T 4   // positions per prefetched tile of the volume sweeps (two tiles in flight)
#endif

// ---------------------------------------------------------------------------------------------
// Row sweep: one wave per (pair, row, chunk), lane = disparity.  MODE 0 reads p (vm) and the
// guide, MODE 1 reads alpha_0..2, beta (AB).  Ext position i (column refl(i - r)) enters the
// running sums; from i = k on, position i - k leaves (read again: it was loaded k positions ago,
// an L1 / L2 hit).
// ---------------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(64) void k_gfcv_rows(const GfCvArgs a) {
    constexpr int T = SM_GFCV_T;
    const int lane = threadIdx.x;
    const int nchunks = (a.D + 63) >> 6;
    const int blk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int b = blk / (a.H * nchunks);
    const int lc = blk - b * a.H * nchunks;
    const int y = lc / nchunks, chunk = lc - y * nchunks;
    const int d = chunk * 64 + lane;
    const bool live = d < a.D;
    const int dd = live ? d : a.D - 1;
    const int W = a.W, D = a.D;
    const size_t npix = (size_t)a.H * W;
    const size_t nvol = npix * D;
    const size_t row0 = ((size_t)b * npix + (size_t)y * W) * D + dd;   // element (b, y, 0, dd)
    const uint32_t* gw = a.px + (size_t)b * a.px_pair_stride + (size_t)y * W;
    double* rs = a.rs;
    const size_t rs_plane = (size_t)a.cap * nvol;   // doubles between channel planes
    const float* ab = a.ab;
    const size_t ab_plane = (size_t)a.cap * nvol;
    const int L = W + 2 * GC_R;   // ext positions

    auto fetch = [&](int i, float (&x)[4]) {
        const int u = refl(i - GC_R, W);
        const size_t e = row0 + (size_t)u * D;
        if (MODE == 0) {
            const float p = a.vm[e];
            const uint32_t w = gw[u];
            x[0] = p;
            x[1] = p * (float)(w & 0xffu);             // mul(src, guideCn[0]) (covSrcGuide)
            x[2] = p * (float)((w >> 8) & 0xffu);
            x[3] = p * (float)((w >> 16) & 0xffu);
        } else {
#pragma unroll
            for (int c = 0; c < 4; c++) x[c] = ab[c * ab_plane + e];
        }
    };
    struct Tile {
        float in[T][4];
        float out[T][4];
    };
    auto load = [&](Tile& t, int i0) {
#pragma unroll
        for (int s = 0; s < T; s++) {
            const int i = min(i0 + s, L - 1);
            fetch(i, t.in[s]);
            fetch(max(i - GC_K, 0), t.out[s]);
        }
    };
    double S[4] = {0, 0, 0, 0};
    auto process = [&](const Tile& t, int i0) {
#pragma unroll
        for (int s = 0; s < T; s++) {
            const int i = i0 + s;
            if (i >= L) break;   // wave-uniform
            if (i < GC_K) {
#pragma unroll
                for (int c = 0; c < 4; c++) S[c] += (double)t.in[s][c];
            } else {
#pragma unroll
                for (int c = 0; c < 4; c++) S[c] += (double)t.in[s][c] - (double)t.out[s][c];
            }
            if (i >= GC_K - 1 && live) {
                const size_t e = row0 - dd + d + (size_t)(i - (GC_K - 1)) * D;
#pragma unroll
                for (int c = 0; c < 4; c++) rs[c * rs_plane + e] = S[c];
            }
        }
    };
    Tile ta, tb;
    load(ta, 0);
    for (int i0 = 0; i0 < L; i0 += 2 * T) {
        load(tb, i0 + T);
        process(ta, i0);
        if (i0 + T >= L) break;
        load(ta, i0 + 2 * T);
        process(tb, i0 + T);
    }
}

// ---------------------------------------------------------------------------------------------
// Column sweep: one wave per (pair, column, chunk).  SUM starts as the first k - 1 reflected
// rows' row sums; output row y adds row y + r, stores (float)(s0 / 361) and drops row y - r.
// MODE 0: mean_p, box(p I_c) -> cov, alpha, beta -> AB.  MODE 1: box(alpha), box(beta) -> q -> vm.
// ---------------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(64) void k_gfcv_cols(const GfCvArgs a) {
    constexpr int T = SM_GFCV_T;
    const int lane = threadIdx.x;
    const int nchunks = (a.D + 63) >> 6;
    const int blk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int b = blk / (a.W * nchunks);
    const int lc = blk - b * a.W * nchunks;
    const int u = lc / nchunks, chunk = lc - u * nchunks;
    const int d = chunk * 64 + lane;
    const bool live = d < a.D;
    const int dd = live ? d : a.D - 1;
    const int H = a.H, W = a.W, D = a.D;
    const size_t npix = (size_t)H * W;
    const size_t nvol = npix * D;
    const size_t col0 = ((size_t)b * npix + u) * D + dd;   // element (b, 0, u, dd)
    const size_t rstep = (size_t)W * D;
    const double* rs = a.rs;
    const size_t rs_plane = (size_t)a.cap * nvol;
    float* ab = a.ab;
    const size_t ab_plane = (size_t)a.cap * nvol;
    const float* pix = a.pix + (size_t)b * 9 * npix + u;
    const uint32_t* gw = a.px + (size_t)b * a.px_pair_stride + u;
    const double scale = 1. / (GC_K * GC_K);

    // output row y from the box means m (MODE 0: alpha, beta -> AB; MODE 1: q -> vm)
    auto emit = [&](int y, const float (&m)[4]) {
        const size_t po = (size_t)y * W;
        const size_t e = col0 - dd + d + (size_t)y * rstep;
        if (MODE == 0) {
            const float mI[3] = {pix[0 * npix + po], pix[1 * npix + po], pix[2 * npix + po]};
            const float iv[6] = {pix[3 * npix + po], pix[4 * npix + po], pix[5 * npix + po],
                                 pix[6 * npix + po], pix[7 * npix + po], pix[8 * npix + po]};
            const float mP = m[0];
            float cov[3];
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const float mm = mP * mI[c];
                cov[c] = m[1 + c] - mm;
            }
            // inverse entry (g, k): 00 01 02 / 01 11 12 / 02 12 22
            const int IX[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
            float al[3];
#pragma unroll
            for (int g = 0; g < 3; g++) {
                float acc = iv[IX[g][0]] * cov[0];
#pragma unroll
                for (int k = 1; k < 3; k++) {
                    const float mm = iv[IX[g][k]] * cov[k];
                    acc = acc + mm;
                }
                al[g] = acc;
            }
            float be = mP;
#pragma unroll
            for (int g = 0; g < 3; g++) {
                const float mm = al[g] * mI[g];
                be = be - mm;
            }
            if (live) {
                ab[0 * ab_plane + e] = al[0];
                ab[1 * ab_plane + e] = al[1];
                ab[2 * ab_plane + e] = al[2];
                ab[3 * ab_plane + e] = be;
            }
        } else {
            const uint32_t w = gw[po];
            const float I[3] = {(float)(w & 0xffu), (float)((w >> 8) & 0xffu), (float)((w >> 16) & 0xffu)};
            float q = m[3];   // box(beta)
#pragma unroll
            for (int g = 0; g < 3; g++) {
                const float mm = m[g] * I[g];
                q = q + mm;
            }
            if (a.solve_all) {   // SolveAll fused (sm_run): its `sum = 0; sum += w * v`
                float sum = 0.f;
                sum += a.scale * q;
                q = sum;
            }
            if (live) a.vm[e] = q;
        }
    };
    double SUM[4] = {0, 0, 0, 0};
#if SM_GFCV_RING
    // The row sums leaving the window (row y - r) are the ones that entered it 2r = 18 rows
    // earlier: a register ring of 18 rows x 4 channels keeps them, so every RS element is read
    // once (the tiled form below reads it twice, the second time 18 rows later, past L2).
    // ring[i] starts as row refl(i - r), the rows the first 18 outputs drop; slot y mod 18.
    constexpr int RK = GC_K - 1, PF = SM_GFCV_PF;
    static_assert(RK % PF == 0, "prefetch slots repeat with the ring");
    double ring[RK][4], nx[PF][4];
#pragma unroll
    for (int i = 0; i < RK; i++) {
        const size_t e = col0 + (size_t)refl(i - GC_R, H) * rstep;
#pragma unroll
        for (int c = 0; c < 4; c++) ring[i][c] = rs[c * rs_plane + e];
    }
#pragma unroll
    for (int i = 0; i < RK; i++)
#pragma unroll
        for (int c = 0; c < 4; c++) SUM[c] += ring[i][c];
    auto fetch = [&](double (&x)[4], int y) {
        const size_t ep = col0 + (size_t)refl(min(y, H - 1) + GC_R, H) * rstep;
#pragma unroll
        for (int c = 0; c < 4; c++) x[c] = rs[c * rs_plane + ep];
    };
#pragma unroll
    for (int k = 0; k < PF; k++) fetch(nx[k], k);
    for (int y0 = 0; y0 < H; y0 += RK) {
#pragma unroll
        for (int s = 0; s < RK; s++) {
            const int y = y0 + s;
            if (y >= H) break;   // wave-uniform
            float m[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const double sp = nx[s % PF][c];
                const double s0 = SUM[c] + sp;
                m[c] = (float)(s0 * scale);
                SUM[c] = s0 - ring[s][c];
                ring[s][c] = sp;
            }
            fetch(nx[s % PF], y + PF);
            emit(y, m);
        }
    }
#else
    for (int i = 0; i < GC_K - 1; i++) {
        const size_t e = col0 + (size_t)refl(i - GC_R, H) * rstep;
#pragma unroll
        for (int c = 0; c < 4; c++) SUM[c] += rs[c * rs_plane + e];
    }
    struct Tile {
        double sp[T][4];
        double sm[T][4];
    };
    auto load = [&](Tile& t, int y0) {
#pragma unroll
        for (int s = 0; s < T; s++) {
            const int y = min(y0 + s, H - 1);
            const size_t ep = col0 + (size_t)refl(y + GC_R, H) * rstep, em = col0 + (size_t)refl(y - GC_R, H) * rstep;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                t.sp[s][c] = rs[c * rs_plane + ep];
                t.sm[s][c] = rs[c * rs_plane + em];
            }
        }
    };
    auto process = [&](const Tile& t, int y0) {
#pragma unroll
        for (int s = 0; s < T; s++) {
            const int y = y0 + s;
            if (y >= H) break;   // wave-uniform
            float m[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const double s0 = SUM[c] + t.sp[s][c];
                m[c] = (float)(s0 * scale);
                SUM[c] = s0 - t.sm[s][c];
            }
            emit(y, m);
        }
    };
    Tile ta, tb;
    load(ta, 0);
    for (int y0 = 0; y0 < H; y0 += 2 * T) {
        load(tb, y0 + T);
        process(ta, y0);
        if (y0 + T >= H) break;
        load(ta, y0 + 2 * T);
        process(tb, y0 + T);
    }
#endif
}

}  // namespace

size_t gfcv_img_scratch_doubles(int H, int W, int n) { return (size_t)n * 9 * H * W; }

void launch_gf_cv(const GfCvArgs& a, int n, hipStream_t st) {
    {
        const int tr = n * 9 * a.H;
        hipLaunchKernelGGL(k_gfcv_img_rows, dim3((tr + 255) / 256), dim3(256), 0, st, a.px, a.px_pair_stride, a.img_rs, a.H,
                           a.W, n);
        const int tc = n * 9 * a.W;
        hipLaunchKernelGGL(k_gfcv_img_cols, dim3((tc + 255) / 256), dim3(256), 0, st, a.img_rs, a.pix, a.H, a.W, n);
        const size_t tp = (size_t)n * a.H * a.W;
        hipLaunchKernelGGL(k_gfcv_pix, dim3((unsigned)((tp + 255) / 256)), dim3(256), 0, st, a.pix, a.H, a.W, n, a.eps);
    }
    const int nchunks = (a.D + 63) / 64;
    hipLaunchKernelGGL(k_gfcv_rows<0>, dim3(a.H * nchunks * n), dim3(64), 0, st, a);
    hipLaunchKernelGGL(k_gfcv_cols<0>, dim3(a.W * nchunks * n), dim3(64), 0, st, a);
    hipLaunchKernelGGL(k_gfcv_rows<1>, dim3(a.H * nchunks * n), dim3(64), 0, st, a);
    hipLaunchKernelGGL(k_gfcv_cols<1>, dim3(a.W * nchunks * n), dim3(64), 0, st, a);
}

}  // namespace sm
