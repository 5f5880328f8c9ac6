// sm_gf.hip — aggregation "GF" (guideFilter, stereoMatching.cpp:4492-4516) in its MY_GUIDE form:
// per disparity slice p, guideFilterCore_matlab(I, p, 9, 0.0001) (cpp:4975-5104), the colour
// guided filter of He et al. with the reference's own BoxFilter / CumSum (cpp:5107-5202):
//
//   BoxFilter(x) = column cumulative sums S (row 0 = 0 + x), out(y) = S(y + r) - S(y - r - 1)
//                  (S(y + r) alone for y <= r, S(H - 1) for y + r >= H), then the same along rows
//   mean_p = box(p) / N, mean_Ip[c] = box(I_c p) / N, cov[c] = mean_Ip[c] - mean_I[c] mean_p
//   a = cov^T (Sigma + eps E)^-1  (double cofactors, per pixel), b = mean_p - sum_c a[c] mean_I[c]
//   q = box(b) / N + sum_c box(a[c]) / N * I_c
//
// gfx950 mapping.  The p-independent per-pixel terms (N, mean_I, the 3x3 inverse's cofactors and
// 1 / DET in double) come from 10 image planes box-filtered once per pair (k_gf_img_v / _h,
// k_gf_pix).  The volume work is four line sweeps over [H][W][D] (lane = disparity, one wave per
// (line, 64-disparity chunk)), each carrying four channels at once:
//   V0: column box of (p, B p, G p, R p)           -> s0..s3
//   H0: row box, then mean_p, cov, a[0..2], b      -> s0..s3 (in place, behind the read front)
//   V1: column box of (a0, a1, a2, b)              -> s0..s3 (in place)
//   H1: row box, then q                            -> vm
// The cumulative sum of a line lives in a register ring of 2r + 2 = 20 slots (r = 9, the
// reference's constant): the loop is unrolled by 20 so every slot index is static; positions past
// the line end add 0, which leaves S(H - 1) in place for the last r outputs.  Every operation is
// the reference's, in its order (float adds of the cumulative sums, IEEE divisions by N, the
// double inverse as written, float products), so the volume is bit-exact to the restatement.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

namespace sm {

namespace {

#ifndef SM_GF_PARTS
#define SM_GF_PARTS 2   // parts a block of GF_RING positions is loaded and processed in (1, 2, 4, 5)
// (same-process A/B, Teddy x16 GF: 1 part 5.05 / 4.56 ms, 2 parts 4.72 / 4.18 ms, 4 parts 5.13 /
// 4.62 ms, 5 parts 4.71 / 4.69 ms; a software-pipelined variant with the next block's inputs in
// flight needed 264-288 VGPRs, one wave per SIMD, and ran 7.5-7.8 ms)
#endif

constexpr int GF_R = 9;                // guideFilterCore_matlab(I, p, 9, eps) (cpp:4509)
constexpr int GF_RING = 2 * GF_R + 2;  // S(j) .. S(j - 2r - 1)

// ---------------------------------------------------------------------------------------------
// Image planes: 0 = ones, 1..3 = B, G, R, 4..9 = BB, BG, BR, GG, GR, RR (var_I order, cpp:5005-5016)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float gf_plane_w(uint32_t w, int k) {   // w = B | G << 8 | R << 16
    const float b = (float)(w & 0xffu), g = (float)((w >> 8) & 0xffu), r = (float)((w >> 16) & 0xffu);
    switch (k) {
        case 0: return 1.0f;
        case 1: return b;
        case 2: return g;
        case 3: return r;
        case 4: return b * b;
        case 5: return b * g;
        case 6: return b * r;
        case 7: return g * g;
        case 8: return g * r;
        default: return r * r;
    }
}

// one thread per (pair, plane, column): column box of the plane into planes[b][k][H][W]
// (the colours come from the packed BGR words k_pack_bgr made in the prep: one dword per row)
__global__ __launch_bounds__(256) void k_gf_img_v(const uint32_t* __restrict__ pxw, float* __restrict__ planes, int H, int W,
                                                  int n, size_t px_pair_stride) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 10 * W) return;
    const int x = t % W, k = (t / W) % 10, b = t / (W * 10);
    const uint32_t* src = pxw + (size_t)b * px_pair_stride + x;
    float* out = planes + ((size_t)b * 10 + k) * H * W + x;
    float ring[GF_RING];
    float S = 0.f;
    // the inputs of a block of rows are loaded while the previous block is summed
    auto fetch = [&](float (&v)[GF_RING], int j0) {
#pragma unroll
        for (int s = 0; s < GF_RING; s++) {
            const int j = j0 + s;
            v[s] = j < H ? gf_plane_w(src[(size_t)j * W], k) : 0.f;
        }
    };
    float vin[GF_RING], nxt[GF_RING];
    fetch(nxt, 0);
    for (int j0 = 0; j0 < H + GF_R; j0 += GF_RING) {
#pragma unroll
        for (int s = 0; s < GF_RING; s++) vin[s] = nxt[s];
        if (j0 + GF_RING < H + GF_R) fetch(nxt, j0 + GF_RING);   // (rows past H read 0)
#pragma unroll
        for (int s = 0; s < GF_RING; s++) {
            const int j = j0 + s;
            if (j < H + GF_R) {
                const float v = vin[s];
                S = (j == 0 ? 0.f : S) + v;   // CumSum(., 1): 0 + x on row 0; past the end + 0 keeps S(H - 1)
                ring[s] = S;
                const int i = j - GF_R;
                if (i >= 0) out[(size_t)i * W] = i >= GF_R + 1 ? S - ring[(s + 1) % GF_RING] : S;
            }
        }
    }
}

// one thread per (pair, plane, row): row box in place.  A wave owns 64 consecutive rows and
// walks them in blocks of GF_RING columns staged through LDS: the block is loaded and the outputs
// stored row segment by row segment across the lanes (coalesced), while each lane runs its row's
// sequential cumulative sum on the LDS copy (a lane per row reading global memory directly makes
// every load instruction touch 64 rows).  Block j0 reads columns j0 .. j0 + 19 and writes the
// outputs of columns j0 - 9 .. j0 + 10, all of which it has already read (in place is safe).
#ifndef SM_GF_IMG_H_LDS
#define SM_GF_IMG_H_LDS 1
#endif
constexpr int GF_HP = GF_RING + 1;   // LDS row pitch (odd: conflict-free column reads)
__global__ __launch_bounds__(64) void k_gf_img_h(float* __restrict__ planes, int H, int W, int n) {
    const int rows = n * 10 * H;
    const int lane = threadIdx.x;
    const int r0 = blockIdx.x * 64;
    if (!SM_GF_IMG_H_LDS) {
        const int t = r0 + lane;
        if (t >= rows) return;
        float* row = planes + (size_t)t * W;   // planes are [b][k][H][W]: thread t owns row t
        float ring[GF_RING];
        float S = 0.f;
        for (int j0 = 0; j0 < W + GF_R; j0 += GF_RING) {
            float vin[GF_RING];
#pragma unroll
            for (int s = 0; s < GF_RING; s++) vin[s] = j0 + s < W ? row[j0 + s] : 0.f;
#pragma unroll
            for (int s = 0; s < GF_RING; s++) {
                const int j = j0 + s;
                if (j < W + GF_R) {
                    if (j < W) S = (j == 0) ? vin[0] : S + vin[s];   // CumSum(., 2): x = 0 copies
                    ring[s] = S;
                    const int i = j - GF_R;
                    if (i >= 0) row[i] = i >= GF_R + 1 ? S - ring[(s + 1) % GF_RING] : S;
                }
            }
        }
        return;
    }
    __shared__ float tin[64 * GF_HP], tout[64 * GF_HP];
    // element m of a lane's share of a block: row (m * 64 + lane) / GF_RING, column % GF_RING
    auto fetch = [&](float (&v)[GF_RING], int j0) {
#pragma unroll
        for (int m = 0; m < GF_RING; m++) {
            const int e = m * 64 + lane, rr = e / GF_RING, cc = e - rr * GF_RING;
            const int j = j0 + cc;
            v[m] = (r0 + rr < rows && j < W) ? planes[(size_t)(r0 + rr) * W + j] : 0.f;
        }
    };
    float nxt[GF_RING];
    fetch(nxt, 0);
    float ring[GF_RING];
    float S = 0.f;
    for (int j0 = 0; j0 < W + GF_R; j0 += GF_RING) {
#pragma unroll
        for (int m = 0; m < GF_RING; m++) {
            const int e = m * 64 + lane, rr = e / GF_RING, cc = e - rr * GF_RING;
            tin[rr * GF_HP + cc] = nxt[m];
        }
        __syncthreads();
        // the next block's loads fly while this block is summed (its columns are >= j0 + 20,
        // past every output this block stores)
        if (j0 + GF_RING < W + GF_R) fetch(nxt, j0 + GF_RING);   // (columns past W read 0)
#pragma unroll
        for (int s = 0; s < GF_RING; s++) {
            const int j = j0 + s;
            if (j < W + GF_R) {
                const float v = tin[lane * GF_HP + s];
                if (j < W) S = (j == 0) ? v : S + v;   // CumSum(., 2): x = 0 copies
                ring[s] = S;
                const int i = j - GF_R;
                tout[lane * GF_HP + s] = i >= GF_R + 1 ? S - ring[(s + 1) % GF_RING] : S;
            }
        }
        __syncthreads();
        // store: tout[row][s] is the output of column j0 + s - GF_R
#pragma unroll
        for (int m = 0; m < GF_RING; m++) {
            const int e = m * 64 + lane, rr = e / GF_RING, cc = e - rr * GF_RING;
            const int i = j0 + cc - GF_R;
            if (r0 + rr < rows && i >= 0 && i < W) planes[(size_t)(r0 + rr) * W + i] = tout[rr * GF_HP + cc];
        }
    }
}

// per pixel: N, mean_I, and the 3x3 inverse's p-independent doubles (cpp:5003-5078)
__global__ __launch_bounds__(256) void k_gf_pix(const float* __restrict__ planes, GfPix* __restrict__ pix, int H, int W, int n,
                                                float eps) {
    const size_t npix = (size_t)H * W;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npix * n) return;
    const size_t b = t / npix, i = t - b * npix;
    const float* pl = planes + b * 10 * npix + i;
    const float N = pl[0];
    float mI[3], var[6];
#pragma unroll
    for (int c = 0; c < 3; c++) mI[c] = pl[(1 + c) * npix] / N;
    int vi = 0;
#pragma unroll
    for (int c0 = 0; c0 < 3; c0++)
#pragma unroll
        for (int c1 = c0; c1 < 3; c1++, vi++) {
            float v = pl[(4 + vi) * npix] / N;
            const float m = mI[c0] * mI[c1];
            var[vi] = v - m;
        }
    const double a11 = var[0] + eps, a12 = var[1], a13 = var[2];
    const double a21 = var[1], a22 = var[3] + eps, a23 = var[4];
    const double a31 = var[2], a32 = var[4], a33 = var[5] + eps;
    GfPix r;
    const double DET = a11 * (a33 * a22 - a32 * a23) - a21 * (a33 * a12 - a32 * a13) + a31 * (a23 * a12 - a22 * a13);
    r.cof[0] = a33 * a22 - a32 * a23;
    r.cof[1] = a31 * a23 - a33 * a21;
    r.cof[2] = a32 * a21 - a31 * a22;
    r.cof[3] = a32 * a13 - a33 * a12;
    r.cof[4] = a33 * a11 - a31 * a13;
    r.cof[5] = a31 * a12 - a32 * a11;
    r.cof[6] = a23 * a12 - a22 * a13;
    r.cof[7] = a21 * a13 - a23 * a11;
    r.cof[8] = a22 * a11 - a21 * a12;
    r.idet = 1 / DET;
    r.N = N;
    r.mI[0] = mI[0];
    r.mI[1] = mI[1];
    r.mI[2] = mI[2];
    pix[t] = r;
}

// ---------------------------------------------------------------------------------------------
// Volume sweeps: one wave per (pair, line, 64-disparity chunk), lane = disparity
// ---------------------------------------------------------------------------------------------
template <bool HORIZ, int MODE>   // MODE 0: first box (from p), MODE 1: second box (from a, b)
__global__ __launch_bounds__(64) void k_gf_sweep(const GfArgs a) {
    const int lane = threadIdx.x;
    const int nchunks = (a.D + 63) >> 6;
    const int lines = HORIZ ? a.H : a.W;
    const int blk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int b = blk / (lines * nchunks);
    const int lc = blk - b * lines * nchunks;
    const int line = lc / nchunks, chunk = lc - line * nchunks;
    const int d = chunk * 64 + lane;
    const bool live = d < a.D;
    const int dd = live ? d : a.D - 1;
    const size_t npix = (size_t)a.H * a.W;
    const int len = HORIZ ? a.W : a.H;
    const size_t pstep = HORIZ ? 1 : (size_t)a.W;            // pixels between positions
    const size_t p0 = (size_t)b * npix + (HORIZ ? (size_t)line * a.W : (size_t)line);
    const size_t vstep = pstep * a.D;
    const size_t v0 = p0 * a.D + dd;
    const uint8_t* px0 = a.bgr + (size_t)b * a.bgr_pair_stride + (HORIZ ? (size_t)line * a.W : (size_t)line) * 3;
    float* const s[4] = {a.s0, a.s1, a.s2, a.s3};

    float ring[4][GF_RING];
    float S[4] = {0.f, 0.f, 0.f, 0.f};
    // blocks of GF_RING positions, each processed in SM_GF_PARTS parts of GF_RING / SM_GF_PARTS
    // (fewer input registers per part: more waves per SIMD; the ring slots stay static)
    constexpr int PART = GF_RING / SM_GF_PARTS;
    for (int j00 = 0; j00 < len + GF_R; j00 += GF_RING)
#pragma unroll
    for (int part = 0; part < SM_GF_PARTS; part++) {
        const int j0 = j00 + part * PART;
        if (j0 >= len + GF_R) break;
        // inputs of this part of the block
        float x[PART][4];
#pragma unroll
        for (int sp = 0; sp < PART; sp++) {
            const int sl = sp;
            const int j = j0 + sl;
            const bool in = j < len;
            const size_t jv = (size_t)(in ? j : len - 1);
            if (!HORIZ && MODE == 0) {
                const float p = a.vm[v0 + jv * vstep];
                const uint8_t* q = px0 + jv * pstep * 3;
                x[sl][0] = p;
                x[sl][1] = (float)q[0] * p;   // multiply(I_ch[c], p) (cpp:4992)
                x[sl][2] = (float)q[1] * p;
                x[sl][3] = (float)q[2] * p;
            } else {
#pragma unroll
                for (int c = 0; c < 4; c++) x[sl][c] = s[c][v0 + jv * vstep];
            }
            if (!in) {
#pragma unroll
                for (int c = 0; c < 4; c++) x[sl][c] = 0.f;
            }
        }
#pragma unroll
        for (int sp = 0; sp < PART; sp++) {
            const int sl = part * PART + sp;   // ring slot (static)
            const int j = j00 + sl;
            if (j >= len + GF_R) break;
            float bx[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                // CumSum: 0 + x at the first row (V), x itself at the first column (H); past the
                // end + 0, which keeps S(len - 1) (S is never -0)
                S[c] = (j == 0) ? (HORIZ ? x[sp][c] : 0.f + x[sp][c]) : S[c] + x[sp][c];
                ring[c][sl] = S[c];
            }
            const int i = j - GF_R;
            if (i < 0) continue;
#pragma unroll
            for (int c = 0; c < 4; c++) bx[c] = i >= GF_R + 1 ? S[c] - ring[c][(sl + 1) % GF_RING] : S[c];
            const size_t vo = v0 + (size_t)i * vstep;
            if (!HORIZ) {
                if (live) {
#pragma unroll
                    for (int c = 0; c < 4; c++) s[c][vo] = bx[c];
                }
                continue;
            }
            const GfPix& P = a.pix[p0 + (size_t)i * pstep];
            const float N = P.N;
            if (MODE == 0) {
                const float mean_p = bx[0] / N;
                double cv[3];
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const float mIp = bx[1 + c] / N;
                    const float m = P.mI[c] * mean_p;
                    cv[c] = (double)(mIp - m);
                }
                float av[3];
#pragma unroll
                for (int c = 0; c < 3; c++)
                    av[c] = (float)(P.idet * (cv[0] * P.cof[3 * c] + cv[1] * P.cof[3 * c + 1] + cv[2] * P.cof[3 * c + 2]));
                float bb = mean_p;
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const float m = av[c] * P.mI[c];
                    bb -= m;
                }
                if (live) {
                    s[0][vo] = av[0];
                    s[1][vo] = av[1];
                    s[2][vo] = av[2];
                    s[3][vo] = bb;
                }
            } else {
                const uint8_t* q = px0 + (size_t)i * 3;
                float out = bx[3] / N;   // q = mean_b (cpp:5097)
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const float ma = bx[c] / N;
                    const float m = ma * (float)q[c];
                    out += m;
                }
                if (a.solve_all) {   // SolveAll fused (sm_run): its `sum = 0; sum += w * v`
                    float sum = 0.f;
                    sum += a.scale * out;
                    out = sum;
                }
                if (live) a.vm[vo] = out;
            }
        }
    }
}

}  // namespace

void launch_gf(const GfArgs& a, int n, hipStream_t st) {
    {
        const int th = n * 10 * a.W;
        hipLaunchKernelGGL(k_gf_img_v, dim3((th + 255) / 256), dim3(256), 0, st, a.px, a.planes, a.H, a.W, n, a.px_pair_stride);
        const int tr = n * 10 * a.H;
        hipLaunchKernelGGL(k_gf_img_h, dim3((tr + 63) / 64), dim3(64), 0, st, a.planes, a.H, a.W, n);
        const size_t tp = (size_t)n * a.H * a.W;
        hipLaunchKernelGGL(k_gf_pix, dim3((unsigned)((tp + 255) / 256)), dim3(256), 0, st, a.planes, a.pix, a.H, a.W, n, a.eps);
    }
    GfArgs g = a;
    const int nchunks = (a.D + 63) / 64;
    hipLaunchKernelGGL((k_gf_sweep<false, 0>), dim3(a.W * nchunks * n), dim3(64), 0, st, g);
    hipLaunchKernelGGL((k_gf_sweep<true, 0>), dim3(a.H * nchunks * n), dim3(64), 0, st, g);
    hipLaunchKernelGGL((k_gf_sweep<false, 1>), dim3(a.W * nchunks * n), dim3(64), 0, st, g);
    hipLaunchKernelGGL((k_gf_sweep<true, 1>), dim3(a.H * nchunks * n), dim3(64), 0, st, g);
}

}  // namespace sm
