// sm_nl.hip — aggregation "NL" (NL(), stereoMatching.cpp:4892-4917): Qingxiong Yang's non-local
// cost aggregation on the minimum spanning tree of the left colour image (NL/NLCCA.cpp:27-96).
//
//   edges      ctmf 3x3 median of each channel with clamped borders (NL/ctmf.c, called with r = 1
//              by qx_mst_kruskals_image::mst), weight = max channel |difference| of 4-neighbours
//   tree       host (sm_nl_tree.cpp): Kruskal + breadth-first orientation + heavy paths
//   filter     qx_tree_filter::filter (NL/qx_tree_filter.cpp:61-117) in double, w = exp(-c / 25.5):
//                up(x)  = C(x) + sum_j up(child_j) * w(child_j)           children in list order
//                fin(x) = w(x) * (fin(parent) - w(x) * up(x)) + up(x),    fin(root) = up(root)
//   NL()       vm = (float)fin(C) / (float)fin(1)   (the ones volume, cpp:4899-4910)
//
// gfx950 mapping: one wave per (heavy path, 64-disparity chunk), lane = disparity, walking the path
// node by node; the child on the same path arrives in a register, the other children (their paths
// finished in earlier rounds) from memory.  A round is one launch; a node's sum keeps the
// reference's child order, so rounds only schedule work and the result is the restatement's bit for
// bit.  Intermediate values are doubles, as in the reference (m_cost_vol is double).
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

namespace sm {

namespace {

__device__ __forceinline__ void cswap(int& a, int& b) {
    const int lo = min(a, b), hi = max(a, b);
    a = lo;
    b = hi;
}

// median of 9 (a classic 19-exchange network)
__device__ __forceinline__ int median9(int p[9]) {
    cswap(p[1], p[2]); cswap(p[4], p[5]); cswap(p[7], p[8]);
    cswap(p[0], p[1]); cswap(p[3], p[4]); cswap(p[6], p[7]);
    cswap(p[1], p[2]); cswap(p[4], p[5]); cswap(p[7], p[8]);
    cswap(p[0], p[3]); cswap(p[5], p[8]); cswap(p[4], p[7]);
    cswap(p[3], p[6]); cswap(p[1], p[4]); cswap(p[2], p[5]);
    cswap(p[4], p[7]); cswap(p[4], p[2]); cswap(p[6], p[4]);
    cswap(p[4], p[2]);
    return p[4];
}

__global__ __launch_bounds__(256) void k_nl_median(const uint8_t* __restrict__ bgr, size_t pair_stride, uint8_t* __restrict__ med,
                                                   int H, int W, int n) {
    const size_t npix = (size_t)H * W;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npix * n) return;
    const size_t b = t / npix, i = t - b * npix;
    const int y = (int)(i / W), x = (int)(i - (size_t)y * W);
    const uint8_t* src = bgr + b * pair_stride;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        int p[9], k = 0;
#pragma unroll
        for (int dy = -1; dy <= 1; dy++)
#pragma unroll
            for (int dx = -1; dx <= 1; dx++) {
                const int yy = min(max(y + dy, 0), H - 1), xx = min(max(x + dx, 0), W - 1);
                p[k++] = src[((size_t)yy * W + xx) * 3 + c];
            }
        med[t * 3 + c] = (uint8_t)median9(p);
    }
}

// edge weights: [pair][H (W-1) horizontal, row by row | (H-1) W vertical, column by column]
__global__ __launch_bounds__(256) void k_nl_edges(const uint8_t* __restrict__ med, uint8_t* __restrict__ ew, int H, int W, int n) {
    const size_t npix = (size_t)H * W;
    const int neh = H * (W - 1), ne = neh + (H - 1) * W;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)ne * n) return;
    const size_t b = t / ne;
    const int e = (int)(t - b * ne);
    int u, v;
    if (e < neh) {
        const int y = e / (W - 1), x = e - y * (W - 1);
        u = y * W + x;
        v = u + 1;
    } else {
        const int k = e - neh, x = k / (H - 1), y = k - x * (H - 1);
        u = y * W + x;
        v = u + W;
    }
    const uint8_t* m = med + b * npix * 3;
    int w = 0;
#pragma unroll
    for (int c = 0; c < 3; c++) w = max(w, abs((int)m[(size_t)v * 3 + c] - (int)m[(size_t)u * 3 + c]));
    ew[t] = (uint8_t)w;
}

// up pass over the paths chains[lo, hi): bottom -> top
__global__ __launch_bounds__(64) void k_nl_up(const NlArgs a, int lo, int P) {
    const int nchunks = (P + 63) >> 6;
    const int ci = a.order_up[lo + blockIdx.x / nchunks];
    const int d = (blockIdx.x % nchunks) * 64 + threadIdx.x;
    if (d >= P) return;
    const int* nodes = a.chain_nodes + a.chain_start[ci];
    const int len = a.chain_len[ci];
    double carry = 0.0;
    for (int t = 0; t < len; t++) {
        const int x = nodes[t];
        double v = P == 1 ? 1.0 : (double)a.vm[(size_t)x * P + d];
        const int nc = a.nchild[x];
        const int hv = a.heavy[x];
        for (int j = 0; j < nc; j++) {
            const int c = a.child[(size_t)x * 4 + j];
            const double w = a.table[a.weight[c]];
            const double cv = (j == hv) ? carry : a.val[(size_t)c * P + d];
            const double m = cv * w;
            v = v + m;
        }
        a.val[(size_t)x * P + d] = v;
        carry = v;
    }
}

// down pass over the paths chains[lo, hi): top -> bottom; writes the final doubles in place and
// the normalised float volume (P = D) or the float weight sums (P = 1)
__global__ __launch_bounds__(64) void k_nl_down(const NlArgs a, int lo, int P) {
    const int nchunks = (P + 63) >> 6;
    const int ci = a.order_down[lo + blockIdx.x / nchunks];
    const int d = (blockIdx.x % nchunks) * 64 + threadIdx.x;
    if (d >= P) return;
    const int* nodes = a.chain_nodes + a.chain_start[ci];
    const int len = a.chain_len[ci];
    double carry = 0.0;
    for (int t = len - 1; t >= 0; t--) {
        const int x = nodes[t];
        const double up = a.val[(size_t)x * P + d];
        const int p = a.parent[x];
        double fin;
        if (p == x) {
            fin = up;                                   // the root
        } else {
            const double w = a.table[a.weight[x]];
            const double fp = (t == len - 1) ? a.val[(size_t)p * P + d] : carry;
            const double m = w * up;
            const double q = fp - m;
            const double r = w * q;
            fin = r + up;
        }
        a.val[(size_t)x * P + d] = fin;
        carry = fin;
        if (P == 1)
            a.wsum[x] = (float)fin;
        else
            a.vm[(size_t)x * P + d] = (float)fin / a.wsum[x];
    }
}

}  // namespace

void launch_nl_edges(const uint8_t* bgr, size_t pair_stride, uint8_t* med, uint8_t* ew, int H, int W, int n, hipStream_t st) {
    const size_t np = (size_t)H * W * n;
    hipLaunchKernelGGL(k_nl_median, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, st, bgr, pair_stride, med, H, W, n);
    const size_t ne = ((size_t)H * (W - 1) + (size_t)(H - 1) * W) * n;
    hipLaunchKernelGGL(k_nl_edges, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st, med, ew, H, W, n);
}

void launch_nl_round(const NlArgs& a, bool up, int lo, int hi, int P, hipStream_t st) {
    if (hi <= lo) return;
    const int nchunks = (P + 63) / 64;
    const dim3 grid((unsigned)((hi - lo) * nchunks));
    if (up)
        hipLaunchKernelGGL(k_nl_up, grid, dim3(64), 0, st, a, lo, P);
    else
        hipLaunchKernelGGL(k_nl_down, grid, dim3(64), 0, st, a, lo, P);
}

}  // namespace sm
