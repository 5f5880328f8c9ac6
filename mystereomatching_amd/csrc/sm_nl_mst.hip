// sm_nl_mst.hip — the NL minimum spanning tree on the GPU (qx_mst_kruskals_image::mst,
// NL/qx_mst_kruskals_image.cpp:167-277): Boruvka rounds over a union-find forest, then every
// pixel's neighbour list in the reference's order.
//
// Why it equals the reference's tree.  Kruskal there visits the edges sorted stably by weight
// (a counting sort), i.e. in increasing order of the key (weight, edge index), which is a strict
// total order; so its tree is THE minimum spanning tree under that key, and every edge that is
// the lightest key leaving some component of a spanning forest of lighter edges belongs to it
// (cut property).  Boruvka adds exactly such edges, so it builds the same edge set.  A pixel's
// neighbour list is its tree edges in Kruskal's acceptance order, which is again increasing key.
//
// Rounds: (1) every pixel offers the keys of its right and down edges, when their endpoints lie
// in different components, to both components' roots (atomic 64-bit minimum); (2) every root
// holding a key marks that edge as a tree edge and unites its two endpoints (lock-free: link the
// larger root under the smaller by compare-and-swap, finds halve paths); (3) every pixel points
// straight at its root, so the next round's offers read each endpoint's root with one load.
// Each round at least halves the number of components of every pair, so ceil(log2(H W)) rounds
// finish; a round in which nothing was united clears the flag the later rounds' kernels test
// first, so they return at once.  (4) one pass builds the neighbour words the host walk reads
// (sm_nl_tree.h): count | direction j << (3 + 2 j) | right weight << 16 | down weight << 24,
// directions 0: +1, 1: -1, 2: +W, 3: -W (one column: the vertical edges use 0 / 1).
// Layout (per batch of nn = n H W pixels, in `scratch`): tree flags of each pixel's right edge
// [nn] and down edge [nn] (bytes), the pixel's (right | down << 8) weights [nn] (u16, the
// vertical weights transposed from k_nl_edges' column-major order), then one flag per round.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_kernels.h"

namespace sm {

namespace {

typedef unsigned long long u64;

__device__ __forceinline__ int ld_par(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_par(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// root of x with path halving
__device__ __forceinline__ int uf_find(int* par, int x) {
    for (;;) {
        const int p = ld_par(par + x);
        if (p == x) return x;
        const int g = ld_par(par + p);
        if (g == p) return p;
        st_par(par + x, g);
        x = g;
    }
}

__device__ __forceinline__ void uf_unite(int* par, int a, int b) {
    for (;;) {
        a = uf_find(par, a);
        b = uf_find(par, b);
        if (a == b) return;
        if (a > b) {
            const int t = a;
            a = b;
            b = t;
        }
        int expect = b;
        if (__hip_atomic_compare_exchange_strong(par + b, &expect, a, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return;
    }
}

// edge indices of k_nl_edges' numbering: horizontal edges row by row, then vertical column by column
__device__ __forceinline__ int edge_right(int y, int x, int W) { return y * (W - 1) + x; }
__device__ __forceinline__ int edge_down(int y, int x, int H, int W) { return H * (W - 1) + x * (H - 1) + y; }

__global__ __launch_bounds__(256) void k_mst_init(const uint8_t* __restrict__ ew, int* __restrict__ par, u64* __restrict__ best,
                                                  uint8_t* __restrict__ scratch, int* __restrict__ live, int H, int W, int n,
                                                  int rounds) {
    const int np = H * W, nn = np * n, ne = H * (W - 1) + (H - 1) * W;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t <= rounds) live[t] = t == 0;
    if (t >= nn) return;
    const int b = t / np, p = t - b * np, y = p / W, x = p - y * W;
    const uint8_t* e = ew + (long)b * ne;
    par[t] = t;
    best[t] = ~0ull;
    scratch[t] = 0;
    scratch[nn + t] = 0;
    const uint32_t wr = x < W - 1 ? e[edge_right(y, x, W)] : 0u;
    const uint32_t wd = y < H - 1 ? e[edge_down(y, x, H, W)] : 0u;
    ((uint16_t*)(scratch + 2 * (long)nn))[t] = (uint16_t)(wr | wd << 8);
}

__global__ __launch_bounds__(256) void k_mst_offer(const int* __restrict__ par, u64* best, const uint8_t* __restrict__ scratch,
                                                   const int* __restrict__ live, int r, int H, int W, int n) {
    if (!live[r]) return;
    const int np = H * W, nn = np * n;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nn) return;
    const int b = t / np, p = t - b * np, y = p / W, x = p - y * W;
    const uint32_t wp = ((const uint16_t*)(scratch + 2 * (long)nn))[t];
    const int ru = par[t];
    if (x < W - 1) {
        const int rv = par[t + 1];
        if (ru != rv) {
            const u64 key = (u64)(wp & 0xffu) << 32 | (uint32_t)edge_right(y, x, W);
            atomicMin(best + ru, key);
            atomicMin(best + rv, key);
        }
    }
    if (y < H - 1) {
        const int rv = par[t + W];
        if (ru != rv) {
            const u64 key = (u64)(wp >> 8) << 32 | (uint32_t)edge_down(y, x, H, W);
            atomicMin(best + ru, key);
            atomicMin(best + rv, key);
        }
    }
}

__global__ __launch_bounds__(256) void k_mst_unite(int* par, u64* __restrict__ best, uint8_t* __restrict__ scratch,
                                                   int* __restrict__ live, int r, int H, int W, int n) {
    if (!live[r]) return;
    const int np = H * W, nn = np * n, neh = H * (W - 1);
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nn) return;
    const u64 key = best[t];
    if (key == ~0ull) return;
    best[t] = ~0ull;
    const int b = t / np, e = (int)(uint32_t)key;
    int u, v;
    if (e < neh) {
        const int y = e / (W - 1), x = e - y * (W - 1);
        u = y * W + x;
        v = u + 1;
        scratch[b * np + u] = 1;
    } else {
        const int k = e - neh, x = k / (H - 1), y = k - x * (H - 1);
        u = y * W + x;
        v = u + W;
        scratch[nn + b * np + u] = 1;
    }
    uf_unite(par, b * np + u, b * np + v);
    live[r + 1] = 1;
}

// every pixel -> its root (parents only move towards the roots, so stale reads still progress)
__global__ __launch_bounds__(256) void k_mst_flatten(int* par, const int* __restrict__ live, int r, int nn) {
    if (!live[r + 1]) return;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nn) return;
    int x = ld_par(par + t);
    for (;;) {
        const int p = ld_par(par + x);
        if (p == x) break;
        x = p;
    }
    st_par(par + t, x);
}

__global__ __launch_bounds__(256) void k_mst_lists(const uint8_t* __restrict__ scratch, uint32_t* __restrict__ adj, int H, int W, int n) {
    const int np = H * W, nn = np * n;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nn) return;
    const int b = t / np, p = t - b * np, y = p / W, x = p - y * W;
    const uint8_t* fr = scratch;
    const uint8_t* fd = scratch + nn;
    const uint16_t* wp = (const uint16_t*)(scratch + 2 * (long)nn);
    // the pixel's tree edges +1, -1, +W, -W as (weight, edge index) keys with the direction in the
    // two low bits (absent: all ones), then a 5-exchange sorting network on increasing key
    const bool in[4] = {x < W - 1 && fr[t], x > 0 && fr[t - 1], y < H - 1 && fd[t], y > 0 && fd[t - W]};
    const uint32_t w[4] = {in[0] ? wp[t] & 0xffu : 0u, in[1] ? wp[t - 1] & 0xffu : 0u, in[2] ? (uint32_t)wp[t] >> 8 : 0u,
                           in[3] ? (uint32_t)wp[t - W] >> 8 : 0u};
    const int ei[4] = {edge_right(y, x, W), edge_right(y, x - 1, W), edge_down(y, x, H, W), edge_down(y - 1, x, H, W)};
    u64 k[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint32_t d = W > 1 ? (uint32_t)c : (uint32_t)(c & 1);
        k[c] = in[c] ? ((u64)w[c] << 32 | (u64)(uint32_t)ei[c] << 2 | d) : ~0ull;
    }
    auto cx = [](u64& a, u64& b) {
        const u64 lo = a < b ? a : b, hi = a < b ? b : a;
        a = lo;
        b = hi;
    };
    cx(k[0], k[1]);
    cx(k[2], k[3]);
    cx(k[0], k[2]);
    cx(k[1], k[3]);
    cx(k[1], k[2]);
    uint32_t a = (uint32_t)wp[t] << 16;   // the pixel's right | down weights
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (k[j] == ~0ull) continue;
        a |= (uint32_t)(k[j] & 3ull) << (3 + 2 * j);
        cnt++;
    }
    adj[t] = a | cnt;
}

}  // namespace

int nl_mst_rounds(int np) {
    int r = 0;
    while ((1 << r) < np) r++;
    return r;
}

size_t nl_mst_scratch_bytes(int H, int W, int n) { return (size_t)4 * H * W * n + 4 * 64; }

void launch_nl_mst(const uint8_t* ew, int H, int W, int n, int* par, unsigned long long* best, uint8_t* scratch,
                   uint32_t* adj, hipStream_t st) {
    const int np = H * W, nn = np * n;
    const unsigned gn = (unsigned)((nn + 255) / 256);
    const int rounds = nl_mst_rounds(np);
    int* live = (int*)(scratch + 4 * (size_t)nn);
    hipLaunchKernelGGL(k_mst_init, dim3(gn), dim3(256), 0, st, ew, par, best, scratch, live, H, W, n, rounds);
    for (int r = 0; r < rounds; r++) {
        hipLaunchKernelGGL(k_mst_offer, dim3(gn), dim3(256), 0, st, par, best, scratch, live, r, H, W, n);
        hipLaunchKernelGGL(k_mst_unite, dim3(gn), dim3(256), 0, st, par, best, scratch, live, r, H, W, n);
        hipLaunchKernelGGL(k_mst_flatten, dim3(gn), dim3(256), 0, st, par, live, r, nn);
    }
    hipLaunchKernelGGL(k_mst_lists, dim3(gn), dim3(256), 0, st, scratch, adj, H, W, n);
}

}  // namespace sm
