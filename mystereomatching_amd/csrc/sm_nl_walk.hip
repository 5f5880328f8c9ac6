// sm_nl_walk.hip — the NL tree walk on the GPU: the breadth-first orientation of each pair's
// minimum spanning tree from pixel 0 (NL/qx_mst_kruskals_image.cpp:229-277, build_tree), cut into
// heavy paths, packed into the records and round tables the tree filter (sm_nl.hip) walks.
//
// The reference orients the tree by a breadth-first walk from pixel 0 and makes every neighbour
// but the parent a child, in list order.  What the filter's arithmetic depends on is only the
// parent of every node and its children's order (qx_tree_filter.cpp:61-117); both are properties
// of the rooted tree, not of the walk that found them, so any traversal that roots the same tree
// at pixel 0 gives the same sums bit for bit.  Here:
//
//   tour      the Euler tour of the tree: arc (p -> q) is followed by the arc out of q that comes
//             after (q -> p) in q's cyclic list; the tour starts at pixel 0's first arc.
//   ranks     list ranking of the tour: the first arc of about one node in WALK_K (by a hash of
//             the node) starts a sublist; every start walks its sublist (k_walk_sub), the starts'
//             list is ranked by pointer jumping over node-indexed arrays (k_walk_jump, ceil(log2)
//             rounds), and the starts walk again writing the ranks (k_walk_rank) -- no atomics.
//   nodes     the arc entering v is the one of v's two arcs to a neighbour with the smaller rank
//             (that neighbour is the parent); subtree size = (rank out - rank in - 1) / 2 + 1;
//             children = the list minus the parent, in list order; the heavy child = the first
//             of the largest (as sm_nl_tree.cpp).
//   preorder  heavy-child-first preorder numbers as root-path sums: pre(v) = pre(parent) + 1 for
//             the heavy child, + 1 + size(heavy) + sizes of the earlier light children otherwise,
//             evaluated by one prefix sum over the tour (+x on entering a child, -x on leaving);
//             the same sum carries the light depth (down level).  A heavy path is then a run of
//             consecutive preorder numbers, stored in reverse (bottom -> top) as the filter reads
//             it: record slot = pair base + (H W - 1 - pre).
//   paths     path bottom = the first leaf at or after a node in preorder (a min-scan), path top
//             of a node = the last top at or before it (a max-scan); the up level of a path
//             (1 + the largest up level of a path hanging off it) is propagated from the deepest
//             light depth upwards, one launch per depth; round tables by counting sort.
// Per batch of n pairs, all on the NL front stream; the host reads back only the round offsets.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>
#include <climits>

#include "sm_kernels.h"

namespace sm {

namespace {

constexpr int WALK_K = 8;         // the first arc of about one node in WALK_K starts a sublist
constexpr long long PRE_MASK = (1LL << 40) - 1;   // tour sums: preorder offset | light depth << 40

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// node g (pair-local index p) starts a sublist at its first arc; pixel 0 (whose first arc is the
// tour's first) always does
__device__ __forceinline__ bool start_node(uint32_t p) { return p == 0 || (mix32(p) & (WALK_K - 1)) == 0; }
__device__ __forceinline__ bool is_start(int a, int base_node) { return (a & 3) == 0 && start_node((uint32_t)((a >> 2) - base_node)); }

__device__ __forceinline__ int dir_delta(uint32_t c, int W) { return c == 0 ? 1 : (c == 1 ? -1 : (c == 2 ? W : -W)); }
__device__ __forceinline__ uint32_t dir_at(uint32_t a, int j) { return (a >> (3 + 2 * j)) & 3u; }
// list position of direction c in neighbour word a (-1 if absent)
__device__ __forceinline__ int list_pos(uint32_t a, uint32_t c) {
    const int cnt = (int)(a & 7u);
    int r = -1;
    for (int j = 0; j < 4; j++)
        if (j < cnt && dir_at(a, j) == c && r < 0) r = j;
    return r;
}
// weight of the edge leaving g in direction c: the right / down field of its left / upper end
__device__ __forceinline__ uint32_t edge_w(const uint32_t* __restrict__ adj, long g, uint32_t c, int W) {
    switch (c) {
    case 0: return (adj[g] >> 16) & 255u;
    case 1: return (adj[g - 1] >> 16) & 255u;
    case 2: return adj[g] >> 24;
    default: return adj[g - W] >> 24;
    }
}

struct WalkBufs {
    int* succ;        // [4 nn] next arc of the tour (-1: the last, -2: no such arc)
    int* rank;        // [4 nn] position in the pair's tour
    int* jn[2];       // [nn] per start node: pointer jumping: next start node, arcs to the tour's end
    int* jd[2];
    int* err;         // set when a tour is not a spanning tree's
    uint8_t* pdir;    // [nn] direction to the parent (4: the root)
    uint8_t* hvf;     // [nn] 1: the heavy child of its parent
    int* size;        // [nn] subtree size
    int* erank;       // [nn] rank of the arc entering the node
    uint32_t* meta;   // [nn] record meta word (nchild | (heavy + 1) << 3 | cdir << 6 | weight << 16)
    uint32_t* wp;     // [nn] children's edge weights
    int* pre;         // [nn] heavy-first preorder number in the pair
    int* dl;          // [nn] light depth (down level)
    long long* tour;  // [n T] +-(offset | light << 40) in tour order
    long long* tsum;  // [n T] inclusive prefix sums
    int* lrev;        // [nn] reversed preorder: position if a leaf, else INT_MAX -> min-scan
    int* lsc;
    int* tp;          // [nn] preorder: position if a path top, else -1 -> max-scan
    int* tsc;
    int* ptop;        // [nn] per top position: the top position of its parent's path (-1 root, -2 no top)
    int* ul;          // [nn] per top position: up level
    int* dlp;         // [nn] per top position: down level
    int* hist;        // [4 (NL_LEVELS + 1)] up / down counts, then cursors
    void* cub;        // hipcub temporary storage
    size_t cub_bytes;
};

__global__ __launch_bounds__(256) void k_walk_succ(const uint32_t* __restrict__ adj, WalkBufs w, int np, int W, long na) {
    const long a = (long)blockIdx.x * 256 + threadIdx.x;
    if (a >= na) return;
    const long g = a >> 2;
    const int j = (int)(a & 3);
    const long b = (long)((int)g / np);   // (node ids < 2^31: 32-bit division)
    const uint32_t x = adj[g];
    if (j >= (int)(x & 7u)) {
        w.succ[a] = -2;
        return;
    }
    const uint32_t c = dir_at(x, j);
    const long q = g + dir_delta(c, W);
    const uint32_t y = adj[q];
    const int jp = list_pos(y, c ^ 1u), cq = (int)(y & 7u);
    const int nj = jp + 1 == cq ? 0 : jp + 1;
    long nx = 4 * q + nj;
    if (q == b * np && nj == 0) nx = -1;   // back at the tour's first arc: the end
    w.succ[a] = jp < 0 ? -1 : (int)nx;
    if (jp < 0) atomicOr(w.err, 1);        // not a symmetric neighbour list
}

// every sublist start walks to the next start: its length and successor start node
__global__ __launch_bounds__(256) void k_walk_sub(WalkBufs w, int np, int nn) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= nn) return;
    const int base = g / np * np;
    if (!start_node((uint32_t)(g - base))) return;
    int cur = w.succ[4 * g], len = 1;
    while (cur >= 0 && !is_start(cur, base)) {
        if (len > 4 * np) {   // a list that is no tour (a cycle without a start): stop, flag it
            atomicOr(w.err, 8);
            cur = -1;
            break;
        }
        cur = w.succ[cur];
        len++;
    }
    w.jn[0][g] = cur < 0 ? -1 : cur >> 2;
    w.jd[0][g] = len;
}

__global__ __launch_bounds__(256) void k_walk_jump(const int* __restrict__ nin, const int* __restrict__ din, int* __restrict__ nout,
                                                   int* __restrict__ dout, int np, int nn) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= nn || !start_node((uint32_t)(g % np))) return;
    int x = nin[g], d = din[g];
    if (x >= 0) {
        d += din[x];
        x = nin[x];
    }
    nout[g] = x;
    dout[g] = d;
}

// the starts walk their sublists again, writing the ranks (2 (H W - 1) arcs per tour)
__global__ __launch_bounds__(256) void k_walk_rank(WalkBufs w, const int* __restrict__ dist, int np, int nn) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= nn) return;
    const int base = g / np * np;
    if (!start_node((uint32_t)(g - base))) return;
    int r = 2 * (np - 1) - dist[g];
    if (g == base && r != 0) atomicOr(w.err, 2);   // the tour from pixel 0 misses arcs
    w.rank[4 * g] = r;
    int cur = w.succ[4 * g];
    for (int steps = 0; cur >= 0 && !is_start(cur, base); steps++) {
        if (steps > 4 * np) {
            atomicOr(w.err, 8);
            break;
        }
        w.rank[cur] = ++r;
        cur = w.succ[cur];
    }
}

// parent direction, entering rank, subtree size
__global__ __launch_bounds__(256) void k_walk_node1(const uint32_t* __restrict__ adj, WalkBufs w, int np, int W, long nn) {
    if (*w.err) return;   // not a spanning tree's tour (flags read by the host): indices below are invalid
    const long g = (long)blockIdx.x * 256 + threadIdx.x;
    if (g >= nn) return;
    const long b = (long)((int)g / np);   // (node ids < 2^31: 32-bit division)
    if (g == b * np) {
        w.pdir[g] = 4;
        w.erank[g] = -1;
        w.size[g] = np;
        return;
    }
    const uint32_t x = adj[g];
    const int cnt = (int)(x & 7u);
    int found = 0;
    for (int j = 0; j < 4; j++) {
        if (j >= cnt) break;
        const uint32_t c = dir_at(x, j);
        const long q = g + dir_delta(c, W);
        const int jp = list_pos(adj[q], c ^ 1u);
        const int rout = w.rank[4 * g + j], rin = w.rank[4 * q + jp];
        if (rin < rout) {
            w.pdir[g] = (uint8_t)c;
            w.erank[g] = rin;
            w.size[g] = (rout - rin - 1) / 2 + 1;
            found++;
        }
    }
    if (found != 1) atomicOr(w.err, 4);
}

// children, heavy child, record words; the children's preorder offsets into the tour
__global__ __launch_bounds__(256) void k_walk_node2(const uint32_t* __restrict__ adj, WalkBufs w, int np, int W, long nn) {
    if (*w.err) return;   // not a spanning tree's tour (flags read by the host): indices below are invalid
    const long g = (long)blockIdx.x * 256 + threadIdx.x;
    if (g >= nn) return;
    const long b = (long)((int)g / np);   // (node ids < 2^31: 32-bit division)
    const uint32_t x = adj[g];
    const int cnt = (int)(x & 7u);
    const uint32_t pd = w.pdir[g];
    int nc = 0, heavy = -1, hs = 0;
    uint32_t cdir = 0, wpk = 0;
    int csz[4], cj[4];
    long cq[4];
    for (int j = 0; j < 4; j++) {
        if (j >= cnt) break;
        const uint32_t c = dir_at(x, j);
        if (c == pd) continue;
        const long q = g + dir_delta(c, W);
        const int sz = w.size[q];
        if (sz > hs) {
            hs = sz;
            heavy = nc;
        }
        cdir |= c << (2 * nc);
        wpk |= edge_w(adj, g, c, W) << (8 * nc);
        csz[nc] = sz;
        cj[nc] = j;
        cq[nc] = q;
        nc++;
    }
    const uint32_t own = pd < 4 ? edge_w(adj, g, pd, W) : 0u;
    w.meta[g] = (uint32_t)nc | (uint32_t)(heavy + 1) << 3 | cdir << 6 | own << 16;
    w.wp[g] = wpk;
    const long T = 2 * (long)(np - 1);
    long long acc = 1 + (long long)hs;   // the first light child follows the heavy child's subtree
    for (int i = 0; i < nc; i++) {
        long long off;
        long long light;
        if (i == heavy) {
            off = 1;
            light = 0;
        } else {
            off = acc;
            acc += csz[i];
            light = 1;
        }
        const long long pk = off | light << 40;
        const uint32_t c = dir_at(x, cj[i]);
        const int e = w.rank[4 * g + cj[i]];                              // g -> child: entering
        const int l = w.rank[4 * cq[i] + list_pos(adj[cq[i]], c ^ 1u)];   // child -> g: leaving
        w.tour[b * T + e] = pk;
        w.tour[b * T + l] = -pk;
        w.hvf[cq[i]] = (uint8_t)(i == heavy);
    }
}

__global__ __launch_bounds__(256) void k_walk_node3(WalkBufs w, int np, long nn) {
    if (*w.err) return;   // not a spanning tree's tour (flags read by the host): indices below are invalid
    const long g = (long)blockIdx.x * 256 + threadIdx.x;
    if (g >= nn) return;
    const long b = (long)((int)g / np);   // (node ids < 2^31: 32-bit division)
    const bool root = g == b * np;
    const long T = 2 * (long)(np - 1);
    long long s = root ? 0 : w.tsum[b * T + w.erank[g]];
    const int pre = (int)(s & PRE_MASK), dl = (int)(s >> 40);
    w.pre[g] = pre;
    w.dl[g] = dl;
    const long pos = b * np + pre;
    w.lrev[nn - 1 - pos] = (w.meta[g] & 7u) == 0 ? (int)pos : INT_MAX;
    w.tp[pos] = (root || !w.hvf[g]) ? (int)pos : -1;
}

// records (bottom -> top per path), path tables per top position
__global__ __launch_bounds__(256) void k_walk_node4(WalkBufs w, int4* __restrict__ rec, int* __restrict__ cstart, int* __restrict__ clen,
                                                    int np, int W, long nn) {
    if (*w.err) return;   // not a spanning tree's tour (flags read by the host): indices below are invalid
    const long g = (long)blockIdx.x * 256 + threadIdx.x;
    if (g >= nn) return;
    const long b = (long)((int)g / np);   // (node ids < 2^31: 32-bit division)
    const bool root = g == b * np;
    const int pre = w.pre[g];
    const long pos = b * np + pre;
    const int hlen = w.lsc[nn - 1 - pos] - (int)pos + 1;
    const long par = root ? g : g + dir_delta(w.pdir[g], W);
    rec[b * np + (np - 1 - pre)] = make_int4((int)g, (int)w.meta[g], (int)w.wp[g], (int)par);
    if (root || !w.hvf[g]) {
        cstart[pos] = (int)(b * np + np - pre - hlen);
        clen[pos] = hlen;
        w.ul[pos] = 0;
        w.dlp[pos] = w.dl[g];
        w.ptop[pos] = root ? -1 : w.tsc[b * np + w.pre[par]];
    } else {
        w.ptop[pos] = -2;
    }
}

__global__ __launch_bounds__(256) void k_walk_ul(WalkBufs w, long nn, int d) {
    if (*w.err) return;   // not a spanning tree's tour (flags read by the host): indices below are invalid
    const long pos = (long)blockIdx.x * 256 + threadIdx.x;
    if (pos >= nn) return;
    const int pt = w.ptop[pos];
    if (pt >= 0 && w.dlp[pos] == d) atomicMax(w.ul + pt, w.ul[pos] + 1);
}

// per-block histograms in LDS, one global atomic per nonzero bin and block
__global__ __launch_bounds__(256) void k_walk_hist(WalkBufs w, long nn) {
    if (*w.err) return;   // (uniform over the block: before any barrier)
    __shared__ int h[2 * NL_LEVELS];
    if (threadIdx.x < 2 * NL_LEVELS) h[threadIdx.x] = 0;
    __syncthreads();
    const long pos = (long)blockIdx.x * 256 + threadIdx.x;
    if (pos < nn && w.ptop[pos] != -2) {
        atomicAdd(h + min(w.ul[pos], NL_LEVELS - 1), 1);
        atomicAdd(h + NL_LEVELS + min(w.dlp[pos], NL_LEVELS - 1), 1);
    }
    __syncthreads();
    if (threadIdx.x < 2 * NL_LEVELS && h[threadIdx.x]) atomicAdd(w.hist + threadIdx.x, h[threadIdx.x]);
}

// offs: up round offsets [NL_LEVELS + 1], down round offsets [NL_LEVELS + 1], error flags
__global__ void k_walk_offs(WalkBufs w, int* __restrict__ offs) {
    if (threadIdx.x != 0) return;
    for (int k = 0; k < 2; k++) {
        int o = 0;
        for (int r = 0; r < NL_LEVELS; r++) {
            const int x = w.hist[k * NL_LEVELS + r];
            offs[k * (NL_LEVELS + 1) + r] = o;
            w.hist[2 * NL_LEVELS + k * NL_LEVELS + r] = o;   // cursor
            o += x;
        }
        offs[k * (NL_LEVELS + 1) + NL_LEVELS] = o;
    }
    offs[2 * (NL_LEVELS + 1)] = *w.err;
}

// counting-sort scatter: a block counts its tops per bin in LDS, reserves each bin's range with
// one global atomic, and places its tops (any order within a round is valid)
__global__ __launch_bounds__(256) void k_walk_scatter(WalkBufs w, int* __restrict__ oup, int* __restrict__ odn, long nn) {
    if (*w.err) return;   // (uniform over the block: before any barrier)
    __shared__ int h[2 * NL_LEVELS];
    if (threadIdx.x < 2 * NL_LEVELS) h[threadIdx.x] = 0;
    __syncthreads();
    const long pos = (long)blockIdx.x * 256 + threadIdx.x;
    const bool top = pos < nn && w.ptop[pos] != -2;
    int bu = 0, bd = 0, iu = 0, id = 0;
    if (top) {
        bu = min(w.ul[pos], NL_LEVELS - 1);
        bd = NL_LEVELS + min(w.dlp[pos], NL_LEVELS - 1);
        iu = atomicAdd(h + bu, 1);
        id = atomicAdd(h + bd, 1);
    }
    __syncthreads();
    if (threadIdx.x < 2 * NL_LEVELS) {
        const int c = h[threadIdx.x];
        h[threadIdx.x] = c ? atomicAdd(w.hist + 2 * NL_LEVELS + threadIdx.x, c) : 0;   // the block's first slot
    }
    __syncthreads();
    if (!top) return;
    oup[h[bu] + iu] = (int)pos;
    odn[h[bd] + id] = (int)pos;
}

struct MinOp {
    __device__ __forceinline__ int operator()(int a, int b) const { return a < b ? a : b; }
};
struct MaxOp {
    __device__ __forceinline__ int operator()(int a, int b) const { return a > b ? a : b; }
};

// carve the scratch (every piece 256-byte aligned); returns the bytes used
size_t carve(uint8_t* base, int H, int W, int n, WalkBufs* w) {
    const size_t np = (size_t)H * W, nn = np * n, na = 4 * nn, nt = (size_t)n * 2 * (np - 1);
    size_t o = 0;
    auto take = [&](size_t bytes) -> void* {
        void* p = base ? base + o : nullptr;
        o += (bytes + 255) / 256 * 256;
        return p;
    };
    WalkBufs t{};
    t.succ = (int*)take(na * 4);
    t.rank = (int*)take(na * 4);
    for (int k = 0; k < 2; k++) {
        t.jn[k] = (int*)take(nn * 4);
        t.jd[k] = (int*)take(nn * 4);
    }
    t.err = (int*)take(4);
    t.pdir = (uint8_t*)take(nn);
    t.hvf = (uint8_t*)take(nn);
    t.size = (int*)take(nn * 4);
    t.erank = (int*)take(nn * 4);
    t.meta = (uint32_t*)take(nn * 4);
    t.wp = (uint32_t*)take(nn * 4);
    t.pre = (int*)take(nn * 4);
    t.dl = (int*)take(nn * 4);
    t.tour = (long long*)take(nt * 8);
    t.tsum = (long long*)take(nt * 8);
    t.lrev = (int*)take(nn * 4);
    t.lsc = (int*)take(nn * 4);
    t.tp = (int*)take(nn * 4);
    t.tsc = (int*)take(nn * 4);
    t.ptop = (int*)take(nn * 4);
    t.ul = (int*)take(nn * 4);
    t.dlp = (int*)take(nn * 4);
    t.hist = (int*)take(4 * NL_LEVELS * 4);
    size_t b1 = 0, b2 = 0, b3 = 0;
    hipcub::DeviceScan::InclusiveSum(nullptr, b1, (long long*)nullptr, (long long*)nullptr, (int)nt);
    hipcub::DeviceScan::InclusiveScan(nullptr, b2, (int*)nullptr, (int*)nullptr, MinOp(), (int)nn);
    hipcub::DeviceScan::InclusiveScan(nullptr, b3, (int*)nullptr, (int*)nullptr, MaxOp(), (int)nn);
    t.cub_bytes = std::max(b1, std::max(b2, b3));
    t.cub = take(t.cub_bytes);
    if (w) *w = t;
    return o;
}

inline unsigned blocks(size_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

size_t nl_walk_scratch_bytes(int H, int W, int n) { return carve(nullptr, H, W, n, nullptr); }

void launch_nl_walk(const uint32_t* adj, int H, int W, int n, uint8_t* scratch, int4* rec, int* chain_start, int* chain_len,
                    int* order_up, int* order_down, int* offs, hipStream_t st) {
    WalkBufs w;
    carve(scratch, H, W, n, &w);
    const int np = H * W;
    const long nn = (long)np * n, na = 4 * nn, nt = (long)n * 2 * (np - 1);
    hipMemsetAsync(w.err, 0, 4, st);
    hipMemsetAsync(w.hist, 0, 4 * NL_LEVELS * 4, st);
    hipLaunchKernelGGL(k_walk_succ, dim3(blocks(na)), dim3(256), 0, st, adj, w, np, W, na);
    hipLaunchKernelGGL(k_walk_sub, dim3(blocks(nn)), dim3(256), 0, st, w, np, (int)nn);
    // pointer jumping over the sublist starts: ceil(log2(starts per pair)) rounds suffice (a pair
    // has at most H W starts)
    int rounds = 0;
    while ((1L << rounds) < (long)np) rounds++;
    int cur = 0;
    for (int r = 0; r < rounds; r++, cur ^= 1)
        hipLaunchKernelGGL(k_walk_jump, dim3(blocks(nn)), dim3(256), 0, st, w.jn[cur], w.jd[cur], w.jn[cur ^ 1], w.jd[cur ^ 1], np, (int)nn);
    hipLaunchKernelGGL(k_walk_rank, dim3(blocks(nn)), dim3(256), 0, st, w, w.jd[cur], np, (int)nn);
    hipLaunchKernelGGL(k_walk_node1, dim3(blocks(nn)), dim3(256), 0, st, adj, w, np, W, nn);
    hipLaunchKernelGGL(k_walk_node2, dim3(blocks(nn)), dim3(256), 0, st, adj, w, np, W, nn);
    size_t cb = w.cub_bytes;
    hipcub::DeviceScan::InclusiveSum(w.cub, cb, w.tour, w.tsum, (int)nt, st);
    hipLaunchKernelGGL(k_walk_node3, dim3(blocks(nn)), dim3(256), 0, st, w, np, nn);
    cb = w.cub_bytes;
    hipcub::DeviceScan::InclusiveScan(w.cub, cb, w.lrev, w.lsc, MinOp(), (int)nn, st);
    cb = w.cub_bytes;
    hipcub::DeviceScan::InclusiveScan(w.cub, cb, w.tp, w.tsc, MaxOp(), (int)nn, st);
    hipLaunchKernelGGL(k_walk_node4, dim3(blocks(nn)), dim3(256), 0, st, w, rec, chain_start, chain_len, np, W, nn);
    // up levels, deepest light depth first (light depth <= log2(H W))
    int maxd = 0;
    while ((1L << maxd) <= np) maxd++;
    for (int d = std::min(maxd, NL_LEVELS - 1); d >= 1; d--)
        hipLaunchKernelGGL(k_walk_ul, dim3(blocks(nn)), dim3(256), 0, st, w, nn, d);
    hipLaunchKernelGGL(k_walk_hist, dim3(blocks(nn)), dim3(256), 0, st, w, nn);
    hipLaunchKernelGGL(k_walk_offs, dim3(1), dim3(64), 0, st, w, offs);
    hipLaunchKernelGGL(k_walk_scatter, dim3(blocks(nn)), dim3(256), 0, st, w, order_up, order_down, nn);
}

}  // namespace sm
