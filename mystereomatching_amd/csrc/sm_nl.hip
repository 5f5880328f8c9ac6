// sm_nl.hip — aggregation "NL" (NL(), stereoMatching.cpp:4892-4917): Qingxiong Yang's non-local
// cost aggregation on the minimum spanning tree of the left colour image (NL/NLCCA.cpp:27-96).
//
//   edges      ctmf 3x3 median of each channel with clamped borders (NL/ctmf.c, called with r = 1
//              by qx_mst_kruskals_image::mst), weight = max channel |difference| of 4-neighbours
//   tree       GPU spanning trees (sm_nl_mst.hip), rooted at pixel 0 and cut into heavy paths on
//              the GPU (sm_nl_walk.hip)
//   filter     qx_tree_filter::filter (NL/qx_tree_filter.cpp:61-117) in double, w = exp(-c / 25.5):
//                up(x)  = C(x) + sum_j up(child_j) * w(child_j)           children in list order
//                fin(x) = w(x) * (fin(parent) - w(x) * up(x)) + up(x),    fin(root) = up(root)
//   NL()       vm = (float)fin(C) / (float)fin(1)   (the ones volume, cpp:4899-4910; fin(1) depends
//              only on the tree and is filtered here too, as one more channel of the same walk)
//
// gfx950 mapping: one wave per (heavy path, 64-disparity chunk), lane = disparity, walking the path
// node by node; the child on the same path arrives in a register, the other children (their paths
// finished in earlier rounds) from memory.  A round is one launch; a node's sum keeps the
// reference's child order, so rounds only schedule work and the result is the restatement's bit for
// bit.  Intermediate values are doubles, as in the reference (m_cost_vol is double).
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sm_device.h"
#include "sm_kernels.h"

#ifndef SM_NL_BLOCK
#define SM_NL_BLOCK 4   // path nodes whose loads are issued together (tuning)
#endif
#ifndef SM_NL_PIPE
#define SM_NL_PIPE 1    // issue the next block's loads before this block's arithmetic (tuning)
#endif
#ifndef SM_NL_BLOCK_SHORT
#define SM_NL_BLOCK_SHORT 2      // ... in rounds of at least SM_NL_SHORT_UNITS (path, chunk) units
#endif
#ifndef SM_NL_SHORT_UNITS
#define SM_NL_SHORT_UNITS 65536
#endif
#ifndef SM_NL_SHORT_UNITS_DN
#define SM_NL_SHORT_UNITS_DN 65536
#endif
#ifndef SM_NL_WAVES
#define SM_NL_WAVES 1   // waves (independent paths) per workgroup (tuning)
#endif

namespace sm {

static_assert(3 * SM_NL_BLOCK <= NL_REC_PAD, "the passes read up to two blocks past a path's ends");

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

// Child j of node x from its direction code (NlArgs::rec): 0 = x + 1, 1 = x - 1, 2 = x + W, 3 = x - W
// (tree edges join 4-neighbours, and node ids are pair * H W + pixel).
__device__ __forceinline__ int nl_child(int x, int meta, int j, int W) {
    const int code = (meta >> (6 + 2 * j)) & 3;
    const int step = (code & 2) ? W : 1;
    return (code & 1) ? x - step : x + step;
}

// Up pass over the paths order_up[lo, ...): bottom -> top.  A path is walked in blocks of K nodes:
// every load of a block (the node's cost, its other children's finished sums, the edge weights)
// is issued before the block's sequential arithmetic, and with SM_NL_PIPE the next block's loads
// are issued before this block's arithmetic, so a long path pays a memory latency per K nodes or
// less instead of a chain of dependent loads per node.  The branches around the loads are uniform
// (scalar); the records themselves are read past the path's end (the next path or zero padding,
// NL_REC_PAD) so that a block's records arrive in one go.
template <int K>
struct NlUpBlock {
    int4 r[K];
    float cost[K];
    double wh[K], lm[K][4];
    double lo[K][4];   // the ones channel's off-path children (uniform across the wave)
};

// issue the block's loads (uniform branches; nothing here waits for them)
template <int K>
__device__ __forceinline__ void nl_up_load(NlUpBlock<K>& B, const NlArgs& a, const int4* __restrict__ R, int b, int len,
                                           int P, int d) {
#pragma unroll
    for (int k = 0; k < K; k++) B.r[k] = R[b + k];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int4 r = B.r[k];
        const int nc = r.y & 7, hv = ((r.y >> 3) & 7) - 1;
        B.cost[k] = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; j++) B.lm[k][j] = B.lo[k][j] = 0.0;
        if (b + k >= len) continue;                     // no loads past the path
        B.cost[k] = a.vc[(size_t)r.x * P + d];
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (j < nc && j != hv) {
                const int ch = nl_child(r.x, r.y, j, a.W);
                B.lm[k][j] = a.val[(size_t)ch * P + d];
                B.lo[k][j] = a.oup[ch];
            }
    }
}

// weights (scalar loads of the table) and the other children's products, once the loads are in
template <int K>
__device__ __forceinline__ void nl_up_weigh(NlUpBlock<K>& B, const double* __restrict__ table) {
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int4 r = B.r[k];
        const int hv = ((r.y >> 3) & 7) - 1;
        B.wh[k] = hv >= 0 ? table[(r.z >> (8 * hv)) & 255] : 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const double t = table[(r.z >> (8 * j)) & 255];
            B.lm[k][j] = B.lm[k][j] * t;
            B.lo[k][j] = B.lo[k][j] * t;
        }
    }
}

// (the ones channel: up(1) = 1 + sum_j up_1(child_j) * w(child_j), the same order; every wave
// of the path computes it, the first lane of chunk 0 stores it)
template <int K>
__device__ __forceinline__ void nl_up_compute(const NlUpBlock<K>& B, const NlArgs& a, int b, int len, int P, int d,
                                              double& carry, double& carry_o) {
#pragma unroll
    for (int k = 0; k < K; k++) {
        if (b + k >= len) break;
        const int4 r = B.r[k];
        const int nc = r.y & 7, hv = ((r.y >> 3) & 7) - 1;
        double v = (double)B.cost[k];
        double vo = 1.0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (j >= nc) break;
            const double m = (j == hv) ? carry * B.wh[k] : B.lm[k][j];
            const double mo = (j == hv) ? carry_o * B.wh[k] : B.lo[k][j];
            v = v + m;
            vo = vo + mo;
        }
        a.val[(size_t)r.x * P + d] = v;
        if (d == 0) a.oup[r.x] = vo;
        carry = v;
        carry_o = vo;
    }
}

// rec and table arrive as restrict kernel arguments so that their uniform loads become scalar
// loads (the struct members carry no aliasing guarantee against the stores to val).
template <int K>
__global__ __launch_bounds__(64 * SM_NL_WAVES) void k_nl_up(const NlArgs a, const int4* __restrict__ rec,
                                                            const double* __restrict__ table, int lo, int nunits, int P) {
    const int nchunks = (P + 63) >> 6;
    const int u = blockIdx.x * SM_NL_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (path, chunk)
    if (u >= nunits) return;
    const int ci = a.order_up[lo + u / nchunks];
    const int d = (u % nchunks) * 64 + (threadIdx.x & 63);
    if (d >= P) return;
    const int4* __restrict__ R = rec + a.chain_start[ci];
    const int len = a.chain_len[ci];
    double carry = 0.0, carry_o = 0.0;
#if SM_NL_PIPE
    NlUpBlock<K> X, Y;
    nl_up_load(X, a, R, 0, len, P, d);
    for (int b = 0; b < len; b += 2 * K) {
        nl_up_load(Y, a, R, b + K, len, P, d);
        nl_up_weigh(X, table);
        nl_up_compute(X, a, b, len, P, d, carry, carry_o);
        if (b + K >= len) break;
        nl_up_load(X, a, R, b + 2 * K, len, P, d);
        nl_up_weigh(Y, table);
        nl_up_compute(Y, a, b + K, len, P, d, carry, carry_o);
    }
#else
    for (int b = 0; b < len; b += K) {
        NlUpBlock<K> X;
        nl_up_load(X, a, R, b, len, P, d);
        nl_up_weigh(X, table);
        nl_up_compute(X, a, b, len, P, d, carry, carry_o);
    }
#endif
}

// Down pass over the paths order_down[lo, ...): top -> bottom, blocked like the up pass; writes
// the final doubles in place and the normalised float volume.  Records before a path's first
// node are the previous path's or zero padding.
template <int K>
struct NlDownBlock {
    int4 r[K];
    double up[K];
    double uo[K];      // the ones channel's up sum (uniform across the wave)
};

template <int K>
__device__ __forceinline__ void nl_down_load(NlDownBlock<K>& B, const NlArgs& a, const int4* __restrict__ R, int b, int P,
                                             int d) {
#pragma unroll
    for (int k = 0; k < K; k++) B.r[k] = R[b - k];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int4 r = B.r[k];
        B.up[k] = 0.0;
        B.uo[k] = 1.0;
        if (b - k < 0) continue;                        // no loads before the path
        B.up[k] = a.val[(size_t)r.x * P + d];
        B.uo[k] = a.oup[r.x];
    }
}

template <int K>
__device__ __forceinline__ void nl_down_compute(const NlDownBlock<K>& B, const NlArgs& a, const double* __restrict__ table,
                                                int b, int P, int d, double& carry, double& carry_o) {
    double w[K];
#pragma unroll
    for (int k = 0; k < K; k++) w[k] = table[(B.r[k].y >> 16) & 255];
#pragma unroll
    for (int k = 0; k < K; k++) {
        if (b - k < 0) break;
        const int4 r = B.r[k];
        double fin, fo;
        if (r.w == r.x) {
            fin = B.up[k];                              // the root
            fo = B.uo[k];
        } else {
            const double m = w[k] * B.up[k];
            const double q = carry - m;
            const double s = w[k] * q;
            fin = s + B.up[k];
            const double mo = w[k] * B.uo[k];
            const double qo = carry_o - mo;
            const double so = w[k] * qo;
            fo = so + B.uo[k];
        }
        a.val[(size_t)r.x * P + d] = fin;
        if (d == 0) a.ofin[r.x] = fo;
        carry = fin;
        carry_o = fo;
        float out = (float)fin / (float)fo;
        if (a.solve_all) {   // SolveAll fused (sm_run): its `sum = 0; sum += w * v`
            float sum = 0.f;
            sum += a.scale * out;
            out = sum;
        }
        a.vm[(size_t)r.x * P + d] = out;
    }
}

template <int K>
__global__ __launch_bounds__(64 * SM_NL_WAVES) void k_nl_down(const NlArgs a, const int4* __restrict__ rec,
                                                              const double* __restrict__ table, int lo, int nunits, int P) {
    const int nchunks = (P + 63) >> 6;
    const int u = blockIdx.x * SM_NL_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (path, chunk)
    if (u >= nunits) return;
    const int ci = a.order_down[lo + u / nchunks];
    const int d = (u % nchunks) * 64 + (threadIdx.x & 63);
    if (d >= P) return;
    const int4* __restrict__ R = rec + a.chain_start[ci];
    const int len = a.chain_len[ci];
    const int4 top = R[len - 1];
    // the top's parent is on a path finished in an earlier round (or the top is the root)
    double carry = top.w == top.x ? 0.0 : a.val[(size_t)top.w * P + d];
    double carry_o = top.w == top.x ? 0.0 : a.ofin[top.w];
#if SM_NL_PIPE
    NlDownBlock<K> X, Y;
    nl_down_load(X, a, R, len - 1, P, d);
    for (int b = len - 1; b >= 0; b -= 2 * K) {
        nl_down_load(Y, a, R, b - K, P, d);
        nl_down_compute(X, a, table, b, P, d, carry, carry_o);
        if (b - K < 0) break;
        nl_down_load(X, a, R, b - 2 * K, P, d);
        nl_down_compute(Y, a, table, b - K, P, d, carry, carry_o);
    }
#else
    for (int b = len - 1; b >= 0; b -= K) {
        NlDownBlock<K> X;
        nl_down_load(X, a, R, b, P, d);
        nl_down_compute(X, a, table, b, P, d, carry, carry_o);
    }
#endif
}


// ---------------------------------------------------------------------------------------------
// Producer / consumer rounds.  The last up rounds and the first down rounds hold a few long
// paths (Teddy: the root's heavy path has ~3000 nodes), and there a wave walking its path waits
// on every block's records and then on the block's data loads (~0.3-0.4 us per node).  In these
// rounds a workgroup of 1 + PC_P PC_C / PC_H waves owns one (path, 64-disparity chunk): producer group p
// (PC_C / PC_H waves, PC_H nodes each) loads the nodes of chunk c (c = p mod PC_P: PC_C nodes'
// records, costs or up sums, the light children's sums and the weights), keeps the loads in flight
// for PC_P - 1 steps and then writes one of two LDS slots -- weighted and pre-summed; the consumer
// wave runs the node chain out of that slot in the next step.  One barrier per step of PC_C nodes; the
// arithmetic and its order are the block kernels' above (bit-exact).
#ifndef SM_NL_PC_UNITS
#define SM_NL_PC_UNITS 512   // rounds of fewer (path, chunk) units use the producer/consumer kernels (0: never)
#endif
#ifndef SM_NL_PC_C
#define SM_NL_PC_C 8         // nodes per chunk (ring slot)
#endif
constexpr int PC_C = SM_NL_PC_C;
#ifndef SM_NL_PC_P
#define SM_NL_PC_P 3         // producer groups: a chunk's loads are issued PC_P - 1 steps before its write
#endif
constexpr int PC_P = SM_NL_PC_P;
constexpr int PC_R = 2;      // ring slots: a slot is read the step after its write, while the next one is written
#ifndef SM_NL_PC_H
#define SM_NL_PC_H 2         // nodes per producer wave (PC_C / PC_H producer waves per group share a chunk)
#endif
constexpr int PC_H = SM_NL_PC_H;
constexpr int PC_NH = PC_C / PC_H;
constexpr int PC_WAVES = 1 + PC_NH * PC_P;
static_assert(PC_WAVES + 2 <= 16 && PC_C % PC_H == 0, "a workgroup holds at most 1024 threads");

struct PcUpSlot {
    int4 rec[PC_C];
    double4 lu[PC_C][64];    // per lane (disparity): {pre, post1, post2, post3} (see below)
    double4 ou[PC_C];        // the ones channel: {pre, post1, post2, post3}
    double wh[PC_C];         // the heavy child's weight (0: none)
};
struct PcDnSlot {
    int4 rec[PC_C];
    double w[PC_C];          // the node's own weight (0 for the root: fin = 0 (carry - 0) + up = up)
    double uo[PC_C];         // the ones channel's up sum
    double up[PC_C][64];
};
// Down rounds: the consumer leaves each node's final sums here; PC_SW store waves divide, scale
// and store them the step after (the division and the three stores are off the chain).
constexpr int PC_SW = 2;
struct PcDnOut {
    double fin[PC_C][64];
    double fo[PC_C];
    int x[PC_C];
};

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double rdlane_f64(double v, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l), hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}

// The up sum of a node is ((cost + m_0) + m_1) + ... in child order, the heavy child's term
// m_hv = carry * w_hv the only one on the chain.  The producer adds the terms before it (pre =
// ((cost + m_0) + ...) + m_(hv-1)) and lines up the ones after it (post1..3, +0 where absent:
// adding +0 leaves every sum unchanged, sums are >= +0), so the consumer's chain is always
// (((pre + carry w_hv) + post1) + post2) + post3 -- the reference's additions in the reference's
// order, no selects or branches (a node without children has w_hv = 0, and pre + 0 = pre).
// Each wave type runs its own step loop (barriers only have to match in number): producer PP
// handles chunks PP, PP + PC_P, ...; its body for chunk c spans steps c .. c + PC_P - 1 -- issue,
// PC_P - 2 idle steps, write -- as straight-line code, so the compiler's wait for the loads sits at
// the write (PC_P - 1 barriers after the issue) and nowhere earlier.
// producer wave w (0-based) = group w % PC_P, half w / PC_P: a compile-time (group, half) pair
template <int W, typename F>
__device__ __forceinline__ void pc_dispatch(int w, F&& f) {
    if constexpr (W < PC_P * PC_NH) {
        if (w == W) f(std::integral_constant<int, W % PC_P>{}, std::integral_constant<int, W / PC_P>{});
        else pc_dispatch<W + 1>(w, f);
    }
}

struct PcCtx {
    const int4* R;
    int len, nst, d, lane;
    bool dok;
};

template <int PP, int HF>
__device__ __forceinline__ void nl_up_producer(PcUpSlot* S, const NlArgs& a, const double* __restrict__ table, const PcCtx& q, int P) {
    constexpr int K0 = HF * PC_H;   // this producer's nodes of a chunk: K0 .. K0 + PC_H - 1
    const int lane = q.lane, d = q.d, len = q.len, nst = q.nst;
    const bool dok = q.dok;
    int step = 0;
    for (; step < PP; step++) __syncthreads();
    int4 rc = make_int4(0, 0, 0, 0);
    if (PP < nst && lane < PC_C) rc = q.R[PP * PC_C + lane];
    for (int c = PP; c < nst; c += PC_P) {
        // step c: issue the loads, then the records of this producer's next chunk (issued last:
        // the next chunk's first readlane then waits for nothing younger)
        float xc[PC_H];
        double xm[PC_H][4];
#pragma unroll
        for (int kk = 0; kk < PC_H; kk++) {
            const int k = K0 + kk;
            const int x = __builtin_amdgcn_readlane(rc.x, k), meta = __builtin_amdgcn_readlane(rc.y, k);
            const int nc = meta & 7, hv = ((meta >> 3) & 7) - 1;
            xc[kk] = 0.0f;
#pragma unroll
            for (int j = 0; j < 4; j++) xm[kk][j] = 0.0;
            if (c * PC_C + k >= len) continue;
            if (dok) xc[kk] = a.vc[(size_t)x * P + d];
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (j < nc && j != hv && dok) xm[kk][j] = a.val[(size_t)nl_child(x, meta, j, a.W) * P + d];
        }
        // lane t < 4 PC_H: child position t % 4 of node K0 + t / 4 (weights of every child, the
        // ones sum of the light ones)
        const int kt = K0 + ((lane >> 2) & (PC_H - 1)), jt = lane & 3;   // (PC_H <= 16)
        const int xk = __shfl(rc.x, kt), mk = __shfl(rc.y, kt), wk = __shfl(rc.z, kt);
        const int nck = mk & 7, hvk = ((mk >> 3) & 7) - 1;
        const bool here = lane < 4 * PC_H && c * PC_C + kt < len && jt < nck;
        const double xw = here ? table[(wk >> (8 * jt)) & 255] : 0.0;
        const double xo = (here && jt != hvk) ? a.oup[nl_child(xk, mk, jt, a.W)] : 0.0;
        int4 rn = make_int4(0, 0, 0, 0);
        if (c + PC_P < nst && lane < PC_C) rn = q.R[(c + PC_P) * PC_C + lane];
        for (int i = 0; i < PC_P - 1; i++) __syncthreads();   // steps c .. c + PC_P - 2: the loads stay in flight
        // step c + PC_P - 1: write the slot's nodes K0 .. K0 + PC_H - 1
        PcUpSlot& B = S[c % PC_R];
        if (lane >= K0 && lane < K0 + PC_H) B.rec[lane] = rc;
        // the ones channel, lane-parallel: lane kk < PC_H sums node K0 + kk's four terms
        {
            const double mo_t = xo * xw;   // lane t: the ones term of position t % 4 of node K0 + t / 4
            const int kk = lane & (PC_H - 1);
            const int hvl = ((__shfl(rc.y, K0 + kk) >> 3) & 7) - 1;
            double t4[4], w4[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                t4[j] = __shfl(mo_t, 4 * kk + j);
                w4[j] = __shfl(xw, 4 * kk + j);
            }
            double pre = 1.0;
#pragma unroll
            for (int j = 0; j < 4; j++) pre = pre + (j < hvl ? t4[j] : 0.0);
            const double p1 = hvl == 0 ? t4[1] : (hvl == 1 ? t4[2] : (hvl == 2 ? t4[3] : 0.0));
            const double p2 = hvl == 0 ? t4[2] : (hvl == 1 ? t4[3] : 0.0);
            const double p3 = hvl == 0 ? t4[3] : 0.0;
            const double wh = hvl == 0 ? w4[0] : (hvl == 1 ? w4[1] : (hvl == 2 ? w4[2] : (hvl == 3 ? w4[3] : 0.0)));
            if (lane < PC_H) {
                B.ou[K0 + kk] = make_double4(pre, p1, p2, p3);
                B.wh[K0 + kk] = wh;
            }
        }
#pragma unroll
        for (int kk = 0; kk < PC_H; kk++) {
            const int k = K0 + kk;
            const int hv = ((__builtin_amdgcn_readlane(rc.y, k) >> 3) & 7) - 1;
            double t4[4];
#pragma unroll
            for (int j = 0; j < 4; j++) t4[j] = xm[kk][j] * rdlane_f64(xw, 4 * kk + j);
            double pre = (double)xc[kk];
#pragma unroll
            for (int j = 0; j < 4; j++) pre = pre + (j < hv ? t4[j] : 0.0);
            const double p1 = hv == 0 ? t4[1] : (hv == 1 ? t4[2] : (hv == 2 ? t4[3] : 0.0));
            const double p2 = hv == 0 ? t4[2] : (hv == 1 ? t4[3] : 0.0);
            const double p3 = hv == 0 ? t4[3] : 0.0;
            B.lu[k][lane] = make_double4(pre, p1, p2, p3);
        }
        __syncthreads();
        step += PC_P;
        rc = rn;
    }
    for (; step < nst + PC_P; step++) __syncthreads();
}

__global__ __launch_bounds__(64 * PC_WAVES, 1) void k_nl_up_pc(const NlArgs a, const int4* __restrict__ rec,
                                                                  const double* __restrict__ table, int lo, int nunits, int P) {
    extern __shared__ __align__(16) unsigned char pc_smem[];
    PcUpSlot* S = (PcUpSlot*)pc_smem;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nchunks = (P + 63) >> 6;
    const int u = blockIdx.x;
    if (u >= nunits) return;
    const int ci = a.order_up[lo + u / nchunks];
    PcCtx q;
    q.lane = lane;
    q.d = (u % nchunks) * 64 + lane;
    q.dok = q.d < P;
    q.R = rec + a.chain_start[ci];
    q.len = a.chain_len[ci];
    q.nst = (q.len + PC_C - 1) / PC_C;
    if (wv > 0) {
        pc_dispatch<0>(wv - 1, [&](auto pp, auto hf) { nl_up_producer<decltype(pp)::value, decltype(hf)::value>(S, a, table, q, P); });
        return;
    }
    __builtin_amdgcn_s_setprio(3);   // the chain: first at its SIMD
    const int len = q.len;
    // lanes past P store out of range (dropped) instead of under an exec mask
    const __amdgpu_buffer_rsrc_t val_r = buf_rsrc(a.val), oup_r = buf_rsrc(a.oup);
    const uint32_t dof = q.dok ? (uint32_t)q.d * 8u : 0x80000000u;
    double carry = 0.0, carry_o = 0.0;
    auto node = [&](const PcUpSlot& B, int k) {
        const int x = __builtin_amdgcn_readfirstlane(B.rec[k].x);
        const double4 L = B.lu[k][lane];
        const double4 O = B.ou[k];
        const double wh = B.wh[k];
        const double v = (((L.x + carry * wh) + L.y) + L.z) + L.w;
        const double vo = (((O.x + carry_o * wh) + O.y) + O.z) + O.w;
        const uint32_t row = (uint32_t)x * (uint32_t)P * 8u;   // (volume < 4 GiB: see launch)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), val_r, dof, row, 0);
        if (lane == 0 && q.d == 0) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, vo), oup_r, 0, (uint32_t)x * 8u, 0);
        carry = v;
        carry_o = vo;
    };
    for (int s = 0; s < q.nst + PC_P; s++) {
        const int c = s - PC_P;
        if (c >= 0) {
            const PcUpSlot& B = S[c % PC_R];
            if ((c + 1) * PC_C <= len) {   // a full slot: straight-line
#pragma unroll
                for (int k = 0; k < PC_C; k++) node(B, k);
            } else {
                for (int k = 0; k < len - c * PC_C; k++) node(B, k);
            }
        }
        __syncthreads();
    }
}

template <int PP, int HF>
__device__ __forceinline__ void nl_down_producer(PcDnSlot* S, const NlArgs& a, const double* __restrict__ table, const PcCtx& q, int P) {
    constexpr int K0 = HF * PC_H;
    const int lane = q.lane, d = q.d, len = q.len, nst = q.nst;
    const bool dok = q.dok;
    int step = 0;
    for (; step < PP; step++) __syncthreads();
    // chunk c holds path positions len - 1 - c PC_C - k, k = 0 .. PC_C - 1 (top -> bottom)
    int4 rc = make_int4(0, 0, 0, 0);
    if (PP < nst && lane < PC_C) rc = q.R[len - 1 - PP * PC_C - lane];
    for (int c = PP; c < nst; c += PC_P) {
        double xu[PC_H];
#pragma unroll
        for (int kk = 0; kk < PC_H; kk++) {
            const int k = K0 + kk;
            const int x = __builtin_amdgcn_readlane(rc.x, k);
            xu[kk] = 0.0;
            if (c * PC_C + k >= len) continue;
            if (dok) xu[kk] = a.val[(size_t)x * P + d];
        }
        double xo = 0.0, xw = 0.0;   // lane k in [K0, K0 + PC_H): node k's ones up sum and own weight (0: root)
        if (lane >= K0 && lane < K0 + PC_H && c * PC_C + lane < len) {
            xo = a.oup[rc.x];
            xw = rc.w == rc.x ? 0.0 : table[(rc.y >> 16) & 255];
        }
        int4 rn = make_int4(0, 0, 0, 0);
        if (c + PC_P < nst && lane < PC_C) rn = q.R[len - 1 - (c + PC_P) * PC_C - lane];
        for (int i = 0; i < PC_P - 1; i++) __syncthreads();
        PcDnSlot& B = S[c % PC_R];
        if (lane >= K0 && lane < K0 + PC_H) {
            B.rec[lane] = rc;
            B.uo[lane] = xo;
            B.w[lane] = xw;
        }
#pragma unroll
        for (int kk = 0; kk < PC_H; kk++) B.up[K0 + kk][lane] = xu[kk];
        __syncthreads();
        step += PC_P;
        rc = rn;
    }
    for (; step < nst + PC_P + 1; step++) __syncthreads();   // (+1: the store waves' last step)
}

__global__ __launch_bounds__(64 * (PC_WAVES + PC_SW), 1) void k_nl_down_pc(const NlArgs a, const int4* __restrict__ rec,
                                                                    const double* __restrict__ table, int lo, int nunits, int P) {
    extern __shared__ __align__(16) unsigned char pc_smem[];
    PcDnSlot* S = (PcDnSlot*)pc_smem;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nchunks = (P + 63) >> 6;
    const int u = blockIdx.x;
    if (u >= nunits) return;
    const int ci = a.order_down[lo + u / nchunks];
    PcCtx q;
    q.lane = lane;
    q.d = (u % nchunks) * 64 + lane;
    q.dok = q.d < P;
    q.R = rec + a.chain_start[ci];
    q.len = a.chain_len[ci];
    q.nst = (q.len + PC_C - 1) / PC_C;
    PcDnOut* O = (PcDnOut*)(pc_smem + PC_R * sizeof(PcDnSlot));
    const int len = q.len;
    if (wv >= PC_WAVES) {
        // store wave: nodes [sw PC_C / PC_SW, (sw + 1) PC_C / PC_SW) of the chunk consumed last step
        constexpr int NPW = PC_C / PC_SW;
        const int k0 = (wv - PC_WAVES) * NPW;
        const __amdgpu_buffer_rsrc_t val_r = buf_rsrc(a.val), vm_r = buf_rsrc(a.vm), ofin_r = buf_rsrc(a.ofin);
        const uint32_t dof8 = q.dok ? (uint32_t)q.d * 8u : 0x80000000u, dof4 = q.dok ? (uint32_t)q.d * 4u : 0x80000000u;
        for (int s = 0; s < q.nst + PC_P + 1; s++) {
            const int cc = s - PC_P - 1;
            if (cc >= 0) {
                const PcDnOut& B = O[cc % 2];
#pragma unroll
                for (int kk = 0; kk < NPW; kk++) {
                    const int k = k0 + kk;
                    if (cc * PC_C + k >= len) break;
                    const double fin = B.fin[k][lane], fo = B.fo[k];
                    const int x = __builtin_amdgcn_readfirstlane(B.x[k]);
                    float out = (float)fin / (float)fo;
                    if (a.solve_all) {   // SolveAll fused (sm_run): its `sum = 0; sum += w * v`
                        float sum = 0.f;
                        sum += a.scale * out;
                        out = sum;
                    }
                    const uint32_t row = (uint32_t)x * (uint32_t)P;
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, fin), val_r, dof8, row * 8u, 0);
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, out), vm_r, dof4, row * 4u, 0);
                    if (lane == 0 && q.d == 0) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, fo), ofin_r, 0, (uint32_t)x * 8u, 0);
                }
            }
            __syncthreads();
        }
        return;
    }
    if (wv > 0) {
        pc_dispatch<0>(wv - 1, [&](auto pp, auto hf) { nl_down_producer<decltype(pp)::value, decltype(hf)::value>(S, a, table, q, P); });
        return;
    }
    __builtin_amdgcn_s_setprio(3);
    double carry = 0.0, carry_o = 0.0;
    {
        // the top's parent is on a path finished in an earlier round (or the top is the root)
        const int4 top = q.R[len - 1];
        if (top.w != top.x) {
            carry = q.dok ? a.val[(size_t)top.w * P + q.d] : 0.0;
            carry_o = a.ofin[top.w];
        }
    }
    auto node = [&](const PcDnSlot& B, PcDnOut& OB, int k) {
        const double up = B.up[k][lane], uo = B.uo[k], w = B.w[k];
        // (the root has w = 0: fin = 0 (carry - 0 up) + up = up, exactly)
        const double fin = w * (carry - w * up) + up;
        const double fo = w * (carry_o - w * uo) + uo;
        OB.fin[k][lane] = fin;
        if (lane == 0) {
            OB.fo[k] = fo;
            OB.x[k] = B.rec[k].x;
        }
        carry = fin;
        carry_o = fo;
    };
    for (int s = 0; s < q.nst + PC_P + 1; s++) {
        const int c = s - PC_P;
        if (c >= 0 && c < q.nst) {
            const PcDnSlot& B = S[c % PC_R];
            PcDnOut& OB = O[c % 2];
            if ((c + 1) * PC_C <= len) {
#pragma unroll
                for (int k = 0; k < PC_C; k++) node(B, OB, k);
            } else {
                for (int k = 0; k < len - c * PC_C; k++) node(B, OB, k);
            }
        }
        __syncthreads();
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
    const int nchunks = (P + 63) / 64, nunits = (hi - lo) * nchunks;
    // (the producer/consumer stores use 32-bit byte offsets into val: volumes below 4 GiB)
    const bool small = (double)a.nodes * P * 8 < 4294967296.0;
    if (nunits < SM_NL_PC_UNITS && small) {
        static bool attr = false;   // LDS above the 64 KiB default
        if (!attr) {
            hipFuncSetAttribute((const void*)k_nl_up_pc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(PC_R * sizeof(PcUpSlot)));
            hipFuncSetAttribute((const void*)k_nl_down_pc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(PC_R * sizeof(PcDnSlot) + 2 * sizeof(PcDnOut)));
            attr = true;
        }
        if (up)
            hipLaunchKernelGGL(k_nl_up_pc, dim3(nunits), dim3(64 * PC_WAVES), PC_R * sizeof(PcUpSlot), st, a, a.rec, a.table, lo, nunits, P);
        else
            hipLaunchKernelGGL(k_nl_down_pc, dim3(nunits), dim3(64 * (PC_WAVES + PC_SW)), PC_R * sizeof(PcDnSlot) + 2 * sizeof(PcDnOut), st, a, a.rec, a.table, lo, nunits, P);
        return;
    }
    const dim3 grid((unsigned)((nunits + SM_NL_WAVES - 1) / SM_NL_WAVES)), block(64 * SM_NL_WAVES);
    constexpr int K = SM_NL_BLOCK;
    // rounds of very many (short) paths: smaller blocks, fewer registers, more waves in flight
    if (nunits >= (up ? SM_NL_SHORT_UNITS : SM_NL_SHORT_UNITS_DN)) {
        constexpr int KS = SM_NL_BLOCK_SHORT;
        if (up)
            hipLaunchKernelGGL((k_nl_up<KS>), grid, block, 0, st, a, a.rec, a.table, lo, nunits, P);
        else
            hipLaunchKernelGGL((k_nl_down<KS>), grid, block, 0, st, a, a.rec, a.table, lo, nunits, P);
        return;
    }
    if (up)
        hipLaunchKernelGGL((k_nl_up<K>), grid, block, 0, st, a, a.rec, a.table, lo, nunits, P);
    else
        hipLaunchKernelGGL((k_nl_down<K>), grid, block, 0, st, a, a.rec, a.table, lo, nunits, P);
}

}  // namespace sm
