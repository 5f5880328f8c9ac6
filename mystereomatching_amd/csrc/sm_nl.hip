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

#include "sm_device.h"
#include "sm_kernels.h"

#ifndef SM_NL_BLOCK
#define SM_NL_BLOCK 4   // path nodes whose loads are issued together (tuning)
#endif
#ifndef SM_NL_PIPE
#define SM_NL_PIPE 1    // issue the next block's loads before this block's arithmetic (tuning)
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
        B.cost[k] = a.vm[(size_t)r.x * P + d];
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
// rounds a workgroup of 1 + PC_P waves owns one (path, 64-disparity chunk): producer wave p loads
// the nodes of ring slot c (c = p mod PC_P: PC_C nodes' records, costs or up sums, the light
// children's sums and the weights), keeps the loads in flight for two steps and then writes the
// slot -- weighted products ready -- into LDS; the consumer wave runs the node chain out of LDS
// three steps after the slot's loads were issued.  One barrier per step of PC_C nodes; the
// arithmetic and its order are the block kernels' above (bit-exact).
#ifndef SM_NL_PC_UNITS
#define SM_NL_PC_UNITS 512   // rounds of fewer (path, chunk) units use the producer/consumer kernels (0: never)
#endif
constexpr int PC_C = 16;     // nodes per ring slot
constexpr int PC_R = 4;      // ring slots (a slot is written 2 steps after its loads, read 1 step later)
constexpr int PC_P = 3;      // producer waves

struct PcUpSlot {
    int4 rec[PC_C];
    double wh[PC_C];         // the heavy child's weight (0: none)
    double lo[PC_C][4];      // the ones channel's light products by child position (0: heavy / none)
    float cost[PC_C][64];
    double lm[PC_C][4][64];  // light products (lane = disparity) by child position (0: heavy / none)
};
struct PcDnSlot {
    int4 rec[PC_C];
    double w[PC_C];          // the node's own weight
    double uo[PC_C];         // the ones channel's up sum
    double up[PC_C][64];
};

__device__ __forceinline__ double rdlane_f64(double v, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l), hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}

// Consumers run a slot's PC_C nodes as straight-line code (the LDS reads of later nodes issue
// ahead of the chain): absent and heavy children hold +0 in the light arrays, and adding +0 leaves
// every sum unchanged (sums are >= +0, never -0), so the child loop needs no branches; the heavy
// child's term is selected at its position in the child order.
__global__ __launch_bounds__(64 * (1 + PC_P), 1) void k_nl_up_pc(const NlArgs a, const int4* __restrict__ rec,
                                                                  const double* __restrict__ table, int lo, int nunits, int P) {
    extern __shared__ __align__(16) unsigned char pc_smem[];
    PcUpSlot* S = (PcUpSlot*)pc_smem;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nchunks = (P + 63) >> 6;
    const int u = blockIdx.x;
    if (u >= nunits) return;
    const int ci = a.order_up[lo + u / nchunks];
    const int d = (u % nchunks) * 64 + lane;
    const bool dok = d < P;
    const int4* __restrict__ R = rec + a.chain_start[ci];
    const int len = a.chain_len[ci];
    const int nst = (len + PC_C - 1) / PC_C;
    double carry = 0.0, carry_o = 0.0;
    // producer state: records of the chunk being loaded (lane t < PC_C: node t) and of the next one
    int4 rc = make_int4(0, 0, 0, 0), rn = make_int4(0, 0, 0, 0);
    float xc[PC_C];
    double xm[PC_C][4];
    double xo = 0.0, xw = 0.0;   // lane t: child position t % 4 of node t / 4: its ones up sum, weight
    double xh = 0.0;             // lane t < PC_C: node t's heavy-child weight
    const int p = wv - 1;
    if (wv > 0 && p < nst && lane < PC_C) rc = R[p * PC_C + lane];
    for (int s = 0; s < nst + 3; s++) {
        if (wv == 0) {
            const int c = s - 3;
            if (c >= 0) {
                const PcUpSlot& B = S[c % PC_R];
#pragma unroll
                for (int k = 0; k < PC_C; k++) {
                    const bool ok = c * PC_C + k < len;
                    const int4 r = B.rec[k];
                    const int x = __builtin_amdgcn_readfirstlane(r.x), meta = __builtin_amdgcn_readfirstlane(r.y);
                    const int hv = ((meta >> 3) & 7) - 1;
                    const double h = carry * B.wh[k], ho = carry_o * B.wh[k];
                    double v = (double)B.cost[k][lane];
                    double vo = 1.0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        v = v + (j == hv ? h : B.lm[k][j][lane]);
                        vo = vo + (j == hv ? ho : B.lo[k][j]);
                    }
                    if (ok) {
                        if (dok) a.val[(size_t)x * P + d] = v;
                        if (d == 0) a.oup[x] = vo;
                        carry = v;
                        carry_o = vo;
                    }
                }
            }
        } else {
            // write the slot whose loads were issued two steps ago
            const int cw = s - 2;
            if (cw >= 0 && cw < nst && cw % PC_P == p) {
                PcUpSlot& B = S[cw % PC_R];
                if (lane < PC_C) {
                    B.rec[lane] = rc;
                    B.wh[lane] = xh;
                }
                B.lo[lane >> 2][lane & 3] = xo * xw;
#pragma unroll
                for (int k = 0; k < PC_C; k++) {
                    B.cost[k][lane] = xc[k];
#pragma unroll
                    for (int j = 0; j < 4; j++) B.lm[k][j][lane] = xm[k][j] * rdlane_f64(xw, 4 * k + j);
                }
                rc = rn;   // the records of this producer's next chunk (cw + PC_P)
            }
            // issue the loads of chunk s (its records were loaded a producer cycle earlier)
            if (s < nst && s % PC_P == p) {
                if (s + PC_P < nst && lane < PC_C) rn = R[(s + PC_P) * PC_C + lane];
#pragma unroll
                for (int k = 0; k < PC_C; k++) {
                    const int x = __builtin_amdgcn_readlane(rc.x, k), meta = __builtin_amdgcn_readlane(rc.y, k);
                    const int nc = meta & 7, hv = ((meta >> 3) & 7) - 1;
                    xc[k] = 0.0f;
#pragma unroll
                    for (int j = 0; j < 4; j++) xm[k][j] = 0.0;
                    if (s * PC_C + k >= len) continue;
                    if (dok) xc[k] = a.vm[(size_t)x * P + d];
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (j < nc && j != hv && dok) xm[k][j] = a.val[(size_t)nl_child(x, meta, j, a.W) * P + d];
                }
                // lane t: child position t % 4 of node t / 4 (weights of every child; the ones sum
                // of the light ones)
                const int kt = lane >> 2, jt = lane & 3;
                const int xk = __shfl(rc.x, kt), mk = __shfl(rc.y, kt), wk = __shfl(rc.z, kt);
                const int nck = mk & 7, hvk = ((mk >> 3) & 7) - 1;
                const bool here = s * PC_C + kt < len && jt < nck;
                xw = here ? table[(wk >> (8 * jt)) & 255] : 0.0;
                xo = (here && jt != hvk) ? a.oup[nl_child(xk, mk, jt, a.W)] : 0.0;
                xh = 0.0;
                if (lane < PC_C && s * PC_C + lane < len) {
                    const int hvl = ((rc.y >> 3) & 7) - 1;
                    if (hvl >= 0) xh = table[(rc.z >> (8 * hvl)) & 255];
                }
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(64 * (1 + PC_P), 1) void k_nl_down_pc(const NlArgs a, const int4* __restrict__ rec,
                                                                    const double* __restrict__ table, int lo, int nunits, int P) {
    extern __shared__ __align__(16) unsigned char pc_smem[];
    PcDnSlot* S = (PcDnSlot*)pc_smem;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nchunks = (P + 63) >> 6;
    const int u = blockIdx.x;
    if (u >= nunits) return;
    const int ci = a.order_down[lo + u / nchunks];
    const int d = (u % nchunks) * 64 + lane;
    const bool dok = d < P;
    const int4* __restrict__ R = rec + a.chain_start[ci];
    const int len = a.chain_len[ci];
    const int nst = (len + PC_C - 1) / PC_C;
    double carry = 0.0, carry_o = 0.0;
    if (wv == 0) {
        // the top's parent is on a path finished in an earlier round (or the top is the root)
        const int4 top = R[len - 1];
        if (top.w != top.x) {
            carry = dok ? a.val[(size_t)top.w * P + d] : 0.0;
            carry_o = a.ofin[top.w];
        }
    }
    int4 rc = make_int4(0, 0, 0, 0), rn = make_int4(0, 0, 0, 0);
    double xu[PC_C];
    double xo = 0.0, xw = 0.0;   // lane t < PC_C: node t's ones up sum and own weight
    const int p = wv - 1;
    // chunk c holds path positions len - 1 - c PC_C - k, k = 0 .. PC_C - 1 (top -> bottom)
    if (wv > 0 && p < nst && lane < PC_C) rc = R[len - 1 - p * PC_C - lane];
    for (int s = 0; s < nst + 3; s++) {
        if (wv == 0) {
            const int c = s - 3;
            if (c >= 0) {
                const PcDnSlot& B = S[c % PC_R];
#pragma unroll
                for (int k = 0; k < PC_C; k++) {
                    const bool ok = c * PC_C + k < len;
                    const int4 r = B.rec[k];
                    const int x = __builtin_amdgcn_readfirstlane(r.x), par = __builtin_amdgcn_readfirstlane(r.w);
                    const double up = B.up[k][lane], uo = B.uo[k], w = B.w[k];
                    const double m = w * up;
                    const double q = carry - m;
                    const double sv = w * q;
                    const double mo = w * uo;
                    const double qo = carry_o - mo;
                    const double so = w * qo;
                    const double fin = par == x ? up : sv + up;   // the root keeps its up sum
                    const double fo = par == x ? uo : so + uo;
                    float out = (float)fin / (float)fo;
                    if (a.solve_all) {   // SolveAll fused (sm_run): its `sum = 0; sum += w * v`
                        float sum = 0.f;
                        sum += a.scale * out;
                        out = sum;
                    }
                    if (ok) {
                        if (d == 0) a.ofin[x] = fo;
                        if (dok) {
                            a.val[(size_t)x * P + d] = fin;
                            a.vm[(size_t)x * P + d] = out;
                        }
                        carry = fin;
                        carry_o = fo;
                    }
                }
            }
        } else {
            const int cw = s - 2;
            if (cw >= 0 && cw < nst && cw % PC_P == p) {
                PcDnSlot& B = S[cw % PC_R];
                if (lane < PC_C) {
                    B.rec[lane] = rc;
                    B.uo[lane] = xo;
                    B.w[lane] = xw;
                }
#pragma unroll
                for (int k = 0; k < PC_C; k++) B.up[k][lane] = xu[k];
                rc = rn;
            }
            if (s < nst && s % PC_P == p) {
                if (s + PC_P < nst && lane < PC_C) rn = R[len - 1 - (s + PC_P) * PC_C - lane];
#pragma unroll
                for (int k = 0; k < PC_C; k++) {
                    const int x = __builtin_amdgcn_readlane(rc.x, k);
                    xu[k] = 0.0;
                    if (s * PC_C + k >= len) continue;
                    if (dok) xu[k] = a.val[(size_t)x * P + d];
                }
                xo = 0.0;
                xw = 0.0;
                if (lane < PC_C && s * PC_C + lane < len) {
                    xo = a.oup[rc.x];
                    xw = table[(rc.y >> 16) & 255];
                }
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
    if (nunits < SM_NL_PC_UNITS) {
        static bool attr = false;   // LDS above the 64 KiB default
        if (!attr) {
            hipFuncSetAttribute((const void*)k_nl_up_pc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(PC_R * sizeof(PcUpSlot)));
            hipFuncSetAttribute((const void*)k_nl_down_pc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(PC_R * sizeof(PcDnSlot)));
            attr = true;
        }
        if (up)
            hipLaunchKernelGGL(k_nl_up_pc, dim3(nunits), dim3(64 * (1 + PC_P)), PC_R * sizeof(PcUpSlot), st, a, a.rec, a.table, lo, nunits, P);
        else
            hipLaunchKernelGGL(k_nl_down_pc, dim3(nunits), dim3(64 * (1 + PC_P)), PC_R * sizeof(PcDnSlot), st, a, a.rec, a.table, lo, nunits, P);
        return;
    }
    const dim3 grid((unsigned)((nunits + SM_NL_WAVES - 1) / SM_NL_WAVES)), block(64 * SM_NL_WAVES);
    constexpr int K = SM_NL_BLOCK;
    if (up)
        hipLaunchKernelGGL((k_nl_up<K>), grid, block, 0, st, a, a.rec, a.table, lo, nunits, P);
    else
        hipLaunchKernelGGL((k_nl_down<K>), grid, block, 0, st, a, a.rec, a.table, lo, nunits, P);
}

}  // namespace sm
