// sm_so.hip — scan-line optimisation, optimization == "so" (stereoMatching.cpp:1091-1105, so()
// cpp:6272-6394): per row, a left-to-right dynamic programme over the disparities with a trace
// of every choice, then a right-to-left backtrack from the last column's minimum.
//
// Forward step at column u (u = 1 .. W-1), per disparity d, with prev = vm(u - 1) already updated:
//   Pn2 = 1.2f, Pn3 = 3.6f, both halved when the mean channel |I(u) - I(u-1)| of I[0] exceeds 15
//   cost_min = prev[d]; candidates in this order, each taken only when strictly smaller:
//     prev[d-1] + Pn2 (d > 0), prev[d+1] + Pn2 (d < D-1), min_d' prev[d'] + Pn3 (first argmin)
//   vm(u)[d] += cost_min;  trace(u)[d] = the chosen disparity
// I[0] is the LEFT colour image for both views (dispOptimize passes I_c; so() reads I[0]).
//
// gfx950 mapping: one wave per (pair, row), lane l owns K consecutive disparities (registers);
// the row minimum is an unsigned-integer DPP reduction (every cost is >= +0, so bit patterns
// order like the floats) plus a ballot for the first index; d +- 1 across lane edges come by DPP
// wave shifts.  Columns are prefetched a tile ahead.  The trace is stored as one byte per element
// (0: d, 1: d - 1, 2: d + 1, 3: the row minimum's index, kept per column), so the backtrack — a
// chain of W dependent reads, inherently sequential — reads one byte and one u16 per column.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

#ifndef SM_SO_LDS_TRACE
#define SM_SO_LDS_TRACE 1
#endif

namespace sm {

namespace {

constexpr int SO_T = 8;   // columns per prefetch tile

__host__ __device__ inline size_t so_lds_words(int W, int K) {   // per wave, in u64 words
    return (size_t)W * 2 * K + ((size_t)W * 2 + 7) / 8;
}

__device__ __forceinline__ float shr1_f(float v) {   // lane l <- lane l - 1 (lane 0 <- FLT_MAX)
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp((int)0x7f7fffff, __builtin_bit_cast(int, v),
                                                                 DPP_WAVE_SHR1, 0xF, 0xF, false));
}
__device__ __forceinline__ float shl1_f(float v) {   // lane l <- lane l + 1 (lane 63 <- FLT_MAX)
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp((int)0x7f7fffff, __builtin_bit_cast(int, v),
                                                                 DPP_WAVE_SHL1, 0xF, 0xF, false));
}

// LT (LDS trace): the choice codes of a row live in LDS as two ballot masks per column and
// per lane slot j (bit l of mask 2j / 2j + 1 = bit 0 / 1 of the code of disparity l K + j), and
// the row-minimum indices as u16; the backtrack's W dependent reads then hit LDS instead of
// global memory (Teddy x16: the chain of ~450 dependent global loads per row dominated the
// kernel), and the byte-wise trace stores disappear.  Used when 4 rows' traces fit in 64 KB.
template <int K, bool LT>
__global__ __launch_bounds__(256) void k_so(const SoArgs a) {
    extern __shared__ __align__(16) uint64_t so_lds[];
    const int lane = threadIdx.x & 63;
    const int row_id = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int H = a.H, W = a.W, D = a.D;
    if (row_id >= a.n * H) return;   // whole waves only: no barrier follows
    const int b = row_id / H, v = row_id - b * H;
    const size_t npix = (size_t)H * W;
    const size_t pix0 = (size_t)b * npix + (size_t)v * W;
    float* vrow = a.vm + pix0 * D;                     // (u, d) at u * D + d
    uint8_t* trow = a.trace + pix0 * D;
    uint16_t* crow = a.cidx + pix0;
    // LT: this wave's trace masks [W][2K] u64, then its row-minimum indices [W] u16
    uint64_t* tl = so_lds + (size_t)(threadIdx.x >> 6) * so_lds_words(W, K);
    uint16_t* cl = (uint16_t*)(tl + (size_t)W * 2 * K);
    const uint32_t* prow = a.px + ((size_t)b * 2) * npix + (size_t)v * W;   // left view's packed BGR
    const int d0 = lane * K;
    bool valid[K];
#pragma unroll
    for (int j = 0; j < K; j++) valid[j] = d0 + j < D;
    float prev[K];
#pragma unroll
    for (int j = 0; j < K; j++) prev[j] = valid[j] ? vrow[d0 + j] : FLT_MAX;

    using Tile = float[SO_T][K];
    auto load_tile = [&](Tile& t, int u0) {
#pragma unroll
        for (int k = 0; k < SO_T; k++) {
            const int u = min(u0 + k, W - 1);
#pragma unroll
            for (int j = 0; j < K; j++) t[k][j] = valid[j] ? vrow[(size_t)u * D + d0 + j] : 0.f;
        }
    };
    auto process = [&](const Tile& t, int u0) {
        // discontinuity flags of the tile's columns: lane k tests column u0 + k
        uint64_t disc;
        {
            const int u = u0 + lane;
            bool f = false;
            if (lane < SO_T && u < W) {
                const uint32_t x = prow[u], y = prow[u - 1];
                float sum = 0.f;
                sum += abs((int)(x & 0xff) - (int)(y & 0xff));
                sum += abs((int)((x >> 8) & 0xff) - (int)((y >> 8) & 0xff));
                sum += abs((int)((x >> 16) & 0xff) - (int)((y >> 16) & 0xff));
                sum /= 3;
                f = sum > 15;
            }
            disc = __ballot(f);
        }
#pragma unroll
        for (int k = 0; k < SO_T; k++) {
            const int u = u0 + k;
            if (u >= W) break;
            const bool dc = (disc >> k) & 1;
            float Pn2 = 1.2f, Pn3 = 3.6f;
            if (dc) {
                Pn2 /= 2;
                Pn3 /= 2;
            }
            // row minimum of prev and its first index (prev lanes past D hold FLT_MAX)
            float lm = prev[0];
            int li = d0;
#pragma unroll
            for (int j = 1; j < K; j++)
                if (prev[j] < lm) {
                    lm = prev[j];
                    li = d0 + j;
                }
            const uint32_t wm = wave_umin(__builtin_bit_cast(uint32_t, lm));
            const uint64_t hit = __ballot(__builtin_bit_cast(uint32_t, lm) == wm);
            const int cidx = __builtin_amdgcn_readlane(li, (int)__builtin_ctzll(hit));
            const float c_min = __builtin_bit_cast(float, wm) + Pn3;
            const float left = shr1_f(prev[K - 1]);    // prev[d0 - 1]
            const float right = shl1_f(prev[0]);       // prev[d0 + K]
            float nv[K];
            uint32_t codes = 0;
#pragma unroll
            for (int j = 0; j < K; j++) {
                const int d = d0 + j;
                const float pm = j > 0 ? prev[j - 1] : left;
                const float pp = j < K - 1 ? prev[j + 1] : right;
                const float c_minus = d > 0 ? pm + Pn2 : FLT_MAX;
                const float c_plus = d < D - 1 ? pp + Pn2 : FLT_MAX;
                float cost_min = prev[j];
                uint32_t code = 0;
                if (c_minus < cost_min) {
                    cost_min = c_minus;
                    code = 1;
                }
                if (c_plus < cost_min) {
                    cost_min = c_plus;
                    code = 2;
                }
                if (c_min < cost_min) {
                    cost_min = c_min;
                    code = 3;
                }
                nv[j] = t[k][j] + cost_min;
                if (LT) {
                    const uint64_t b0 = __ballot(code & 1u), b1 = __ballot(code & 2u);
                    if (lane == 0) {
                        tl[(size_t)u * 2 * K + 2 * j] = b0;
                        tl[(size_t)u * 2 * K + 2 * j + 1] = b1;
                    }
                    continue;
                }
                codes |= code << (8 * (j & 3));
                if ((j & 3) == 3 || j == K - 1) {   // flush the codes of disparities base .. j
                    const int base = j & ~3;
                    uint8_t* tp = trow + (size_t)u * D + d0 + base;
                    if (j - base == 3 && (D & 3) == 0 && d0 + base + 3 < D) {
                        *(uint32_t*)tp = codes;      // 4-byte aligned: D % 4 == 0 and d0 + base % 4 == 0
                    } else {
#pragma unroll
                        for (int q = 0; q <= (j & 3); q++)
                            if (d0 + base + q < D) tp[q] = (uint8_t)(codes >> (8 * q));
                    }
                    codes = 0;
                }
            }
            if (lane == 0) {
                if (LT)
                    cl[u] = (uint16_t)cidx;
                else
                    crow[u] = (uint16_t)cidx;
            }
#pragma unroll
            for (int j = 0; j < K; j++) {
                prev[j] = valid[j] ? nv[j] : FLT_MAX;
                if (a.keep_final && valid[j]) vrow[(size_t)u * D + d0 + j] = nv[j];
            }
        }
    };
    Tile ta, tb;   // explicit ping-pong (no dynamically indexed register arrays)
    load_tile(ta, 1);
    for (int u0 = 1; u0 < W; u0 += 2 * SO_T) {
        if (u0 + SO_T < W) load_tile(tb, u0 + SO_T);
        process(ta, u0);
        if (u0 + SO_T >= W) break;
        if (u0 + 2 * SO_T < W) load_tile(ta, u0 + 2 * SO_T);
        process(tb, u0 + SO_T);
    }
    // backtrack: first minimum of the last column, then one trace read per column
    int dmin;
    {
        float lm = prev[0];
        int li = d0;
#pragma unroll
        for (int j = 1; j < K; j++)
            if (prev[j] < lm) {
                lm = prev[j];
                li = d0 + j;
            }
        const uint32_t wm = wave_umin(__builtin_bit_cast(uint32_t, lm));
        const uint64_t hit = __ballot(__builtin_bit_cast(uint32_t, lm) == wm);
        dmin = __builtin_amdgcn_readlane(li, (int)__builtin_ctzll(hit));
    }
    __threadfence_block();   // this wave's trace stores are visible to its own loads
    int16_t* drow = a.disp + pix0;
    int outv = 0;            // lane (u & 63) of the current 64-column group holds disp[u]
    int u = W - 1;
    outv = lane == (u & 63) ? dmin : outv;
    for (; u > 0; u--) {
        int code, ci;
        if (LT) {   // uniform LDS reads: the two masks of dmin's slot and the column's row minimum
            const int l = dmin / K, j = dmin - l * K;
            const uint64_t m0 = tl[(size_t)u * 2 * K + 2 * j], m1 = tl[(size_t)u * 2 * K + 2 * j + 1];
            code = (int)((m0 >> l) & 1u) | (int)(((m1 >> l) & 1u) << 1);
            ci = cl[u];
        } else {
            code = trow[(size_t)u * D + dmin];
            ci = crow[u];
        }
        dmin = code == 0 ? dmin : (code == 1 ? dmin - 1 : (code == 2 ? dmin + 1 : ci));
        const int t = u - 1;
        if ((t & 63) == 63) {   // the group of columns t + 1 .. has been filled: flush it
            const int g = t + 1;
            if (g + lane < W) drow[g + lane] = (int16_t)outv;
        }
        outv = lane == (t & 63) ? dmin : outv;
    }
    if (lane < W) drow[lane] = (int16_t)outv;   // group 0 (columns 0 .. 63)
}

}  // namespace

void launch_so(const SoArgs& a, hipStream_t st) {
    const int rows = a.n * a.H;
    dim3 grid((unsigned)((rows + 3) / 4));
    const int k = (a.D + 63) / 64;
    const int kk = k <= 1 ? 1 : (k <= 2 ? 2 : (k <= 4 ? 4 : (k <= 8 ? 8 : 16)));
    const size_t shm = 4 * so_lds_words(a.W, kk) * 8;
    const bool lt = shm <= 64 * 1024 && SM_SO_LDS_TRACE;
    const size_t sh = lt ? shm : 0;
#define SM_SO_LAUNCH(KV)                                                              \
    do {                                                                              \
        if (lt) hipLaunchKernelGGL((k_so<KV, true>), grid, dim3(256), sh, st, a);     \
        else hipLaunchKernelGGL((k_so<KV, false>), grid, dim3(256), 0, st, a);       \
    } while (0)
    if (kk == 1) SM_SO_LAUNCH(1);
    else if (kk == 2) SM_SO_LAUNCH(2);
    else if (kk == 4) SM_SO_LAUNCH(4);
    else if (kk == 8) SM_SO_LAUNCH(8);
    else SM_SO_LAUNCH(16);
#undef SM_SO_LAUNCH
}

}  // namespace sm
