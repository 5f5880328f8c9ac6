// sm_sgm.hip — semi-global matching path sweeps with the path sum and WTA fused in.
//
// Reference: sgm (stereoMatching.cpp:6204-6224) runs costScan (cpp:1983-2029) for the direction
// table rv = {+1,-1,0,0,+1,+1,-1,-1}, ru = {0,0,+1,-1,-1,+1,+1,-1} (numOfDirec = 4 by default),
// updateCost<float> (h:2206-2280) per pixel, then gen_sgm_vm (cpp:2031-2056) sums the path
// volumes in path order and gen_dispFromVm (cpp:3928-3967) takes the first strict minimum.
// For a pixel p whose predecessor p + r is inside the image:
//   m = min_d Lr(p+r, d);  P1, P2 = 1, 3 (/4 if max_c |I(p) - I(p+r)| > 15);  P1' = P1 - m
//   Lr(p, d) = C(p, d) + min(min(Lr(p+r,d) - m, Lr(p+r,d-1) + P1'), min(Lr(p+r,d+1) + P1', P2))
// (out-of-range d neighbours are FLT_MAX); a path starts with Lr = C.
//
// gfx950 mapping.  One wave walks one scan line of a direction (the previous pixel of each step
// is the wave's own previous step), lane l holding disparities [l*K, l*K + K).  The path minimum
// m is a DPP + permlane wave reduction, the d +/- 1 neighbours cross lanes with DPP wave_shr/shl —
// no LDS anywhere.  Path order is kept by running the directions as consecutive launches that
// accumulate into one sum volume: path 0 writes acc = 0 + L0, middle paths acc += Li, and the
// last path adds its Li, takes the WTA in registers and writes only the int16 disparity (and the
// summed volume when the caller asks for it).  The next T steps of C and acc are prefetched into
// registers; the colour-difference penalty flags of every pixel come from the prep kernel.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "sm_device.h"
#include "sm_kernels.h"

// Steps prefetched per tile (two tiles in flight).  Large-D launches have few waves per SIMD
// (one line per wave, or four per wave in k_sgm_rows), so their tiles are deep.
#ifndef SM_SGM_ROWS_T1
#define SM_SGM_ROWS_T1 8
#endif
#ifndef SM_SGM_ROWS_T2
#define SM_SGM_ROWS_T2 4
#endif
#ifndef SM_SGM_ROWS_T3
#define SM_SGM_ROWS_T3 2
#endif
#ifndef SM_SGM_ROWS_T4
#define SM_SGM_ROWS_T4 2
#endif
#ifndef SM_SGM_T_K1
#define SM_SGM_T_K1 16
#endif
#ifndef SM_SGM_T_K3
#define SM_SGM_T_K3 5
#endif
#ifndef SM_SGM_T_K4
#define SM_SGM_T_K4 4
#endif
#ifndef SM_SGM_VEC_MIN_D
#define SM_SGM_VEC_MIN_D 128
#endif
#ifndef SM_SGM_T_V4
#define SM_SGM_T_V4 8
#endif
#ifndef SM_SGM_T_BIG
#define SM_SGM_T_BIG 2
#endif

namespace sm {

template <int K>
__device__ __forceinline__ float dpp_shr1(float v) {  // lane l <- lane l-1; lane 0 <- FLT_MAX
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, FLT_MAX),
                                                                 __builtin_bit_cast(int, v), DPP_WAVE_SHR1, 0xF, 0xF, false));
}
template <int K>
__device__ __forceinline__ float dpp_shl1(float v) {  // lane l <- lane l+1; lane 63 <- FLT_MAX
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, FLT_MAX),
                                                                 __builtin_bit_cast(int, v), DPP_WAVE_SHL1, 0xF, 0xF, false));
}

template <int K, int T>
struct SgmTile {
    float c[T][K];
    float acc[T][K];
    uint32_t fl;  // lane t < T: penalty flags of the pixel of step j0 + t
};

template <int K, int MODE, int T, bool FULL, bool VEC>
__global__ __launch_bounds__(256) void k_sgm(const SgmArgs a) {
    constexpr bool SG = (MODE & SGM_SIGNED) != 0;
    // VEC (D % 4 == 0, K % 4 == 0): each lane's K consecutive disparities move as K / 4 dwordx4
    // accesses, so a step of a line is one contiguous D * 4-byte access per volume
    constexpr int KV = VEC ? K / 4 : 1;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int H = a.H, W = a.W, D = a.D;
    const int b = blockIdx.y;
    const int rv = a.rv, ru = a.ru;
    int nlines, v0, u0;
    if (rv == 0) {
        nlines = H;
        v0 = wave;
        u0 = ru > 0 ? W - 1 : 0;
    } else if (ru == 0) {
        nlines = W;
        u0 = wave;
        v0 = rv > 0 ? H - 1 : 0;
    } else {
        nlines = W + H - 1;
        const int vedge = rv > 0 ? H - 1 : 0, uedge = ru > 0 ? W - 1 : 0;
        if (wave < W) {
            v0 = vedge;
            u0 = wave;
        } else {
            const int k = wave - W;
            v0 = rv > 0 ? k : k + 1;
            u0 = uedge;
        }
    }
    if (wave >= nlines) return;  // wave-uniform
    int steps;
    {
        const int nv = rv > 0 ? v0 + 1 : (rv < 0 ? H - v0 : 1 << 30);
        const int nu = ru > 0 ? u0 + 1 : (ru < 0 ? W - u0 : 1 << 30);
        steps = min(nv, nu);
    }
    const int pstep = -rv * W - ru;  // pixel index delta per step (walk = -r)
    const size_t npix = (size_t)H * W;
    const size_t p0 = (size_t)v0 * W + u0;
    const int d0 = lane * K;
    // per-element load/store bases: elements past D read a clamped (valid) address and store to
    // a private dummy slot (VEC: the store is skipped), so no scalar store is predicated
    const float* cbase = a.vm + ((size_t)b * npix + p0) * D;
    float* abase = a.acc + ((size_t)b * npix + p0) * D;
    float* fbase = a.vm + ((size_t)b * npix + p0) * D;
    const uint8_t* flbase = a.flags + (size_t)b * npix + p0;
    int16_t* dbase = a.disp + (size_t)b * npix + p0;
    const long vstep = (long)pstep * D;
    int ld[K];          // load column (clamped to a valid address)
    bool val[K];
    float* ap[K];       // store targets: real element or this lane's dummy slot (stride 0)
    float* fp[K];
    long sst[K];
    bool cval[KV];      // VEC: chunk inside D
    int ldc[KV];        // VEC: chunk load column (clamped)
#pragma unroll
    for (int k = 0; k < K; k++) {
        val[k] = d0 + k < D;
        ld[k] = val[k] ? d0 + k : D - 1;
        ap[k] = val[k] ? abase + d0 + k : a.dummy + ((lane * K + k) & 63);
        fp[k] = val[k] ? fbase + d0 + k : a.dummy + ((lane * K + k) & 63);
        sst[k] = val[k] ? vstep : 0;
    }
#pragma unroll
    for (int c = 0; c < KV; c++) {
        cval[c] = d0 + 4 * c < D;
        ldc[c] = cval[c] ? d0 + 4 * c : D - 4;
    }
    int dacc = -1;      // lane s holds the disparity of step j0 + s until the tile's store
    const float p1 = a.p1, p2 = a.p2;
    const float p1r = p1 / (float)a.redu, p2r = p2 / (float)a.redu;  // updateCost: P1 /= reduCoeffi1
    const int dir = a.dir;

    auto clampi = [&](int s) { return s < steps ? s : steps - 1; };
    auto load = [&](SgmTile<K, T>& t, int j0) {
#pragma unroll
        for (int s = 0; s < T; s++) {
            const long off = (long)clampi(j0 + s) * vstep;
            if (VEC) {
#pragma unroll
                for (int c = 0; c < KV; c++) {
                    const float4 v = ld_stream4(cbase + off + ldc[c]);
                    t.c[s][4 * c + 0] = v.x;
                    t.c[s][4 * c + 1] = v.y;
                    t.c[s][4 * c + 2] = v.z;
                    t.c[s][4 * c + 3] = v.w;
                    if (!(MODE & SGM_FIRST)) {
                        const float4 q = ld_stream4(abase + off + ldc[c]);
                        t.acc[s][4 * c + 0] = q.x;
                        t.acc[s][4 * c + 1] = q.y;
                        t.acc[s][4 * c + 2] = q.z;
                        t.acc[s][4 * c + 3] = q.w;
                    }
                }
            } else {
#pragma unroll
                for (int k = 0; k < K; k++) {
                    t.c[s][k] = ld_stream(cbase + off + ld[k]);
                    if (!(MODE & SGM_FIRST)) t.acc[s][k] = ld_stream(abase + off + ld[k]);
                }
            }
        }
        t.fl = flbase[(long)clampi(j0 + min(lane, T - 1)) * pstep];
    };
    auto store = [&](float* base, float* const* pk, int j, const float* f) {
        if (VEC) {
#pragma unroll
            for (int c = 0; c < KV; c++)
                if (FULL || cval[c])
                    st_stream4(base + (long)j * vstep + d0 + 4 * c, make_float4(f[4 * c + 0], f[4 * c + 1], f[4 * c + 2], f[4 * c + 3]));
        } else {
#pragma unroll
            for (int k = 0; k < K; k++) st_stream(pk[k] + (long)j * sst[k], f[k]);
        }
    };

    float Lp[K];
#pragma unroll
    for (int k = 0; k < K; k++) Lp[k] = FLT_MAX;

    // All path costs are >= +0 (C >= 0; Lp - m >= 0; Lp[d +/- 1] + (P1 - m) >= 0 because
    // fl(P1 - m) >= -m; P2 > 0), so every min below is an exact unsigned min on the bit patterns.
    // SIGNED (guided-filter costs, which can be negative but are never -0 or NaN, nor are the
    // sums of them): v_min_f32 minima, which then equal the reference's std::min exactly.
    // Out-of-range neighbours (d - 1 < 0, d + 1 >= D) hold FLT_MAX from the DPP shift's bound
    // value or the padded lanes; FLT_MAX + (P1 - m) never undercuts P2 <= 3, so those terms
    // cannot win the min and need no separate select.
    auto step = [&](const SgmTile<K, T>& t, int s, int j, bool start) {
        float L[K];
        if (start) {
#pragma unroll
            for (int k = 0; k < K; k++) L[k] = (FULL || val[k]) ? t.c[s][k] : FLT_MAX;
        } else {
            const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)t.fl, s);
            const bool pen = (fl >> dir) & 1u;
            const float P1 = pen ? p1r : p1, P2 = pen ? p2r : p2;
            float lm = Lp[0];
#pragma unroll
            for (int k = 1; k < K; k++) lm = SG ? fminf(lm, Lp[k]) : fmin_pos(lm, Lp[k]);
            const float m = SG ? wave_min(lm) : wave_min_pos(lm);   // wave-uniform
            const float P1m = P1 - m;
            const float left = dpp_shr1<K>(Lp[K - 1]);
            const float right = dpp_shl1<K>(Lp[0]);
#pragma unroll
            for (int k = 0; k < K; k++) {
                const float prev = (k == 0) ? left : Lp[k - 1];
                const float next = (k == K - 1) ? right : Lp[k + 1];
                const float S1 = Lp[k] - m;
                const float S2 = prev + P1m;
                const float S3 = next + P1m;
                const float mm = SG ? fminf(fminf(S1, S2), fminf(S3, P2)) : fmin_pos(fmin_pos(S1, S2), fmin_pos(S3, P2));
                const float Lk = t.c[s][k] + mm;
                L[k] = (FULL || val[k]) ? Lk : FLT_MAX;
            }
        }
        float f[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const float prev = (MODE & SGM_FIRST) ? 0.f : t.acc[s][k];
            f[k] = prev + L[k];   // sum += Lr[num] (cpp:2046-2049); padded lanes stay FLT_MAX
        }
        if (MODE & SGM_LAST) {
            if (MODE & SGM_KEEP) store(fbase, fp, j, f);
            float bm = f[0];
            int bi = d0;
#pragma unroll
            for (int k = 1; k < K; k++)
                if (bm > f[k]) {
                    bm = f[k];
                    bi = d0 + k;
                }
            // first minimum: lowest lane holding the wave minimum, then that lane's first index
            // (padded lanes hold FLT_MAX and only match when every cost is FLT_MAX -> -1)
            const float wm = SG ? wave_min(bm) : wave_min_pos(bm);
            const uint64_t hit = __ballot(bm == wm);
            const int widx = __builtin_amdgcn_readlane(bi, (int)__builtin_ctzll(hit));
            const int dsel = (wm < FLT_MAX) ? widx : -1;
            dacc = (lane == s) ? dsel : dacc;
        } else {
            store(abase, ap, j, f);
        }
#pragma unroll
        for (int k = 0; k < K; k++) Lp[k] = L[k];
    };

    auto process = [&](const SgmTile<K, T>& t, int j0) {
        if (j0 > 0 && j0 + T <= steps) {
#pragma unroll
            for (int s = 0; s < T; s++) step(t, s, j0 + s, false);
        } else {
#pragma unroll
            for (int s = 0; s < T; s++)
                if (j0 + s < steps) step(t, s, j0 + s, j0 + s == 0);
        }
        if (MODE & SGM_LAST) {  // one store instruction per tile for the int16 disparities
            if (lane < T && j0 + lane < steps) dbase[(long)(j0 + lane) * pstep] = (int16_t)dacc;
        }
    };

    SgmTile<K, T> ta, tb;
    load(ta, 0);
    for (int j0 = 0; j0 < steps; j0 += 2 * T) {
        load(tb, j0 + T);
        process(ta, j0);
        load(ta, j0 + 2 * T);
        process(tb, j0 + T);
    }
}

// ---------------------------------------------------------------------------------------
// Straight paths (rv == 0 or ru == 0) with D % 4 == 0: four lines per wave, one DPP row of 16
// lanes per line, K = 4 * KV consecutive disparities per lane.  Every step of a wave then moves
// 4 x 256 B per volume with dwordx4 accesses (uniform tile base + 32-bit lane offset), the path minimum is a 4-stage DPP row
// reduction, d +/- 1 neighbours cross lanes with row_shr / row_shl (whose row boundaries are
// the line boundaries), and the colour-difference flag of each line's pixel reaches its row
// with one ds_bpermute.  Arithmetic and its order are those of k_sgm.
// ---------------------------------------------------------------------------------------
enum : int { DPP_ROW_SHL1 = 0x101, DPP_ROW_SHR1 = 0x111 };

template <int CTRL>
__device__ __forceinline__ float row_shift(float v) {  // lane l <- lane l -/+ 1 within its row; FLT_MAX at the row end
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, FLT_MAX),
                                                                 __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t row_umin(uint32_t v) {  // every lane: min over its row of 16
    v = umin_dpp<DPP_QUAD_1032>(v);
    v = umin_dpp<DPP_QUAD_2301>(v);
    v = umin_dpp<DPP_ROW_HALF_MIRROR>(v);
    return umin_dpp<DPP_ROW_MIRROR>(v);
}

__device__ __forceinline__ float row_fmin(float v) {  // every lane: min over its row of 16 (any sign)
    v = fminf(v, dpp_f<DPP_QUAD_1032>(v));
    v = fminf(v, dpp_f<DPP_QUAD_2301>(v));
    v = fminf(v, dpp_f<DPP_ROW_HALF_MIRROR>(v));
    return fminf(v, dpp_f<DPP_ROW_MIRROR>(v));
}

template <int KV, int T>
struct RowTile {
    float c[T][4 * KV];
    float acc[T][4 * KV];
    uint32_t fl;  // lane l16 < T: flags of the row's pixel at step j0 + l16
};

template <int KV, int MODE, int T, bool FULLC>
__global__ __launch_bounds__(256) void k_sgm_rows(const SgmArgs a) {
    constexpr int K = 4 * KV;
    constexpr bool SG = (MODE & SGM_SIGNED) != 0;   // costs of either sign (GF): float mins
    auto mn = [](float x, float y) { return SG ? fminf(x, y) : fmin_pos(x, y); };
    auto rmin = [](float x) { return SG ? row_fmin(x) : __builtin_bit_cast(float, row_umin(__builtin_bit_cast(uint32_t, x))); };
    const int lane = threadIdx.x & 63, row = lane >> 4, l16 = lane & 15;
    const int H = a.H, W = a.W, D = a.D;
    const bool vert = a.ru == 0;                      // lines are columns
    const bool neg = vert ? a.rv > 0 : a.ru > 0;      // walk starts at the far end
    const int nl = vert ? W : H, steps = vert ? H : W;
    const int wpp = (nl + 3) >> 2;
    // wave index made provably uniform: buffer resources must live in SGPRs (a VGPR-resident
    // resource makes the compiler wrap every access in a readfirstlane loop)
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256 + threadIdx.x) >> 6));
    const int b = wave / wpp;
    if (b >= a.n) return;                             // wave-uniform
    const int w = wave - b * wpp;
    const int line0 = 4 * w;
    const bool line_ok = line0 + row < nl;
    const int line = line_ok ? line0 + row : nl - 1;
    const size_t npix = (size_t)H * W;
    const long step_px = vert ? W : 1;                // pixels between consecutive steps
    const long line_px = vert ? 1 : W;                // pixels between consecutive lines
    // pixel of (line, step j) relative to the pair: vert (v, u) = (neg ? H-1-j : j, line)
    auto pix = [&](int ln, int j) -> long {
        const int t = neg ? steps - 1 - j : j;
        return vert ? (long)t * W + ln : (long)ln * W + t;
    };
    const int d0 = l16 * K;
    const uint32_t rowoff = (uint32_t)((line - line0) * line_px * D * 4);
    uint32_t voff[KV];                                 // lane byte offset of each 4-disparity chunk
    bool cval[KV];                                     // chunk inside D (D % 4 == 0: all or nothing)
#pragma unroll
    for (int c = 0; c < KV; c++) {
        cval[c] = d0 + 4 * c < D;
        voff[c] = rowoff + (uint32_t)(d0 + 4 * c) * 4u;  // chunks past D read the next pixel (padded allocation)
    }
    const bool st_ok = line_ok;                        // rows past the last line never store
    const uint32_t sstride = (uint32_t)(step_px * D * 4);
    const float* vmp = a.vm + (size_t)b * npix * D;
    float* accp = a.acc + (size_t)b * npix * D;
    const uint8_t* flp = a.flags + (size_t)b * npix;
    int16_t* dp = a.disp + (size_t)b * npix;
    const float p1 = a.p1, p2 = a.p2;
    const float p1r = p1 / (float)a.redu, p2r = p2 / (float)a.redu;
    const int dir = a.dir;

    // tile geometry: the lowest-address pixel of steps j0 .. j0+T-1 (clamped to the line) is the
    // resource base; step s sits at soff(s) bytes above it
    // (prefetched tiles may start past the line end: every step clamps to the last pixel, so no
    // address ever leaves the line)
    auto tile_base = [&](int j0) -> long { return pix(line0, neg ? min(j0 + T - 1, steps - 1) : min(j0, steps - 1)); };
    auto soff = [&](int j0, int s) -> uint32_t {
        const int js = min(j0 + s, steps - 1);
        const int rel = neg ? min(j0 + T - 1, steps - 1) - js : js - min(j0, steps - 1);
        return (uint32_t)rel * sstride;
    };
    auto load = [&](RowTile<KV, T>& t, int j0) {
        const long bp = tile_base(j0);
        const char* rc = (const char*)(vmp + bp * D);
        const char* ra = (const char*)(accp + bp * D);
#pragma unroll
        for (int s = 0; s < T; s++) {
            const uint32_t so = soff(j0, s);
#pragma unroll
            for (int c = 0; c < KV; c++) {
                const float4 v = ld_stream4((const float*)(rc + so + voff[c]));
                t.c[s][4 * c + 0] = v.x;
                t.c[s][4 * c + 1] = v.y;
                t.c[s][4 * c + 2] = v.z;
                t.c[s][4 * c + 3] = v.w;
                if (!(MODE & SGM_FIRST)) {
                    const float4 q = ld_stream4((const float*)(ra + so + voff[c]));
                    t.acc[s][4 * c + 0] = q.x;
                    t.acc[s][4 * c + 1] = q.y;
                    t.acc[s][4 * c + 2] = q.z;
                    t.acc[s][4 * c + 3] = q.w;
                }
            }
        }
        t.fl = flp[pix(line, min(j0 + min(l16, T - 1), steps - 1))];
    };

    float Lp[K];
#pragma unroll
    for (int k = 0; k < K; k++) Lp[k] = FLT_MAX;
    int dacc = -1;

    auto step = [&](const RowTile<KV, T>& t, int s, bool start, float* f) {
        float L[K];
        if (start) {
#pragma unroll
            for (int k = 0; k < K; k++) L[k] = cval[k / 4] ? t.c[s][k] : FLT_MAX;
        } else {
            const uint32_t fl = (uint32_t)__builtin_amdgcn_ds_bpermute(row * 64 + s * 4, (int)t.fl);  // row's lane s
            const bool pen = (fl >> dir) & 1u;
            const float P1 = pen ? p1r : p1, P2 = pen ? p2r : p2;
            float lm = Lp[0];
#pragma unroll
            for (int k = 1; k < K; k++) lm = mn(lm, Lp[k]);
            const float m = rmin(lm);
            const float P1m = P1 - m;
            const float left = row_shift<DPP_ROW_SHR1>(Lp[K - 1]);
            const float right = row_shift<DPP_ROW_SHL1>(Lp[0]);
#pragma unroll
            for (int k = 0; k < K; k++) {
                const float prev = (k == 0) ? left : Lp[k - 1];
                const float next = (k == K - 1) ? right : Lp[k + 1];
                const float S1 = Lp[k] - m;
                const float S2 = prev + P1m;
                const float S3 = next + P1m;
                const float mm = mn(mn(S1, S2), mn(S3, P2));
                const float Lk = t.c[s][k] + mm;
                L[k] = cval[k / 4] ? Lk : FLT_MAX;
            }
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const float prev = (MODE & SGM_FIRST) ? 0.f : t.acc[s][k];
            f[k] = prev + L[k];
            Lp[k] = L[k];
        }
    };

    auto store4 = [&](char* r, uint32_t so, const float* f) {
#pragma unroll
        for (int c = 0; c < KV; c++)
            if (FULLC || cval[c]) st_stream4((float*)(r + so + voff[c]), make_float4(f[4 * c + 0], f[4 * c + 1], f[4 * c + 2], f[4 * c + 3]));
    };

    auto process = [&](const RowTile<KV, T>& t, int j0) {
        const long bp = tile_base(j0);
        char* rout = (char*)((MODE & SGM_LAST) ? (float*)vmp + bp * D : accp + bp * D);
#pragma unroll
        for (int s = 0; s < T; s++) {
            if (j0 + s >= steps) break;                   // wave-uniform
            float f[K];
            step(t, s, j0 + s == 0, f);
            const uint32_t so = soff(j0, s);
            if ((!(MODE & SGM_LAST) || (MODE & SGM_KEEP)) && st_ok) store4(rout, so, f);
            if (MODE & SGM_LAST) {
                // first minimum of the row: lowest lane of the row holding its minimum, then that
                // lane's first index (chunks past D hold FLT_MAX: -1 when everything is FLT_MAX)
                float bm = f[0];
                int bi = d0;
#pragma unroll
                for (int k = 1; k < K; k++)
                    if (bm > f[k]) {
                        bm = f[k];
                        bi = d0 + k;
                    }
                const float wm = rmin(bm);
                const uint64_t hit = __ballot(bm == wm);
                const uint32_t rmask = (uint32_t)(hit >> (row * 16)) & 0xffffu;
                const int src = row * 16 + __builtin_ctz(rmask);
                const int widx = __builtin_amdgcn_ds_bpermute(src * 4, bi);
                const int dsel = (wm < FLT_MAX) ? widx : -1;
                dacc = (l16 == s) ? dsel : dacc;
            }
        }
        if (MODE & SGM_LAST) {
            if (line_ok && l16 < T && j0 + l16 < steps) dp[pix(line, j0 + l16)] = (int16_t)dacc;
        }
    };

    RowTile<KV, T> ta, tb;
    load(ta, 0);
    for (int j0 = 0; j0 < steps; j0 += 2 * T) {
        load(tb, j0 + T);
        process(ta, j0);
        if (j0 + T >= steps) break;
        load(ta, j0 + 2 * T);
        process(tb, j0 + T);
    }
}

template <int KV, bool FULLC, int S>
static void launch_rows_m(const SgmArgs& a, int mode, dim3 grid, hipStream_t st) {
    constexpr int T = KV == 1 ? SM_SGM_ROWS_T1 : (KV == 2 ? SM_SGM_ROWS_T2 : (KV == 3 ? SM_SGM_ROWS_T3 : SM_SGM_ROWS_T4));
    switch (mode) {
        case SGM_FIRST: hipLaunchKernelGGL((k_sgm_rows<KV, S | SGM_FIRST, T, FULLC>), grid, dim3(256), 0, st, a); break;
        case SGM_LAST: hipLaunchKernelGGL((k_sgm_rows<KV, S | SGM_LAST, T, FULLC>), grid, dim3(256), 0, st, a); break;
        case SGM_LAST | SGM_KEEP: hipLaunchKernelGGL((k_sgm_rows<KV, S | SGM_LAST | SGM_KEEP, T, FULLC>), grid, dim3(256), 0, st, a); break;
        case SGM_FIRST | SGM_LAST: hipLaunchKernelGGL((k_sgm_rows<KV, S | SGM_FIRST | SGM_LAST, T, FULLC>), grid, dim3(256), 0, st, a); break;
        case SGM_FIRST | SGM_LAST | SGM_KEEP:
            hipLaunchKernelGGL((k_sgm_rows<KV, S | SGM_FIRST | SGM_LAST | SGM_KEEP, T, FULLC>), grid, dim3(256), 0, st, a);
            break;
        default: hipLaunchKernelGGL((k_sgm_rows<KV, S, T, FULLC>), grid, dim3(256), 0, st, a); break;
    }
}

template <int KV, bool FULLC>
static void launch_rows_f(const SgmArgs& a, int mode, int n, hipStream_t st) {
    const int nl = a.ru == 0 ? a.W : a.H;
    const int waves = (nl + 3) / 4 * n;
    dim3 grid((waves + 3) / 4);
    if ((mode & SGM_LAST) && a.keep_final) mode |= SGM_KEEP;
    if (a.signed_costs)
        launch_rows_m<KV, FULLC, SGM_SIGNED>(a, mode, grid, st);
    else
        launch_rows_m<KV, FULLC, 0>(a, mode, grid, st);
}

template <int KV>
static void launch_rows(const SgmArgs& a, int mode, int n, hipStream_t st) {
    if (a.D == 16 * 4 * KV)
        launch_rows_f<KV, true>(a, mode, n, st);
    else
        launch_rows_f<KV, false>(a, mode, n, st);
}

template <int K, bool FULL, bool VEC = false>
static void launch_kf(const SgmArgs& a, int mode, int n, hipStream_t st) {
    const int nlines = a.rv == 0 ? a.H : (a.ru == 0 ? a.W : a.W + a.H - 1);
    dim3 grid((nlines + 3) / 4, n);
    constexpr int T = VEC ? (K == 4 ? SM_SGM_T_V4 : SM_SGM_T_BIG)
                          : (K >= 8 ? SM_SGM_T_BIG : (K == 3 ? SM_SGM_T_K3 : (K == 4 ? SM_SGM_T_K4 : (K == 1 ? SM_SGM_T_K1 : 16 / K))));
    if ((mode & SGM_LAST) && a.keep_final) mode |= SGM_KEEP;
    switch (mode) {
        case SGM_FIRST: hipLaunchKernelGGL((k_sgm<K, SGM_FIRST, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
        case SGM_LAST: hipLaunchKernelGGL((k_sgm<K, SGM_LAST, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
        case SGM_LAST | SGM_KEEP: hipLaunchKernelGGL((k_sgm<K, SGM_LAST | SGM_KEEP, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
        case SGM_FIRST | SGM_LAST: hipLaunchKernelGGL((k_sgm<K, SGM_FIRST | SGM_LAST, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
        case SGM_FIRST | SGM_LAST | SGM_KEEP:
            hipLaunchKernelGGL((k_sgm<K, SGM_FIRST | SGM_LAST | SGM_KEEP, T, FULL, VEC>), grid, dim3(256), 0, st, a);
            break;
        default: hipLaunchKernelGGL((k_sgm<K, 0, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
    }
}

template <int K, bool FULL, bool VEC = false>
static void launch_kf_signed(const SgmArgs& a, int mode, int n, hipStream_t st) {
    const int nlines = a.rv == 0 ? a.H : (a.ru == 0 ? a.W : a.W + a.H - 1);
    dim3 grid((nlines + 3) / 4, n);
    constexpr int T = VEC ? (K == 4 ? SM_SGM_T_V4 : SM_SGM_T_BIG)
                          : (K >= 8 ? SM_SGM_T_BIG : (K == 3 ? SM_SGM_T_K3 : (K == 4 ? SM_SGM_T_K4 : (K == 1 ? SM_SGM_T_K1 : 16 / K))));
    constexpr int S = SGM_SIGNED;
    if ((mode & SGM_LAST) && a.keep_final) mode |= SGM_KEEP;
    switch (mode) {
        case SGM_FIRST: hipLaunchKernelGGL((k_sgm<K, S | SGM_FIRST, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
        case SGM_LAST: hipLaunchKernelGGL((k_sgm<K, S | SGM_LAST, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
        case SGM_LAST | SGM_KEEP: hipLaunchKernelGGL((k_sgm<K, S | SGM_LAST | SGM_KEEP, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
        case SGM_FIRST | SGM_LAST: hipLaunchKernelGGL((k_sgm<K, S | SGM_FIRST | SGM_LAST, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
        case SGM_FIRST | SGM_LAST | SGM_KEEP:
            hipLaunchKernelGGL((k_sgm<K, S | SGM_FIRST | SGM_LAST | SGM_KEEP, T, FULL, VEC>), grid, dim3(256), 0, st, a);
            break;
        default: hipLaunchKernelGGL((k_sgm<K, S, T, FULL, VEC>), grid, dim3(256), 0, st, a); break;
    }
}

template <int K>
static void launch_k(const SgmArgs& a, int mode, int n, hipStream_t st) {
    if (a.signed_costs) {
        if (a.D == 64 * K)
            launch_kf_signed<K, true>(a, mode, n, st);
        else
            launch_kf_signed<K, false>(a, mode, n, st);
        return;
    }
    if (a.D == 64 * K)
        launch_kf<K, true>(a, mode, n, st);
    else
        launch_kf<K, false>(a, mode, n, st);
}

// Lanes-per-line layout for straight paths with D <= SM_SGM_VEC_MIN_D.  Measured on MI355X
// (Teddy x16): faster for the vertical paths and the last (WTA) path, slower for the middle
// horizontal one, whose K = 1 sweep already streams whole rows.  Larger D runs every direction
// one line per wave with dwordx4 lanes
// (k_sgm VEC): the four-lines-per-wave layout leaves too few waves in flight there
// (tools/ubench_sgm.hip, KITTI D = 192: 3.5 TB/s with 4 lines per wave vs 5.0 TB/s with one).
static int rows_kv(const SgmArgs& a, int mode) {
    if ((a.rv != 0 && a.ru != 0) || a.D % 4 != 0 || a.D > SM_SGM_VEC_MIN_D) return 0;
    if (!(a.ru == 0 || (mode & SGM_LAST))) return 0;
    const int K = (a.D + 15) / 16;
    return (K + 3) / 4;
}

// ---------------------------------------------------------------------------------------
// Checkpointed path pairs.  The path sum is ((L0 + L1) + L2) + L3 ... (gen_sgm_vm,
// cpp:2031-2056; 0 + L0 == L0), and paths 0 / 1 (2 / 3) walk one line direction both ways, so a
// pair needs no L volume in memory: pass A walks the pair's first path and keeps its L only at
// the end of every segment of S steps; pass B walks the second path segment by segment and
// first recomputes the first path's S values of the segment from the checkpoint before it —
// the same operations on the same inputs, hence the same bits — then combines both in
// registers.  Per element: A reads C (4 B + 4 / S for the checkpoints); B of pair (0, 1) reads C
// and writes L0 + L1 (8 B + 4 / S); B of pair (2, 3) reads C and L0 + L1 and writes the map
// (8 B + 4 / S) or, with 8 paths, the running sum (12 B + 4 / S): 24 B instead of the four
// sweeps' 8 + 12 + 12 + 8, for half again the recursion arithmetic, which sweeps that wait on
// memory have to spare.  Paths 4 .. 7 (8 paths) then run as k_sgm / k_sgm_rows sweeps.
// Segment k of pass B covers the first path's steps [steps - (k+1) S, steps - k S) (the last
// segment may start before step 0); checkpoint slot k holds the first path's L at step
// steps - (k+1) S - 1, i.e. at the end of the A tile before it.
// Layouts: D in (128, 256]: k_sgm<4, ..., VEC>'s, one line per wave, four consecutive
// disparities per lane (dwordx4); D <= 128: k_sgm_rows's, four lines per wave, a DPP row of 16
// lanes per line, 4 KV disparities per lane.  D % 4 == 0 throughout.
// Diagonal pair (8 paths, one line per wave): paths 4 and 6 walk the anti-diagonals both ways,
// but the sum puts L5 between them: (((acc + L4) + L5) + L6) + L7.  Path 5 (the other diagonal
// family) therefore runs as an SGM_FIRST sweep that stores L5 itself (4 + 4 B), pass A walks path
// 4 (4 B), pass B walks path 6 with L4 recomputed and reads acc and L5 (16 B), and the last path
// stays a sweep (8 B): 32 B + checkpoints instead of the three sweeps' 12 + 12 + 12 + 8.  Lines
// are k_sgm's diagonals of the first path (W + H - 1 of them, 1 .. min(H, W) steps; checkpoint
// slots strided by the longest), segments of SM_SGM_CK_SD steps.
// ---------------------------------------------------------------------------------------
#ifndef SM_SGM_CK
#define SM_SGM_CK 1
#endif
#ifndef SM_SGM_CK_S
#define SM_SGM_CK_S 8        // segment steps (layouts with 4 disparities per lane)
#endif
#ifndef SM_SGM_CK_S2
#define SM_SGM_CK_S2 4       // segment steps with 8 disparities per lane (D in (64, 128])
#endif

#ifndef SM_SGM_CK_DIAG
#define SM_SGM_CK_DIAG 1     // 8 paths, 128 < D <= 256: the diagonal pair (4, 6) checkpointed too
#endif
#ifndef SM_SGM_CK_SD
#define SM_SGM_CK_SD 4       // segment steps of the diagonal pair (its pass B also holds L5's segment)
#endif

bool sgm_ck_ok(int D, int paths) { return SM_SGM_CK && (paths == 4 || paths == 8) && D <= 256 && D % 4 == 0; }
static int ck_kv(int D) { return D > SM_SGM_VEC_MIN_D ? 0 : ((D + 15) / 16 + 3) / 4; }   // 0: one line per wave
int sgm_ck_seg(int D) { return ck_kv(D) == 2 ? SM_SGM_CK_S2 : SM_SGM_CK_S; }
bool sgm_ck_diag_ok(int D, int paths) { return SM_SGM_CK_DIAG && paths == 8 && sgm_ck_ok(D, paths) && ck_kv(D) == 0; }
int sgm_ck_diag_seg() { return SM_SGM_CK_SD; }

template <int KV, bool ROWS, bool FULL, bool SG>
struct CkStep {
    static constexpr int K = 4 * KV;
    float p1, p2, p1r, p2r;
    bool cv[KV];   // the lane's c-th chunk of four disparities lies inside D
    __device__ __forceinline__ float mn(float x, float y) const { return SG ? fminf(x, y) : fmin_pos(x, y); }
    __device__ __forceinline__ float line_min(float x) const {
        if (ROWS) return SG ? row_fmin(x) : __builtin_bit_cast(float, row_umin(__builtin_bit_cast(uint32_t, x)));
        return SG ? wave_min(x) : wave_min_pos(x);
    }
    // one step of updateCost (h:2206-2280): k_sgm's / k_sgm_rows's step, operation for operation
    __device__ __forceinline__ void run(float (&L)[K], const float (&Lp)[K], const float (&c)[K], bool pen, bool start) const {
        if (start) {
#pragma unroll
            for (int k = 0; k < K; k++) L[k] = (FULL || cv[k / 4]) ? c[k] : FLT_MAX;
            return;
        }
        const float P1 = pen ? p1r : p1, P2 = pen ? p2r : p2;
        float lm = Lp[0];
#pragma unroll
        for (int k = 1; k < K; k++) lm = mn(lm, Lp[k]);
        const float m = line_min(lm);
        const float P1m = P1 - m;
        const float left = ROWS ? row_shift<DPP_ROW_SHR1>(Lp[K - 1]) : dpp_shr1<K>(Lp[K - 1]);
        const float right = ROWS ? row_shift<DPP_ROW_SHL1>(Lp[0]) : dpp_shl1<K>(Lp[0]);
#pragma unroll
        for (int k = 0; k < K; k++) {
            const float prev = (k == 0) ? left : Lp[k - 1];
            const float next = (k == K - 1) ? right : Lp[k + 1];
            const float S1 = Lp[k] - m;
            const float S2 = prev + P1m;
            const float S3 = next + P1m;
            const float mm = mn(mn(S1, S2), mn(S3, P2));
            const float Lk = c[k] + mm;
            L[k] = (FULL || cv[k / 4]) ? Lk : FLT_MAX;
        }
    }
};

template <int K>
__device__ __forceinline__ void cpk(float (&d)[K], const float (&s)[K]) {
#pragma unroll
    for (int k = 0; k < K; k++) d[k] = s[k];
}

template <int S, int MODE, int KV, bool ROWS, bool FULL>
__global__ __launch_bounds__(256) void k_sgm_ck(const SgmArgs a) {
    static_assert(ROWS || KV == 1, "one line per wave: four disparities per lane");
    constexpr int K = 4 * KV;
    constexpr int LPL = ROWS ? 16 : 64;   // lanes per line
    constexpr bool SG = (MODE & SGM_SIGNED) != 0;
    constexpr bool LAST = (MODE & SGM_LAST) != 0;
    constexpr bool ACC_IN = LAST || (MODE & CK_MID) != 0;
    constexpr bool LX = (MODE & CK_X) != 0;   // L5 between the pair's paths (diagonal pair)
    const int lane = threadIdx.x & 63;
    const int row = ROWS ? lane >> 4 : 0, ll = ROWS ? lane & 15 : lane;
    const int H = a.H, W = a.W, D = a.D;
    const bool diag = !ROWS && a.rv != 0 && a.ru != 0;   // the diagonal pair: one line per wave only
    const bool horiz = a.rv == 0;
    const int nl = diag ? W + H - 1 : (horiz ? H : W);
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256 + threadIdx.x) >> 6));
    int b, line;
    bool line_ok;
    if (ROWS) {   // 1-D grid over (pair, group of four lines)
        const int wpp = (nl + 3) >> 2;
        b = wave / wpp;
        if (b >= a.n) return;                 // wave-uniform
        const int l = 4 * (wave - b * wpp) + row;
        line_ok = l < nl;
        line = line_ok ? l : nl - 1;          // rows past the last line run a copy and store nothing
    } else {      // 2-D grid: (line, pair)
        b = blockIdx.y;
        if (wave >= nl) return;               // wave-uniform
        line = wave;
        line_ok = true;
    }
    int v0, u0, steps;
    if (!diag) {
        v0 = horiz ? line : (a.rv > 0 ? H - 1 : 0);
        u0 = horiz ? (a.ru > 0 ? W - 1 : 0) : line;
        steps = horiz ? W : H;
    } else {   // k_sgm's diagonal lines of the first path: W from the edge row, then H - 1 from the edge column
        if (line < W) {
            v0 = a.rv > 0 ? H - 1 : 0;
            u0 = line;
        } else {
            const int k = line - W;
            v0 = a.rv > 0 ? k : k + 1;
            u0 = a.ru > 0 ? W - 1 : 0;
        }
        steps = min(a.rv > 0 ? v0 + 1 : H - v0, a.ru > 0 ? u0 + 1 : W - u0);
    }
    const int pstep = -a.rv * W - a.ru;       // pixel delta per step of the pair's FIRST path
    const size_t npix = (size_t)H * W;
    const size_t p0 = (size_t)v0 * W + u0;
    const long vstep = (long)pstep * D;
    const int d0 = ll * K;
    CkStep<KV, ROWS, FULL, SG> st;
    st.p1 = a.p1;
    st.p2 = a.p2;
    st.p1r = a.p1 / (float)a.redu;
    st.p2r = a.p2 / (float)a.redu;
    int ldc[KV];                              // chunk load column (chunks past D: a valid one)
#pragma unroll
    for (int c = 0; c < KV; c++) {
        st.cv[c] = d0 + 4 * c < D;
        ldc[c] = st.cv[c] ? d0 + 4 * c : D - 4;
    }
    const float* cld = a.vm + ((size_t)b * npix + p0) * D;
    const float* ald = a.acc + ((size_t)b * npix + p0) * D;
    float* ast = a.acc + ((size_t)b * npix + p0) * D;
    float* fst = a.vm + ((size_t)b * npix + p0) * D;
    const uint8_t* flbase = a.flags + (size_t)b * npix + p0;
    int16_t* dbase = a.disp + (size_t)b * npix + p0;
    const int nseg = (steps + S - 1) / S;     // segments of the line (= its checkpoint slots)
    const int nslot = diag ? (min(H, W) + S - 1) / S : nseg;   // slot stride per line
    float* ckl = a.ck + ((size_t)b * nl + line) * (size_t)nslot * D;
    const float* xld = LX ? a.lx + ((size_t)b * npix + p0) * D : nullptr;
    const int dirA = a.dir, dirB = a.dir2;
    auto clampj = [&](int j) { return j < 0 ? 0 : (j >= steps ? steps - 1 : j); };
    auto pen = [&](uint32_t fl, int s, int dir) {
        const uint32_t f = ROWS ? (uint32_t)__builtin_amdgcn_ds_bpermute(row * 64 + s * 4, (int)fl)   // the row's lane s
                                : (uint32_t)__builtin_amdgcn_readlane((int)fl, s);
        return ((f >> dir) & 1u) != 0;
    };
    auto ldK = [&](float (&d)[K], const float* base, long off) {
#pragma unroll
        for (int c = 0; c < KV; c++) {
            const float4 v = ld_stream4(base + off + ldc[c]);
            d[4 * c + 0] = v.x;
            d[4 * c + 1] = v.y;
            d[4 * c + 2] = v.z;
            d[4 * c + 3] = v.w;
        }
    };
    auto stK = [&](float* base, long off, const float (&f)[K]) {
        if (!line_ok) return;
#pragma unroll
        for (int c = 0; c < KV; c++)
            if (FULL || st.cv[c]) st_stream4(base + off + d0 + 4 * c, make_float4(f[4 * c + 0], f[4 * c + 1], f[4 * c + 2], f[4 * c + 3]));
    };
    auto flag_of = [&](int j0) { return (uint32_t)flbase[(long)clampj(j0 + min(ll, S - 1)) * pstep]; };

    if constexpr ((MODE & CK_A) != 0) {
        // pass A: the first path; tile t covers steps [steps - (nseg - t) S, ... + S), so every
        // tile but the last ends on a checkpoint (slot nseg - t - 2)
        struct Tl {
            float c[S][K];
            uint32_t fl;   // lane s < S (of each line): flags of the tile's step s
        };
        auto load = [&](Tl& t, int tt) {
            const int j0 = steps - (nseg - tt) * S;
#pragma unroll
            for (int s = 0; s < S; s++) ldK(t.c[s], cld, (long)clampj(j0 + s) * vstep);
            t.fl = flag_of(j0);
        };
        float Lp[K];
#pragma unroll
        for (int k = 0; k < K; k++) Lp[k] = FLT_MAX;
        auto process = [&](const Tl& t, int tt) {
            const int j0 = steps - (nseg - tt) * S;
            if (j0 > 0) {
#pragma unroll
                for (int s = 0; s < S; s++) {
                    float L[K];
                    st.run(L, Lp, t.c[s], pen(t.fl, s, dirA), false);
                    cpk(Lp, L);
                }
            } else {
#pragma unroll
                for (int s = 0; s < S; s++)
                    if (j0 + s >= 0) {
                        float L[K];
                        st.run(L, Lp, t.c[s], pen(t.fl, s, dirA), j0 + s == 0);
                        cpk(Lp, L);
                    }
            }
            if (tt <= nseg - 2) stK(ckl, (long)(nseg - tt - 2) * D, Lp);
        };
        Tl ta, tb;
        load(ta, 0);
        for (int tt = 0; tt < nseg; tt += 2) {
            load(tb, tt + 1);
            process(ta, tt);
            load(ta, tt + 2);
            if (tt + 1 < nseg) process(tb, tt + 1);
        }
    } else {
        // pass B: the second path, segment k = the first path's steps [aj0, aj0 + S), walked
        // from aj0 + S - 1 down; the first path's L over the segment is recomputed in registers
        struct Sg {
            float c[S][K];
            float acc[ACC_IN ? S : 1][K];   // the running sum (pair (2, 3))
            float lx[LX ? S : 1][K];        // L5 (diagonal pair)
            float ck[K];                    // the first path's L at step aj0 - 1
            uint32_t fl;
        };
        auto load = [&](Sg& g, int k) {
            const int aj0 = steps - (k + 1) * S;
#pragma unroll
            for (int s = 0; s < S; s++) {
                const long off = (long)clampj(aj0 + s) * vstep;
                ldK(g.c[s], cld, off);
                if (ACC_IN) ldK(g.acc[s], ald, off);
                if (LX) ldK(g.lx[s], xld, off);
            }
            ldK(g.ck, ckl, (long)(k < nseg - 1 ? k : 0) * D);
            // chunks past D: checkpoints are only stored inside D, and those lanes must hold
            // FLT_MAX (the d + 1 neighbour of the last disparity) as in pass A
#pragma unroll
            for (int q = 0; q < K; q++) g.ck[q] = (FULL || st.cv[q / 4]) ? g.ck[q] : FLT_MAX;
            g.fl = flag_of(aj0);
        };
        float Lp[K];
#pragma unroll
        for (int k = 0; k < K; k++) Lp[k] = FLT_MAX;
        int dacc = -1;   // LAST: lane s (of each line) holds the disparity of segment step s
        auto emit = [&](const Sg& g, int s, int j, const float (&LA)[K], const float (&LB)[K]) {
            float f[K];
#pragma unroll
            for (int q = 0; q < K; q++)
                f[q] = LX ? ((g.acc[s][q] + LA[q]) + g.lx[s][q]) + LB[q] : (ACC_IN ? (g.acc[s][q] + LA[q]) + LB[q] : LA[q] + LB[q]);
            if (!LAST) {
                stK(ast, (long)j * vstep, f);
                return;
            }
            if (MODE & SGM_KEEP) stK(fst, (long)j * vstep, f);
            // first minimum: the lowest lane of the line holding its minimum, then that lane's
            // first index (lanes past D hold FLT_MAX or more: -1 only when everything does)
            float bm = f[0];
            int bi = d0;
#pragma unroll
            for (int q = 1; q < K; q++)
                if (bm > f[q]) {
                    bm = f[q];
                    bi = d0 + q;
                }
            const float wm = st.line_min(bm);
            const uint64_t hit = __ballot(bm == wm);
            int widx;
            if (ROWS) {
                const uint32_t rmask = (uint32_t)(hit >> (row * 16)) & 0xffffu;
                widx = __builtin_amdgcn_ds_bpermute((row * 16 + __builtin_ctz(rmask)) * 4, bi);
            } else {
                widx = __builtin_amdgcn_readlane(bi, (int)__builtin_ctzll(hit));
            }
            const int dsel = (wm < FLT_MAX) ? widx : -1;
            dacc = (ll == s) ? dsel : dacc;
        };
        auto process = [&](const Sg& g, int k) {
            const int aj0 = steps - (k + 1) * S;
            float LA[S][K];
            if (k > 0 && aj0 > 0) {   // neither path starts inside the segment
#pragma unroll
                for (int s = 0; s < S; s++) {
                    if (s == 0)
                        st.run(LA[0], g.ck, g.c[0], pen(g.fl, 0, dirA), false);
                    else
                        st.run(LA[s], LA[s - 1], g.c[s], pen(g.fl, s, dirA), false);
                }
#pragma unroll
                for (int s = S - 1; s >= 0; s--) {
                    float L[K];
                    st.run(L, Lp, g.c[s], pen(g.fl, s, dirB), false);
                    cpk(Lp, L);
                    emit(g, s, aj0 + s, LA[s], L);
                }
            } else {
                float prev[K];
                cpk(prev, g.ck);
#pragma unroll
                for (int s = 0; s < S; s++)
                    if (aj0 + s >= 0) {
                        st.run(LA[s], prev, g.c[s], pen(g.fl, s, dirA), aj0 + s == 0);
                        cpk(prev, LA[s]);
                    }
#pragma unroll
                for (int s = S - 1; s >= 0; s--)
                    if (aj0 + s >= 0) {
                        float L[K];
                        st.run(L, Lp, g.c[s], pen(g.fl, s, dirB), aj0 + s == steps - 1);
                        cpk(Lp, L);
                        emit(g, s, aj0 + s, LA[s], L);
                    }
            }
            if (LAST) {   // one store instruction per segment (and line) for the int16 disparities
                if (line_ok && ll < S && aj0 + ll >= 0) dbase[(long)(aj0 + ll) * pstep] = (int16_t)dacc;
            }
        };
        Sg ga, gb;
        load(ga, 0);
        for (int k = 0; k < nseg; k += 2) {
            load(gb, k + 1);
            process(ga, k);
            load(ga, k + 2);
            if (k + 1 < nseg) process(gb, k + 1);
        }
    }
}

template <int S, int MODE, int KV, bool ROWS, bool FULL>
static void launch_ck_one(const SgmArgs& a, hipStream_t st) {
    const int nl = (a.rv != 0 && a.ru != 0) ? a.W + a.H - 1 : (a.rv == 0 ? a.H : a.W);
    if (ROWS) {
        const int waves = (nl + 3) / 4 * a.n;
        hipLaunchKernelGGL((k_sgm_ck<S, MODE, KV, ROWS, FULL>), dim3((waves + 3) / 4), dim3(256), 0, st, a);
    } else {
        hipLaunchKernelGGL((k_sgm_ck<S, MODE, KV, ROWS, FULL>), dim3((nl + 3) / 4, a.n), dim3(256), 0, st, a);
    }
}
template <int S, int KV, bool ROWS, bool FULL, int SGN>
static void launch_ck_f(const SgmArgs& a, int mode, hipStream_t st) {
    switch (mode) {
        case CK_A: return launch_ck_one<S, SGN | CK_A, KV, ROWS, FULL>(a, st);
        case CK_B: return launch_ck_one<S, SGN | CK_B, KV, ROWS, FULL>(a, st);
        case CK_B | CK_MID: return launch_ck_one<S, SGN | CK_B | CK_MID, KV, ROWS, FULL>(a, st);
        case CK_B | CK_MID | CK_X:
            if constexpr (!ROWS) return launch_ck_one<S, SGN | CK_B | CK_MID | CK_X, KV, ROWS, FULL>(a, st);
            return;
        case CK_B | SGM_LAST: return launch_ck_one<S, SGN | CK_B | SGM_LAST, KV, ROWS, FULL>(a, st);
        default: return launch_ck_one<S, SGN | CK_B | SGM_LAST | SGM_KEEP, KV, ROWS, FULL>(a, st);
    }
}
template <int S, int KV, bool ROWS, bool FULL>
static void launch_ck_s(const SgmArgs& a, int mode, hipStream_t st) {
    if (a.signed_costs)
        launch_ck_f<S, KV, ROWS, FULL, SGM_SIGNED>(a, mode, st);
    else
        launch_ck_f<S, KV, ROWS, FULL, 0>(a, mode, st);
}
// mode: CK_A, CK_B (acc = L_first + L_second), CK_B | CK_MID (8 paths: acc = (acc + L2) + L3),
// CK_B | SGM_LAST (the map; SGM_KEEP added here when the final volume is kept)
void launch_sgm_ck(const SgmArgs& a, int mode, int n, hipStream_t st) {
    SgmArgs b = a;
    b.n = n;
    if ((mode & SGM_LAST) && a.keep_final) mode |= SGM_KEEP;
    if (a.rv != 0 && a.ru != 0) {   // the diagonal pair (sgm_ck_diag_ok: one line per wave)
        if (a.D == 256) return launch_ck_s<SM_SGM_CK_SD, 1, false, true>(b, mode, st);
        return launch_ck_s<SM_SGM_CK_SD, 1, false, false>(b, mode, st);
    }
    switch (ck_kv(a.D)) {
        case 0:
            if (a.D == 256) return launch_ck_s<SM_SGM_CK_S, 1, false, true>(b, mode, st);
            return launch_ck_s<SM_SGM_CK_S, 1, false, false>(b, mode, st);
        case 1:
            if (a.D == 64) return launch_ck_s<SM_SGM_CK_S, 1, true, true>(b, mode, st);
            return launch_ck_s<SM_SGM_CK_S, 1, true, false>(b, mode, st);
        default:
            if (a.D == 128) return launch_ck_s<SM_SGM_CK_S2, 2, true, true>(b, mode, st);
            return launch_ck_s<SM_SGM_CK_S2, 2, true, false>(b, mode, st);
    }
}

void launch_sgm_path(const SgmArgs& a, int mode, int n, hipStream_t st) {
    SgmArgs b = a;
    b.n = n;
    switch (rows_kv(a, mode)) {
        case 1: return launch_rows<1>(b, mode, n, st);
        case 2: return launch_rows<2>(b, mode, n, st);
        case 3: return launch_rows<3>(b, mode, n, st);
        case 4: return launch_rows<4>(b, mode, n, st);
        default: break;
    }
    if (a.D > SM_SGM_VEC_MIN_D && a.D <= 256 && a.D % 4 == 0) {  // one line per wave, dwordx4 per lane
        if (a.signed_costs) {
            if (a.D == 256)
                launch_kf_signed<4, true, true>(b, mode, n, st);
            else
                launch_kf_signed<4, false, true>(b, mode, n, st);
            return;
        }
        if (a.D == 256)
            launch_kf<4, true, true>(b, mode, n, st);
        else
            launch_kf<4, false, true>(b, mode, n, st);
        return;
    }
    switch (sgm_k_for(a.D)) {
        case 1: launch_k<1>(a, mode, n, st); break;
        case 2: launch_k<2>(a, mode, n, st); break;
        case 3: launch_k<3>(a, mode, n, st); break;
        case 4: launch_k<4>(a, mode, n, st); break;
        case 6: launch_k<6>(a, mode, n, st); break;
        case 8: launch_k<8>(a, mode, n, st); break;
        case 12: launch_k<12>(a, mode, n, st); break;
        default: launch_k<16>(a, mode, n, st); break;
    }
}

}  // namespace sm
