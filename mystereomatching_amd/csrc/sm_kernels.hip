// sm_kernels.hip — hand-written gfx950 kernels for the census / CBCA / SGM / WTA hot path.
//
// Layout in HBM (per pair b, all packed):
//   bgr   [b][view][H][W][3] u8  gray [b][view][H][W] u8   (view 0 = left, 1 = right)
//   code  [b][view][H][W] ulonglong2   (census words 0,1; genCensusCode_NC_Sur h:867-934)
//   (gradients, calGrad / calGrad_y cpp:271-386: recomputed from gray by the cost kernel)
//   arms  [b][view][plane][H][W] u32 (L | R<<16, U | D<<16; calHorVerDis cpp:2959-3050)
//   vm    [b][H][W][D] f32       (d innermost, as the reference's CV_32FC(D), cpp:2080)
//   acc   [b][H][W][D] f32       (SGM path sum in path order, gen_sgm_vm cpp:2031-2056)
//   disp  [b][H][W] i16          (DP[0], gen_dispFromVm cpp:3928-3967)
// Every float op below is written in the reference's evaluation order and the file is compiled
// with -ffp-contract=off, so results are bit-identical to the scalar CPU path.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sm_device.h"
#include "sm_kernels.h"

namespace sm {

__constant__ uint64_t c_exp_tab[32] = SM_EXPF_TABLE;

__device__ inline float dev_expf(float x) { return expf_glibc(x, c_exp_tab); }

// ---------------------------------------------------------------------------------------
// K0: per-pixel prep of both views: k_pack_bgr (packed BGR), k_pack_arms (arm-walk words and
// the SGM colour-difference penalty flags), then k_prep: census code, x/y gradients and cross
// arms from LDS tiles.  Block = 64 x 16 pixels, 256 threads (4 pixels each).  Gray tile with
// the census halo (REFLECT_101 applied while filling it, as copyMakeBorder does, h:870-871);
// arm-walk strips with an L_out halo along each axis.  Teddy x16, rocprof, same box: 0.261 ->
// 0.229 ms for the three kernels (census unrolled for the default window, LDS walks, tile
// fills with 8 loads in flight per thread).
// ---------------------------------------------------------------------------------------
constexpr int PREP_TX = 64, PREP_TY = 16;

__device__ __forceinline__ bool color_ok_packed(uint32_t x, uint32_t y, int t) {
    return abs((int)(x & 0xff) - (int)(y & 0xff)) <= t && abs((int)((x >> 8) & 0xff) - (int)((y >> 8) & 0xff)) <= t &&
           abs((int)(x >> 16) - (int)(y >> 16)) <= t;
}
__device__ __forceinline__ int color_d1(uint32_t x, uint32_t y) {
    return max(max(abs((int)(x & 0xff) - (int)(y & 0xff)), abs((int)((x >> 8) & 0xff) - (int)((y >> 8) & 0xff))),
               abs((int)(x >> 16) - (int)(y >> 16)));
}

// BGR bytes -> one packed u32 per pixel (B | G << 8 | R << 16) for every view of every pair.
__global__ void k_pack_bgr(const uint8_t* __restrict__ bgr, uint32_t* __restrict__ px, size_t total) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const uint8_t* p = bgr + i * 3;
        px[i] = p[0] | (p[1] << 8) | (p[2] << 16);
    }
}

// Same, four pixels per thread: three aligned dword loads (12 bytes) and one dwordx4 store.
__global__ void k_pack_bgr4(const uint32_t* __restrict__ bgr, uint4* __restrict__ px, size_t quads) {
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += (size_t)gridDim.x * blockDim.x) {
        const uint32_t w0 = bgr[3 * q], w1 = bgr[3 * q + 1], w2 = bgr[3 * q + 2];
        px[q] = make_uint4(w0 & 0xffffffu, (w0 >> 24) | ((w1 & 0xffffu) << 8), (w1 >> 16) | ((w2 & 0xffu) << 16), w2 >> 8);
    }
}

// Arm-walk words (calHorVerDis, cpp:2959-3050).  A walk step compares the step pixel with the
// centre under threshold t and with the previous step pixel under C_D.  k_pack_arms writes two
// planes whose words hold the pixel in 10-bit fields (B | G << 10 | R << 20) and the C_D test
// against the walk's previous pixel, precomputed once per pixel and axis:
//   pxh bit 30: (p, p + 1) within C_D (an L walk reaches p from p + 1), bit 31: (p, p - 1) (R walk)
//   pxv bit 30: (p, p + W) (U walk), bit 31: (p, p - W) (D walk); 0 where the partner is outside.
// The centre test is one guard-bit subtraction for all three channels: with M = 1 | 1 << 10 |
// 1 << 20, A = C + (512 + t) M - P and B = C + (511 - t) M - P keep every field in [1, 1022]
// for -1 <= t <= 255 (no borrow crosses a field; the flag bits only borrow upwards), and
// bit 9 of A's field c is set iff C_c - P_c >= -t, bit 9 of B's field clear iff C_c - P_c <= t.
// So a step passes iff ((A & ~B) & B9) | (P & flag) == B9 | flag — words outside the image are
// 0 and fail on the flag, which replaces the reference's border test.
constexpr uint32_t ARM_M = 1u | (1u << 10) | (1u << 20);
constexpr uint32_t ARM_B9 = ARM_M << 9;

__device__ __forceinline__ uint32_t pack10(uint32_t p) {   // B | G << 8 | R << 16 -> 10-bit fields
    return (p & 0xffu) | ((p & 0xff00u) << 2) | ((p & 0xff0000u) << 4);
}

// One thread per pixel (grid x: 256-pixel row segments, y: rows, z: images).  Also writes the
// SGM colour-difference penalty flags (updateCost, h:2223-2229): bit i set when the neighbour
// towards direction i (rv/ru tables of sgm, cpp:6207-6208) is inside and its max-channel
// difference exceeds sgm_corDifThres — of the left image, and of the right image when vm[1] is
// optimised too (leftFirst = false compares I_c[1], h:2224).
#ifndef SM_PACK_ROWS
#define SM_PACK_ROWS 4   // rows per thread (short one-row blocks were latency-bound: 33 us on Teddy x16)
#endif
__device__ __forceinline__ void pack_arms_pixel(const PrepArgs& a, int arms, int img, int v, int u);

__global__ __launch_bounds__(256) void k_pack_arms(const PrepArgs a, int arms) {
    const int u = blockIdx.x * 256 + threadIdx.x;
    if (u >= a.W) return;
#pragma unroll
    for (int r = 0; r < SM_PACK_ROWS; r++) {
        const int v = blockIdx.y * SM_PACK_ROWS + r;
        if (v < a.H) pack_arms_pixel(a, arms, blockIdx.z, v, u);
    }
}

__device__ __forceinline__ void pack_arms_pixel(const PrepArgs& a, int arms, int img, int v, int u) {
    const int H = a.H, W = a.W;
    const size_t npix = (size_t)H * W;
    const int b = img >> 1, view = img & 1;
    const size_t i = (size_t)img * npix + (size_t)v * W + u;
    const uint32_t* pc = a.px + i;
    const uint32_t c = pc[0];
    const bool inL = u > 0, inR = u + 1 < W, inU = v > 0, inD = v + 1 < H;
    const uint32_t pl = inL ? pc[-1] : c, pr = inR ? pc[1] : c, pu = inU ? pc[-W] : c, pd = inD ? pc[W] : c;
    if (arms) {
        const uint32_t f = pack10(c);
        uint32_t h = f, vv = f;
        if (inR && color_ok_packed(c, pr, a.C_D)) h |= 1u << 30;
        if (inL && color_ok_packed(c, pl, a.C_D)) h |= 1u << 31;
        if (inD && color_ok_packed(c, pd, a.C_D)) vv |= 1u << 30;
        if (inU && color_ok_packed(c, pu, a.C_D)) vv |= 1u << 31;
        a.pxh[i] = h;
        a.pxv[i] = vv;
    }
    if (a.do_flags && (view == 0 || a.flags1)) {
        const int t = a.cor_thres;
        uint32_t fl = 0;
        // directions 0..7: (rv, ru) = (+1,0) (-1,0) (0,+1) (0,-1) (+1,-1) (+1,+1) (-1,+1) (-1,-1)
        if (inD && color_d1(c, pd) > t) fl |= 1u;
        if (inU && color_d1(c, pu) > t) fl |= 2u;
        if (inR && color_d1(c, pr) > t) fl |= 4u;
        if (inL && color_d1(c, pl) > t) fl |= 8u;
        if (inD && inL && color_d1(c, pc[W - 1]) > t) fl |= 16u;
        if (inD && inR && color_d1(c, pc[W + 1]) > t) fl |= 32u;
        if (inU && inR && color_d1(c, pc[1 - W]) > t) fl |= 64u;
        if (inU && inL && color_d1(c, pc[-1 - W]) > t) fl |= 128u;
        (view == 0 ? a.flags : a.flags1)[(size_t)b * npix + (size_t)v * W + u] = (uint8_t)fl;
    }
}

// prep LDS: gray tile (census/gradient halo), then the arm strips (STRIPS): hs = the tile's 16
// rows over columns u0 - Lo .. u0 + 63 + Lo, vs = its 64 columns over rows v0 - Lo .. v0 + 15 + Lo
__host__ __device__ inline int prep_gray_bytes(int rv, int ru) {
    const int hv = rv > 1 ? rv : 1, hu = ru > 1 ? ru : 1;
    return ((PREP_TX + 2 * hu) * (PREP_TY + 2 * hv) + 15) / 16 * 16;
}
__host__ __device__ inline int prep_strip_words(int Lo) {
    return PREP_TY * (PREP_TX + 2 * Lo) + (PREP_TY + 2 * Lo) * PREP_TX;
}
// guard-bit test of two pack10 words (see ARM_M above): every channel within t, -1 <= t <= 255
__device__ __forceinline__ bool ok10(uint32_t c, uint32_t p, uint32_t ka, uint32_t kb) {
    return (((c + ka - p) & ~(c + kb - p)) & ARM_B9) == ARM_B9;
}
constexpr uint32_t PREP_OUT = 0xffffffffu;   // packed-pixel strips: a pixel outside the image

#ifndef SM_PREP_WALK
#define SM_PREP_WALK 1    // arm-walk steps whose LDS reads are issued together (tuning)
#endif
// census code (genCensusCode_NC_Sur, h:867-934) and x/y gradients of one pixel; g = the pixel in
// the block's gray tile (row stride gw, REFLECT_101 halo of max(rv, 1) rows / max(ru, 1) columns)
template <int TRV, int TRU, int TRING>
__device__ __forceinline__ void prep_census_grad(const PrepArgs& a, const uint8_t* g, int gw, int rv, int ru, int ring,
                                                 int u, int v, size_t o) {
    const int H = a.H, W = a.W;
    if (TRV >= 0 && a.do_census) {
        // compile-time geometry: every bit's position is a constant, so the bits go into four
        // 32-bit accumulators (acc = 2 acc + bit: a compare and an add-with-carry per bit)
        // instead of a 64-bit shift register; the words are then assembled exactly as the
        // reference's 64-bit chunks (MSB first, a partial last chunk in the low bits)
        const int c = g[0];
        uint32_t acc[4] = {0, 0, 0, 0};
        int k = 0;
#pragma unroll
        for (int dv = -rv; dv <= rv; dv++)
#pragma unroll
            for (int du = -ru; du <= ru; du++, k++)
                acc[k >> 5] = acc[k >> 5] + acc[k >> 5] + (uint32_t)(c < (int)g[dv * gw + du]);
        if (ring) {
            const int dvs[9] = {-1, -1, -1, 0, 1, 1, 1, 0, -1};
            const int dus[9] = {-1, 0, 1, 1, 1, 0, -1, -1, -1};
#pragma unroll
            for (int i = 0; i < 8; i++, k++)
                acc[k >> 5] = acc[k >> 5] + acc[k >> 5] +
                              (uint32_t)((int)g[dvs[i] * gw + dus[i]] < (int)g[dvs[i + 1] * gw + dus[i + 1]]);
        }
        const int nb0 = k < 64 ? k : 64, nb1 = k - nb0;   // bits of chunk 0 and chunk 1
        const uint64_t w0 = nb0 > 32 ? ((uint64_t)acc[0] << (nb0 - 32)) | acc[1] : acc[0];
        const uint64_t w1 = nb1 > 32 ? ((uint64_t)acc[2] << (nb1 - 32)) | acc[3] : acc[2];
        a.code[o] = make_ulonglong2(w0, w1);
    } else if (a.do_census) {
        const int c = g[0];
        uint64_t w[2] = {0, 0};
        uint64_t cs = 0;
        int step = 0, dep = 0;
#pragma unroll
        for (int dv = -rv; dv <= rv; dv++)
#pragma unroll
            for (int du = -ru; du <= ru; du++) {
                if (step > 63) {
                    w[dep & 1] = cs;
                    cs = 0;
                    step = 0;
                    dep++;
                }
                cs <<= 1;
                if (c - (int)g[dv * gw + du] < 0) cs++;
                step++;
            }
        if (ring) {
            const int dvs[9] = {-1, -1, -1, 0, 1, 1, 1, 0, -1};
            const int dus[9] = {-1, 0, 1, 1, 1, 0, -1, -1, -1};
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int pre = g[dvs[i] * gw + dus[i]], aft = g[dvs[i + 1] * gw + dus[i + 1]];
                if (step > 63) {
                    w[dep & 1] = cs;
                    cs = 0;
                    step = 0;
                    dep++;
                }
                cs <<= 1;
                if (pre - aft < 0) cs++;
                step++;
            }
        }
        if (step > 0) w[dep & 1] = cs;
        a.code[o] = make_ulonglong2(w[0], w[1]);
    }
}

// gradients of image pixel (v, u) (calGrad / calGrad_y single-channel, cpp:271-350): half the
// central difference inside, the one-sided difference on the border rows / columns (a 1-pixel
// wide image has 0, as the prep halo's reflection gave).  The cost kernel evaluates them from the
// gray plane when it stages a row, so no gradient plane goes through HBM.
__device__ __forceinline__ float2 grad_at(const uint8_t* G, int v, int u, int H, int W) {
    const uint8_t* row = G + (size_t)v * W;
    float gxv, gyv;
    if (W == 1)
        gxv = 0.f;
    else if (u == 0)
        gxv = (float)((int)row[1] - (int)row[0]);
    else if (u == W - 1)
        gxv = (float)((int)row[u] - (int)row[u - 1]);
    else
        gxv = 0.5f * (float)((int)row[u + 1] - (int)row[u - 1]);
    if (H == 1)
        gyv = 0.f;
    else if (v == 0)
        gyv = (float)((int)row[W + u] - (int)row[u]);
    else if (v == H - 1)
        gyv = (float)((int)row[u] - (int)row[u - W]);
    else
        gyv = 0.5f * (float)((int)row[W + u] - (int)row[u - W]);
    return make_float2(gxv, gyv);
}

// One arm walk over an LDS strip of arm-walk words (calHorVerDis, cpp:2959-3050): sp = the centre
// pixel's word, sst = the step between words, fb = the C_D flag bit of this direction, (ca, cb) the
// centre's guard-bit operands for steps <= Lin (C_D) and beyond (C_D_out).  Returns the first step
// that fails (1 .. Lo + 1).
__device__ __forceinline__ int strip_walk(const uint32_t* sp, int sst, uint32_t fb, uint32_t ca1, uint32_t cb1, uint32_t ca2,
                                          uint32_t cb2, int Lin, int Lo) {
    const uint32_t want = ARM_B9 | fb;
    auto pass = [&](uint32_t p, uint32_t ca, uint32_t cb) { return ((((ca - p) & ~(cb - p)) & ARM_B9) | (p & fb)) == want; };
    int arm = 1;
#if SM_PREP_WALK > 1
    // chunks of SM_PREP_WALK steps: a chunk's LDS reads are issued together, then its first
    // failing step (or Lo + 1) ends the walk
    for (;;) {
        uint32_t pw[SM_PREP_WALK];
#pragma unroll
        for (int j = 0; j < SM_PREP_WALK; j++) pw[j] = sp[min(arm + j, Lo) * sst];
        int ff = SM_PREP_WALK;
#pragma unroll
        for (int j = SM_PREP_WALK - 1; j >= 0; j--) {
            const int st = arm + j;
            const bool in1 = st <= Lin;
            if (st > Lo || !pass(pw[j], in1 ? ca1 : ca2, in1 ? cb1 : cb2)) ff = j;
        }
        arm += ff;
        if (ff < SM_PREP_WALK) break;
    }
#else
    for (; arm <= Lin; arm++)
        if (!pass(sp[arm * sst], ca1, cb1)) break;
    if (arm > Lin)
        for (; arm <= Lo; arm++)
            if (!pass(sp[arm * sst], ca2, cb2)) break;
#endif
    return arm;
}
// Two walks from one centre (the split prep's L / R and U / D pairs) advanced together in chunks
// of SM_PREP_WALK2 steps: both chunks' LDS reads are issued before either is tested, so a thread
// has 2 x SM_PREP_WALK2 reads in flight instead of one dependent read per step.  Same results as
// two strip_walk calls (a chunk's first failing step ends that walk; steps past Lo fail).
#ifndef SM_PREP_WALK2
#define SM_PREP_WALK2 4
#endif
__device__ __forceinline__ void strip_walk2(const uint32_t* sp, int sa, uint32_t fa, int sb, uint32_t fb, uint32_t ca1,
                                            uint32_t cb1, uint32_t ca2, uint32_t cb2, int Lin, int Lo, int& arm_a,
                                            int& arm_b) {
    constexpr int CW = SM_PREP_WALK2 > 0 ? SM_PREP_WALK2 : 1;
    auto first_fail = [&](const uint32_t (&pw)[CW], int arm, uint32_t f) {
        const uint32_t want = ARM_B9 | f;
        int ff = CW;
#pragma unroll
        for (int j = CW - 1; j >= 0; j--) {
            const int st = arm + j;
            const bool in1 = st <= Lin;
            const uint32_t ca = in1 ? ca1 : ca2, cb = in1 ? cb1 : cb2;
            const bool ok = ((((ca - pw[j]) & ~(cb - pw[j])) & ARM_B9) | (pw[j] & f)) == want;
            if (st > Lo || !ok) ff = j;
        }
        return ff;
    };
    int a = 1, b = 1;
    bool da = false, db = false;
    while (!(da && db)) {
        uint32_t pa[CW], pb[CW];
#pragma unroll
        for (int j = 0; j < CW; j++) {
            pa[j] = sp[min(a + j, Lo) * sa];
            pb[j] = sp[min(b + j, Lo) * sb];
        }
        if (!da) {
            const int ff = first_fail(pa, a, fa);
            a += ff;
            da = ff < CW;
        }
        if (!db) {
            const int ff = first_fail(pb, b, fb);
            b += ff;
            db = ff < CW;
        }
    }
    arm_a = a;
    arm_b = b;
}
// The arm length kept from a walk that failed at step `arm` (cpp:3035-3046): the walked length
// when it reaches minL, else the longest length <= minL that stays inside the image.
__device__ __forceinline__ int arm_final(int arm, int minL, int u, int v, int du, int dv, int W, int H) {
    if (--arm >= minL) return arm;
    for (int len = minL; len >= 0; len--)
        if (u + len * du >= 0 && u + len * du <= W - 1 && v + len * dv >= 0 && v + len * dv <= H - 1) return len;
    return 0;
}
// TRV/TRU/TRING >= 0: census geometry fixed at compile time (the default 7 x 9 window with the
// ring bits), so the bit loop unrolls into straight-line compares with immediate LDS offsets;
// -1: the runtime geometry.  STRIPS: arm walks over the LDS strips (else over global memory).
// (Making the arm-walk words and flags inside this kernel, so the pxh / pxv planes never reach
// memory, was bit-exact and slower: tools/experiments/prep_fused_words.patch.)
template <int TRV, int TRU, int TRING, bool STRIPS>
__global__ __launch_bounds__(256) void k_prep(const PrepArgs a) {
    extern __shared__ __align__(16) unsigned char prep_raw[];
    const int H = a.H, W = a.W, Lo = a.L_out;
    const int rv = TRV >= 0 ? TRV : a.rv, ru = TRU >= 0 ? TRU : a.ru;
    const int ring = TRING >= 0 ? TRING : a.ring;
    const int u0 = blockIdx.x * PREP_TX, v0 = blockIdx.y * PREP_TY;
    const int b = blockIdx.z >> 1, view = blockIdx.z & 1;
    const size_t npix = (size_t)H * W;
    const size_t img = (size_t)b * 2 + view;
    const uint8_t* G = a.gray + img * npix;
    const uint32_t* P = a.px + img * npix;
    // gray tile: rows v0-hv .. v0+TY+hv, cols u0-hu .. u0+TX+hu, REFLECT_101 applied on fill
    const int hv = max(rv, 1), hu = max(ru, 1);
    const int gw = PREP_TX + 2 * hu, gh = PREP_TY + 2 * hv;
    uint8_t* gt = prep_raw;
    const int tid = threadIdx.x;
    // Tile fills: the loads of FB entries per thread are issued before any of them is stored, so a
    // block waits on global-memory latency a few times instead of once per entry.
    constexpr int FB = 8;
    auto fill = [&](auto* dst, int count, auto&& load) {
        for (int i0 = 0; i0 < count; i0 += FB * 256) {
            uint32_t r[FB];
#pragma unroll
            for (int k = 0; k < FB; k++) {
                const int i = i0 + k * 256 + tid;
                r[k] = i < count ? load(i) : 0u;
            }
#pragma unroll
            for (int k = 0; k < FB; k++) {
                const int i = i0 + k * 256 + tid;
                if (i < count) dst[i] = (std::remove_reference_t<decltype(dst[0])>)r[k];
            }
        }
    };
    if (a.do_census)
        fill(gt, gw * gh, [&](int i) -> uint32_t {
            const int ty = i / gw, tx = i - ty * gw;
            const int vv = reflect101(v0 - hv + ty, H), uu = reflect101(u0 - hu + tx, W);
            return G[(size_t)vv * W + uu];
        });
    const int hsw = PREP_TX + 2 * Lo;
    uint32_t* hs = (uint32_t*)(prep_raw + prep_gray_bytes(rv, ru));
    uint32_t* vs = hs + PREP_TY * hsw;
    if (STRIPS && a.do_arms) {
        const uint32_t* PH = a.pxh + img * npix;
        const uint32_t* PV = a.pxv + img * npix;
        // hs rows are hsw = 64 + 2 Lo words long (runtime): row index by a float reciprocal
        // instead of an integer division (exact for i < 2^22: the +0.5 keeps the product's
        // rounding from crossing an integer)
        const float rinv = 1.0f / (float)hsw;
        fill(hs, PREP_TY * hsw, [&](int i) -> uint32_t {
            const int r = (int)(((float)i + 0.5f) * rinv), vv = v0 + r, uu = u0 - Lo + (i - r * hsw);
            return (vv < H && (unsigned)uu < (unsigned)W) ? PH[(size_t)vv * W + uu] : 0u;
        });
        fill(vs, (PREP_TY + 2 * Lo) * PREP_TX, [&](int i) -> uint32_t {
            const int vv = v0 - Lo + (i >> 6), uu = u0 + (i & 63);
            return ((unsigned)vv < (unsigned)H && uu < W) ? PV[(size_t)vv * W + uu] : 0u;
        });
    }
    __syncthreads();
    const int x = tid & 63;
    for (int yy = tid >> 6; yy < PREP_TY; yy += 4) {
        const int u = u0 + x, v = v0 + yy;
        if (u >= W || v >= H) continue;
        const size_t o = img * npix + (size_t)v * W + u;
        prep_census_grad<TRV, TRU, TRING>(a, gt + (yy + hv) * gw + (x + hu), gw, rv, ru, ring, u, v, o);
        const uint32_t* pc = P + (size_t)v * W + u;
        // cross arms (calHorVerDis 7-arg, cpp:2959-3050), direction order L, R, U, D; the walks
        // read the packed image (lanes = consecutive pixels, so every step is one coalesced load)
        if (a.do_arms) {
            uint32_t packed = 0;
            // strip walks: centre words and the two thresholds' guard-bit operands
            const uint32_t* hc = hs + yy * hsw + (x + Lo);
            const uint32_t* vc = vs + (yy + Lo) * PREP_TX + x;
            const uint32_t center = pc[0];
            const uint32_t cf = pack10(center);
            const int t1 = min(max(a.C_D, -1), 255), t2 = min(max(a.C_D_out, -1), 255);
            const uint32_t ca1 = cf + (uint32_t)(512 + t1) * ARM_M, cb1 = cf + (uint32_t)(511 - t1) * ARM_M;
            const uint32_t ca2 = cf + (uint32_t)(512 + t2) * ARM_M, cb2 = cf + (uint32_t)(511 - t2) * ARM_M;
            const int Lin = min(a.L, Lo);
#pragma unroll
            for (int direc = 0; direc < 4; direc++) {
                const int du = direc == 0 ? -1 : (direc == 1 ? 1 : 0);
                const int dv = direc == 2 ? -1 : (direc == 3 ? 1 : 0);
                int arm = 1;
                if (STRIPS) {
                    const uint32_t fb = (direc == 0 || direc == 2) ? (1u << 30) : (1u << 31);
                    arm = strip_walk(direc < 2 ? hc : vc, direc == 0 ? -1 : (direc == 1 ? 1 : (direc == 2 ? -PREP_TX : PREP_TX)),
                                     fb, ca1, cb1, ca2, cb2, Lin, Lo);
                } else {
                    const int off = dv * W + du;
                    uint32_t prev = center;
                    for (; arm <= Lo; arm++) {
                        const int va = v + arm * dv, ua = u + arm * du;
                        if (va < 0 || va >= H || ua < 0 || ua >= W) break;
                        const uint32_t cur = pc[arm * off];
                        const bool nb = color_ok_packed(cur, prev, a.C_D);
                        const bool ip = color_ok_packed(center, cur, arm <= a.L ? a.C_D : a.C_D_out);
                        if (!nb || !ip) break;
                        prev = cur;
                    }
                }
                packed |= (uint32_t)arm_final(arm, a.minL, u, v, du, dv, W, H) << (8 * direc);
            }
            // two u16-pair planes: (L | R << 16) and (U | D << 16)
            uint32_t* planes = (uint32_t*)a.arms + img * 2 * npix + (size_t)v * W + u;
            planes[0] = (packed & 0xffu) | ((packed >> 8 & 0xffu) << 16);
            planes[npix] = (packed >> 16 & 0xffu) | ((packed >> 24) << 16);
        }
    }
}


// ---------------------------------------------------------------------------------------
// Split prep (SM_PREP_SPLIT): two kernels that make the arm-walk words in LDS from the colour
// bytes, so no packed plane (px / pxh / pxv) goes through HBM, and whose tiles are long along
// their walk axis, so the walk halo is re-read 1.3-2.1 times instead of the 16-row tile's 5.3:
//   k_prep_h  tiles of 256 columns x 8 rows: census, the SGM penalty flags and the
//             L / R arms (arm plane 0), from a gray tile and a strip of packed pixels (rows
//             v0 - 1 .. v0 + 4, columns u0 - Lo - 1 .. u0 + 256 + Lo);
//   k_prep_v  tiles of 64 columns x 128 rows: the U / D arms (arm plane 1) from a strip of rows
//             v0 - Lo - 1 .. v0 + 128 + Lo.
// The packed-BGR plane is made (k_pack_bgr) only for the kernels that read it (GF, so, refine).
// ---------------------------------------------------------------------------------------
#ifndef SM_PREP_SPLIT
#define SM_PREP_SPLIT 1
#endif
#ifndef SM_PREP_HTH
#define SM_PREP_HTH 8    // k_prep_h tile rows (4 -> 8: gray / colour halo re-reads 2.5 / 1.5 -> 1.75 / 1.25)
#endif
#ifndef SM_PREP_VTH
#define SM_PREP_VTH 128  // k_prep_v tile rows (64 -> 128: colour strip re-read 2.1 -> 1.55; prep
                         // 0.772 -> 0.736 ms at full resolution, profiles/r6/prep)
#endif
constexpr int PH_TW = 256, PH_TH = SM_PREP_HTH, PV_TW = 64, PV_TH = SM_PREP_VTH;
#ifndef SM_PREP_QUAD
#define SM_PREP_QUAD 1   // strips filled four pixels per load_quad_bgr (else three byte loads per pixel)
#endif
__host__ __device__ inline int preph_gray_bytes(int rv, int ru) {
    const int hv = rv > 1 ? rv : 1, hu = ru > 1 ? ru : 1;
    return ((PH_TW + 2 * hu) * (PH_TH + 2 * hv) + 15) / 16 * 16;
}
__host__ __device__ inline int preph_hc(int Lo) { return PH_TW + 2 * Lo + 2; }
__host__ __device__ inline int preph_bytes(int rv, int ru, int Lo) { return preph_gray_bytes(rv, ru) + 4 * (PH_TH + 2) * preph_hc(Lo); }
__host__ __device__ inline int prepv_bytes(int Lo) { return 4 * (PV_TH + 2 * Lo + 2) * PV_TW; }

// packed pixel (pack10) of image pixel (vv, uu) from the colour bytes, PREP_OUT outside the image
__device__ __forceinline__ uint32_t pack10_at(const uint8_t* bgr, int vv, int uu, int H, int W) {
    if ((unsigned)vv >= (unsigned)H || (unsigned)uu >= (unsigned)W) return PREP_OUT;
    const uint8_t* q = bgr + ((size_t)vv * W + uu) * 3;
    return (uint32_t)q[0] | ((uint32_t)q[1] << 10) | ((uint32_t)q[2] << 20);
}
// Four consecutive pixels' colours (B | G << 8 | R << 16 each) from the 12 bytes at q, any
// alignment: four dword loads from the dword below q and three byte-aligning funnel shifts (the
// colour allocation carries a 16-byte tail pad for the fourth dword)
__device__ __forceinline__ uint4 load_quad_bgr(const uint8_t* q) {
    const uintptr_t ad = (uintptr_t)q;
    const uint32_t* d = (const uint32_t*)(ad & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(ad & 3u);
    const uint32_t w0 = d[0], w1 = d[1], w2 = d[2], w3 = d[3];
    const uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, sh), x1 = __builtin_amdgcn_alignbyte(w2, w1, sh),
                   x2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
    return make_uint4(x0 & 0xffffffu, (x0 >> 24) | ((x1 & 0xffffu) << 8), (x1 >> 16) | ((x2 & 0xffu) << 16), x2 >> 8);
}
// Fill `rows` rows of a packed-pixel strip (pack10 words, PREP_OUT outside the image) covering
// columns c0 .. c0 + width - 1 of image rows r0 .. r0 + rows - 1, row stride `stride` words:
// quads of four columns from one load_quad_bgr each, four quads per thread in flight.
__device__ __forceinline__ void fill_strip_quads(uint32_t* dst, int stride, const uint8_t* C, int r0, int rows, int c0,
                                                 int width, int H, int W) {
    const int qpr = (width + 3) >> 2;   // quads per row (the last may be partial)
    const int nq = rows * qpr;
    for (int i0 = 0; i0 < nq; i0 += 4 * 256) {
        uint4 px[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int i = i0 + k * 256 + (int)threadIdx.x;
            const int r = i / qpr, x = 4 * (i - r * qpr), vv = r0 + r, uu = c0 + x;
            // whole quad inside the image: one funnel-shifted load; else per-pixel bytes
            const bool row_in = i < nq && (unsigned)vv < (unsigned)H;
            if (row_in && uu >= 0 && uu + 3 < W) {
                px[k] = load_quad_bgr(C + ((size_t)vv * W + uu) * 3);
            } else {
                uint32_t t[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int u = uu + j;
                    const uint8_t* b = C + ((size_t)vv * W + u) * 3;
                    t[j] = (row_in && (unsigned)u < (unsigned)W) ? ((uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16))
                                                               : 0xffffffffu;
                }
                px[k] = make_uint4(t[0], t[1], t[2], t[3]);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int i = i0 + k * 256 + (int)threadIdx.x;
            if (i >= nq) continue;
            const int r = i / qpr, x = 4 * (i - r * qpr);
            const uint32_t v[4] = {px[k].x, px[k].y, px[k].z, px[k].w};
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (x + j < width) dst[r * stride + x + j] = v[j] == 0xffffffffu ? PREP_OUT : pack10(v[j]);
        }
    }
}
// arm-walk word of packed pixel p (k_pack_arms): bit 30 / 31 = its C_D test against the walk's
// previous pixel nb30 / nb31 (the neighbour towards the walk's start); 0 outside the image
__device__ __forceinline__ uint32_t walk_word(uint32_t p, uint32_t nb30, uint32_t nb31, uint32_t ka, uint32_t kb) {
    if (p == PREP_OUT) return 0u;
    uint32_t w = p;
    if (nb30 != PREP_OUT && ok10(p, nb30, ka, kb)) w |= 1u << 30;
    if (nb31 != PREP_OUT && ok10(p, nb31, ka, kb)) w |= 1u << 31;
    return w;
}
// tile fill with the loads of FB entries per thread issued before any of them is stored
template <typename T, typename F>
__device__ __forceinline__ void prep_fill(T* dst, int count, F&& load) {
    constexpr int FB = 8;
    for (int i0 = 0; i0 < count; i0 += FB * 256) {
        uint32_t r[FB];
#pragma unroll
        for (int k = 0; k < FB; k++) {
            const int i = i0 + k * 256 + (int)threadIdx.x;
            r[k] = i < count ? load(i) : 0u;
        }
#pragma unroll
        for (int k = 0; k < FB; k++) {
            const int i = i0 + k * 256 + (int)threadIdx.x;
            if (i < count) dst[i] = (T)r[k];
        }
    }
}

template <int TRV, int TRU, int TRING>
__global__ __launch_bounds__(256) void k_prep_h(const PrepArgs a) {
    extern __shared__ __align__(16) unsigned char prep_raw[];
    const int H = a.H, W = a.W, Lo = a.do_arms ? a.L_out : 0;
    const int rv = TRV >= 0 ? TRV : a.rv, ru = TRU >= 0 ? TRU : a.ru;
    const int ring = TRING >= 0 ? TRING : a.ring;
    const int u0 = blockIdx.x * PH_TW, v0 = blockIdx.y * PH_TH;
    const int b = blockIdx.z >> 1, view = blockIdx.z & 1;
    const size_t npix = (size_t)H * W;
    const size_t img = (size_t)b * 2 + view;
    const int tid = threadIdx.x;
    const int hv = max(rv, 1), hu = max(ru, 1);
    const int gw = PH_TW + 2 * hu, gh = PH_TH + 2 * hv;
    uint8_t* gt = prep_raw;
    const bool words = a.do_arms;
    const bool flags = a.do_flags && (view == 0 || a.flags1);
    if (a.do_census) {
        const uint8_t* G = a.gray + img * npix;
        prep_fill(gt, gw * gh, [&](int i) -> uint32_t {
            const int ty = i / gw, tx = i - ty * gw;
            return G[(size_t)reflect101(v0 - hv + ty, H) * W + reflect101(u0 - hu + tx, W)];
        });
    }
    const int hc = preph_hc(Lo);
    uint32_t* PH = (uint32_t*)(prep_raw + preph_gray_bytes(rv, ru));   // [PH_TH + 2][hc]
    if (words || flags) {
        const uint8_t* C = a.bgr + img * npix * 3;
        if (SM_PREP_QUAD) {
            fill_strip_quads(PH, hc, C, v0 - 1, PH_TH + 2, u0 - Lo - 1, hc, H, W);
        } else {
            const float rinv = 1.0f / (float)hc;   // row by a float reciprocal (exact for i < 2^22)
            prep_fill(PH, (PH_TH + 2) * hc, [&](int i) -> uint32_t {
                const int r = (int)(((float)i + 0.5f) * rinv);
                return pack10_at(C, v0 - 1 + r, u0 - Lo - 1 + (i - r * hc), H, W);
            });
        }
    }
    __syncthreads();
    if (flags) {   // SGM penalty flags (updateCost, h:2223-2229) from the packed pixels and their rim
        const int tf = min(max(a.cor_thres, -1), 255);
        const uint32_t fa = (uint32_t)(512 + tf) * ARM_M, fb = (uint32_t)(511 - tf) * ARM_M;
        const int u = u0 + tid;
        // directions 0..7: (rv, ru) = (+1,0) (-1,0) (0,+1) (0,-1) (+1,-1) (+1,+1) (-1,+1) (-1,-1)
        const int offs[8] = {hc, -hc, 1, -1, hc - 1, hc + 1, 1 - hc, -1 - hc};
#pragma unroll
        for (int yy = 0; yy < PH_TH; yy++) {
            const int v = v0 + yy;
            if (u >= W || v >= H) continue;
            const uint32_t* q = PH + (yy + 1) * hc + tid + Lo + 1;
            const uint32_t c = q[0];
            uint32_t fl = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t nb = q[offs[k]];
                if (nb != PREP_OUT && !ok10(c, nb, fa, fb)) fl |= 1u << k;
            }
            (view == 0 ? a.flags : a.flags1)[(size_t)b * npix + (size_t)v * W + u] = (uint8_t)fl;
        }
    }
    if (words) {
        // the walk rows' words, computed into registers and written over the packed pixels after
        // every thread has read its neighbours
        const int tc = min(max(a.C_D, -1), 255);
        const uint32_t ka = (uint32_t)(512 + tc) * ARM_M, kb = (uint32_t)(511 - tc) * ARM_M;
        constexpr int MH = (PH_TH * (PH_TW + 128) + 255) / 256;   // Lo <= 64
        const int nw = hc - 2, nh = PH_TH * nw;
        const float winv = 1.0f / (float)nw;
        uint32_t wh[MH];
#pragma unroll
        for (int m = 0; m < MH; m++) {
            const int i = m * 256 + tid;
            if (i < nh) {
                const int r = (int)(((float)i + 0.5f) * winv);
                const uint32_t* q = PH + (r + 1) * hc + (i - r * nw) + 1;
                wh[m] = walk_word(q[0], q[1], q[-1], ka, kb);
            }
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < MH; m++) {
            const int i = m * 256 + tid;
            if (i < nh) {
                const int r = (int)(((float)i + 0.5f) * winv);
                PH[(r + 1) * hc + (i - r * nw) + 1] = wh[m];
            }
        }
        __syncthreads();
    }
    const int u = u0 + tid;
    if (u >= W) return;
    const int t1 = min(max(a.C_D, -1), 255), t2 = min(max(a.C_D_out, -1), 255);
    const int Lin = min(a.L, Lo);
#pragma unroll 1
    for (int yy = 0; yy < PH_TH; yy++) {
        const int v = v0 + yy;
        if (v >= H) break;
        const size_t o = img * npix + (size_t)v * W + u;
        prep_census_grad<TRV, TRU, TRING>(a, gt + (yy + hv) * gw + (tid + hu), gw, rv, ru, ring, u, v, o);
        if (words) {   // L and R arms (calHorVerDis 7-arg, cpp:2959-3050): arm plane 0 = L | R << 16
            const uint32_t* q = PH + (yy + 1) * hc + tid + Lo + 1;
            const uint32_t cf = q[0] & 0x3fffffffu;
            const uint32_t ca1 = cf + (uint32_t)(512 + t1) * ARM_M, cb1 = cf + (uint32_t)(511 - t1) * ARM_M;
            const uint32_t ca2 = cf + (uint32_t)(512 + t2) * ARM_M, cb2 = cf + (uint32_t)(511 - t2) * ARM_M;
            int wl, wr;
            if (SM_PREP_WALK2 > 0) {
                strip_walk2(q, -1, 1u << 30, 1, 1u << 31, ca1, cb1, ca2, cb2, Lin, Lo, wl, wr);
            } else {
                wl = strip_walk(q, -1, 1u << 30, ca1, cb1, ca2, cb2, Lin, Lo);
                wr = strip_walk(q, 1, 1u << 31, ca1, cb1, ca2, cb2, Lin, Lo);
            }
            const int al = arm_final(wl, a.minL, u, v, -1, 0, W, H);
            const int ar = arm_final(wr, a.minL, u, v, 1, 0, W, H);
            ((uint32_t*)a.arms)[img * 2 * npix + (size_t)v * W + u] = (uint32_t)al | ((uint32_t)ar << 16);
        }
    }
}

__global__ __launch_bounds__(256) void k_prep_v(const PrepArgs a) {
    extern __shared__ __align__(16) unsigned char prep_raw[];
    const int H = a.H, W = a.W, Lo = a.L_out;
    const int u0 = blockIdx.x * PV_TW, v0 = blockIdx.y * PV_TH;
    const int b = blockIdx.z >> 1, view = blockIdx.z & 1;
    const size_t npix = (size_t)H * W;
    const size_t img = (size_t)b * 2 + view;
    const int tid = threadIdx.x;
    uint32_t* PV = (uint32_t*)prep_raw;   // [PV_TH + 2 Lo + 2][PV_TW]: rows v0 - Lo - 1 ..
    const uint8_t* C = a.bgr + img * npix * 3;
    if (SM_PREP_QUAD) {
        fill_strip_quads(PV, PV_TW, C, v0 - Lo - 1, PV_TH + 2 * Lo + 2, u0, PV_TW, H, W);
    } else {
        prep_fill(PV, (PV_TH + 2 * Lo + 2) * PV_TW,
                  [&](int i) -> uint32_t { return pack10_at(C, v0 - Lo - 1 + (i >> 6), u0 + (i & 63), H, W); });
    }
    __syncthreads();
    {
        const int tc = min(max(a.C_D, -1), 255);
        const uint32_t ka = (uint32_t)(512 + tc) * ARM_M, kb = (uint32_t)(511 - tc) * ARM_M;
        constexpr int MV = ((PV_TH + 128) * PV_TW + 255) / 256;   // Lo <= 64
        const int nv = (PV_TH + 2 * Lo) * PV_TW;
        uint32_t wv[MV];
#pragma unroll
        for (int m = 0; m < MV; m++) {
            const int i = m * 256 + tid;
            if (i < nv) {
                const uint32_t* q = PV + PV_TW + i;
                wv[m] = walk_word(q[0], q[PV_TW], q[-PV_TW], ka, kb);
            }
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < MV; m++) {
            const int i = m * 256 + tid;
            if (i < nv) PV[PV_TW + i] = wv[m];
        }
        __syncthreads();
    }
    const int x = tid & 63, u = u0 + x;
    if (u >= W) return;
    const int t1 = min(max(a.C_D, -1), 255), t2 = min(max(a.C_D_out, -1), 255);
    const int Lin = min(a.L, Lo);
    uint32_t* plane1 = (uint32_t*)a.arms + img * 2 * npix + npix;
#pragma unroll 1
    for (int yy = tid >> 6; yy < PV_TH; yy += 4) {
        const int v = v0 + yy;
        if (v >= H) break;
        // U and D arms: arm plane 1 = U | D << 16
        const uint32_t* q = PV + (yy + Lo + 1) * PV_TW + x;
        const uint32_t cf = q[0] & 0x3fffffffu;
        const uint32_t ca1 = cf + (uint32_t)(512 + t1) * ARM_M, cb1 = cf + (uint32_t)(511 - t1) * ARM_M;
        const uint32_t ca2 = cf + (uint32_t)(512 + t2) * ARM_M, cb2 = cf + (uint32_t)(511 - t2) * ARM_M;
        int wu, wd;
        if (SM_PREP_WALK2 > 0) {
            strip_walk2(q, -PV_TW, 1u << 30, PV_TW, 1u << 31, ca1, cb1, ca2, cb2, Lin, Lo, wu, wd);
        } else {
            wu = strip_walk(q, -PV_TW, 1u << 30, ca1, cb1, ca2, cb2, Lin, Lo);
            wd = strip_walk(q, PV_TW, 1u << 31, ca1, cb1, ca2, cb2, Lin, Lo);
        }
        const int au = arm_final(wu, a.minL, u, v, 0, -1, W, H);
        const int ad = arm_final(wd, a.minL, u, v, 0, 1, W, H);
        plane1[(size_t)v * W + u] = (uint32_t)au | ((uint32_t)ad << 16);
    }
}

// strip walks when the strips fit comfortably: L_out <= 64 is <= 49 KB of LDS per block (the
// default 34 takes 30 KB: five blocks per CU); longer arms walk global memory
static bool prep_strips(int L_out) { return L_out >= 0 && L_out <= 64; }

size_t prep_smem_bytes(int rv, int ru, int L_out) {
    return (size_t)prep_gray_bytes(rv, ru) +
           (prep_strips(L_out) ? 4 * (size_t)prep_strip_words(L_out) : 0);
}

template <int TRV, int TRU, int TRING>
static void launch_prep_g(const PrepArgs& a, dim3 grid, size_t shm, bool strips, hipStream_t st) {
    if (strips)
        hipLaunchKernelGGL((k_prep<TRV, TRU, TRING, true>), grid, dim3(256), shm, st, a);
    else
        hipLaunchKernelGGL((k_prep<TRV, TRU, TRING, false>), grid, dim3(256), shm, st, a);
}

static void launch_prep_split(const PrepArgs& a, int n, hipStream_t st) {
    const int Lo = a.do_arms ? a.L_out : 0;
    const dim3 gh((a.W + PH_TW - 1) / PH_TW, (a.H + PH_TH - 1) / PH_TH, 2 * n);
    const size_t shh = (size_t)preph_bytes(a.rv, a.ru, Lo);
    if (a.rv == 3 && a.ru == 4 && a.ring == 1)   // the reference's default census window (cpp:815)
        hipLaunchKernelGGL((k_prep_h<3, 4, 1>), gh, dim3(256), shh, st, a);
    else
        hipLaunchKernelGGL((k_prep_h<-1, -1, -1>), gh, dim3(256), shh, st, a);
    if (a.do_arms) {
        const dim3 gv((a.W + PV_TW - 1) / PV_TW, (a.H + PV_TH - 1) / PV_TH, 2 * n);
        hipLaunchKernelGGL(k_prep_v, gv, dim3(256), (size_t)prepv_bytes(a.L_out), st, a);
    }
}

void launch_prep(const PrepArgs& a, int n, hipStream_t st) {
    const bool strips = a.do_arms && prep_strips(a.L_out);
    const bool split = SM_PREP_SPLIT && (strips || !a.do_arms);
    if (split && !a.pack_px) {
        launch_prep_split(a, n, st);
        return;
    }
    const size_t total = (size_t)n * 2 * a.H * a.W;
    size_t blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (((uintptr_t)a.bgr & 3) == 0 && ((uintptr_t)a.px & 15) == 0) {
        const size_t quads = total / 4;
        size_t qb = (quads + 255) / 256;
        if (qb > 4096) qb = 4096;
        if (quads) hipLaunchKernelGGL(k_pack_bgr4, dim3((unsigned)qb), dim3(256), 0, st, (const uint32_t*)a.bgr, (uint4*)a.px, quads);
        if (total % 4)   // the last one to three pixels
            hipLaunchKernelGGL(k_pack_bgr, dim3(1), dim3(64), 0, st, a.bgr + quads * 12, a.px + quads * 4, total % 4);
    } else {
        hipLaunchKernelGGL(k_pack_bgr, dim3((unsigned)blocks), dim3(256), 0, st, a.bgr, a.px, total);
    }
    if (split) {
        launch_prep_split(a, n, st);
        return;
    }
    if (strips || a.do_flags)   // arm-walk planes and the SGM penalty flags
        hipLaunchKernelGGL(k_pack_arms, dim3((a.W + 255) / 256, (a.H + SM_PACK_ROWS - 1) / SM_PACK_ROWS, 2 * n), dim3(256), 0,
                           st, a, (int)strips);
    dim3 grid((a.W + PREP_TX - 1) / PREP_TX, (a.H + PREP_TY - 1) / PREP_TY, 2 * n);
    const size_t shm = (size_t)prep_gray_bytes(a.rv, a.ru) +
                       (strips ? 4 * (size_t)prep_strip_words(a.L_out) : 0);
    if (a.rv == 3 && a.ru == 4 && a.ring == 1)   // the reference's default census window (cpp:815)
        launch_prep_g<3, 4, 1>(a, grid, shm, strips, st);
    else
        launch_prep_g<-1, -1, -1>(a, grid, shm, strips, st);
}

// ---------------------------------------------------------------------------------------
// K1: cost volume of one view.  Block = one row segment of P pixels x all D disparities.
// The "fixed" pixel is (v,u) of image `view`; its candidate ("moving") pixel is (v, u - d) in
// the right image for view 0 and (v, u + d) in the left image for view 1.  Per-pixel inputs of
// the P fixed and P + D - 1 moving pixels are staged in LDS once, then each wave writes D
// contiguous floats of one pixel (coalesced).
//   census  gen_cenVM_XOR (h:936-981); grad calgradvm (cpp:388-455);
//   AD      gen_ad_sd_vm (cpp:2468-2509);   fusion gen_vm_from2vm_exp (cpp:3566-3590).
// exp(-C/lam) (C integer 0..128) and exp(-AD/lam) (AD = s/3, s integer 0..765) come from LUTs
// built on the host with libm expf (staged in LDS); the gradient term is sm::expf_glibc_core,
// whose result is discarded when -G/lamG < -17.5: then expf(-G/lamG) <= 2^-25 and
// fl(t - e) == t for every t = fl(2 - e0) in [1, 2), so the reference's value is t itself.
// The element loop is branch-free: out-of-range candidates (u - d < 0 or u + d >= W) read a
// zero-filled staged record and select the reference's out-of-range cost afterwards; without
// the adaptive weights the weights are 1, and 1 * x + 1 * y == x + y exactly.  lamG == 1 (the
// default) skips the division, since -G / 1 == -G.
// ---------------------------------------------------------------------------------------
#ifndef SM_COST_STORE_AUX
#define SM_COST_STORE_AUX 2   // buffer store cache policy: slc = non-temporal (see SM_ST_AUX, sm_device.h)
#endif
#ifndef SM_COST_SPLIT
#define SM_COST_SPLIT 1
#endif
#ifndef SM_COST_ONE_PAIR
#define SM_COST_ONE_PAIR 1   // D <= 64: two focus pixels per trip (profiles/r5t/ab_one.log)
#endif
#ifndef SM_COST_ONE_FAST
#define SM_COST_ONE_FAST 1   // D <= 64: FAST elements too, with two pixels per trip (Teddy x16 0.169 -> 0.166 ms)
#endif
#ifndef SM_COST_UNROLL
#define SM_COST_UNROLL 1
#endif
#ifndef SM_COST_ND
#define SM_COST_ND 1   // D = 128 / 192 / 256: element loop unrolled at compile time (k_cost<..., ND>)
#endif
// Pixels of a row segment per block (at most; launch_cost splits a row into equal segments of
// at most this many): D <= 64 amortises the P + D - 1 moving-pixel staging over up to 240 pixels
// (Teddy x16, same-process A/B: 128 -> 0.195-0.203 ms, 160 -> 0.186, 192 -> 0.187-0.191, 225 (two
// equal segments of the 450-pixel row) -> 0.170-0.179, 240 -> 0.182-0.188, 256 (256 + 194) ->
// 0.205-0.213); larger D takes up to 192 (full res, same process: 64 -> 3.26-3.34 ms, 96 -> 3.24,
// 128 -> 3.21-3.25, 192 -> 3.13-3.25; KITTI D = 192: 0.366 -> 0.360 ms).
#ifndef SM_COST_P_ONE
#define SM_COST_P_ONE 240
#endif
#ifndef SM_COST_P_MULTI
#define SM_COST_P_MULTI 192
#endif
__host__ __device__ constexpr int cost_p(bool one) { return one ? SM_COST_P_ONE : SM_COST_P_MULTI; }
constexpr int LUT_A_N = 129, LUT_B_N = 766;

// LDS layout of a cost block.  Moving pixel i (position mbase + i, every candidate of the
// block's P pixels: q - mbase is in [0, P + D - 1) by construction) is a record of the CW
// 32-bit census words in use (CW = ceil(bits / 32), at least 2) followed by gx | BGR and gy:
// one 16-byte uint4 for CW = 2 (one ds_read_b128 per element), two for CW = 3, 4.  Positions
// outside the image hold zeros (the out-of-range select discards them).  Focus-pixel values are
// wave-uniform reads, once per pixel.
template <int CW>
__host__ __device__ constexpr int cost_rec_u4() { return CW <= 2 ? 1 : 2; }

// Select-free gradient elements (NOSEL = censusGrad with >= 3 census words and OORZ): an
// out-of-range candidate's staged record carries gx = gy = 1e30 and a census count bias of
// icd, so the element's own arithmetic yields the reference's out-of-range value without a
// select: min(|f - 1e30|, T) = T per axis (T = grad_trunc, 500) makes G >= 0.999 T (the host
// enables the path only when -0.999 T / lamG < -17.5, so e1 rounds away exactly as it does for
// the reference's 707.1068), and popc + icd >= icd
// picks LUT entry icd (the LUT holds 2 - expf(-C / lamCen) and is clamped at icd, so no min
// is needed either).  The exponential's input is clamped at -100 instead of selecting 0 below
// -17.5: expf_glibc_core is exact down to -103.9, and every value below 2^-25 leaves
// fl(t - e) == t (see above).  Saves the range test, three selects and a min per element.
constexpr int LUT_T_N = 260;   // >= 128 census bits + icd (<= 128) + 1
// The out-of-range sentinel gradient (NOSEL): |f - S| for a real gradient f in [-255, 255] lies in
// [S - 255, S + 255] = [295, 805]; with the truncation min(., T) the element's G is then >= 0.999
// min(T, 295) (the host's NOSEL test), and unclamped (FAST below) G <= 677.5.
constexpr float COST_OOR_GRAD = 550.0f;
// FAST elements (NOSEL, lamG == 1, adaptive weights, T >= 382.5, focus pixel off the image border): the gradient
// images are 0.5 (I[+1] - I[-1]) inside the image and full differences on its border rows and
// columns (calGrad, cpp:271-350), so an interior focus pixel has |gx|, |gy| <= 127.5 and a
// candidate in the same row |gx| <= 255, |gy| <= 127.5: |dx| <= 382.5 <= T and |dy| <= 255, the
// truncation is the identity, and wa |dx| == |fl(wa dx)| (wa, wb > 0; round-to-nearest is
// symmetric), so G = |fl(wa dx)| + |fl(wb dy)| takes one packed subtract, one packed multiply and
// one add with both operands' abs modifiers.  With wa + wb = 1 (up to 2^-24), G <= 382.5 for real
// candidates and <= 677.5 for the sentinel (unit weights could reach 1355), so -G >= -700 keeps expf_glibc_core's exponent field from wrapping without the -100
// clamp (below -103.9 the core returns a double < 2^-149 that rounds to 0 or the least
// subnormal, which fl(t - e) absorbs like the reference's exact value).  The census count
// starts from the record's bias word and accumulates through three v_bcnt_u32_b32 (one chain).
#ifndef SM_COST_FAST
#define SM_COST_FAST 1
#endif
// The cost kernel's LDS copy of the 2^(i/32) table sits in static LDS (a link-time address), so
// its byte offset (ki % 32) * 8 is one SDWA shift with a byte-0 destination select
// ((ki << 3) & 0xff) and the table's address goes into the ds_read's offset field.
struct LdsExpTab {
    const uint64_t* p;
};
__device__ __forceinline__ uint64_t exp_tab_at(const LdsExpTab& t, uint64_t ki) {
    uint32_t off;
    asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD"
        : "=v"(off) : "v"((uint32_t)ki));
    return *(const uint64_t*)((const char*)t.p + off);
}
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

// ND > 0: D == 64 * ND, the element loop fully unrolled (LDS and store offsets become immediates;
// no loop counter, compare or pointer increments: 35 -> ~29 VALU per element at D = 256)
template <int METHOD, bool LAM1, int CW, bool ONE, bool OORZ, int ND = 0>
__global__ __launch_bounds__(256) void k_cost(const CostArgs a) {
    extern __shared__ __align__(16) unsigned char cs_raw[];
    // static LDS (link-time addresses: table reads take the offset field): the 2^(i/32) table
    // and the census / AD exponential LUTs
    __shared__ uint64_t etab[32];
    __shared__ float luts[LUT_A_N + LUT_B_N];
    constexpr int RW = cost_rec_u4<CW>();
    constexpr int COST_P = cost_p(ONE);
    constexpr bool NOSEL = METHOD == SM_M_CENSUS_GRAD && OORZ && CW >= 3;
    const int D = a.D, W = a.W, H = a.H;
    const int nbx = (W + a.seg - 1) / a.seg;
    const int blk = xcd_swizzle(blockIdx.x, gridDim.x);  // neighbouring segments share an XCD's L2
    const int bx = blk % nbx, rest = blk / nbx;
    const int v = rest % H, b = rest / H;
    const int u0 = bx * a.seg;
    const int np = min(a.seg, W - u0);         // <= COST_P, the LDS layout's capacity
    const int nm = np + D - 1;                      // moving pixels needed
    const int sgn = a.view == 0 ? 1 : -1;           // moving position = u - sgn * d
    const int mbase = a.view == 0 ? u0 - (D - 1) : u0;
    const size_t npix = (size_t)H * W;
    const int fview = a.view, mview = 1 - a.view;
    const size_t frow = ((size_t)b * 2 + fview) * npix + (size_t)v * W;
    const size_t mrow = ((size_t)b * 2 + mview) * npix + (size_t)v * W;
    constexpr bool CEN = METHOD != SM_M_AD;
    constexpr bool GRAD = METHOD == SM_M_CENSUS_GRAD;
    constexpr bool ADM = METHOD == SM_M_AD || METHOD == SM_M_AD_CENSUS;
    uint4* mrec = (uint4*)cs_raw;                                // [(P + D - 1) * RW]
    ulonglong2* fcode = (ulonglong2*)(mrec + RW * (COST_P + D - 1));  // [P]
    // SM_COST_SPLIT: records of 2 uint4 (CW = 3, 4) live as two planes, so a lane's record
    // reads are 16-byte (plane A) and 8 / 16-byte (plane B) strided instead of 32-byte strided
    // (half the LDS banks per pass: 2-way conflicts on every element)
    constexpr bool SPLIT = SM_COST_SPLIT && RW == 2;
    uint4* mrecB4 = mrec + (COST_P + D - 1);                     // plane B (SPLIT), CW = 4
    uint2* mrecB2 = (uint2*)mrecB4;                              // plane B (SPLIT), CW = 3
    auto recA = [&](int i) -> uint4& { return SPLIT ? mrec[i] : mrec[RW * i]; };
    float* fgx = (float*)(fcode + COST_P);                       // [P]
    float* fgy = fgx + COST_P;
    float* fwa = fgy + COST_P;                                   // adaptive weight a (1 if off)
    float* fwb = fwa + COST_P;                                   // 1 - a (1 if off)
    uint32_t* fbgr = (uint32_t*)(fwb + COST_P);                  // [P]
    float* luta = luts;                                          // [LUT_A_N]
    float* lutb = luta + LUT_A_N;                                // [LUT_B_N]
    const int tid = threadIdx.y * 64 + threadIdx.x;
    const float cd = a.census_default;
    const int icd = (int)cd;                        // (int)fminf(pc, cd) == min(pc, (int)cd) for integer pc >= 0
    if (GRAD && tid < 32) etab[tid] = c_exp_tab[tid];
    if (NOSEL)   // luta's region (LUT_A_N + LUT_B_N floats) holds the clamped 2 - e0 table
        for (int i = tid; i < LUT_T_N; i += 256) luta[i] = 2.0f - a.lut[min(i, icd)];
    else if (CEN)
        for (int i = tid; i < LUT_A_N; i += 256) luta[i] = a.lut[i];
    if (METHOD == SM_M_AD_CENSUS)
        for (int i = tid; i < LUT_B_N; i += 256) lutb[i] = a.lut[1024 + i];
    for (int i = tid; i < np; i += 256) {
        const int u = u0 + i;
        if (CEN) fcode[i] = a.code[frow + u];
        if (GRAD) {
            const float2 gr = grad_at(a.gray + frow - (size_t)v * W, v, u, H, W);
            fgx[i] = gr.x;
            fgy[i] = gr.y;
            float wa = 1.f, wb = 1.f;
            if (a.grad_adaptive) {
                const uint32_t* planes = (const uint32_t*)a.arms + ((size_t)b * 2 + fview) * 2 * npix + (size_t)v * W + u;
                const uint32_t ph = planes[0], pv = planes[npix];
                float sH = (float)min(ph & 0xffffu, ph >> 16);
                float sV = (float)min(pv & 0xffffu, pv >> 16);
                if (sH == 0) sH = 1;
                if (sV == 0) sV = 1;
                wa = sH / (sH + sV);
                wb = 1.0f - wa;
            }
            fwa[i] = wa;
            fwb[i] = wb;
        }
        if (ADM) {
            const uint8_t* p = a.bgr + (frow + u) * 3;
            fbgr[i] = p[0] | (p[1] << 8) | (p[2] << 16);
        }
    }
    for (int i = tid; i < nm; i += 256) {
        const int q = mbase + i;
        ulonglong2 c = make_ulonglong2(0, 0);
        uint32_t w2 = 0, w3 = 0, bias = 0;
        if (q >= 0 && q < W) {
            if (CEN) c = a.code[mrow + q];
            if (GRAD) {
                const float2 gr = grad_at(a.gray + mrow - (size_t)v * W, v, q, H, W);
                w2 = __float_as_uint(gr.x);
                w3 = __float_as_uint(gr.y);
            }
            if (ADM) {
                const uint8_t* p = a.bgr + (mrow + q) * 3;
                w2 = p[0] | (p[1] << 8) | (p[2] << 16);
            }
        } else if (NOSEL) {   // out-of-range candidate: see NOSEL above
            w2 = w3 = __float_as_uint(COST_OOR_GRAD);
            bias = (uint32_t)icd;
        }
        if (CW == 4) {
            recA(i) = make_uint4((uint32_t)c.x, (uint32_t)(c.x >> 32), (uint32_t)c.y, (uint32_t)(c.y >> 32));
            if (SPLIT) mrecB4[i] = make_uint4(w2, w3, bias, 0);
            else mrec[2 * i + 1] = make_uint4(w2, w3, bias, 0);
        } else if (CW == 3 && NOSEL) {   // {census words, bias} and {gx, gy} (one 8-byte read)
            recA(i) = make_uint4((uint32_t)c.x, (uint32_t)(c.x >> 32), (uint32_t)c.y, bias);
            if (SPLIT) mrecB2[i] = make_uint2(w2, w3);
            else mrec[2 * i + 1] = make_uint4(w2, w3, 0, 0);
        } else if (CW == 3) {
            recA(i) = make_uint4((uint32_t)c.x, (uint32_t)(c.x >> 32), (uint32_t)c.y, w2);
            if (SPLIT) mrecB2[i] = make_uint2(w3, bias);
            else mrec[2 * i + 1] = make_uint4(w3, bias, 0, 0);
        } else {
            mrec[i] = make_uint4((uint32_t)c.x, (uint32_t)(c.x >> 32), w2, w3);
        }
    }
    __syncthreads();
    const int lane = threadIdx.x;
    if (ONE && lane >= D) return;                   // D <= 64: one disparity per lane; no barrier follows
    const float* out = a.vm + ((size_t)b * npix + (size_t)v * W + u0) * D;
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(out, np * D * 4);
    // the wave's pixel index is uniform: loop control and the store's pixel offset stay scalar
    const int wy = __builtin_amdgcn_readfirstlane((int)threadIdx.y);
    // FAST: interior rows, T >= 382.5, adaptive weights (wa + wb <= 1 + 2^-24 bounds the sentinel's G)
    const bool fast_rows = v > 0 && v < H - 1 && a.grad_trunc >= 382.5f && a.grad_adaptive;
    // (ND > 0) the lane's record index at pl = 0: a pixel's records start pl records later
    const int mil_lane = (sgn > 0 ? u0 - lane - 64 * (ND - 1) : u0 + lane) - mbase;
    // one focus pixel (pl: its index in the segment) with FAST or general elements
    auto one = [&](int pl, auto fastc) {
        const int u = u0 + pl;
        const ulonglong2 cf = CEN ? fcode[pl] : make_ulonglong2(0, 0);
        float fx = 0.f, fy = 0.f, wa = 0.f, wb = 0.f;
        uint32_t fc = 0;
        if (GRAD) {
            fx = fgx[pl];
            fy = fgy[pl];
            wa = fwa[pl];
            wb = fwb[pl];
        }
        if (ADM) fc = fbgr[pl];
        // element at staged record mi (moving position q = mbase + mi = u - sgn * d, zeros when out
        // of range), stored at byte voff + soff of the pixel's row (voff = d * 4 - soff's part)
        auto elem = [&](auto fastc, int mi, uint32_t voff, uint32_t soff) {
            constexpr bool FAST = decltype(fastc)::value;
            const int q = mi + mbase;
            if constexpr (NOSEL) {
                typedef float f2 __attribute__((ext_vector_type(2)));
                const uint4 r0 = recA(mi);
                uint32_t pc;
                uint2 gw;
                if constexpr (CW == 3) {
                    gw = SPLIT ? mrecB2[mi] : *(const uint2*)&mrec[RW * mi + 1];
                    pc = r0.w;                         // icd for out-of-range candidates, else 0
                } else {
                    const uint4 r1 = SPLIT ? mrecB4[mi] : mrec[RW * mi + 1];
                    pc = r1.z;
                    gw = make_uint2(r1.x, r1.y);
                }
                pc = bcnt_acc((uint32_t)cf.x ^ r0.x, pc);
                pc = bcnt_acc((uint32_t)(cf.x >> 32) ^ r0.y, pc);
                pc = bcnt_acc((uint32_t)cf.y ^ r0.z, pc);
                if (CW == 4) pc = bcnt_acc((uint32_t)(cf.y >> 32) ^ r0.w, pc);
                const f2 dv = f2{fx, fy} - f2{__uint_as_float(gw.x), __uint_as_float(gw.y)};
                float g;
                if constexpr (FAST) {
                    const f2 tv = f2{wa, wb} * dv;
                    g = fabsf(tv.x) + fabsf(tv.y);
                } else {
                    const f2 tv = f2{wa, wb} * f2{fminf(fabsf(dv.x), a.grad_trunc), fminf(fabsf(dv.y), a.grad_trunc)};
                    g = tv.x + tv.y;
                }
                // (-fminf(g, 100) == fmaxf(-g, -100): both paths end in a negated conversion)
                const float xg = LAM1 ? (FAST ? -g : -fminf(g, 100.0f)) : fmaxf(-g / a.lam2, -100.0f);
                const float t = luta[pc];                       // fl(2 - expf(-min(pc, icd) / lamCen))
                const float ex = expf_glibc_core(xg, LdsExpTab{etab});
                const float res = t - ex;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, res), ro, voff, soff,
                                                      SM_COST_STORE_AUX);
                return;
            }
            const bool oor = (unsigned)q >= (unsigned)W;
            const uint4 r0 = recA(mi);
            uint32_t w2 = r0.z, w3 = r0.w;
            uint32_t pc = 0;
            if (CEN) {
                pc = __popc((uint32_t)cf.x ^ r0.x) + __popc((uint32_t)(cf.x >> 32) ^ r0.y);
                if (CW >= 3) pc += __popc((uint32_t)cf.y ^ r0.z);
                if (CW == 4) pc += __popc((uint32_t)(cf.y >> 32) ^ r0.w);
            }
            if (CW == 3) {
                w2 = r0.w;
                w3 = SPLIT ? mrecB2[mi].x : ((const uint32_t*)mrec)[4 * (RW * mi + 1)];
            } else if (CW == 4) {
                const uint4 r1 = SPLIT ? mrecB4[mi] : mrec[RW * mi + 1];
                w2 = r1.x;
                w3 = r1.y;
            }
            float res;
            if (METHOD == SM_M_CENSUS) {
                res = oor ? cd : fminf((float)pc, cd);
            } else if (GRAD) {
                const float dx = fminf(fabsf(fx - __uint_as_float(w2)), a.grad_trunc);
                const float dy = fminf(fabsf(fy - __uint_as_float(w3)), a.grad_trunc);
                const float t1 = wa * dx;
                const float t2 = wb * dy;
                float g0 = t1 + t2;
                asm volatile("" : "+v"(g0));              // keep the element loop branch-free
                const float g = oor ? a.grad_oor : g0;
                const int ci = oor ? icd : min((int)pc, icd);
                const float e0 = luta[ci];                // expf(-C / lamCen)
                const float xg = LAM1 ? -g : -g / a.lam2;
                const float ex = expf_glibc_core(xg, LdsExpTab{etab}); // expf(-G / lamG)
                const float e1 = xg >= -17.5f ? ex : 0.f;
                const float t = 2.0f - e0;
                res = t - e1;
            } else {
                const uint32_t y = w2;
                const int s3 = abs((int)(fc & 0xff) - (int)(y & 0xff)) +
                               abs((int)((fc >> 8) & 0xff) - (int)((y >> 8) & 0xff)) + abs((int)(fc >> 16) - (int)(y >> 16));
                if (METHOD == SM_M_AD) {
                    res = oor ? a.ad_trunc : fminf((float)s3 / 3.0f, a.ad_trunc);
                } else {
                    const float e0 = oor ? a.ad_oor_exp : lutb[s3];
                    const int ci = oor ? icd : min((int)pc, icd);
                    const float e1 = luta[ci];
                    const float t = 2.0f - e0;
                    res = t - e1;
                }
            }
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, res), ro, voff, soff,
                                                  SM_COST_STORE_AUX);
        };
        auto pixel = [&](auto fastc) {
            if constexpr (ONE) {
                elem(fastc, u - sgn * lane - mbase, lane * 4, pl * D * 4);
            } else if constexpr (ND > 0) {
                // element k takes disparity d = lane + 64 kk with kk = k (left view) or ND - 1 - k (right
                // view), so that its record index is mil + 64 (ND - 1 - k) in both views: the LDS reads
                // take non-negative immediate offsets from one per-lane base, the stores a uniform soffset
                const int mil = mil_lane + pl;
#pragma unroll
                for (int k = 0; k < ND; k++) {
                    const int kk = sgn > 0 ? k : ND - 1 - k;
                    elem(fastc, mil + 64 * (ND - 1 - k), lane * 4, (uint32_t)(pl * D * 4 + kk * 256));
                }
            } else {
                const int qstep = sgn * 64;
                int q = u - sgn * lane;
                for (int d = lane; d < D; d += 64, q -= qstep) elem(fastc, q - mbase, d * 4, pl * D * 4);
            }
        };
        pixel(fastc);
    };
    // FAST (see COST_OOR_GRAD): a wave-uniform choice per focus pixel; the general elements are
    // valid for every pixel.  (Two pixels per trip: no fewer instructions per element.)
    // (for ONE only with two pixels per trip: one element per lane and pixel leaves the table
    // read's latency exposed, Teddy x16 0.164 -> 0.178 ms, profiles/r5n/ab3_teddy.log)
    constexpr bool FASTOK = SM_COST_FAST && NOSEL && LAM1 && (!ONE || SM_COST_ONE_FAST);
    int pl = wy;
    if constexpr (ONE && SM_COST_ONE_PAIR) {
        // D <= 64: pixels pl and pl + 4 per trip, two independent elements per lane
        for (; pl + 4 < np; pl += 8) {
            const int u = u0 + pl;
            if (FASTOK && fast_rows && u > 0 && u + 4 < W - 1) {
                one(pl, std::integral_constant<bool, FASTOK>{});
                one(pl + 4, std::integral_constant<bool, FASTOK>{});
            } else {
                one(pl, std::false_type{});
                one(pl + 4, std::false_type{});
            }
        }
    }
#pragma unroll SM_COST_UNROLL
    for (; pl < np; pl += 4) {
        const int u = u0 + pl;
        if (FASTOK && fast_rows && u > 0 && u < W - 1)
            one(pl, std::integral_constant<bool, FASTOK>{});
        else
            one(pl, std::false_type{});
    }
}

size_t cost_smem_bytes(int D, int cwords) {
    const int COST_P = cost_p(D <= 64);
    const size_t nm = COST_P + D - 1;
    return 16 * (cwords > 2 ? 2 : 1) * nm + 16 * COST_P + 4 * 5 * COST_P;   // (+ the static tables)
}

// SolveAll with PY_LVL = 1 as a standalone pass (used by the reference-ordered API):
// vm = 0 + invWgt * vm (cpp:2189-2201).
__global__ void k_scale(float* __restrict__ vm, size_t n, float w) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float sum = 0.f;
        sum += w * vm[i];
        vm[i] = sum;
    }
}

// WTA alone (optimization == "" / aggregation-only runs): one wave per pixel.
template <int K>
__global__ __launch_bounds__(256) void k_wta(const float* __restrict__ vm, int16_t* __restrict__ disp, int H, int W, int D) {
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const size_t npix = (size_t)H * W;
    const int b = blockIdx.y;
    if ((size_t)wave >= npix) return;
    const float* f = vm + ((size_t)b * npix + wave) * D;
    const int d0 = lane * K;
    float bm = FLT_MAX;
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < K; k++)
        if (d0 + k < D && bm > f[d0 + k]) {
            bm = f[d0 + k];
            bi = d0 + k;
        }
    const float wm = wave_min(bm);
    const uint64_t hit = __ballot(bm == wm);   // lowest lane holding the minimum = first index
    const int widx = __builtin_amdgcn_readlane(bi, (int)__builtin_ctzll(hit));
    if (lane == 0) disp[(size_t)b * npix + wave] = (int16_t)((wm < FLT_MAX) ? widx : -1);
}

// div_area vs IEEE: block y = divisor, threads sweep the 2^23 mantissas of exponent exp2
__global__ void k_div_check(int exp2, unsigned long long* __restrict__ bad) {
    const uint32_t b = blockIdx.y + 1;
    const uint32_t ebits = (uint32_t)(exp2 + 127) << 23;
    uint32_t nbad = 0;
    for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < (1u << 23); m += gridDim.x * blockDim.x) {
        const float a = __builtin_bit_cast(float, ebits | m);
        const float fast = div_area(a, b);
        const float ref = a / (float)b;
        nbad += __builtin_bit_cast(uint32_t, fast) != __builtin_bit_cast(uint32_t, ref);
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

void launch_div_check(int exp2, int bmax, unsigned long long* bad, hipStream_t st) {
    hipLaunchKernelGGL(k_div_check, dim3(64, bmax), dim3(256), 0, st, exp2, bad);
}

__global__ void k_expf_range(uint32_t first, uint32_t n, float* __restrict__ out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[i] = dev_expf(__builtin_bit_cast(float, first + i));
}

// Measured HBM ceiling for the roofline: a dwordx4 copy, each workgroup moving
// whole 16 KB blocks (256 lanes x 4 dwordx4 in flight per lane), non-temporal loads and stores
// like the volume sweeps, XCD-ordered so that consecutive blocks share an XCD's L2.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy_x4(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t nblk) {
    const size_t stride = gridDim.x;
    for (size_t b = xcd_swizzle(blockIdx.x, gridDim.x); b < nblk; b += stride) {
        const size_t i0 = b * 1024 + threadIdx.x;
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = __builtin_nontemporal_load(in + i0 + 256 * k);
#pragma unroll
        for (int k = 0; k < 4; k++) __builtin_nontemporal_store(v[k], out + i0 + 256 * k);
    }
}

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
void launch_copy_x4(const void* in, void* out, size_t bytes, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_copy_x4, dim3(grid), dim3(256), 0, st, (const u32x4*)in, (u32x4*)out, bytes / 16384);
}

template <int METHOD, bool LAM1, int CW, bool OORZ>
static void launch_cost_z(const CostArgs& a, dim3 grid, dim3 block, size_t shm, hipStream_t st) {
    if (a.D <= 64)
        hipLaunchKernelGGL((k_cost<METHOD, LAM1, CW, true, OORZ>), grid, block, shm, st, a);
#if SM_COST_ND
    else if (a.D == 256)
        hipLaunchKernelGGL((k_cost<METHOD, LAM1, CW, false, OORZ, 4>), grid, block, shm, st, a);
    else if (a.D == 192)
        hipLaunchKernelGGL((k_cost<METHOD, LAM1, CW, false, OORZ, 3>), grid, block, shm, st, a);
    else if (a.D == 128)
        hipLaunchKernelGGL((k_cost<METHOD, LAM1, CW, false, OORZ, 2>), grid, block, shm, st, a);
#endif
    else
        hipLaunchKernelGGL((k_cost<METHOD, LAM1, CW, false, OORZ>), grid, block, shm, st, a);
}

template <int METHOD, bool LAM1, int CW>
static void launch_cost_nw(const CostArgs& a, dim3 grid, dim3 block, size_t shm, hipStream_t st) {
    // select-free elements (NOSEL in k_cost): an out-of-range pair's G is at least
    // fl(wa m) + fl(wb m) >= 0.999 m, m = min(T, COST_OOR_GRAD - 255) (T = grad_trunc,
    // wa + fl(1 - wa) = 1 up to 2^-24), and its exponential
    // must still round away: xg = -G (lamG == 1) or -G / lamG below -17.5; the clamped
    // 2 - e0 table covers counts up to 128 + icd
    const float gmin = 0.999f * fminf(a.grad_trunc, COST_OOR_GRAD - 255.0f);
    const float xg = LAM1 ? -gmin : -gmin / a.lam2;
    if constexpr (METHOD == SM_M_CENSUS_GRAD && CW >= 3) {
        if (xg < -17.5f && a.grad_trunc < 1e29f && (int)a.census_default <= 128 && (int)a.census_default >= 0)
            return launch_cost_z<METHOD, LAM1, CW, true>(a, grid, block, shm, st);
    }
    launch_cost_z<METHOD, LAM1, CW, false>(a, grid, block, shm, st);
}

template <int METHOD, bool LAM1>
static void launch_cost_m(const CostArgs& a, dim3 grid, dim3 block, size_t shm, hipStream_t st) {
    if (METHOD == SM_M_AD || a.cwords <= 2)
        launch_cost_nw<METHOD, LAM1, 2>(a, grid, block, shm, st);
    else if (a.cwords == 3)
        launch_cost_nw<METHOD, LAM1, 3>(a, grid, block, shm, st);
    else
        launch_cost_nw<METHOD, LAM1, 4>(a, grid, block, shm, st);
}

void launch_cost(const CostArgs& a0, int method, int n, hipStream_t st) {
    // equal segments of at most cost_p pixels (a 450-pixel row: two of 225, not 128 x 3 + 66)
    CostArgs a = a0;
    const int P = cost_p(a.D <= 64);
    const int nb = (a.W + P - 1) / P;
    a.seg = (a.W + nb - 1) / nb;
    dim3 grid((unsigned)(nb * a.H * n));
    dim3 block(64, 4);
    const size_t shm = cost_smem_bytes(a.D, method == SM_M_AD ? 2 : a.cwords);
    switch (method) {
        case SM_M_CENSUS_GRAD:
            if (a.lam2 == 1.0f)
                launch_cost_m<SM_M_CENSUS_GRAD, true>(a, grid, block, shm, st);
            else
                launch_cost_m<SM_M_CENSUS_GRAD, false>(a, grid, block, shm, st);
            break;
        case SM_M_CENSUS: launch_cost_m<SM_M_CENSUS, false>(a, grid, block, shm, st); break;
        case SM_M_AD_CENSUS: launch_cost_m<SM_M_AD_CENSUS, false>(a, grid, block, shm, st); break;
        default: launch_cost_m<SM_M_AD, false>(a, grid, block, shm, st); break;
    }
}

void launch_scale(float* vm, size_t n, float w, hipStream_t st) {
    size_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_scale, dim3((unsigned)blocks), dim3(256), 0, st, vm, n, w);
}

int sgm_k_for(int D) {
    const int k = (D + 63) / 64;
    if (k <= 4) return k;
    if (k <= 6) return 6;
    if (k <= 8) return 8;
    if (k <= 12) return 12;
    return 16;
}

void launch_wta(const float* vm, int16_t* disp, int n, int H, int W, int D, hipStream_t st) {
    const size_t npix = (size_t)H * W;
    dim3 grid((unsigned)((npix + 3) / 4), n);
    switch (sgm_k_for(D)) {
        case 1: hipLaunchKernelGGL(k_wta<1>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 2: hipLaunchKernelGGL(k_wta<2>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 3: hipLaunchKernelGGL(k_wta<3>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 4: hipLaunchKernelGGL(k_wta<4>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 6: hipLaunchKernelGGL(k_wta<6>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 8: hipLaunchKernelGGL(k_wta<8>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 12: hipLaunchKernelGGL(k_wta<12>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        default: hipLaunchKernelGGL(k_wta<16>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
    }
}

void launch_expf_range(uint32_t first, uint32_t n, float* out, hipStream_t st) {
    hipLaunchKernelGGL(k_expf_range, dim3(4096), dim3(256), 0, st, first, n, out);
}

float expf_host(float x) {
    static const uint64_t tab[32] = SM_EXPF_TABLE;
    return expf_glibc(x, tab);
}

}  // namespace sm
