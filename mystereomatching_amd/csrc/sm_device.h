// sm_device.h — device helpers shared by the hot-path kernels (gfx950 / CDNA4).
//
// * sm_expf: the host libm's expf, restated in fp64 so that device results are bit-identical
//   to the CPU reference's `exp(float)` (stereoMatching.cpp:3585 resolves to expf).  The host
//   libm is glibc 2.35; its x86_64 expf (FMA ifunc variant) evaluates 2^(k/32)·p(r) in double:
//   r = fma(InvLn2N, x, -kd), degree-3 polynomial in fma form.  The 2^(i/32) table entries are
//   the correctly rounded doubles (generated with mpmath, see tools/gen_expf_table.py).  The
//   restatement was checked against libm on every negative float down to -0x1.9fe368p6f
//   (1,120,924,085 inputs, 0 mismatches) on the build host, and the device build is checked
//   over the same range on the GPU box (tests/test_gpu_parity.py::test_device_expf_exhaustive).
// * sm_reflect101: OpenCV borderInterpolate(BORDER_REFLECT_101) (copyMakeBorder, h:870-871).
// * wave64 reductions built on DPP + gfx950 permlane swaps (no LDS round trip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SM_EXPF_TABLE                                                                    \
    {0x3ff0000000000000ULL, 0x3fefd9b0d3158574ULL, 0x3fefb5586cf9890fULL, 0x3fef9301d0125b51ULL, \
     0x3fef72b83c7d517bULL, 0x3fef54873168b9aaULL, 0x3fef387a6e756238ULL, 0x3fef1e9df51fdee1ULL, \
     0x3fef06fe0a31b715ULL, 0x3feef1a7373aa9cbULL, 0x3feedea64c123422ULL, 0x3feece086061892dULL, \
     0x3feebfdad5362a27ULL, 0x3feeb42b569d4f82ULL, 0x3feeab07dd485429ULL, 0x3feea47eb03a5585ULL, \
     0x3feea09e667f3bcdULL, 0x3fee9f75e8ec5f74ULL, 0x3feea11473eb0187ULL, 0x3feea589994cce13ULL, \
     0x3feeace5422aa0dbULL, 0x3feeb737b0cdc5e5ULL, 0x3feec49182a3f090ULL, 0x3feed503b23e255dULL, \
     0x3feee89f995ad3adULL, 0x3feeff76f2fb5e47ULL, 0x3fef199bdd85529cULL, 0x3fef3720dcef9069ULL, \
     0x3fef5818dcfba487ULL, 0x3fef7c97337b9b5fULL, 0x3fefa4afa2a490daULL, 0x3fefd0765b6e4540ULL}

#ifndef SM_EXPF_VEC
#define SM_EXPF_VEC 1   // assemble 2^(k/32) from two 32-bit words (4 VALU fewer per call than 64-bit ops)
#endif
#ifndef SM_EXPF_FMA_SHIFT
#define SM_EXPF_FMA_SHIFT 1
#endif

namespace sm {

// entry ki % 32 of the 2^(i/32) table (overloaded for the cost kernel's LDS copy)
template <typename Tab>
__host__ __device__ inline uint64_t exp_tab_at(const Tab& tab, uint64_t ki) { return tab[ki % 32]; }

// expf core; `tab` is the 32-entry 2^(i/32) table (device: __constant__, host: static).
// Main path only: valid for -0x1.9fe368p6 <= x <= 0x1.62e42ep6 (callers that cannot be outside
// that range, or that discard such results, skip the special cases).
template <typename Tab>
__host__ __device__ inline float expf_glibc_core(float x, const Tab& tab) {
    const double InvLn2N = 0x1.71547652b82fep+0 * 32;
    const double SHIFT = 0x1.8p+52;
    const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32;
    const double C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32;
    const double C2 = 0x1.62e42ff0c52d6p-1 / 32;
    double xd = (double)x;
#if SM_EXPF_FMA_SHIFT
    // kd = round(InvLn2N * xd) through one fma instead of a rounded product plus SHIFT: equal
    // to glibc's result on every float the device path sees (tests/test_gpu_parity.py,
    // test_device_expf_exhaustive: all of [-104, -0])
    double kd = __builtin_fma(InvLn2N, xd, SHIFT);
#else
    double z = InvLn2N * xd;
    double kd = z + SHIFT;
#endif
    uint64_t ki = __builtin_bit_cast(uint64_t, kd);
    kd -= SHIFT;
    double r = __builtin_fma(InvLn2N, xd, -kd);
    const uint64_t t = exp_tab_at(tab, ki);
    // t += ki << 47: the shifted term's low word is 0, so only the high word changes (one
    // 32-bit add instead of a 64-bit shift and add); the words are assembled as a 2-vector so
    // that no 64-bit shift / or is emitted for the pair
#if SM_EXPF_VEC
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 tw = {(uint32_t)t, (uint32_t)(t >> 32) + ((uint32_t)ki << 15)};
    double s = __builtin_bit_cast(double, tw);
#else
    double s = __builtin_bit_cast(double, (t & 0xffffffffull) | ((uint64_t)((uint32_t)(t >> 32) + ((uint32_t)ki << 15)) << 32));
#endif
    double zz = __builtin_fma(C0, r, C1);
    double r2 = r * r;
    double y = __builtin_fma(C2, r, 1.0);
    y = __builtin_fma(zz, r2, y);
    y = y * s;
    return (float)y;
}

template <typename Tab>
__host__ __device__ inline float expf_glibc(float x, const Tab& tab) {
    // Special cases of glibc's expf for |x| >= 88 that the main path does not cover.
    if (x < -0x1.9fe368p6f) return 0.0f;           // underflow (also -inf)
    if (x > 0x1.62e42ep6f) return __builtin_inff(); // overflow (never reached on the hot path)
    return expf_glibc_core(x, tab);
}

__host__ __device__ inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    do {
        if (p < 0)
            p = -p;
        else
            p = 2 * len - p - 2;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// XCD-aware block order (speed only, never correctness): the dispatcher deals workgroups
// round-robin over the 8 XCDs, so hardware block `orig` runs on XCD group orig % 8.  This
// bijection gives each XCD group a contiguous range of logical blocks, so neighbouring lines
// that read the same arm / image rows share one XCD's L2.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
    const int xcd = orig & 7, idx = orig >> 3, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Buffer-instruction access (gfx9 resource word 3 = 0x00020000, 32-bit data).  The range limit
// is 2^31 - 1 bytes, so a lane offset of 0x80000000 turns its load into 0 and drops its store.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, int num_bytes = 0x7fffffff) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, num_bytes, 0x00020000);
}
#ifndef SM_LD_AUX
#define SM_LD_AUX 0   // cache policy of streaming volume loads (tuning)
#endif
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, SM_LD_AUX));
}
__device__ __forceinline__ uint32_t buf_ld_u32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0);
}
// Volume stores are streaming: every pass writes a W x H x D volume larger than the 256 MB
// Infinity Cache, read back only by the next pass.  SM_ST_AUX = 2 (slc = "nt" on gfx950) sends
// them with the non-temporal policy, as does SM_NT_STORES for the SGM path sums.  Measured (Teddy
// x16, same box): the pass after a plain-store pass runs slower while the Infinity Cache writes
// back the previous pass's dirty lines — cost volume nt: h_scan 0.314 -> 0.272 ms; CBCA nt:
// -0.005 ms per sweep; SGM nt: path1 0.392 -> 0.370 ms; 3.53 -> ~3.43 ms per step together.
#ifndef SM_ST_AUX
#define SM_ST_AUX 2
#endif
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)voff, (int)soff, SM_ST_AUX);
}
#ifndef SM_NT_STORES
#define SM_NT_STORES 1
#endif
__device__ __forceinline__ void st_stream(float* p, float v) {
#if SM_NT_STORES
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
#ifndef SM_NT_LOADS
#define SM_NT_LOADS 1   // SGM C / path-sum loads non-temporal: last path 0.302 -> 0.249 ms (Teddy x16)
#endif
__device__ __forceinline__ float ld_stream(const float* p) {
#if SM_NT_LOADS
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
__device__ __forceinline__ float4 ld_stream4(const float* p) {
#if SM_NT_LOADS
    return make_float4(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1), __builtin_nontemporal_load(p + 2),
                       __builtin_nontemporal_load(p + 3));
#else
    return *(const float4*)p;
#endif
}
__device__ __forceinline__ void st_stream4(float* p, float4 v) {
#if SM_NT_STORES
    __builtin_nontemporal_store(v.x, p);
    __builtin_nontemporal_store(v.y, p + 1);
    __builtin_nontemporal_store(v.z, p + 2);
    __builtin_nontemporal_store(v.w, p + 3);
#else
    *(float4*)p = v;
#endif
}

// a / b for a float a >= 0 and an integer 1 <= b < 2^16 (CBCA support areas), correctly
// rounded like IEEE division, in 4 instructions instead of the 11 of the general sequence:
//   y = rcp(b) (|rel. error| <= 2^-22 suffices), q0 = RN(a y), r = a - q0 b (exact), q = RN(q0 + r y).
// Proof: with Q = a / b, |Q - q0| <= 4.5 ulp(Q), r is a multiple of ulp(q0) below 2^24 of them,
// so the fma's r is exact and q0 + r y = Q + (Q - q0) e with |(Q - q0) e| <= 2^-19.8 ulp(Q).  A
// midpoint M of Q's binade satisfies b Q - b M = integer * ulp(Q) / 2 and is never hit exactly
// (b M has more than 24 significant bits unless b is a power of two, where q0 is already
// exact), so |Q - M| >= ulp(Q) / (2 b) >= 2^-17 ulp(Q) > the perturbation: RN(q0 + r y) =
// RN(Q).  Needs q0 and r representable without underflow: a == 0 or a >= 2^-110
// (div_area_needs_ieee tells the caller when to use the IEEE division instead).
// tests/test_gpu_parity.py::test_div_area_exhaustive checks it against IEEE on the device.
__device__ __forceinline__ float div_area(float a, uint32_t b) {
    const float bf = (float)b;
    const float y = __builtin_amdgcn_rcpf(bf);
    const float q0 = a * y;
    const float r = __builtin_fmaf(-q0, bf, a);
    return __builtin_fmaf(r, y, q0);
}
__device__ __forceinline__ bool div_area_needs_ieee(float a) {  // 0 < |a| < 2^-110
    return (__builtin_bit_cast(uint32_t, a) & 0x7fffffffu) - 1u < 0x087fffffu;
}

// wave64 cross-lane helpers (device only)
// DPP controls (GFX9 encoding).
enum : int {
    DPP_QUAD_1032 = 0xB1,     // quad_perm [1,0,3,2]
    DPP_QUAD_2301 = 0x4E,     // quad_perm [2,3,0,1]
    DPP_ROW_HALF_MIRROR = 0x141,
    DPP_ROW_MIRROR = 0x140,
    DPP_WAVE_SHL1 = 0x130,    // lane i <- lane i+1
    DPP_WAVE_SHR1 = 0x138,    // lane i <- lane i-1
};

template <int CTRL>
__device__ inline float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ inline int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

// gfx950 v_permlane16_swap / v_permlane32_swap with both operands = v: the two results hold,
// at every lane, the values of the two rows (resp. halves) that the instruction pairs, so
// min(r[0], r[1]) is the min over that pair whichever operand receives which row.
__device__ inline unsigned perm16_min_u(unsigned v, bool is_float) {
    auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    if (is_float) return __builtin_bit_cast(unsigned, fminf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1])));
    return (unsigned)min((int)r[0], (int)r[1]);
}
__device__ inline unsigned perm32_min_u(unsigned v, bool is_float) {
    auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    if (is_float) return __builtin_bit_cast(unsigned, fminf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1])));
    return (unsigned)min((int)r[0], (int)r[1]);
}

// Min over the wave of NON-NEGATIVE floats (and +inf / FLT_MAX): their IEEE order is the
// unsigned order of the bit patterns, so the reduction runs on v_min_u32 (no NaN
// canonicalisation) and ends with the GFX9 row broadcasts; the result is wave-uniform.
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint32_t umin_dpp(uint32_t v) {
    return min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffffu, (int)v, CTRL, ROWS, 0xF, false));
}
enum : int { DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143 };
__device__ __forceinline__ uint32_t wave_umin(uint32_t v) {
    v = umin_dpp<DPP_QUAD_1032>(v);
    v = umin_dpp<DPP_QUAD_2301>(v);
    v = umin_dpp<DPP_ROW_HALF_MIRROR>(v);
    v = umin_dpp<DPP_ROW_MIRROR>(v);          // every lane: its row's min
    v = umin_dpp<DPP_ROW_BCAST15, 0xA>(v);    // rows 1, 3 also see rows 0, 2
    v = umin_dpp<DPP_ROW_BCAST31, 0xC>(v);    // rows 2, 3 also see row 1: lane 63 = wave min
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ float wave_min_pos(float v) {
    return __builtin_bit_cast(float, wave_umin(__builtin_bit_cast(uint32_t, v)));
}
__device__ __forceinline__ float fmin_pos(float a, float b) {  // a, b >= +0
    return __builtin_bit_cast(float, min(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b)));
}

// Full-wave min; every lane receives the result.  min is exact, so the combine order is free.
__device__ inline float wave_min(float v) {
    v = fminf(v, dpp_f<DPP_QUAD_1032>(v));
    v = fminf(v, dpp_f<DPP_QUAD_2301>(v));
    v = fminf(v, dpp_f<DPP_ROW_HALF_MIRROR>(v));
    v = fminf(v, dpp_f<DPP_ROW_MIRROR>(v));
    v = __builtin_bit_cast(float, perm16_min_u(__builtin_bit_cast(unsigned, v), true));
    v = __builtin_bit_cast(float, perm32_min_u(__builtin_bit_cast(unsigned, v), true));
    return v;
}
__device__ inline int wave_min_i(int v) {
    v = min(v, dpp_i<DPP_QUAD_1032>(v));
    v = min(v, dpp_i<DPP_QUAD_2301>(v));
    v = min(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = min(v, dpp_i<DPP_ROW_MIRROR>(v));
    v = (int)perm16_min_u((unsigned)v, false);
    v = (int)perm32_min_u((unsigned)v, false);
    return v;
}


}  // namespace sm
