// sm_sgm2.hip — the default 4-path SGM (sgm, stereoMatching.cpp:6204-6224) in two 2-D wavefront
// passes instead of four path sweeps.
//
// The reference runs costScan (cpp:1983-2029) for the directions r = (+1,0), (-1,0), (0,+1), (0,-1)
// (cpp:6207-6208, numOfDirec = 4) and sums the path volumes in that order,
// vm = (((0 + L0) + L1) + L2) + L3 (gen_sgm_vm, cpp:2031-2056), then takes the WTA.  L0 (previous
// pixel below) and L2 (previous pixel to the right) both run in reverse raster order; L1 (above)
// and L3 (left) in raster order.  So:
//   pass A (reverse raster): L0 and L2 from C      -> acc = 0 + L0, l2v = L2     (R 4 + W 8 B/elem)
//   pass B (raster):         L1 and L3 from C, then (((acc + L1) + l2v) + L3) -> WTA  (R 12 B/elem)
// 24 B per volume element instead of the four sweeps' 8 + 12 + 12 + 8 = 40 B; every value and
// every sum is the reference's, in its order, so the maps are bit-identical to the path sweeps.
//
// gfx950 mapping.  A workgroup owns a strip of R consecutive rows (in the pass's row order), one
// wave per row, lane l holding disparities [l K, l K + K) (D = 64 K).  A wave walks its row in
// tiles of TC columns carrying the horizontal path in registers (path minimum by DPP wave
// reduction, d +/- 1 by DPP wave shifts, as k_sgm does).  The vertical path's state of a column
// flows from row to row: wave r processes tile t in phase t + r, one workgroup barrier per phase,
// and hands each column's vertical L to wave r + 1 through an LDS double buffer.  Between strips
// the last row's vertical L goes through global memory: it is stored with device-scope
// coherence (sc1 -- pass A's acc output itself, pass B's L1 over the acc entry it has just read),
// then the strip's progress counter is raised (device-scope atomic store after the stores have
// completed); the next strip's first wave waits for tile t + 1 of its predecessor before loading
// tile t + 1's values with sc1 loads (one tile of slack, so those loads are prefetched like the
// tile's costs).  Strips are handed out by an atomic ticket in chain order, so a waiting strip's
// predecessor is always already running: no dependence on dispatch order, no deadlock.  Every
// wait is bounded: a wait that exceeds SM_SGM2_SPIN polls raises an abort flag that releases all
// waiters (the kernel then ends and the host reports the abort), so a fault can never hang the GPU.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

#ifndef SM_SGM2_R
#define SM_SGM2_R 8          // rows (waves) per strip
#endif
#ifndef SM_SGM2_TC
#define SM_SGM2_TC 2         // columns per tile (= the skew between consecutive rows)
#endif
#ifndef SM_SGM2_SPIN
#define SM_SGM2_SPIN (1 << 21)   // polls (an atomic load + s_sleep 2 each, ~1-2 us) before a wait gives up
#endif

namespace sm {

namespace {

constexpr int SG2_SYNC_HDR = 4;   // sync words: [0] ticket, [1] abort, [2..3] spare, then progress

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// K consecutive floats of a lane through a buffer resource (aux: cache policy)
template <int K, int AUX>
__device__ __forceinline__ void ldK(__amdgpu_buffer_rsrc_t r, uint32_t off, float* x) {
    if constexpr (K == 4) {
        const f4v v = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX));
        x[0] = v.x, x[1] = v.y, x[2] = v.z, x[3] = v.w;
    } else if constexpr (K == 2) {
        const f2v v = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, AUX));
        x[0] = v.x, x[1] = v.y;
    } else {
        x[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, AUX));
    }
}
template <int K, int AUX>
__device__ __forceinline__ void stK(__amdgpu_buffer_rsrc_t r, uint32_t off, const float* x) {
    if constexpr (K == 4) {
        const f4v v = {x[0], x[1], x[2], x[3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r, (int)off, 0, AUX);
    } else if constexpr (K == 2) {
        const f2v v = {x[0], x[1]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), r, (int)off, 0, AUX);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, x[0]), r, (int)off, 0, AUX);
    }
}

constexpr int AUX_NT = 2;     // non-temporal (streaming volumes)
constexpr int AUX_DEV = 16;   // sc1: device-scope coherent (the strip exchange rows)

template <int K, int TC>
struct Sg2Tile {
    float c[TC][K];    // C
    float a0[TC][K];   // pass B: acc = 0 + L0
    float a2[TC][K];   // pass B: L2
    float xv[TC][K];   // first wave of a strip: the previous strip's vertical L for this tile
    uint32_t fl[TC];   // penalty flags of the tile's pixels (wave-uniform)
};

template <int K, int R, int TC, bool PB, bool SG, bool KEEP>
__global__ __launch_bounds__(64 * R) void k_sgm2(const Sgm2Args a) {
    extern __shared__ float xch[];   // [R - 1][2][TC][64 K]: vertical L handed from wave r to r + 1
    __shared__ int s_ticket;
    const int lane = threadIdx.x & 63;
    const int r = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int H = a.H, W = a.W, D = a.D;
    const int NS = (H + R - 1) / R;
    uint32_t* const sync = a.sync;
    if (threadIdx.x == 0) s_ticket = (int)atomicAdd(&sync[0], 1u);
    __syncthreads();
    const int ticket = __builtin_amdgcn_readfirstlane(s_ticket);
    const int b = ticket % a.n, s = ticket / a.n;
    // processing-order row g; image row v (pass A walks up from the bottom, pass B down)
    const int g = s * R + r;
    const bool rvalid = g < H;
    const int v = rvalid ? (PB ? g : H - 1 - g) : (PB ? H - 1 : 0);
    const bool first_row = g == 0;                       // path start of the vertical path
    const bool xin = r == 0 && s > 0;                    // vertical predecessor from the previous strip
    const bool xout = r == R - 1 && s + 1 < NS;          // publish the vertical L for the next strip
    const int ntiles = (W + TC - 1) / TC;
    const size_t npix = (size_t)H * W;
    const size_t rowe = ((size_t)b * npix + (size_t)v * W) * D;   // element (b, v, 0, 0)
    const int rowbytes = W * D * 4;
    const __amdgpu_buffer_rsrc_t rC = buf_rsrc(a.vm + rowe, rowbytes);
    const __amdgpu_buffer_rsrc_t rA = buf_rsrc(a.acc + rowe, rowbytes);
    const __amdgpu_buffer_rsrc_t rL = buf_rsrc(a.l2v + rowe, rowbytes);
    const int vprev = PB ? v - 1 : v + 1;                // the previous strip's last row (xin)
    const __amdgpu_buffer_rsrc_t rX = buf_rsrc(a.acc + ((size_t)b * npix + (size_t)(xin ? vprev : v) * W) * D, rowbytes);
    const uint8_t* flrow = a.flags + (size_t)b * npix + (size_t)v * W;
    int16_t* drow = a.disp + (size_t)b * npix + (size_t)v * W;
    uint32_t* const prog_in = sync + SG2_SYNC_HDR + (size_t)b * NS + (s > 0 ? s - 1 : 0);
    uint32_t* const prog_out = sync + SG2_SYNC_HDR + (size_t)b * NS + s;
    const int dir_v = PB ? 1 : 0, dir_h = PB ? 3 : 2;    // direction-table indices (cpp:6207-6208)
    const float p1 = a.p1, p2 = a.p2;
    const float p1r = p1 / (float)a.redu, p2r = p2 / (float)a.redu;   // updateCost: P1 /= reduCoeffi1
    const uint32_t lo = (uint32_t)lane * K * 4;          // lane byte offset inside a pixel
    auto col = [&](int j) { return PB ? j : W - 1 - j; };   // column of step j

    // bounded wait for the previous strip's progress counter (wave-uniform)
    auto wait_prog = [&](uint32_t need) {
        for (int tries = 0;; tries++) {
            const uint32_t pv = (uint32_t)__builtin_amdgcn_readfirstlane(
                (int)__hip_atomic_load(prog_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (pv >= need) break;
            const uint32_t ab = (uint32_t)__builtin_amdgcn_readfirstlane(
                (int)__hip_atomic_load(&sync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (ab) break;
            if (tries >= SM_SGM2_SPIN) {
                __hip_atomic_store(&sync[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        // order only: the exchange loads below read through the caches (sc1)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };

    auto load = [&](Sg2Tile<K, TC>& t, int ti) {
        if (xin) wait_prog((uint32_t)min(ti + 1, ntiles));   // tile ti of the previous strip published
#pragma unroll
        for (int st = 0; st < TC; st++) {
            const int j = min(ti * TC + st, W - 1);
            const uint32_t off = (uint32_t)col(j) * D * 4 + lo;
            ldK<K, AUX_NT>(rC, off, t.c[st]);
            if (PB) {
                ldK<K, AUX_NT>(rA, off, t.a0[st]);
                ldK<K, AUX_NT>(rL, off, t.a2[st]);
            }
            if (xin) ldK<K, AUX_DEV>(rX, off, t.xv[st]);
            t.fl[st] = flrow[col(j)];
        }
    };

    float Lh[K];            // horizontal path: L of the previous step of this row
    float mh = 0.f;         // its minimum over d
#pragma unroll
    for (int k = 0; k < K; k++) Lh[k] = FLT_MAX;
    auto mn = [](float x, float y) { return SG ? fminf(x, y) : fmin_pos(x, y); };
    auto wmin = [&](const float* x) {
        float m = x[0];
#pragma unroll
        for (int k = 1; k < K; k++) m = mn(m, x[k]);
        return SG ? wave_min(m) : wave_min_pos(m);
    };
    // updateCost (h:2206-2280): L = C + min(min(Lp - m, Lp[d-1] + (P1 - m)), min(Lp[d+1] + (P1 - m), P2))
    auto update = [&](const float* C, const float* Lp, float m, bool pen, float* L) {
        const float P1 = pen ? p1r : p1, P2 = pen ? p2r : p2;
        const float P1m = P1 - m;
        const float left = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, FLT_MAX),
                                                                                   __builtin_bit_cast(int, Lp[K - 1]), DPP_WAVE_SHR1, 0xF, 0xF, false));
        const float right = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, FLT_MAX),
                                                                                    __builtin_bit_cast(int, Lp[0]), DPP_WAVE_SHL1, 0xF, 0xF, false));
#pragma unroll
        for (int k = 0; k < K; k++) {
            const float prev = k == 0 ? left : Lp[k - 1];
            const float next = k == K - 1 ? right : Lp[k + 1];
            const float S1 = Lp[k] - m;
            const float S2 = prev + P1m;
            const float S3 = next + P1m;
            L[k] = C[k] + mn(mn(S1, S2), mn(S3, P2));
        }
    };

    int dacc = -1;   // lane st < TC: the disparity of the tile's step st (pass B)
    auto process = [&](const Sg2Tile<K, TC>& t, int ti, int p) {
        const float* xin_buf = r > 0 ? xch + ((size_t)((r - 1) * 2 + ((p - 1) & 1)) * TC) * 64 * K : nullptr;
        float* xout_buf = r < R - 1 ? xch + ((size_t)(r * 2 + (p & 1)) * TC) * 64 * K : nullptr;
#pragma unroll
        for (int st = 0; st < TC; st++) {
            const int j = ti * TC + st;
            if (j >= W) break;   // wave-uniform
            const uint32_t off = (uint32_t)col(j) * D * 4 + lo;
            const uint32_t fl = t.fl[st];
            // vertical path: the previous row's L of this column
            float Lv[K];
            if (first_row) {
#pragma unroll
                for (int k = 0; k < K; k++) Lv[k] = t.c[st][k];
            } else {
                float Lp[K];
                if (r > 0) {
#pragma unroll
                    for (int k = 0; k < K; k++) Lp[k] = xin_buf[st * 64 * K + lane * K + k];
                } else {
#pragma unroll
                    for (int k = 0; k < K; k++) Lp[k] = t.xv[st][k];
                }
                update(t.c[st], Lp, wmin(Lp), (fl >> dir_v) & 1u, Lv);
            }
            // horizontal path: this row's previous step
            float Lq[K];
            if (j == 0) {
#pragma unroll
                for (int k = 0; k < K; k++) Lq[k] = t.c[st][k];
            } else {
                update(t.c[st], Lh, mh, (fl >> dir_h) & 1u, Lq);
            }
#pragma unroll
            for (int k = 0; k < K; k++) Lh[k] = Lq[k];
            if (r < R - 1) {
#pragma unroll
                for (int k = 0; k < K; k++) xout_buf[st * 64 * K + lane * K + k] = Lv[k];
            }
            if (!PB) {
                float f[K];
#pragma unroll
                for (int k = 0; k < K; k++) f[k] = 0.f + Lv[k];   // sum = 0; sum += L0 (cpp:2046-2049)
                if (xout)
                    stK<K, AUX_DEV>(rA, off, f);                   // also the next strip's input
                else
                    stK<K, AUX_NT>(rA, off, f);
                stK<K, AUX_NT>(rL, off, Lq);
            } else {
                float f[K];
#pragma unroll
                for (int k = 0; k < K; k++) {
                    float x = t.a0[st][k] + Lv[k];   // acc + L1
                    x = x + t.a2[st][k];             // + L2
                    f[k] = x + Lq[k];                // + L3
                }
                if (KEEP) stK<K, AUX_NT>(rC, off, f);
                if (xout) stK<K, AUX_DEV>(rA, off, Lv);   // the next strip's input (acc entry read above)
                // WTA (cpp:3928-3967): first strict minimum over d
                float bm = f[0];
                int bi = lane * K;
#pragma unroll
                for (int k = 1; k < K; k++)
                    if (bm > f[k]) {
                        bm = f[k];
                        bi = lane * K + k;
                    }
                const float wm = SG ? wave_min(bm) : wave_min_pos(bm);
                const uint64_t hit = __ballot(bm == wm);
                const int widx = __builtin_amdgcn_readlane(bi, (int)__builtin_ctzll(hit));
                const int dsel = (wm < FLT_MAX) ? widx : -1;
                dacc = (lane == st) ? dsel : dacc;
            }
            mh = wmin(Lq);
        }
        if (PB && lane < TC && ti * TC + lane < W) drow[col(ti * TC + lane)] = (int16_t)dacc;
        if (xout) {
            // publish tile ti: every store of this wave (the sc1 exchange row included) completes
            // first, then the counter (device-scope atomic store)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_s_waitcnt(0 | (0x7 << 4) | (0xf << 8));   // vmcnt(0)
            if (lane == 0) __hip_atomic_store(prog_out, (uint32_t)(ti + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };

    // phases: wave r processes tile p - r; tile t + 1's loads are issued while tile t is processed
    Sg2Tile<K, TC> ta, tb;
    if (r == 0 && rvalid) load(ta, 0);
    const int nphase = ntiles + R - 1;
    auto phase = [&](Sg2Tile<K, TC>& cur, Sg2Tile<K, TC>& nxt, int p) {
        const int ti = p - r;
        if (rvalid && ti >= -1 && ti + 1 < ntiles) load(nxt, ti + 1);
        if (rvalid && ti >= 0 && ti < ntiles) process(cur, ti, p);
        __syncthreads();
    };
    for (int p = 0; p < nphase; p += 2) {
        phase(ta, tb, p);
        if (p + 1 < nphase) phase(tb, ta, p + 1);
    }
}

template <int K, bool PB, bool SG, bool KEEP>
void launch_k2(const Sgm2Args& a, hipStream_t st) {
    constexpr int R = SM_SGM2_R, TC = SM_SGM2_TC;
    const int NS = (a.H + R - 1) / R;
    const size_t shm = (size_t)(R - 1) * 2 * TC * 64 * K * 4;
    hipLaunchKernelGGL((k_sgm2<K, R, TC, PB, SG, KEEP>), dim3(a.n * NS), dim3(64 * R), shm, st, a);
}

template <int K>
void launch_pass(const Sgm2Args& a, bool pass_b, hipStream_t st) {
    if (!pass_b) {
        if (a.signed_costs) launch_k2<K, false, true, false>(a, st);
        else launch_k2<K, false, false, false>(a, st);
    } else if (a.keep_final) {
        if (a.signed_costs) launch_k2<K, true, true, true>(a, st);
        else launch_k2<K, true, false, true>(a, st);
    } else {
        if (a.signed_costs) launch_k2<K, true, true, false>(a, st);
        else launch_k2<K, true, false, false>(a, st);
    }
}

}  // namespace

bool sgm2_supported(int D, int paths) { return paths == 4 && (D == 64 || D == 128 || D == 256); }
size_t sgm2_sync_words(int H, int n) { return SG2_SYNC_HDR + (size_t)n * ((H + SM_SGM2_R - 1) / SM_SGM2_R); }

hipError_t launch_sgm2_pass(const Sgm2Args& a, bool pass_b, hipStream_t st) {
    // the ticket, the abort flag and every strip's progress start at 0 (the abort flag is kept:
    // a pass after an aborted one must not run on its half-written volumes)
    hipError_t e = hipMemsetAsync(a.sync, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(a.sync + SG2_SYNC_HDR, 0, (sgm2_sync_words(a.H, a.n) - SG2_SYNC_HDR) * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    switch (a.D / 64) {
        case 1: launch_pass<1>(a, pass_b, st); break;
        case 2: launch_pass<2>(a, pass_b, st); break;
        default: launch_pass<4>(a, pass_b, st); break;
    }
    return hipGetLastError();
}

}  // namespace sm
