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

#include <type_traits>

#include "sm_device.h"
#include "sm_kernels.h"

#ifndef SM_SGM2_R
#define SM_SGM2_R 8          // rows (waves) per strip
#endif
#ifndef SM_SGM2_TC
#define SM_SGM2_TC 2         // columns per tile (= the skew between consecutive rows)
#endif
#ifndef SM_SGM2_PF
#define SM_SGM2_PF 3         // tiles whose loads are in flight ahead of the one processed (<= 5), pass A
#endif
#ifndef SM_SGM2_PF_B
#define SM_SGM2_PF_B 2       // the same for pass B (three volumes per tile: <= 128 VGPRs, two blocks per CU)
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
};

// s_waitcnt with vmcnt(n) only (expcnt / lgkmcnt left at their maxima)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}
__device__ __forceinline__ void compiler_fence() { __asm__ __volatile__("" ::: "memory"); }

template <int K, int R, int TC, int PF, bool PB, bool SG, bool KEEP>
__global__ __launch_bounds__(64 * R) void k_sgm2(const Sgm2Args a) {
    constexpr int NB = PF + 1;                         // tiles in the register ring
    constexpr int NLT = TC * (PB ? 3 : 1);             // vector-memory loads per tile (C [+ acc, l2v])
    extern __shared__ float xch[];   // [R - 1][2][TC][64 K] vertical L from wave r to r + 1, then the flags
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
    int16_t* drow = a.disp + (size_t)b * npix + (size_t)v * W;
    uint32_t* const prog_in = sync + SG2_SYNC_HDR + (size_t)b * NS + (s > 0 ? s - 1 : 0);
    uint32_t* const prog_out = sync + SG2_SYNC_HDR + (size_t)b * NS + s;
    const int dir_v = PB ? 1 : 0, dir_h = PB ? 3 : 2;    // direction-table indices (cpp:6207-6208)
    const float p1 = a.p1, p2 = a.p2;
    const float p1r = p1 / (float)a.redu, p2r = p2 / (float)a.redu;   // updateCost: P1 /= reduCoeffi1
    const uint32_t lo = (uint32_t)lane * K * 4;          // lane byte offset inside a pixel
    auto col = [&](int j) { return PB ? j : W - 1 - j; };   // column of step j

    // the row's penalty flags (two bits: this pass's vertical and horizontal directions) in LDS,
    // so that no flag load joins the counted vector-memory loads of the tiles
    uint8_t* const flg = (uint8_t*)(xch + (size_t)(R - 1) * 2 * TC * 64 * K) + (size_t)r * ((W + 3) & ~3);
    if (rvalid) {
        const __amdgpu_buffer_rsrc_t rF = buf_rsrc(a.flags + (size_t)b * npix + (size_t)v * W, W);
        for (int i = lane * 4; i < W; i += 256) {
            if (i + 4 <= W) {   // (a dword reaching past the resource's range would read as 0)
                *(uint32_t*)(flg + i) = __builtin_amdgcn_raw_buffer_load_b32(rF, i, 0, 0);
            } else {
                for (int k = i; k < W; k++) flg[k] = __builtin_amdgcn_raw_buffer_load_b8(rF, k, 0, 0);
            }
        }
        wait_vm<0>();
    }

    // The previous strip's progress as last seen, and an asynchronous poll of it issued at the
    // start of every phase (before the phase's other loads) and read when a tile's values are
    // needed, so that the counter's round trip overlaps the phase instead of stalling it.
    uint32_t seen = 0;
    uint32_t poll_v = 0;
    bool poll_out = false;
    auto poll_issue = [&]() {
        if (!poll_out) {
            poll_v = __hip_atomic_load(prog_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            poll_out = true;
        }
    };
    // bounded wait for the previous strip's progress counter (wave-uniform)
    auto wait_prog = [&](uint32_t need) {
        if (seen >= need) return;
        if (poll_out) {
            seen = max(seen, (uint32_t)__builtin_amdgcn_readfirstlane((int)poll_v));
            poll_out = false;
            if (seen >= need) {
                compiler_fence();
                return;
            }
        }
        for (int tries = 0;; tries++) {
            const uint32_t pv = (uint32_t)__builtin_amdgcn_readfirstlane(
                (int)__hip_atomic_load(prog_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            seen = pv;
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
        compiler_fence();   // the exchange loads below read through the caches (sc1)
    };
    auto load = [&](Sg2Tile<K, TC>& t, int ti) {   // NLT loads (clamped past the row end)
#pragma unroll
        for (int st = 0; st < TC; st++) {
            const uint32_t off = (uint32_t)col(min(ti * TC + st, W - 1)) * D * 4 + lo;
            ldK<K, AUX_NT>(rC, off, t.c[st]);
            if (PB) {
                ldK<K, AUX_NT>(rA, off, t.a0[st]);
                ldK<K, AUX_NT>(rL, off, t.a2[st]);
            }
        }
    };
    auto load_x = [&](Sg2Tile<K, TC>& t, int ti) {   // the previous strip's values of tile ti
        wait_prog((uint32_t)(ti + 1));
#pragma unroll
        for (int st = 0; st < TC; st++)
            ldK<K, AUX_DEV>(rX, (uint32_t)col(min(ti * TC + st, W - 1)) * D * 4 + lo, t.xv[st]);
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
            const uint32_t fl = flg[col(j)];
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
    };

    // Phases: wave r processes its tile q in phase q + r (one barrier per phase: wave r first
    // passes r idle phases, then its ntiles tiles, then R - 1 - r idle phases).  A tile's loads
    // are issued PF tiles ahead, after the stores of the tile just processed, so that the
    // publishing wave can wait for its exchange stores (vmcnt counts in issue order) without
    // waiting for the prefetches: it raises its progress counter for tile q - 1 at the start of
    // tile q's phase.  The first wave of a later strip fetches the previous strip's values one
    // tile ahead, before the prefetches.
    Sg2Tile<K, TC> tl[NB];
    if (rvalid) {
#pragma unroll
        for (int q = 0; q < PF; q++)
            if (q < ntiles) load(tl[q], q);
        if (xin) load_x(tl[0], 0);
    }
    for (int i = 0; i < r; i++) __syncthreads();
    bool pending = false;   // xout: tile q - 1's exchange stores issued, counter not raised yet
    int pend_loads = 0;     // loads issued after those stores
    auto publish = [&](int q) {
        if (!pending) return;
        if (pend_loads) wait_vm<NLT>();   // the exchange stores, not the NLT prefetch loads after them
        else wait_vm<0>();
        compiler_fence();
        if (lane == 0) __hip_atomic_store(prog_out, (uint32_t)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pending = false;
    };
    auto step_q = [&](auto SLOT, int q) {
        constexpr int sl = decltype(SLOT)::value;
        const int p = q + r;
        if (rvalid) {
            if (xout) publish(q);
            if (xin) poll_issue();
            process(tl[sl], q, p);
            compiler_fence();
            if (xin && q + 1 < ntiles) load_x(tl[(sl + 1) % NB], q + 1);
            const bool more = q + PF < ntiles;
            if (more) load(tl[(sl + PF) % NB], q + PF);
            if (xout) {
                pending = true;
                pend_loads = more ? NLT : 0;
            }
        }
        __syncthreads();
    };
    for (int q0 = 0; q0 < ntiles; q0 += NB) {
        step_q(std::integral_constant<int, 0>{}, q0);
#define SG2_SLOT(I) \
        if constexpr (NB > I) { if (q0 + I < ntiles) step_q(std::integral_constant<int, I>{}, q0 + I); }
        SG2_SLOT(1)
        SG2_SLOT(2)
        SG2_SLOT(3)
        SG2_SLOT(4)
        SG2_SLOT(5)
#undef SG2_SLOT
    }
    if (rvalid && xout) publish(ntiles);
    for (int i = r + 1; i < R; i++) __syncthreads();
}

template <int K, bool PB, bool SG, bool KEEP>
void launch_k2(const Sgm2Args& a, hipStream_t st) {
    constexpr int R = SM_SGM2_R, TC = SM_SGM2_TC, PF = PB ? SM_SGM2_PF_B : SM_SGM2_PF;
    const int NS = (a.H + R - 1) / R;
    const size_t shm = (size_t)(R - 1) * 2 * TC * 64 * K * 4 + (size_t)R * ((a.W + 3) & ~3);
    hipLaunchKernelGGL((k_sgm2<K, R, TC, PF, PB, SG, KEEP>), dim3(a.n * NS), dim3(64 * R), shm, st, a);
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

// D = 64 K (K = 1, 2, 4); the row's flags live in LDS next to the hand-over buffers (W <= 8192)
bool sgm2_supported(int D, int paths, int W) { return paths == 4 && (D == 64 || D == 128 || D == 256) && W <= 8192; }
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
