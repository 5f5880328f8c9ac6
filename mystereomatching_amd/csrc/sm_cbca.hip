// sm_cbca.hip — cross-based cost aggregation (CBCA) as fused, prefetched line sweeps.
//
// Reference: cbca_core (stereoMatching.cpp:5585-5666) runs per iteration two 1-D passes, each
//   gen1DCumu   (cpp:3896-3926)  S[i] = S[i-1] + x[i]              (sequential prefix, in place)
//   cal1DCost   (h:1643-1715)    out[i] = S[i+head] - S[i-tail-1]  (or S[i+head] at the border)
// with the left/right intersection arms (genTrueHorVerArms, cpp:2794-2845), then divides by the
// integer support area (genfinalVm_cbca, cpp:3969-3992).  Iteration 0 runs H then V, iteration 1
// V then H, so the pass sequence for 2 iterations is  H-scan | V-norm, V-scan | H-norm.
//
// gfx950 mapping.  One wave owns one (line, 64-disparity chunk); lane = disparity.  The prefix
// sum is evaluated sequentially along the line exactly as the reference does, and its values are
// kept in an LDS ring, so each 1-D pass is ONE read and ONE write of the volume (the reference:
// two reads, two writes and a full-volume temporary).  Kernel modes:
//   CB_SCAN       first pass of an iteration:            vm <- diff(prefix(vm))
//   CB_NORM       last pass of an iteration:             vm <- diff(prefix(vm)) / area  [* SolveAll]
//   CB_NORM_SCAN  last pass of iteration k fused with the first pass of iteration k+1 (both run
//                 along the same direction): two S rings, one sweep instead of two.
// Areas are integers (< 2^16): after the first pass of an iteration the area of (p,d) is
// tail+head+1 of that pass's intersection arms, so the normalising pass prefix-sums that value
// modulo 2^16 in a u16 ring next to S — no area volume is ever stored.
//
// Instruction budget (the sweeps are issue-bound at 3-6 waves per CU):
//  * arms are stored as two u16-pair planes per pixel, (L | R<<16) and (U | D<<16), so the
//    intersection of a pair is one v_pk_min_u16 against the uniform reference-pixel word;
//  * H sweeps: the pixel's own arm pair of a tile position is a broadcast LDS read; the other
//    image's pair of lane d at position q is A1[q - d] (left view) / A1[q + d] (right view), a
//    window that shifts by one word per position, kept in a mirrored LDS ring (one lane-vector
//    load of the tile's T new words per set);
//  * V sweeps: the own pair comes by v_readlane from the tile's lane-vector load, the other
//    image's pairs (column u -/+ d of each row) are register gathers;
//  * ring slots of a window's two ends are one packed u16 pair and each LDS address one
//    v_mad_u32_u16 (see slot_pair / ring_at).
// Scheduling: the next PF tiles of T positions (volume values, arm words) are loaded while the
// current tile is processed; inside a tile all ring writes precede all ring reads, so a tile
// costs one LDS round trip per stage.  Rings hold 2*lag + T + 1 slots rounded up to a multiple of T.
//
// Rejected designs (same-process A/B) live as patches in tools/experiments/:
// workgroup-staged V arm words, several waves / columns per block, persistent V sweeps, a per-tile
// safe-dividend test, and the timing probes that located the V gathers' cost.
#include <float.h>
#include <algorithm>
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

namespace sm {

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pkmin(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(us2, a), __builtin_bit_cast(us2, b)));
}

// Positions per tile (T) and tiles prefetched ahead (PF), chosen by same-box sweeps
// (tools/build_variants.sh).  Scans: T = 24, one tile ahead.  Normalising sweeps: T = 10 with two
// tiles in flight — their rings (2 lag + T + 1 slots of S plus a u16 area ring) then fit five
// waves per CU instead of four (Teddy x16: h_norm 0.459 -> 0.425 ms, v_norm 0.505 -> 0.480 ms).
// NORM_SCAN: T = 12, two (H) / three (V) tiles in flight, fastest among T = 6-20, PF = 1-3
// (profiles/r3c, r3i): full resolution v_norm + v_scan 12.20 -> 11.09 ms fused.
#ifndef SM_CB_T_SCAN_H
#define SM_CB_T_SCAN_H 24
#endif
#ifndef SM_CB_T_SCAN_V
#define SM_CB_T_SCAN_V 24
#endif
#ifndef SM_CB_T_NORM_H
#define SM_CB_T_NORM_H 10
#endif
#ifndef SM_CB_T_NORM_V
#define SM_CB_T_NORM_V 10
#endif
#ifndef SM_CB_T_NS
#define SM_CB_T_NS 12
#endif
#ifndef SM_CB_PF_SCAN_H
#define SM_CB_PF_SCAN_H 1
#endif
#ifndef SM_CB_PF_SCAN_V
#define SM_CB_PF_SCAN_V 1
#endif
#ifndef SM_CB_PF_NORM_H
#define SM_CB_PF_NORM_H 2
#endif
#ifndef SM_CB_PF_NORM_V
#define SM_CB_PF_NORM_V 2
#endif
#ifndef SM_CB_PF_NS_H
#define SM_CB_PF_NS_H 2
#endif
#ifndef SM_CB_PF_NS_V
#define SM_CB_PF_NS_V 3
#endif

// v_mad_u32_u16 with op_sel: a.half * b.lo + c (one VALU per ring address)
template <int HI>
__device__ __forceinline__ uint32_t mad_u32_u16(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    if (HI)
        asm("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    else
        asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}

// H sweeps: mirrored span ring of R = 63 + T words per set (every word written at i and i + R),
// so a read at start + offset never wraps; a tile loads only its T new words.
__host__ __device__ constexpr int cbca_win_ring(int T) { return 63 + T; }
__host__ __device__ constexpr int cbca_tile(bool horiz, int mode) {
    return mode == CB_SCAN ? (horiz ? SM_CB_T_SCAN_H : SM_CB_T_SCAN_V)
                           : (mode == CB_NORM ? (horiz ? SM_CB_T_NORM_H : SM_CB_T_NORM_V) : SM_CB_T_NS);
}

template <bool HORIZ, int MODE>
struct CbCfg {
    static constexpr int T = cbca_tile(HORIZ, MODE);
    static constexpr int PF = MODE == CB_SCAN ? (HORIZ ? SM_CB_PF_SCAN_H : SM_CB_PF_SCAN_V)
                                              : (MODE == CB_NORM ? (HORIZ ? SM_CB_PF_NORM_H : SM_CB_PF_NORM_V) : (HORIZ ? SM_CB_PF_NS_H : SM_CB_PF_NS_V));
    // arm sets: 0 = pass pair at i (= j - lag), 1 = perpendicular pair at j, 2 = pass pair at j - 2 lag
    static constexpr int NSETS = MODE == CB_SCAN ? 1 : (MODE == CB_NORM ? 2 : 3);
};

// ring slots: >= 2*lag + T + 1 (a whole tile is written before any of it is read) and a multiple
// of T (a tile's write slots never wrap)
__host__ __device__ inline int cbca_ring(int lag, bool horiz, int mode) {
    const int T = cbca_tile(horiz, mode);
    return (2 * lag + T + 1 + T - 1) / T * T;
}
// dynamic LDS in 4-byte words: S ring(s) of ring x 64 floats, then the u16 area ring (6 bytes
// per slot and lane; 8-byte {S, area} records were measured slower: one wave less per CU), then
// (H sweeps) the staged arm words of one tile: per set T own words and the mirrored span ring
__host__ __device__ inline int cbca_ring_words(int lag, bool horiz, int mode) {
    const int ring = cbca_ring(lag, horiz, mode);
    const int floats = mode == CB_NORM_SCAN ? 2 : 1;
    const int u16s = mode == CB_SCAN ? 0 : 1;
    return ring * 64 * floats + ring * 32 * u16s;
}
__host__ __device__ inline int cbca_win_words(bool horiz, int mode) {
    if (!horiz) return 0;   // V sweeps: own words by v_readlane, gathers in registers
    const int T = cbca_tile(horiz, mode);
    const int nsets = mode == CB_SCAN ? 1 : (mode == CB_NORM ? 2 : 3);
    return nsets * (T + 2 * cbca_win_ring(T));
}
__host__ __device__ inline int cbca_smem_words(int lag, bool horiz, int mode) {
    return cbca_ring_words(lag, horiz, mode) + cbca_win_words(horiz, mode);
}

template <bool HORIZ, int T, int NSETS>
struct CbTile {
    float x[T];                        // vm at positions j0 .. j0+T-1
    uint32_t a0[NSETS];                // lane k < T: own arm pair at position (j0 + k - off)
    uint32_t a1w[HORIZ ? NSETS : 1];   // H: lane k < T: the span ring's k-th new word
    uint32_t a1[HORIZ ? 1 : NSETS][T]; // V: other image's arm pair at (row j0 + k - off, u -/+ d)
};

// RV: the right view's volume vm[1] (cbca_core's LOR = 1, run when Do_refine): the pixel's own
// arms are the right image's, and lane d pairs them with the LEFT image's arms at u + d
// (HVL_INTERSECTION[1], cpp:2794-2845) — zero once u + d >= W.
template <bool HORIZ, int MODE, bool FULL, bool SCALE, bool RV, int LAGC = 0>
struct CbLine {
    static constexpr int T = CbCfg<HORIZ, MODE>::T;
    static_assert(T <= 64, "a line's own arm words of a tile are one lane each");
    static constexpr int NSETS = CbCfg<HORIZ, MODE>::NSETS;
    using Tile = CbTile<HORIZ, T, NSETS>;
    // REUSE2 (V NORM_SCAN at the reference's lag, a compile-time LAGC): the scan stage's pass
    // intersection at position j is the norm stage's at j - lag (both are the pass pair of row
    // j - 2 lag), so the sweep keeps the last four tiles' norm intersections in registers and
    // drops the third set's own-arm load, readlane, pkmin and 64-word gather per position
    // (full resolution 11.15 -> 9.91 ms, profiles/r3l, r3m).
    static constexpr bool REUSE2 = LAGC > 0 && !HORIZ && MODE == CB_NORM_SCAN;
    // RING8 (H NORM at the reference's lag, a compile-time LAGC): the ring holds 8 tiles
    // (2 lag + T + 1 = 79 -> 80 slots at T = 10), so an 8-tile loop knows every tile's ring slots at
    // compile time: the window slots of position k are (constant - tail - 1, constant + head),
    // with no per-position scalar wrap (4 SALU per position) and no ws bookkeeping
    static constexpr bool RING8 = LAGC > 0 && HORIZ && MODE == CB_NORM &&
                                  (2 * LAGC + T + 1 + T - 1) / T * T == 8 * T;
    static_assert(!REUSE2 || (CbCfg<HORIZ, MODE>::PF == 3 && LAGC + T - 1 <= 4 * T),
                  "the history is the last four tiles of the four-tile loop");

    // Volume and V-sweep arm accesses are buffer instructions: the tile's first position in the
    // resource base, lane + k * stride in a loop-invariant VGPR.  Loads are not clamped: the
    // resource's range ends at the allocation's end (reads past it return 0; those positions are
    // never output) and the arm planes carry a 2 * lag row front pad for set positions < 0.
    const char* xline;        // byte address of (line, position 0, chunk's first disparity)
    const char* xend;         // end of the volume allocation
    const char* aend;         // end of the arm allocation
    uint32_t xo[T];           // lane's load offset of tile position k (lanes past D re-read D - 1)
    uint32_t ao[HORIZ ? 1 : T];  // V: lane's arm offset (column u -/+ d) of tile position k
    uint32_t ov;              // lane's store offset (lanes past D: out of range, dropped)
    uint32_t vsb;             // bytes between consecutive positions
    int lane;
    __amdgpu_buffer_rsrc_t A0r[NSETS];  // own-image arm-pair plane of each set over the line
    __amdgpu_buffer_rsrc_t A1r[NSETS];  // H: other-image plane over the line
    const char* A1v[NSETS];     // V: other-image plane, row 0 (uniform)
    int pstride, line, len, lag, ring;
    int c64;                  // first disparity of the chunk
    uint32_t* wown;           // H: own arm words of the tile, T per set
    uint32_t* wspan;          // H: the other image's mirrored span ring, 2 R per set
    float S1, S2;
    uint32_t Acc;
    int ws;                   // ring slot of the tile's first position
    int wrs;                  // span-ring slot of the current tile's first word (j0 mod R)
    float* r1;
    float* r2;
    uint16_t* ra;
    uint32_t o1, o2, oa;      // LDS address of this lane's slot-0 entry in r1, r2, ra
    float scale;
    uint32_t ph[REUSE2 ? 4 : 1][REUSE2 ? T : 1];   // REUSE2: pass intersections of the last 4 tiles

    __device__ __forceinline__ int set_off(int s) const { return s == 0 ? lag : (s == 1 ? 0 : 2 * lag); }

    // resource for the tile whose first position is pos0 (may lie before the line: only
    // positions inside it are ever stored)
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(int pos0) const {
        return buf_rsrc(xline + (long)pos0 * (long)vsb);
    }
    __device__ __forceinline__ static __amdgpu_buffer_rsrc_t bounded_rsrc(const char* base, const char* end) {
        // the clamp of end - base to [0, 2^31 - 1] on 32-bit halves: 64-bit signed compares of
        // scalars would go through the VALU
        const long room = end - base;
        const int hi = (int)(room >> 32);
        const uint32_t lo = (uint32_t)room;
        const int range = hi < 0 ? 0 : ((hi > 0 || lo > 0x7fffffffu) ? 0x7fffffff : (int)lo);
        return buf_rsrc(base, range);
    }
    // `in` false: an out-of-range offset (the store is dropped), so that guarded and unguarded
    // tiles issue the same vector-memory sequence and the loops' vmcnt waits stay exact
    __device__ __forceinline__ void store_tile(const __amdgpu_buffer_rsrc_t& r, int k, float v, bool in = true) const {
        if (FULL)
            buf_st(r, in ? xo[k] : 0x80000000u, 0, v);
        else
            buf_st(r, in ? ov : 0x80000000u, (uint32_t)k * vsb, v);
    }

    // Tile loads: positions past the line end read the next line (or 0 past the allocation);
    // their prefix values are never read.
    // (MASK: bit 0 the volume rows, bit 1 + s arm set s; HN2's waves load their parts)
    template <int MASK = 0xff>
    __device__ __forceinline__ void load(Tile& t, int j0) const {
        const __amdgpu_buffer_rsrc_t rx = bounded_rsrc(xline + (long)j0 * (long)vsb, xend);
        if constexpr (MASK & 1) {
#pragma unroll
        for (int k = 0; k < T; k++)   // normalising sweeps: non-temporal volume loads (v_norm 0.466 -> 0.434 ms)
            t.x[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, (int)xo[k], 0, MODE == CB_SCAN ? SM_LD_AUX : 2));
        }
        // lane-vector arm loads: positions outside the line read 0 (an out-of-range offset) --
        // for the other image's arms that is the reference's zeroed intersection when u - d < 0.
        // The offset is a select, never a wrapped negative sum: the range check does not wrap,
        // and the compiler would otherwise move constant parts of a sum into the immediate field.
#pragma unroll
        for (int s = 0; s < NSETS; s++) {
            if (REUSE2 && s == 2) continue;
            if (!(MASK & (2 << s))) continue;
            const int base = j0 - set_off(s);
            // (only lanes k < T are read back; the others stay off the memory system, which
            // matters for the strided column loads of vertical sweeps)
            const int p0 = base + lane;
            t.a0[s] = buf_ld_u32(A0r[s], (lane < T && (unsigned)p0 < (unsigned)len) ? (uint32_t)(p0 * pstride) * 4u : 0x80000000u, 0);
            if constexpr (HORIZ) {
                // the other image's arm pairs that lanes c64 .. c64 + 63 pair with at positions
                // base .. base + T - 1: left view q = p - d in [base - c64 - 63, base - c64 + T - 1],
                // right view q = p + d in [base + c64, base + c64 + 63 + T - 1]; 0 outside the line.
                // The tile's T new words are q0 + 63 .. q0 + 62 + T.
                const int q0 = RV ? base + c64 : base - c64 - 63;
                const int qn = q0 + 63 + lane;
                t.a1w[s] = buf_ld_u32(A1r[s], (lane < T && (unsigned)qn < (unsigned)len) ? (uint32_t)qn * 4u : 0x80000000u, 0);
            } else {
                const __amdgpu_buffer_rsrc_t ra1 = bounded_rsrc(A1v[s] + (long)base * (long)(pstride * 4), aend);
#pragma unroll
                for (int k = 0; k < T; k++) t.a1[s][k] = __builtin_amdgcn_raw_buffer_load_b32(ra1, (int)ao[k], 0, 0);
            }
        }
    }

    // intersection arm pair of set s at tile position k
    __device__ __forceinline__ uint32_t isect(const Tile& t, int s, int k) const {
        if constexpr (!HORIZ) {
            const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)t.a0[s], k);
            return pkmin(a0, t.a1[s][k]);
        } else {
            constexpr int R = cbca_win_ring(T);
            const uint32_t a0 = wown[s * T + k];   // broadcast read
            const uint32_t a1 = wspan[s * 2 * R + wrs + (RV ? k + lane : k + 63 - lane)];
            return pkmin(a0, a1);
        }
    }
    // H sweeps: stage the tile's arm words in LDS (one wave: its LDS accesses complete in order)
    __device__ __forceinline__ void stage(const Tile& t) {
        if constexpr (HORIZ) {
            constexpr int R = cbca_win_ring(T);
#pragma unroll
            for (int s = 0; s < NSETS; s++) {
                if (lane < T) wown[s * T + lane] = t.a0[s];
                uint32_t* sp = wspan + s * 2 * R;
                const int w = wrs + 63 + lane;           // < 2 R
                const int i = w >= R ? w - R : w;
                if (lane < T) {
                    sp[i] = t.a1w[s];
                    sp[i + R] = t.a1w[s];
                }
            }
        }
    }

    __device__ __forceinline__ int uwrap(int s) const {  // uniform slot, any s in (-2 ring, 3 ring)
        s = s < 0 ? s + ring : s;
        s = s < 0 ? s + ring : s;
        s = s >= ring ? s - ring : s;
        return s >= ring ? s - ring : s;
    }
    // (tail slot | head slot << 16) of intersection pair p at uniform slot c < 2 ring: with
    // p = (tail | head << 16), (p ^ 0xffff) + (c, c) is (c - tail - 1, c + head) modulo 2^16, and
    // one packed add of (ring, -ring) plus a packed minimum wraps both ends into [0, ring)
    __device__ __forceinline__ uint32_t slot_pair(uint32_t p, int c) const {
        c = c >= ring ? c - ring : c;   // c < 2 ring: then c + head < 2 ring, c - tail - 1 > -ring
        const us2 q = __builtin_bit_cast(us2, p ^ 0xffffu) + us2{(unsigned short)c, (unsigned short)c};
        const us2 w = q + us2{(unsigned short)ring, (unsigned short)(-ring)};
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(q, w));
    }
    // slot_pair for a compile-time slot c < ring of an 8-tile ring (RING8): one packed add of the
    // constant (c, c), the wrap of both ends as in slot_pair
    __device__ __forceinline__ uint32_t slot_pair_c(uint32_t p, int c) const {
        constexpr int RINGC = 8 * T;
        const us2 q = __builtin_bit_cast(us2, p ^ 0xffffu) + us2{(unsigned short)c, (unsigned short)c};
        const us2 w = q + us2{(unsigned short)RINGC, (unsigned short)(-RINGC)};
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(q, w));
    }
    // LDS element of a ring of 4-byte / 2-byte entries at slot = half H_ of sp, for this lane;
    // RG: 0 = r1, 1 = r2 (floats), 2 = ra (u16).  One v_mad_u32_u16 of the half with the ring's
    // bytes per slot and the lane's slot-0 address.
    template <int H_, int RG, typename E = typename std::conditional<RG == 2, uint16_t, float>::type>
    __device__ __forceinline__ E ring_at(uint32_t sp) const {
        const uint32_t o = RG == 2 ? oa : (RG == 1 ? o2 : o1);
        // (an integer LDS address cast to an LDS pointer: no base add in front of the read)
        typedef __attribute__((address_space(3))) const E lds_e;
        return *(lds_e*)(size_t)mad_u32_u16<H_>(sp, 64u * (uint32_t)sizeof(E), o);
    }

    // (last pass only) SolveAll's `sum = 0; sum += w * v` (cpp:2189-2201): 0 + x == x for every
    // x except -0, and no CBCA value is ever -0 (costs are >= +0, prefix sums of them too, and
    // x - x rounds to +0), so the add is dropped.
    __device__ __forceinline__ float finish_norm(float q) const { return SCALE ? scale * q : q; }

    // ---------------- one tile of T positions, branch-free ------------------------------------
    // Every tile runs the same straight-line code.  Inputs past the line end are clamped loads
    // whose prefix values are never read (heads stop at the border); positions before the line
    // start read the zeroed ring, which is exactly the reference's border case
    // out = S[i + head] (cal1DCost, h:1643-1715).  Only the two ends of a line (GUARD) test
    // whether an output position exists before storing it.
    template <bool GUARD, int R, int RC = -1>
    __device__ __forceinline__ void tile(const Tile& t, int j0) {
        uint32_t pi[T], pi2[T];
        // ring % T == 0 and ws % T == 0, so the tile's write slots ws .. ws+T-1 never wrap
        // (RC >= 0: the tile's slot in the 8-tile ring cycle, all slots compile-time constants)
        constexpr int RINGC = 8 * T;
        const int wsv = RC >= 0 ? RC * T : ws;
        float* w1 = r1 + wsv * 64 + lane;
        uint16_t* wa = ra + wsv * 64 + lane;
        const int si0 = RC >= 0 ? (RC * T - LAGC + 2 * RINGC) % RINGC : uwrap(ws - lag);   // slot of i = j0 - lag
        // (NORM_SCAN: r2 holds position p's S2 at slot (p + lag) mod ring, so the tile's S2 writes
        // are slots ws .. ws + T - 1 and the slot of i2 = j0 - 2 lag in r2 is si0)
        const int i0 = j0 - lag;
        const __amdgpu_buffer_rsrc_t ob = tile_rsrc(i0);
        stage(t);
        // phase A: inputs j0 .. j0+T-1 (+ arm windows)
#pragma unroll
        for (int k = 0; k < T; k++) {
            S1 = S1 + t.x[k];
            w1[k * 64] = S1;
            pi[k] = isect(t, 0, k);
            if (MODE != CB_SCAN) {
                const uint32_t pp = isect(t, 1, k);
                // only Acc mod 2^16 is ever read (u16 ring): Acc + pp + 1 adds lo + 1 (and hi << 16),
                // the dot adds lo + hi exactly; one udot2 + one add instead of shift, add, add3
                Acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, pp), us2{1, 1}, Acc, false) + 1u;
                wa[k * 64] = (uint16_t)Acc;
            }
            if (MODE == CB_NORM_SCAN && !REUSE2) pi2[k] = isect(t, 2, k);
        }
        if constexpr (REUSE2) {
            // position j0 + k - LAGC lies in tile R + dt (dt < 0) at index k - LAGC - dt T
#pragma unroll
            for (int k = 0; k < T; k++) {
                const int q = k - LAGC;
                const int dt = -((-q + T - 1) / T);
                pi2[k] = ph[(R + dt + 8) & 3][q - dt * T];
            }
#pragma unroll
            for (int k = 0; k < T; k++) ph[R][k] = pi[k];
        }
        // phase B: first-stage outputs at i = j - lag (reads batched, then arithmetic)
        float shv[T], stv[T];
        uint32_t ahv[T], atv[T];
#pragma unroll
        for (int k = 0; k < T; k++) {
            const uint32_t sp = RC >= 0 ? slot_pair_c(pi[k], (si0 + k) % RINGC)
                                        : slot_pair(pi[k], si0 + k);   // slots of i - tail - 1, i + head
            shv[k] = ring_at<1, 0>(sp);
            stv[k] = ring_at<0, 0>(sp);
            if (MODE != CB_SCAN) {
                ahv[k] = ring_at<1, 2>(sp);
                atv[k] = ring_at<0, 2>(sp);
            }
        }
        if (MODE == CB_SCAN) {
#pragma unroll
            for (int k = 0; k < T; k++)
                store_tile(ob, k, shv[k] - stv[k], !GUARD || (unsigned)(i0 + k) < (unsigned)len);
        } else {
            // genfinalVm_cbca's division (cpp:3969-3992) by the integer area, through div_area
            // (sm_device.h); tiles holding a dividend below its proven range redo the IEEE
            // division (a uniform branch that never runs on real costs)
            float dv[T], qv[T];
            uint32_t av[T];
#pragma unroll
            for (int k = 0; k < T; k++) {
                dv[k] = shv[k] - stv[k];
                av[k] = (ahv[k] - atv[k]) & 0xffffu;
                qv[k] = div_area(dv[k], av[k]);
            }
            // dividends are >= +0 (prefix sums of costs >= 0; S - S = +0), so "0 < dv < 2^-110"
            // is "bits(dv) - 1 < 0x087fffff" (unsigned); the tile's minimum of bits - 1 decides it
            uint32_t tmin = 0xffffffffu;
#pragma unroll
            for (int k = 0; k < T; k++) tmin = min(tmin, __builtin_bit_cast(uint32_t, dv[k]) - 1u);
            if (__ballot(tmin < 0x087fffffu)) {
#pragma unroll
                for (int k = 0; k < T; k++) qv[k] = dv[k] / (float)av[k];
            }
#pragma unroll
            for (int k = 0; k < T; k++) {
                if (MODE == CB_NORM) {
                    store_tile(ob, k, finish_norm(qv[k]), !GUARD || (unsigned)(i0 + k) < (unsigned)len);
                } else {
                    float y = qv[k];                              // final value of iteration k at i
                    if (GUARD) y = (i0 + k >= 0) ? y : 0.f;       // nothing accumulates before the line
                    S2 = S2 + y;                                  // prefix of iteration k+1's first pass
                    r2[(ws + k) * 64 + lane] = S2;
                }
            }
        }
        // phase C (NS): second-stage outputs at i2 = j - 2 lag
        if (MODE == CB_NORM_SCAN) {
            float s2h[T], s2t[T];
#pragma unroll
            for (int k = 0; k < T; k++) {
                const uint32_t sp = slot_pair(pi2[k], si0 + k);
                s2h[k] = ring_at<1, 1>(sp);
                s2t[k] = ring_at<0, 1>(sp);
            }
            const int i20 = j0 - 2 * lag;
            const __amdgpu_buffer_rsrc_t ob2 = tile_rsrc(i20);
#pragma unroll
            for (int k = 0; k < T; k++)
                store_tile(ob2, k, s2h[k] - s2t[k], !GUARD || (unsigned)(i20 + k) < (unsigned)len);
        }
        if (RC < 0) ws = (ws + T == ring) ? 0 : ws + T;
        wrs = (wrs + T >= cbca_win_ring(T)) ? wrs + T - cbca_win_ring(T) : wrs + T;
    }

    // ---- HN2: H NORM at the reference's lag as two waves per line (RING8's 8-tile ring cycle) ----
    // Each wave stages (and reads) only its own arm set's words: set 0 (pass pairs, stage B) on the
    // second wave, set 1 (perpendicular pairs, the area) on the first; the S1 / area rings are shared.
    template <int S>
    __device__ __forceinline__ void stage_set(const Tile& t) {
        constexpr int R = cbca_win_ring(T);
        if (lane < T) wown[S * T + lane] = t.a0[S];
        uint32_t* sp = wspan + S * 2 * R;
        const int w = wrs + 63 + lane;
        const int i = w >= R ? w - R : w;
        if (lane < T) {
            sp[i] = t.a1w[S];
            sp[i + R] = t.a1w[S];
        }
    }
    __device__ __forceinline__ void adv_span() {
        wrs = (wrs + T >= cbca_win_ring(T)) ? wrs + T - cbca_win_ring(T) : wrs + T;
    }
    // stage A's register part (first wave): the S1 and area prefixes of the tile's positions
    __device__ __forceinline__ void hn_a_vals(const Tile& t, float (&s1v)[T], uint16_t (&acv)[T]) {
#pragma unroll
        for (int k = 0; k < T; k++) {
            S1 = S1 + t.x[k];
            s1v[k] = S1;
            const uint32_t pp = isect(t, 1, k);
            Acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, pp), us2{1, 1}, Acc, false) + 1u;
            acv[k] = (uint16_t)Acc;
        }
    }
    template <int RC>
    __device__ __forceinline__ void hn_a_write(const float (&s1v)[T], const uint16_t (&acv)[T]) {
        float* w1 = r1 + RC * T * 64 + lane;
        uint16_t* wa = ra + RC * T * 64 + lane;
#pragma unroll
        for (int k = 0; k < T; k++) {
            w1[k * 64] = s1v[k];
            wa[k * 64] = acv[k];
        }
    }
    // stage B (second wave): the window slot pairs of the tile's outputs i = j - lag ...
    template <int RC>
    __device__ __forceinline__ void hn_b_slots(const Tile& t, uint32_t (&sp)[T]) const {
        constexpr int RINGC = 8 * T;
        constexpr int si0 = (RC * T - LAGC + 2 * RINGC) % RINGC;
#pragma unroll
        for (int k = 0; k < T; k++) sp[k] = slot_pair_c(isect(t, 0, k), (si0 + k) % RINGC);
    }
    // ... their S1 / area window reads ...
    __device__ __forceinline__ void hn_b_read(const uint32_t (&sp)[T], float (&shv)[T], float (&stv)[T],
                                              uint32_t (&ahv)[T], uint32_t (&atv)[T]) const {
#pragma unroll
        for (int k = 0; k < T; k++) {
            shv[k] = ring_at<1, 0>(sp[k]);
            stv[k] = ring_at<0, 0>(sp[k]);
            ahv[k] = ring_at<1, 2>(sp[k]);
            atv[k] = ring_at<0, 2>(sp[k]);
        }
    }
    // ... and genfinalVm_cbca's division (+ SolveAll's scale) and the stores, as in tile()
    template <bool GUARD>
    __device__ __forceinline__ void hn_b_finish(int j0, const float (&shv)[T], const float (&stv)[T],
                                                const uint32_t (&ahv)[T], const uint32_t (&atv)[T]) const {
        const int i0 = j0 - lag;
        const __amdgpu_buffer_rsrc_t ob = tile_rsrc(i0);
        float dv[T], qv[T];
        uint32_t av[T];
#pragma unroll
        for (int k = 0; k < T; k++) {
            dv[k] = shv[k] - stv[k];
            av[k] = (ahv[k] - atv[k]) & 0xffffu;
            qv[k] = div_area(dv[k], av[k]);
        }
        uint32_t tmin = 0xffffffffu;
#pragma unroll
        for (int k = 0; k < T; k++) tmin = min(tmin, __builtin_bit_cast(uint32_t, dv[k]) - 1u);
        if (__ballot(tmin < 0x087fffffu)) {
#pragma unroll
            for (int k = 0; k < T; k++) qv[k] = dv[k] / (float)av[k];
        }
#pragma unroll
        for (int k = 0; k < T; k++) store_tile(ob, k, finish_norm(qv[k]), !GUARD || (unsigned)(i0 + k) < (unsigned)len);
    }

    template <int R = 0, int RC = -1>   // R: the tile's slot in the four-tile loop (REUSE2 history)
    __device__ __forceinline__ void process(const Tile& t, int j0) {
        constexpr int stages = MODE == CB_NORM_SCAN ? 2 : 1;
        const int last_out = j0 + T - 1 - lag * stages;        // last output position of the tile
        if (j0 - lag >= 0 && last_out < len && (MODE != CB_NORM_SCAN || j0 - 2 * lag >= 0))
            tile<false, R, RC>(t, j0);
        else
            tile<true, R, RC>(t, j0);
    }
};

// ---------------------------------------------------------------------------------------------
// V NORM_SCAN at the reference's lag (LAG = cbca_crossL_out = 34, h:266): the fused sweep that
// runs iteration 0's V normalisation and iteration 1's V scan (full resolution, 1080p).  Same
// arithmetic, order and ring contents as CbLine<false, CB_NORM_SCAN, ...>; what differs is the
// instruction budget of a position and the order the stages of neighbouring tiles are issued in
// (the sweep runs at one wave per SIMD: its rings allow three waves per CU, so every LDS round
// trip a wave waits for is lost issue time):
//  * a tile's work is four stages: A (rows j0 .. j0+T-1 into the S1 / area rings, the tile's
//    pass intersections), B1 (the window slots and S1 / area reads of the normalised outputs at
//    i = j - LAG), B2 (division, S2 prefix and ring writes) and C (the scan outputs at
//    i2 = j - 2 LAG: S2 reads, differences, stores).  They are software-pipelined over
//    tiles: body n issues A(n + 1) while B1(n)'s reads are in flight, and B1(n + 1)'s slot
//    arithmetic and reads while C(n)'s reads are in flight, so each wait for an LDS read
//    finds the reads long returned.  LDS accesses of one wave complete in issue order, so
//    A(n + 1)'s ring writes cannot overtake B1(n)'s reads of the slots they reuse: the rings
//    keep their size (2 LAG + T + 1 slots);
//  * ring reads take the tile position k from the LDS instruction's immediate offset.  The slot
//    pair of a window is computed once per position against the tile's uniform base C (one
//    v_pk_mad_u16 + a packed wrap), and C-relative slot + k may pass the ring's end by up to
//    T - 2 slots: the first T - 1 slots are mirrored past the end (written again by the tile that
//    writes ring slot 0), so no position needs scalar slot arithmetic;
//  * S2 holds position p at slot p mod R like S1, so the scan stage's window at i2 = j - 2 LAG
//    sits at the very slots the norm stage's window at i = (j - LAG) - LAG read LAG positions
//    earlier: the loop keeps those S1 read addresses (head, tail) of the last NH tiles, and the
//    scan stage reads S2 at them plus the ring distance (an LDS immediate);
//  * T = 7, so that the two S rings, the u16 area ring and their mirrors still fit three waves
//    per CU (83 slots x 10 B x 64 lanes); three tiles of loads in flight; a six-tile loop;
//  * tile resources advance incrementally: the volume base by T rows (tiles past the line read
//    nothing; the allocations carry tail pads for the tiles that straddle the end), the arm
//    gathers and own-arm loads through fixed per-plane resources with a uniform row offset;
//  * CHECK = false when the host has proven that every dividend is 0 or >= 2^-110 (iteration
//    0's normalisation of costs >= 2^-24: cbca_div_safe in sm_capi.cpp), so the tiny-dividend
//    test of the area division is dropped.
#ifndef SM_CB_T_NSV
#define SM_CB_T_NSV 7
#endif
#ifndef SM_CB_NSV_VMWAIT
#define SM_CB_NSV_VMWAIT 1   // one explicit vmcnt wait per tile for the stage-A inputs
#endif
// s_waitcnt immediate (gfx9 encoding) waiting for vmcnt <= n only
__host__ __device__ constexpr int nsv_vmcnt(int n) { return ((n >> 4) << 14) | (0xf << 8) | (0x7 << 4) | (n & 0xf); }
static_assert(nsv_vmcnt(60) == 0xCF7C, "s_waitcnt encoding");
constexpr int NSV_LAG = 34;
#ifndef SM_CB_NSV2_PRIO
#define SM_CB_NSV2_PRIO 2   // NsV2: s_setprio of the second wave (full res 7.12-7.46 -> 7.05-7.17 ms, Teddy 0.543 -> 0.540, profiles/r5pr)
#endif
#ifndef SM_CB_NSV2_PIPE
#define SM_CB_NSV2_PIPE 1   // NsV2's second wave software-pipelined over tiles (cbca_run_nsv2; same-process A/B
                            // with placement trials, profiles/r6i: 7.10-7.19 -> 6.87-7.09 ms at like placements)
#endif
#ifndef SM_CB_NSV2_SPLIT
#define SM_CB_NSV2_SPLIT 2   // (pipelined) B1 positions read before C(n-1)'s stores: 4 reads each, <= 15 in flight
#endif
#ifndef SM_CB_NSV_LA
#define SM_CB_NSV_LA 3   // NsV tiles in flight (same-process A/B of the two-wave sweep, profiles/r5la: 2 7.09-7.14, 3 7.03-7.04, 4 9.79-9.81 ms)
#endif
#ifndef SM_CB_RING8_LA
#define SM_CB_RING8_LA 6   // RING8 tiles in flight (same-process A/B, profiles/r5q: LA 3 5.11-5.18, 4 5.10, 5 5.10, 6 5.02-5.10, 7 5.13 ms)
#endif
#ifndef SM_CB_RING8
#define SM_CB_RING8 1   // H NORM at lag 34 through CbLine::RING8 (0: the runtime-ring sweep, A/B builds)
#endif
constexpr int cbca_nsv_ring() { return (2 * NSV_LAG + SM_CB_T_NSV + 1 + SM_CB_T_NSV - 1) / SM_CB_T_NSV * SM_CB_T_NSV; }
constexpr int cbca_nsv_phys() { return cbca_nsv_ring() + SM_CB_T_NSV - 1; }
// dynamic LDS in 4-byte words: r1, r2 (P x 64 floats each), ra (P x 64 u16)
constexpr int cbca_nsv_smem_words() { return cbca_nsv_phys() * (64 + 64 + 32); }

template <bool RV, bool CHECK>
struct NsV {
    static constexpr int T = SM_CB_T_NSV;
    static constexpr int LAG = NSV_LAG;
    static constexpr int R = cbca_nsv_ring();            // logical ring slots (multiple of T)
    static constexpr int P = cbca_nsv_phys();            // physical slots: R + the mirror of 0 .. T-2
    static constexpr int DTMIN = -((LAG + T - 1) / T);   // oldest tile a saved address is reused from
    static constexpr int NH = -DTMIN + 1;                // tiles in the loop = history depth
    static constexpr int SHIFT = (T - (2 * LAG) % T) % T;   // the tile grid starts at row -SHIFT
    static_assert(NH % 3 == 0, "three load buffers rotate through the loop");
    static_assert(2 * LAG + T + 1 <= R && R % T == 0, "ring");
    static_assert((T + (LAG + T - 1)) / T <= NH, "history");

    struct Tile {
        float x[T];           // vm at rows j0 .. j0+T-1
        uint32_t a0[2];       // lane k < T: own arm pair, set 0 at row j0 + k - LAG, set 1 at row j0 + k
        uint32_t a1[2][T];    // the other image's pair at (row, u -/+ d)
    };
    struct Norm {             // B1 -> B2: the S1 and area window ends of a tile's outputs
        float sh[T], st[T];
        us2 ah[(T + 1) / 2], at[(T + 1) / 2];   // position k in half k % 2 of word k / 2
    };

    // volume
    const char* xld;          // (pair, row jld, column u, chunk): the next tile to load
    const char* xst;          // (pair, row j0 - 2 LAG, ...): the scan outputs of the next tile to store
    int jld;                  // first row of the next tile to load
    uint32_t vsb;             // bytes per row
    int rows_avail;           // rows from row 0 that lie inside the allocation (+ tail pad)
    uint32_t xo[T];           // lane offset of tile row k
    // arms: fixed resources over the own / other plane of each set, starting `pad` rows before row 0
    __amdgpu_buffer_rsrc_t A0r[2], A1r[2];
    uint32_t rowb;            // bytes per arm row (W * 4)
    uint32_t rld;             // (jld + pad rows) * rowb: row offset of the next tile's set-1 arms
    uint32_t rld_max;         // its clamp: tiles past the line end re-read rows inside the tail pad
    uint32_t aown;            // own loads: lane k < T -> row k of the tile (else out of range)
    uint32_t ao[T];           // gathers: column u -/+ d of tile row k (out of range outside the image)
    int lane, len;
    int jst;                  // first scan-output row of the next tile to store (j0 - 2 LAG)
    int jnm;                  // first normalised-output row of the next tile's stage B2 (j0 - LAG)
    // rings
    uint32_t o1, oa;          // LDS byte address of this lane's slot-0 entry in r1, ra
    float* r1;
    float* r2;
    uint16_t* ra;
    uint32_t RR;              // (R, -R) mod 2^16
    float S1, S2;
    uint32_t Acc;
    int wsa;                  // ring slot of the next stage-A tile's first input row (multiple of T)
    uint32_t hh[NH][T], ht[NH][T];   // S1 head / tail addresses read by the last NH tiles' B1

    // loads the next tile (tiles are loaded in order, T rows apart); FIRST: the tile at row
    // -SHIFT, whose rows before the line read 0 (out-of-range offsets)
    // (MASK: 1 = the volume rows, 2 = arm set 0, 4 = arm set 1; NsV2's waves load their parts)
    template <bool FIRST = false, int MASK = 7>
    __device__ __forceinline__ void load(Tile& t) {
        // tiles whose rows pass the allocation (only ever past the line end) read 0
        if constexpr (MASK & 1) {
            const __amdgpu_buffer_rsrc_t rx = buf_rsrc(xld, jld + T <= rows_avail ? 0x7fffffff : 0);
#pragma unroll
            for (int k = 0; k < T; k++)
                t.x[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, (FIRST && k < SHIFT) ? (int)0x80000000 : (int)xo[k], 0, 2));
        }
#pragma unroll
        for (int s = 0; s < 2; s++) {
            if (!(MASK & (2 << s))) continue;
            // (stage C's set 0 lies LAG rows further back: its clamp LAG rows further on)
            const uint32_t rl = min(rld, rld_max);
            const uint32_t roff = s == 0 ? rl - (uint32_t)LAG * rowb : rl;   // rows >= -2 LAG: >= 0
            t.a0[s] = __builtin_amdgcn_raw_buffer_load_b32(A0r[s], (int)aown, (int)roff, 0);
#pragma unroll
            for (int k = 0; k < T; k++) t.a1[s][k] = __builtin_amdgcn_raw_buffer_load_b32(A1r[s], (int)ao[k], (int)roff, 0);
        }
        xld += (long)T * (long)vsb;
        jld += T;
        rld += (uint32_t)T * rowb;
    }

    // (C - 1 - tail, C + head) of pair p wrapped into [0, R): the window's tail and head slots
    // relative to the tile's first output (tile position k adds k, served by the mirror)
    // (ccr = cc + (R, -R): two independent v_pk_mad_u16 and a v_pk_min_u16; a dependent
    // v_pk_add_u16 between them costs an s_nop pair per position on gfx950)
    __device__ __forceinline__ uint32_t slots(uint32_t p, uint32_t cc, uint32_t ccr) const {
        // (a v_pk_mad_u16: tail * 0xffff + C - 1, head * 1 + C)
        const us2 q = __builtin_bit_cast(us2, p) * us2{0xffff, 1} + __builtin_bit_cast(us2, cc);
        const us2 w = __builtin_bit_cast(us2, p) * us2{0xffff, 1} + __builtin_bit_cast(us2, ccr);
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(q, w));
    }
    // ring slot of output row i0 = j0 - LAG of the tile whose first input row sits at slot ws
    __device__ __forceinline__ static int out_slot(int ws) { return ws - LAG < 0 ? ws - LAG + R : ws - LAG; }

    // stage B1: window slots of the normalised outputs at i = j - LAG (C: their first slot) and
    // their S1 / area reads; the S1 addresses are kept for the scan stage LAG positions later
    template <int RT>
    __device__ __forceinline__ void stage_b1(const uint32_t (&pi)[T], int C, Norm& nm) {
        typedef __attribute__((address_space(3))) const float lds_f;
        typedef __attribute__((address_space(3))) const uint16_t lds_h;
        const uint32_t cc = ((uint32_t)(C - 1) & 0xffffu) | ((uint32_t)C << 16);
        const uint32_t ccr = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, cc) + __builtin_bit_cast(us2, RR));
        // (all slot pairs first: the dependent packed ops of one position are not adjacent,
        // which would cost s_nop wait states)
        uint32_t spv[T];
#pragma unroll
        for (int k = 0; k < T; k++) spv[k] = slots(pi[k], cc, ccr);
#pragma unroll
        for (int k = 0; k < T; k++) {
            const uint32_t sp = spv[k];
            const uint32_t a1h = mad_u32_u16<1>(sp, 256u, o1), a1t = mad_u32_u16<0>(sp, 256u, o1);
            hh[RT][k] = a1h;
            ht[RT][k] = a1t;
            nm.sh[k] = ((lds_f*)(size_t)a1h)[k * 64];
            nm.st[k] = ((lds_f*)(size_t)a1t)[k * 64];
            // (two positions' u16 ends share a register: the second a d16-hi read)
            nm.ah[k / 2][k % 2] = ((lds_h*)(size_t)mad_u32_u16<1>(sp, 128u, oa))[k * 64];
            nm.at[k / 2][k % 2] = ((lds_h*)(size_t)mad_u32_u16<0>(sp, 128u, oa))[k * 64];
        }
    }

    // stage B2: genfinalVm_cbca's division (cpp:3969-3992) of the outputs of tile j0, their
    // prefix S2 (iteration k+1's scan input) into the S2 ring at slots C .. C+T-1
    __device__ __forceinline__ void stage_b2(const Norm& nm, int C) {
        float qv[T], dv[T];
        uint32_t av[T];
        // div_area (sm_device.h) on position pairs as packed f32 / u16 ops: the same
        // operations element by element (v_pk_add_f32, v_pk_sub_u16, v_pk_mul_f32, v_pk_fma_f32)
        typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int j = 0; j < T / 2; j++) {
            const f2 d = f2{nm.sh[2 * j], nm.sh[2 * j + 1]} - f2{nm.st[2 * j], nm.st[2 * j + 1]};
            const us2 a = nm.ah[j] - nm.at[j];                     // areas modulo 2^16
            const f2 bf = f2{(float)a.x, (float)a.y};
            const f2 y = f2{__builtin_amdgcn_rcpf(bf.x), __builtin_amdgcn_rcpf(bf.y)};
            const f2 q0 = d * y;
            const f2 r = __builtin_elementwise_fma(-q0, bf, d);
            const f2 q = __builtin_elementwise_fma(r, y, q0);
            dv[2 * j] = d.x;
            dv[2 * j + 1] = d.y;
            qv[2 * j] = q.x;
            qv[2 * j + 1] = q.y;
            av[2 * j] = a.x;
            av[2 * j + 1] = a.y;
        }
        if constexpr (T % 2) {
            dv[T - 1] = nm.sh[T - 1] - nm.st[T - 1];
            const us2 a = nm.ah[T / 2] - nm.at[T / 2];
            av[T - 1] = a.x;
            qv[T - 1] = div_area(dv[T - 1], av[T - 1]);
        }
        if constexpr (CHECK) {
            // dividends are >= +0, so "0 < dv < 2^-110" is "bits(dv) - 1 < 0x087fffff" (unsigned)
            uint32_t tmin = 0xffffffffu;
#pragma unroll
            for (int k = 0; k < T; k++) tmin = min(tmin, __builtin_bit_cast(uint32_t, dv[k]) - 1u);
            if (__ballot(tmin < 0x087fffffu)) {
#pragma unroll
                for (int k = 0; k < T; k++) qv[k] = dv[k] / (float)av[k];
            }
        }
        // nothing accumulates before the line: outputs at rows < 0 read the arm rows before their
        // plane (the previous plane's last rows, not a zero pad) and are set to +0 -- a uniform
        // branch taken by the first tiles only, out of line, with no memory operation in it
        if (__builtin_expect(jnm < 0, 0)) {
#pragma unroll
            for (int k = 0; k < T; k++) qv[k] = (jnm + k >= 0) ? qv[k] : 0.f;
        }
        jnm += T;
        // (C + k may pass R: the mirror slots; a logical slot below T - 1 is kept in both copies)
        float s2v[T];
        float* w2 = r2 + C * 64 + lane;
#pragma unroll
        for (int k = 0; k < T; k++) {
            S2 = S2 + qv[k];
            s2v[k] = S2;
            w2[k * 64] = S2;
        }
        if (__builtin_expect(C + T - 1 >= R || C <= T - 2, 0)) {   // two of the R / T tile positions
#pragma unroll
            for (int k = 0; k < T; k++) {
                if (C + k >= R) r2[(C + k - R) * 64 + lane] = s2v[k];
                if (C + k <= T - 2) r2[(C + k + R) * 64 + lane] = s2v[k];
            }
        }
    }

    // NsV2 pipelined (SM_CB_NSV2_PIPE): B1's window addresses are formed a tile ahead (they need
    // only the pass arms and the slot base), so that after the barrier "A(n) written" the reads
    // issue back to back; the S1 ends go to the saved-address history hh / ht[RT] as in stage_b1
    struct B1Addr {
        uint32_t ah[T], at[T];   // the area ring's head / tail addresses
    };
    template <int RT>
    __device__ __forceinline__ void b1_addr(const uint32_t (&pi)[T], int C, B1Addr& ad) {
        const uint32_t cc = ((uint32_t)(C - 1) & 0xffffu) | ((uint32_t)C << 16);
        const uint32_t ccr = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, cc) + __builtin_bit_cast(us2, RR));
        uint32_t spv[T];
#pragma unroll
        for (int k = 0; k < T; k++) spv[k] = slots(pi[k], cc, ccr);
#pragma unroll
        for (int k = 0; k < T; k++) {
            hh[RT][k] = mad_u32_u16<1>(spv[k], 256u, o1);
            ht[RT][k] = mad_u32_u16<0>(spv[k], 256u, o1);
            ad.ah[k] = mad_u32_u16<1>(spv[k], 128u, oa);
            ad.at[k] = mad_u32_u16<0>(spv[k], 128u, oa);
        }
    }
    template <int RT, int K0, int K1>
    __device__ __forceinline__ void b1_read(const B1Addr& ad, Norm& nm) const {
        typedef __attribute__((address_space(3))) const float lds_f;
        typedef __attribute__((address_space(3))) const uint16_t lds_h;
#pragma unroll
        for (int k = K0; k < K1; k++) {
            nm.sh[k] = ((lds_f*)(size_t)hh[RT][k])[k * 64];
            nm.st[k] = ((lds_f*)(size_t)ht[RT][k])[k * 64];
            nm.ah[k / 2][k % 2] = ((lds_h*)(size_t)ad.ah[k])[k * 64];
            nm.at[k / 2][k % 2] = ((lds_h*)(size_t)ad.at[k])[k * 64];
        }
    }

    // stage C reads: the scan outputs at i2 = j - 2 LAG, read at the norm stage's S1 addresses
    // of position j - LAG (tile RT + dt, index q - dt T) plus the ring distance P slots
    template <int RT>
    __device__ __forceinline__ void stage_c_read(float (&s2h)[T], float (&s2t)[T]) const {
        typedef __attribute__((address_space(3))) const float lds_f;
#pragma unroll
        for (int k = 0; k < T; k++) {
            const int q = k - LAG;
            const int dt = -((-q + T - 1) / T);
            const int src = (RT + dt + 4 * NH) % NH, idx = q - dt * T;
            s2h[k] = ((lds_f*)(size_t)hh[src][idx])[(idx + P) * 64];
            s2t[k] = ((lds_f*)(size_t)ht[src][idx])[(idx + P) * 64];
        }
    }
    // stage C stores: the tile's rows jst .. jst+T-1 through a resource whose range ends at the
    // line end (rows past it are dropped by the range check) and is empty for tiles before the
    // line (the tile grid starts SHIFT rows early so that no tile straddles row 0 of the scan
    // outputs): every tile issues the same T stores and no branch
    __device__ __forceinline__ void stage_c_store(const float (&s2h)[T], const float (&s2t)[T]) {
        // (jst < 0 or jst >= len: nothing of the tile is in the line -- the tiles that run past
        // the line end must not store into the rows after it, the next pair's or past the
        // allocation; a tile with 0 < len - jst < T keeps only its rows before the end)
        const int left = len - jst;
        const int range = (unsigned)jst >= (unsigned)len ? 0 : (left >= T ? 0x7fffffff : left * (int)vsb);
        const __amdgpu_buffer_rsrc_t ob2 = buf_rsrc(xst, range);
        xst += (long)T * (long)vsb;
        jst += T;
#pragma unroll
        for (int k = 0; k < T; k++) buf_st(ob2, xo[k], 0, s2h[k] - s2t[k]);
    }

    __device__ __forceinline__ static void launder(Tile& t) {
        static_assert(T == 7, "launder lists the 23 registers of a T = 7 tile");
        asm volatile("" : "+v"(t.x[0]), "+v"(t.x[1]), "+v"(t.x[2]), "+v"(t.x[3]), "+v"(t.x[4]), "+v"(t.x[5]),
                          "+v"(t.x[6]), "+v"(t.a0[0]), "+v"(t.a0[1]), "+v"(t.a1[0][0]), "+v"(t.a1[0][1]),
                          "+v"(t.a1[0][2]), "+v"(t.a1[0][3]), "+v"(t.a1[0][4]), "+v"(t.a1[0][5]), "+v"(t.a1[0][6]),
                          "+v"(t.a1[1][0]), "+v"(t.a1[1][1]), "+v"(t.a1[1][2]), "+v"(t.a1[1][3]), "+v"(t.a1[1][4]),
                          "+v"(t.a1[1][5]), "+v"(t.a1[1][6]));
    }
    // (NsV2 pipelined: each wave waits for its own part of a tile only)
    __device__ __forceinline__ static void launder_set1(Tile& t) {   // volume rows + set 1 (stage A)
        static_assert(T == 7, "launder lists a T = 7 tile");
        asm volatile("" : "+v"(t.x[0]), "+v"(t.x[1]), "+v"(t.x[2]), "+v"(t.x[3]), "+v"(t.x[4]), "+v"(t.x[5]),
                          "+v"(t.x[6]), "+v"(t.a0[1]), "+v"(t.a1[1][0]), "+v"(t.a1[1][1]), "+v"(t.a1[1][2]),
                          "+v"(t.a1[1][3]), "+v"(t.a1[1][4]), "+v"(t.a1[1][5]), "+v"(t.a1[1][6]));
    }
    __device__ __forceinline__ static void launder_set0(Tile& t) {   // set 0 (B1, C)
        static_assert(T == 7, "launder lists a T = 7 tile");
        asm volatile("" : "+v"(t.a0[0]), "+v"(t.a1[0][0]), "+v"(t.a1[0][1]), "+v"(t.a1[0][2]), "+v"(t.a1[0][3]),
                          "+v"(t.a1[0][4]), "+v"(t.a1[0][5]), "+v"(t.a1[0][6]));
    }
    // T stores that store nothing (out-of-range offsets)
    __device__ __forceinline__ void dummy_stores() const {
        const __amdgpu_buffer_rsrc_t r = buf_rsrc(xst, 0);
#pragma unroll
        for (int k = 0; k < T; k++) buf_st(r, 0x80000000u + 4u * k, 0, 0.f);   // (distinct: not merged)
    }

    // NsV2's second wave: the pass intersections of a tile (stage A's pi without the rings)
    __device__ __forceinline__ void pass_isect(const Tile& t, uint32_t (&pi)[T]) const {
#pragma unroll
        for (int k = 0; k < T; k++) pi[k] = pkmin((uint32_t)__builtin_amdgcn_readlane((int)t.a0[0], k), t.a1[0][k]);
    }
    // NsV2's first wave: stage A as its register part (the S1 and area prefixes of the tile's
    // rows) and its ring writes, so that the writes alone wait for the second wave's B1 reads
    struct AVals {
        float s1v[T];
        uint16_t acv[T];
    };
    __device__ __forceinline__ void stage_a_values(const Tile& t, AVals& v) {
#pragma unroll
        for (int k = 0; k < T; k++) {
            S1 = S1 + t.x[k];
            v.s1v[k] = S1;
            const uint32_t pp = pkmin((uint32_t)__builtin_amdgcn_readlane((int)t.a0[1], k), t.a1[1][k]);
            Acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, pp), us2{1, 1}, Acc, false) + 1u;
            v.acv[k] = (uint16_t)Acc;
        }
    }
    __device__ __forceinline__ void stage_a_write(const AVals& v) {
        float* w1 = r1 + wsa * 64 + lane;
        uint16_t* wa = ra + wsa * 64 + lane;
#pragma unroll
        for (int k = 0; k < T; k++) {
            w1[k * 64] = v.s1v[k];
            wa[k * 64] = v.acv[k];
        }
        if (__builtin_expect(wsa == 0, 0)) {
#pragma unroll
            for (int k = 0; k < T - 1; k++) {
                r1[(R + k) * 64 + lane] = v.s1v[k];
                ra[(R + k) * 64 + lane] = v.acv[k];
            }
        }
        wsa = wsa + T == R ? 0 : wsa + T;
    }
};

// the line's state (both NsV forms); the caller zeroes the rings
template <bool RV, bool CHECK>
__device__ __forceinline__ void nsv_setup(NsV<RV, CHECK>& L, const CbcaArgs& a, const int blk, float* smem) {
    using L_t = NsV<RV, CHECK>;
    constexpr int T = L_t::T;
    const int nchunks = a.D / 64;
    const int per_pair = a.W * nchunks;
    const int b = blk / per_pair;
    const int lc = blk - b * per_pair;
    const int u = lc % a.W, chunk = lc / a.W;   // chunk-major (see cbca_run_line)
    const size_t npix = (size_t)a.H * a.W;
    L.vsb = (uint32_t)(a.W * a.D * 4);
    const char* xbase = (const char*)(a.vm + ((size_t)b * npix + u) * a.D + (size_t)chunk * 64);
    constexpr int J0 = -L_t::SHIFT;                 // first tile row
    L.xld = xbase + (long)J0 * (long)L.vsb;
    L.jld = J0;
    L.jst = J0 - 2 * L_t::LAG;
    L.jnm = J0 - L_t::LAG;
    L.xst = xbase + (long)(J0 - 2 * L_t::LAG) * (long)L.vsb;
    {
        const long room = (const char*)a.vm_end - xbase;   // bytes from row 0 to the allocation end
        const long rows = room / (long)L.vsb;
        L.rows_avail = rows > 0x3fffffffL ? 0x3fffffff : (int)rows;
    }
#pragma unroll
    for (int k = 0; k < T; k++) L.xo[k] = (uint32_t)L.lane * 4u + (uint32_t)k * L.vsb;
    L.len = a.H;
    L.rowb = (uint32_t)a.W * 4u;
    L.rld = (uint32_t)(a.arm_pad_rows + J0) * L.rowb;   // (the pad holds 2 LAG rows: J0 - LAG >= -2 LAG)
    // the arm allocation's tail pad holds 2 LAG + 64 rows after the last plane; a tile starting
    // past row len + LAG has all its arm rows (set 0: rows - LAG, set 1: rows) at or past the line
    // end, where no stored output reads them: such tiles re-read the rows of the tile at len + LAG
    L.rld_max = (uint32_t)(a.arm_pad_rows + L.len + L_t::LAG) * L.rowb;
    const int dl = chunk * 64 + L.lane;
    const int own = RV ? 2 : 0, other = RV ? 0 : 2;
    const long pad = (long)a.arm_pad_rows * L.rowb;
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const int pl = s == 0 ? 1 : 0;   // V sweeps: pass pair = (U | D) plane 1, perpendicular = plane 0
        // (distinct, all effectively unbounded ranges: with one shared upper half the compiler
        // re-forms the four descriptors from it with s_mov pairs in every tile)
        L.A0r[s] = buf_rsrc((const char*)(a.arms + ((size_t)b * 4 + own + pl) * npix + u) - pad, 0x7fffffff - 2 * s);
        L.A1r[s] = buf_rsrc((const char*)(a.arms + ((size_t)b * 4 + other + pl) * npix) - pad, 0x7ffffffe - 2 * s);
    }
    L.aown = L.lane < T ? (uint32_t)L.lane * L.rowb : 0x80000000u;
    {
        const bool out = RV ? u + dl >= a.W : u - dl < 0;
        const uint32_t col = (uint32_t)(RV ? u + dl : u - dl) * 4u;
#pragma unroll
        for (int k = 0; k < T; k++) L.ao[k] = out ? 0x80000000u : col + (uint32_t)k * L.rowb;
    }
    L.r1 = smem;
    L.r2 = smem + L_t::P * 64;
    L.ra = (uint16_t*)(smem + L_t::P * 128);
    {
        typedef __attribute__((address_space(3))) char lds_c;
        L.o1 = (uint32_t)(size_t)(lds_c*)L.r1 + 4u * (uint32_t)L.lane;
        L.oa = (uint32_t)(size_t)(lds_c*)L.ra + 2u * (uint32_t)L.lane;
    }
    L.RR = (uint32_t)L_t::R | ((uint32_t)(65536 - L_t::R) << 16);
#pragma unroll
    for (int r = 0; r < L_t::NH; r++)
#pragma unroll
        for (int k = 0; k < T; k++) L.hh[r][k] = L.ht[r][k] = L.o1;   // rows before the line: any in-ring address (outputs < 0 are not stored)
    L.S1 = L.S2 = 0.f;
    L.Acc = 0;
    L.wsa = 0;
}

// NsV2: the same sweep as two waves per line sharing the line's rings (one workgroup of 128).
// A single NsV wave is issue-bound at one wave per SIMD (its rings allow three lines per CU);
// two waves per line double the issuing waves without more LDS.  Wave 0 runs stage A (volume
// rows and perpendicular arms -> S1 / area rings), wave 1 the pass intersections, B1, B2 and C.
// Per tile n two workgroup barriers: after A(n) (its ring writes done) and after B1(n) (its ring
// reads done, the only reads A(n + 1) can overwrite: B1(n) spans rows j0 - 2 lag - 1 .. j0 + T - 1
// of the R-slot ring).  The first wave computes A(n + 1)'s prefixes beside B1(n) and only its
// ring writes wait for B1(n)'s barrier, so the second wave's B1, B2, C are the critical path.
// Both waves run the same tiles and one extra barrier each (the first wave's at the end, the
// second's at the start), so they pass the same barriers in the same order.
__device__ __forceinline__ void nsv2_bar_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void nsv2_bar() { asm volatile("s_barrier" ::: "memory"); }

// Diagnostic builds only (-DSM_CB_NSV_TRACE=1, tools/nsv_trace.py): per-wave sums of shader-clock
// cycles spent in each phase of a tile, read back through sm_debug_nsv_trace.  s_memtime is a
// scalar-memory read whose result waits for lgkmcnt(0), so the phase boundaries sit where the
// sweep waits for its LDS operations anyway (one exception noted below).
#ifndef SM_CB_NSV_TRACE
#define SM_CB_NSV_TRACE 0
#endif
#if SM_CB_NSV_TRACE
constexpr int NSV_TRACE_BLOCKS = 1 << 16, NSV_TRACE_PH = 8;
__device__ unsigned long long g_nsv_trace[NSV_TRACE_BLOCKS * 2 * NSV_TRACE_PH];
struct NsvTrace {
    unsigned long long acc[NSV_TRACE_PH] = {}, t = 0;
    __device__ __forceinline__ void start() { t = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void mark(int ph) {
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
        acc[ph] += t2 - t;
        t = t2;
    }
    __device__ __forceinline__ void flush(int blk, int wid, int tiles) {
        if ((threadIdx.x & 63) == 0 && blk < NSV_TRACE_BLOCKS) {
            unsigned long long* o = g_nsv_trace + ((size_t)blk * 2 + wid) * NSV_TRACE_PH;
            for (int i = 0; i < NSV_TRACE_PH - 1; i++) o[i] = acc[i];
            o[NSV_TRACE_PH - 1] = (unsigned long long)tiles;
        }
    }
};
#define NSV_TR(x) x
#else
#define NSV_TR(x)
#endif

template <bool RV, bool CHECK>
__device__ __forceinline__ void cbca_run_nsv2(const CbcaArgs& a, const int blk, float* smem) {
    using L_t = NsV<RV, CHECK>;
    using Tile = typename L_t::Tile;
    constexpr int T = L_t::T;
    constexpr int J0 = -L_t::SHIFT;
    constexpr int LA = SM_CB_NSV_LA;
    static_assert(LA >= 2 && LA <= 6, "NsV look-ahead");
    static_assert(L_t::NH == 6, "the loops below are written for six tiles");
    L_t L;
    L.lane = (int)threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    nsv_setup(L, a, blk, smem);
    for (int w = (int)threadIdx.x; w < cbca_nsv_smem_words(); w += 128) smem[w] = 0.f;   // rows before the line
    __syncthreads();
    const int nst = L.len + 2 * L_t::LAG;
    Tile tq[6];
    if (wid == 0) {
        // stage A: tile n's rows into the rings, then the two barriers of tile n
        L.template load<true, 5>(tq[0]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 1; k < LA; k++) {
            L.template load<false, 5>(tq[k]);
            __builtin_amdgcn_sched_barrier(0);
        }
        NSV_TR(NsvTrace tr; tr.start(); int tiles = 0;)
        const int nst0 = SM_CB_NSV2_PIPE ? nst + T : nst;   // (the pipelined second wave's extra step)
        for (int j0 = J0; j0 < nst0; j0 += 6 * T) {
            auto step = [&](auto rc) {
                constexpr int n = decltype(rc)::value;
                L.template load<false, 5>(tq[(n + LA) % 6]);
#if SM_CB_NSV_VMWAIT && SM_CB_NSV2_PIPE
                L_t::launder_set1(tq[n]);
#elif SM_CB_NSV_VMWAIT
                L_t::launder(tq[n]);
#endif
                typename L_t::AVals v;
                L.stage_a_values(tq[n], v);
                NSV_TR(tr.mark(0);)   // loads issued, tile n waited for, A(n) values
                nsv2_bar();        // B1(n - 1) read
                NSV_TR(tr.mark(1);)   // waiting for B1(n - 1)
                L.stage_a_write(v);
                nsv2_bar_lgkm();   // A(n) written
                NSV_TR(tr.mark(2); tiles++;)   // ring writes + lgkm + barrier
            };
            step(std::integral_constant<int, 0>{});
            step(std::integral_constant<int, 1>{});
            step(std::integral_constant<int, 2>{});
            step(std::integral_constant<int, 3>{});
            step(std::integral_constant<int, 4>{});
            step(std::integral_constant<int, 5>{});
        }
        nsv2_bar();   // (pairs with the second wave's last "B1 read")
        NSV_TR(tr.flush(blk, 0, tiles);)
    } else {
#if SM_CB_NSV2_PRIO
        __builtin_amdgcn_s_setprio(SM_CB_NSV2_PRIO);   // the second wave carries the critical chain
#endif
#if SM_CB_NSV2_PIPE
        // Software-pipelined over tiles: step n = X1(n) | B1(n) reads, first positions | C(n-1)'s
        // differences and stores (its reads, issued in step n-1, long returned) | B1(n) reads, the
        // rest | tile n+1's loads and pass intersections | X2(n) | B2(n) | C(n) reads (not waited
        // for) | B1(n+1)'s addresses.  So B1's LDS latency hides C(n-1)'s stores, C's LDS latency
        // hides the barrier and B1(n+1)'s issue, and the window X1(n) -> X2(n), in which the first
        // wave waits, holds only B1's reads.  C(n) of the last tile needs one more step.
        {
            typename L_t::Norm nm;
            typename L_t::B1Addr ad;
            int C = L_t::out_slot(0);
            L.jst -= T;   // step 0 stores "C(-1)": rows before the line, out of range
            L.xst -= (long)T * (long)L.vsb;
            float s2h[T], s2t[T];
            uint32_t pi[T];
#pragma unroll
            for (int k = 0; k < T; k++) s2h[k] = s2t[k] = 0.f;
            // (the steady state's vmcnt sequence: T stores, then a tile's loads)
            L.template load<false, 2>(tq[0]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 1; k <= LA; k++) {
                L.dummy_stores();
                __builtin_amdgcn_sched_barrier(0);
                L.template load<false, 2>(tq[k]);
                __builtin_amdgcn_sched_barrier(0);
            }
            L_t::launder_set0(tq[0]);
            L.pass_isect(tq[0], pi);
            L.template b1_addr<0>(pi, C, ad);
            nsv2_bar();   // (pairs with the first wave's "B1(-1) read")
            const int nst1 = nst + T;
            NSV_TR(NsvTrace tr; tr.start(); int tiles = 0;)
            for (int j0 = J0; j0 < nst1; j0 += 6 * T) {
                auto step = [&](auto rc) {
                    constexpr int n = decltype(rc)::value;
                    nsv2_bar();                                       // X1(n): A(n) written
                    NSV_TR(tr.mark(0);)   // X2(n-1) -> X1(n): B2, C issue, B1 addresses, X1 wait (+ C(n-1) read wait)
                    L.template b1_read<n, 0, SM_CB_NSV2_SPLIT>(ad, nm);
                    __builtin_amdgcn_sched_barrier(0);
                    L.stage_c_store(s2h, s2t);                        // C(n-1)
                    __builtin_amdgcn_sched_barrier(0);
                    L.template b1_read<n, SM_CB_NSV2_SPLIT, T>(ad, nm);
                    __builtin_amdgcn_sched_barrier(0);
                    L.template load<false, 2>(tq[(n + LA + 1) % 6]);
                    L_t::launder_set0(tq[(n + 1) % 6]);
                    L.pass_isect(tq[(n + 1) % 6], pi);
                    nsv2_bar_lgkm();                                  // X2(n): B1(n) read
                    NSV_TR(tr.mark(1); tiles++;)   // X1(n) -> X2(n): B1 reads, C(n-1) stores, loads, isect, X2
                    L.stage_b2(nm, C);                                // B2(n)
                    L.template stage_c_read<n>(s2h, s2t);             // C(n)
                    C = C + T >= L_t::R ? C + T - L_t::R : C + T;
                    L.template b1_addr<(n + 1) % 6>(pi, C, ad);       // (tile n + 1)
                };
                step(std::integral_constant<int, 0>{});
                step(std::integral_constant<int, 1>{});
                step(std::integral_constant<int, 2>{});
                step(std::integral_constant<int, 3>{});
                step(std::integral_constant<int, 4>{});
                step(std::integral_constant<int, 5>{});
            }
            NSV_TR(tr.flush(blk, 1, tiles);)
            return;
        }
#endif
        typename L_t::Norm nm;
        int C = L_t::out_slot(0);
        L.template load<false, 2>(tq[0]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 1; k < LA; k++) {
            L.template load<false, 2>(tq[k]);
            __builtin_amdgcn_sched_barrier(0);
#if SM_CB_NSV_VMWAIT
            L.dummy_stores();   // the stores of "C(k - LA)": step 0 sees the steady-state sequence
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
        nsv2_bar();   // (pairs with the first wave's "B1(-1) read")
        NSV_TR(NsvTrace tr; tr.start(); int tiles = 0;)
        for (int j0 = J0; j0 < nst; j0 += 6 * T) {
            auto step = [&](auto rc) {
                constexpr int n = decltype(rc)::value;
                L.template load<false, 2>(tq[(n + LA) % 6]);
#if SM_CB_NSV_VMWAIT
                L_t::launder(tq[n]);
#endif
                uint32_t pi[T];
                L.pass_isect(tq[n], pi);
                NSV_TR(tr.mark(0);)   // loads issued, tile n waited for, pass intersections
                nsv2_bar();                                   // A(n) written
                NSV_TR(tr.mark(1);)   // waiting for A(n)
                L.template stage_b1<n>(pi, C, nm);            // B1(n)
                nsv2_bar_lgkm();                              // B1(n) read
                NSV_TR(tr.mark(2);)   // B1 issue + LDS latency + barrier
                L.stage_b2(nm, C);                            // B2(n)
                NSV_TR(tr.mark(3);)   // B2 (includes its ring writes' completion: the one perturbation)
                float s2h[T], s2t[T];
                L.template stage_c_read<n>(s2h, s2t);         // C(n)
                C = C + T >= L_t::R ? C + T - L_t::R : C + T;
                L.stage_c_store(s2h, s2t);
                NSV_TR(tr.mark(4); tiles++;)   // C reads + their latency + stores issued
            };
            step(std::integral_constant<int, 0>{});
            step(std::integral_constant<int, 1>{});
            step(std::integral_constant<int, 2>{});
            step(std::integral_constant<int, 3>{});
            step(std::integral_constant<int, 4>{});
            step(std::integral_constant<int, 5>{});
        }
        NSV_TR(tr.flush(blk, 1, tiles);)
    }
}

template <bool RV, bool CHECK>
__global__ __launch_bounds__(128) void k_cbca_nsv2(const CbcaArgs a) {
    extern __shared__ float smem[];
    cbca_run_nsv2<RV, CHECK>(a, xcd_swizzle(blockIdx.x, gridDim.x), smem);
}
// the line's state, zeroed rings and the H sweeps' span-ring prologue; returns the sweep length
// (both waves of HN2 run it: they write the same values)
template <bool HORIZ, int MODE, bool FULL, bool SCALE, bool RV, int LAGC>
__device__ __forceinline__ int cbca_line_setup(CbLine<HORIZ, MODE, FULL, SCALE, RV, LAGC>& L, const CbcaArgs& a,
                                               const int blk, float* smem, const int prologue_sets = 0xff) {
    constexpr int T = CbCfg<HORIZ, MODE>::T;
    constexpr int NSETS = CbCfg<HORIZ, MODE>::NSETS;
    L.lane = (int)threadIdx.x & 63;
    const int nchunks = (a.D + 63) / 64;
    const int nlines = HORIZ ? a.H : a.W;
    const int per_pair = nlines * nchunks;
    const int b = blk / per_pair;
    const int lc = blk - b * per_pair;
    // V sweeps run chunk-major: the blocks resident on one XCD are consecutive columns of ONE
    // disparity chunk, whose other-image spans [u - c64 - 63, u - c64] overlap almost entirely
    // (full resolution: v_norm fetches 20.8 -> 13.4 GB per launch for 12.3 GB of volume)
    const int line = HORIZ ? lc / nchunks : lc % nlines;
    const int chunk = HORIZ ? lc - line * nchunks : lc / nlines;
    L.line = line;
    const size_t npix = (size_t)a.H * a.W;
    const size_t first_pix = HORIZ ? (size_t)L.line * a.W : (size_t)L.line;
    L.pstride = HORIZ ? 1 : a.W;
    L.vsb = (uint32_t)(L.pstride * a.D * 4);
    L.xline = (const char*)(a.vm + ((size_t)b * npix + first_pix) * a.D + (size_t)chunk * 64);
    const int dl = chunk * 64 + L.lane;  // true disparity (also for masked lanes)
    {
        const uint32_t xv = FULL ? (uint32_t)L.lane * 4u : (uint32_t)min(L.lane, a.D - 1 - chunk * 64) * 4u;
#pragma unroll
        for (int k = 0; k < T; k++) L.xo[k] = xv + (uint32_t)k * L.vsb;
        L.ov = (FULL || dl < a.D) ? (uint32_t)L.lane * 4u : 0x80000000u;
    }
    L.xend = (const char*)a.vm_end;
    L.aend = (const char*)a.arms_end;
    // arm planes: [b][view][plane][npix]; plane 0 = (L | R<<16), plane 1 = (U | D<<16)
    // own = this view's image, other = the image it is matched against
    const int pass_plane = HORIZ ? 0 : 1, perp_plane = HORIZ ? 1 : 0;
    const int own = RV ? 2 : 0, other = RV ? 0 : 2;
    const uint32_t* planeL = a.arms + ((size_t)b * 4) * npix + first_pix;
    const int line_bytes = (((HORIZ ? a.W : a.H) - 1) * L.pstride + 1) * 4;
#pragma unroll
    for (int s = 0; s < NSETS; s++) {
        const int pl = (s == 1) ? perp_plane : pass_plane;
        L.A0r[s] = buf_rsrc(planeL + (size_t)(own + pl) * npix, line_bytes);
        L.A1r[s] = buf_rsrc(planeL + (size_t)(other + pl) * npix, line_bytes);
        L.A1v[s] = (const char*)(a.arms + ((size_t)b * 4 + other + pl) * npix);
    }
    if constexpr (!HORIZ) {
        // other image's column: u - d (left view) or u + d (right view); lanes whose column lies
        // outside the image get an out-of-range offset, so their gathers return the reference's
        // zeroed intersection (cpp:2794-2845) without a mask per position
        const int u = L.line;
        const bool out = RV ? u + dl >= a.W : u - dl < 0;
        const uint32_t col = (uint32_t)(RV ? u + dl : u - dl) * 4u;
#pragma unroll
        for (int k = 0; k < T; k++) L.ao[k] = out ? 0x80000000u : col + (uint32_t)(k * a.W * 4);
    }
    L.c64 = chunk * 64;
    L.len = HORIZ ? a.W : a.H;
    L.lag = a.lag;
    L.ring = cbca_ring(a.lag, HORIZ, MODE);
    if constexpr (std::remove_reference_t<decltype(L)>::REUSE2) {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int k = 0; k < T; k++) L.ph[r][k] = 0u;   // positions before the line: zero arms
    }
    const int ring_words = cbca_ring_words(a.lag, HORIZ, MODE);
    float* const mine = smem;
    L.r1 = mine;
    L.r2 = mine + (size_t)L.ring * 64;
    L.ra = (uint16_t*)(mine + (size_t)L.ring * 64 * (MODE == CB_NORM_SCAN ? 2 : 1));
    {
        typedef __attribute__((address_space(3))) char lds_c;
        L.o1 = (uint32_t)(size_t)(lds_c*)L.r1 + 4u * (uint32_t)L.lane;
        L.o2 = (uint32_t)(size_t)(lds_c*)L.r2 + 4u * (uint32_t)L.lane;
        L.oa = (uint32_t)(size_t)(lds_c*)L.ra + 2u * (uint32_t)L.lane;
    }
    L.wown = (uint32_t*)(mine + ring_words);
    L.wspan = L.wown + NSETS * T;
    L.scale = a.scale;
    {   // zero the rings: reads of positions before the line start then yield S = 0, area = 0
        const int words = cbca_smem_words(a.lag, HORIZ, MODE);
        for (int w = L.lane; w < words; w += 64) mine[w] = 0.f;
    }
    __syncthreads();  // orders the float ring stores before the u16 ring reads
    L.S1 = L.S2 = 0.f;
    L.Acc = 0;
    L.ws = 0;
    L.wrs = 0;
    if constexpr (HORIZ) {
        // span-ring prologue: the first tile's words q0 .. q0 + 62 of every set (the tiles add the rest)
        constexpr int R = cbca_win_ring(T);
#pragma unroll
        for (int s = 0; s < NSETS; s++) {
            if (!(prologue_sets & (1 << s))) continue;   // (HN2: each wave its own set's words)
            const int base = -L.set_off(s);
            const int q = (RV ? base + L.c64 : base - L.c64 - 63) + L.lane;
            const uint32_t w = buf_ld_u32(L.A1r[s], (L.lane < 63 && (unsigned)q < (unsigned)L.len) ? (uint32_t)q * 4u : 0x80000000u, 0);
            if (L.lane < 63) {
                L.wspan[s * 2 * R + L.lane] = w;
                L.wspan[s * 2 * R + L.lane + R] = w;
            }
        }
    }
    return L.len + a.lag * (MODE == CB_NORM_SCAN ? 2 : 1);
}

template <bool HORIZ, int MODE, bool FULL, bool SCALE, bool RV, int LAGC>
__device__ __forceinline__ void cbca_run_line(const CbcaArgs& a, const int blk, float* smem) {
    CbLine<HORIZ, MODE, FULL, SCALE, RV, LAGC> L;
    constexpr int T = CbCfg<HORIZ, MODE>::T;
    const int nst = cbca_line_setup(L, a, blk, smem);
    typename CbLine<HORIZ, MODE, FULL, SCALE, RV, LAGC>::Tile ta, tb, tc, td;
    // The loops have no exit but their condition and the prologue's tiles are loaded in order:
    // otherwise the compiler's vmcnt waits at the loop head are conservative and the first tile
    // of every trip waits for later tiles' loads too.  Tiles past the line end run (up to PF of
    // them): their loads are bounded or read the next line, their stores are out of range.
    if constexpr (decltype(L)::RING8) {
        // H NORM at lag 34: eight tiles per trip (one ring cycle), tile k in buffer k, LA tiles in
        // flight (the buffer a load fills was consumed LA - 8 tiles before, LA <= 7)
        typename CbLine<HORIZ, MODE, FULL, SCALE, RV, LAGC>::Tile tq[8];
        constexpr int LA = SM_CB_RING8_LA;
        static_assert(LA >= 1 && LA <= 7, "RING8 look-ahead");
#pragma unroll
        for (int k = 0; k < LA; k++) {
            L.load(tq[k], k * T);
            __builtin_amdgcn_sched_barrier(0);
        }
        for (int j0 = 0; j0 < nst; j0 += 8 * T) {
            auto step = [&](auto kc) {
                constexpr int k = decltype(kc)::value;
                L.load(tq[(k + LA) % 8], j0 + (k + LA) * T);
                L.template process<0, k>(tq[k], j0 + k * T);
            };
            step(std::integral_constant<int, 0>{});
            step(std::integral_constant<int, 1>{});
            step(std::integral_constant<int, 2>{});
            step(std::integral_constant<int, 3>{});
            step(std::integral_constant<int, 4>{});
            step(std::integral_constant<int, 5>{});
            step(std::integral_constant<int, 6>{});
            step(std::integral_constant<int, 7>{});
        }
    } else if constexpr (CbCfg<HORIZ, MODE>::PF == 3) {
        L.load(ta, 0);
        __builtin_amdgcn_sched_barrier(0);
        L.load(tb, T);
        __builtin_amdgcn_sched_barrier(0);
        L.load(tc, 2 * T);
        __builtin_amdgcn_sched_barrier(0);
        for (int j0 = 0; j0 < nst; j0 += 4 * T) {
            L.load(td, j0 + 3 * T);
            L.template process<0>(ta, j0);
            L.load(ta, j0 + 4 * T);
            L.template process<1>(tb, j0 + T);
            L.load(tb, j0 + 5 * T);
            L.template process<2>(tc, j0 + 2 * T);
            L.load(tc, j0 + 6 * T);
            L.template process<3>(td, j0 + 3 * T);
        }
    } else if constexpr (CbCfg<HORIZ, MODE>::PF == 2) {
        L.load(ta, 0);
        __builtin_amdgcn_sched_barrier(0);
        L.load(tb, T);
        __builtin_amdgcn_sched_barrier(0);
        for (int j0 = 0; j0 < nst; j0 += 3 * T) {
            L.load(tc, j0 + 2 * T);
            L.process(ta, j0);
            L.load(ta, j0 + 3 * T);
            L.process(tb, j0 + T);
            L.load(tb, j0 + 4 * T);
            L.process(tc, j0 + 2 * T);
        }
    } else {
        L.load(ta, 0);
        __builtin_amdgcn_sched_barrier(0);
        for (int j0 = 0; j0 < nst; j0 += 2 * T) {
            L.load(tb, j0 + T);
            L.process(ta, j0);
            L.load(ta, j0 + 2 * T);
            L.process(tb, j0 + T);
        }
    }
}

// HN2: the H normalising sweep at the reference's lag (RING8) as two waves per line sharing the
// S1 / area rings (a workgroup of 128), the split NsV2 made for the V sweep: the first wave runs
// stage A (volume rows, perpendicular arm set, S1 and area prefixes, ring writes), the second the
// pass arm set, the window slot pairs, the ring reads, the division, SolveAll's scale and the
// stores.  Per tile n two workgroup barriers: X1(n) after A(n)'s ring writes, X2(n) after B(n)'s
// ring reads (the only reads A(n + 1) can overwrite: 2 lag + T + 1 <= 8 T slots).  The second wave
// issues tile n + 1's set-0 staging and pass intersections while B(n)'s reads are in flight, and
// runs B(n)'s division and stores while the first wave writes A(n + 1).
#ifndef SM_CB_HN2
#define SM_CB_HN2 1   // H NORM at lag 34 as HN2 (two waves per line; same-process A/B with placement trials,
                      // profiles/r6/ab_hn2_fullres.txt: 5.00-5.02 -> 4.53-4.55 ms; 0: the one-wave RING8 sweep)
#endif
#ifndef SM_CB_HN2_LA
#define SM_CB_HN2_LA 4   // HN2 tiles in flight (8 buffers; LA 6: 4.54-4.55 ms, 4: 4.53-4.55)
#endif
#ifndef SM_CB_HN2_PRIO
#define SM_CB_HN2_PRIO 2   // s_setprio of the second wave
#endif
template <bool FULL, bool SCALE, bool RV>
__device__ __forceinline__ void cbca_run_hn2(const CbcaArgs& a, const int blk, float* smem) {
    using L_t = CbLine<true, CB_NORM, FULL, SCALE, RV, 34>;
    static_assert(L_t::RING8, "HN2 runs the 8-tile ring cycle");
    constexpr int T = L_t::T;
    constexpr int LA = SM_CB_HN2_LA;
    static_assert(LA >= 1 && LA <= 7, "HN2 look-ahead");
    L_t L;
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int nst = cbca_line_setup(L, a, blk, smem, wid == 0 ? 2 : 1);
    __syncthreads();   // (both waves' setup writes done)
    typename L_t::Tile tq[8];
    const int lag = L.lag;
    if (wid == 0) {
#pragma unroll
        for (int k = 0; k < LA; k++) {
            L.template load<1 | 4>(tq[k], k * T);
            __builtin_amdgcn_sched_barrier(0);
        }
        for (int j0 = 0; j0 < nst; j0 += 8 * T) {
            auto step = [&](auto kc) {
                constexpr int k = decltype(kc)::value;
                L.template load<1 | 4>(tq[(k + LA) % 8], j0 + (k + LA) * T);
                L.template stage_set<1>(tq[k]);
                float s1v[T];
                uint16_t acv[T];
                L.hn_a_vals(tq[k], s1v, acv);
                L.adv_span();
                nsv2_bar();        // X2(n - 1): B(n - 1) read
                L.template hn_a_write<k>(s1v, acv);
                nsv2_bar_lgkm();   // X1(n): A(n) written
            };
            step(std::integral_constant<int, 0>{});
            step(std::integral_constant<int, 1>{});
            step(std::integral_constant<int, 2>{});
            step(std::integral_constant<int, 3>{});
            step(std::integral_constant<int, 4>{});
            step(std::integral_constant<int, 5>{});
            step(std::integral_constant<int, 6>{});
            step(std::integral_constant<int, 7>{});
        }
        nsv2_bar();   // (pairs with the second wave's last X2)
    } else {
#if SM_CB_HN2_PRIO
        __builtin_amdgcn_s_setprio(SM_CB_HN2_PRIO);
#endif
#pragma unroll
        for (int k = 0; k < LA; k++) {
            L.template load<2>(tq[k], k * T);
            __builtin_amdgcn_sched_barrier(0);
        }
        uint32_t sp[T];
        L.template stage_set<0>(tq[0]);
        L.template hn_b_slots<0>(tq[0], sp);
        L.adv_span();
        nsv2_bar();   // X2(-1)
        for (int j0 = 0; j0 < nst; j0 += 8 * T) {
            auto step = [&](auto kc) {
                constexpr int k = decltype(kc)::value;
                nsv2_bar();                                   // X1(n): A(n) written
                float shv[T], stv[T];
                uint32_t ahv[T], atv[T];
                L.hn_b_read(sp, shv, stv, ahv, atv);          // B(n)
                // tile n + 1: loads LA ahead, its set-0 words and slot pairs (reads in flight with B(n)'s)
                L.template load<2>(tq[(k + LA) % 8], j0 + (k + LA) * T);
                L.template stage_set<0>(tq[(k + 1) % 8]);
                uint32_t sp2[T];
                L.template hn_b_slots<(k + 1) % 8>(tq[(k + 1) % 8], sp2);
                L.adv_span();
                nsv2_bar_lgkm();                              // X2(n): B(n) read
                const int jt = j0 + k * T;
                if (jt - lag >= 0 && jt + T - 1 - lag < L.len)
                    L.template hn_b_finish<false>(jt, shv, stv, ahv, atv);
                else
                    L.template hn_b_finish<true>(jt, shv, stv, ahv, atv);
#pragma unroll
                for (int q = 0; q < T; q++) sp[q] = sp2[q];
            };
            step(std::integral_constant<int, 0>{});
            step(std::integral_constant<int, 1>{});
            step(std::integral_constant<int, 2>{});
            step(std::integral_constant<int, 3>{});
            step(std::integral_constant<int, 4>{});
            step(std::integral_constant<int, 5>{});
            step(std::integral_constant<int, 6>{});
            step(std::integral_constant<int, 7>{});
        }
    }
}

template <bool FULL, bool SCALE, bool RV>
__global__ __launch_bounds__(128) void k_cbca_hn2(const CbcaArgs a) {
    extern __shared__ float smem[];
    cbca_run_hn2<FULL, SCALE, RV>(a, xcd_swizzle(blockIdx.x, gridDim.x), smem);
}

template <bool HORIZ, int MODE, bool FULL, bool SCALE, bool RV, int LAGC = 0>
__global__ __launch_bounds__(64) void k_cbca(const CbcaArgs a) {
    extern __shared__ float smem[];
    const int slot = xcd_swizzle(blockIdx.x, gridDim.x);   // neighbouring lines on one XCD
    cbca_run_line<HORIZ, MODE, FULL, SCALE, RV, LAGC>(a, slot, smem);
}

template <bool HORIZ, int MODE, bool SCALE, int LAGC>
static void launch_lag(const CbcaArgs& a, int n, hipStream_t st) {
    const int nchunks = (a.D + 63) / 64;
    const int nlines = (HORIZ ? a.H : a.W) * nchunks * n;
    const size_t shm = 4 * (size_t)cbca_smem_words(a.lag, HORIZ, MODE);
    const bool full = a.D % 64 == 0;
    dim3 grid(nlines), block(64);
    if (a.view == 0) {
        if (full) hipLaunchKernelGGL((k_cbca<HORIZ, MODE, true, SCALE, false, LAGC>), grid, block, shm, st, a);
        else hipLaunchKernelGGL((k_cbca<HORIZ, MODE, false, SCALE, false, LAGC>), grid, block, shm, st, a);
    } else {
        if (full) hipLaunchKernelGGL((k_cbca<HORIZ, MODE, true, SCALE, true, LAGC>), grid, block, shm, st, a);
        else hipLaunchKernelGGL((k_cbca<HORIZ, MODE, false, SCALE, true, LAGC>), grid, block, shm, st, a);
    }
}

// NsV's prerequisites: the reference's lag, whole 64-disparity chunks, arm-plane offsets in 31 bits
static bool nsv_ok(const CbcaArgs& a) {
    return a.lag == NSV_LAG && a.D % 64 == 0 && a.arm_pad_rows == 2 * NSV_LAG &&
           (double)(a.H + 4 * NSV_LAG + 64) * a.W * 4.0 < 2147483647.0;
}

template <bool HORIZ, int MODE, bool SCALE>
static void launch_scaled(const CbcaArgs& a, int n, hipStream_t st) {
    // V NORM_SCAN at the reference's cbca_crossL_out (h:266): NsV, else the REUSE2 instantiation
    if constexpr (!HORIZ && MODE == CB_NORM_SCAN) {
        if (nsv_ok(a)) {
            dim3 grid(a.W * (a.D / 64) * n), block(128);   // two waves per line
            const size_t shm = 4 * (size_t)cbca_nsv_smem_words();
            if (a.view == 0) {
                if (a.div_safe) hipLaunchKernelGGL((k_cbca_nsv2<false, false>), grid, block, shm, st, a);
                else hipLaunchKernelGGL((k_cbca_nsv2<false, true>), grid, block, shm, st, a);
            } else {
                if (a.div_safe) hipLaunchKernelGGL((k_cbca_nsv2<true, false>), grid, block, shm, st, a);
                else hipLaunchKernelGGL((k_cbca_nsv2<true, true>), grid, block, shm, st, a);
            }
            return;
        }
        if (a.lag == 34) return launch_lag<HORIZ, MODE, SCALE, 34>(a, n, st);
    }
#if SM_CB_RING8
    // H NORM at the reference's lag: the compile-time 8-tile ring cycle (CbLine::RING8)
    if constexpr (HORIZ && MODE == CB_NORM) {
        if (a.lag == 34 && SM_CB_HN2) {   // two waves per line (HN2)
            dim3 grid(a.H * ((a.D + 63) / 64) * n), block(128);
            const size_t shm = 4 * (size_t)cbca_smem_words(a.lag, true, CB_NORM);
            const bool full = a.D % 64 == 0;
            if (a.view == 0) {
                if (full) hipLaunchKernelGGL((k_cbca_hn2<true, SCALE, false>), grid, block, shm, st, a);
                else hipLaunchKernelGGL((k_cbca_hn2<false, SCALE, false>), grid, block, shm, st, a);
            } else {
                if (full) hipLaunchKernelGGL((k_cbca_hn2<true, SCALE, true>), grid, block, shm, st, a);
                else hipLaunchKernelGGL((k_cbca_hn2<false, SCALE, true>), grid, block, shm, st, a);
            }
            return;
        }
        if (a.lag == 34) return launch_lag<HORIZ, MODE, SCALE, 34>(a, n, st);
    }
#endif
    launch_lag<HORIZ, MODE, SCALE, 0>(a, n, st);
}

template <bool HORIZ, int MODE>
static void launch_mode(const CbcaArgs& a, int n, hipStream_t st) {
    if constexpr (MODE == CB_NORM) {
        if (a.apply_scale) return launch_scaled<HORIZ, MODE, true>(a, n, st);
    }
    launch_scaled<HORIZ, MODE, false>(a, n, st);
}

void launch_cbca(const CbcaArgs& a, bool horiz, int mode, int n, hipStream_t st) {
    if (horiz) {
        if (mode == CB_SCAN) launch_mode<true, CB_SCAN>(a, n, st);
        else if (mode == CB_NORM) launch_mode<true, CB_NORM>(a, n, st);
        else launch_mode<true, CB_NORM_SCAN>(a, n, st);
    } else {
        if (mode == CB_SCAN) launch_mode<false, CB_SCAN>(a, n, st);
        else if (mode == CB_NORM) launch_mode<false, CB_NORM>(a, n, st);
        else launch_mode<false, CB_NORM_SCAN>(a, n, st);
    }
}

}  // namespace sm

#if SM_CB_NSV_TRACE
// diagnostic builds only: [block][wave][phase] cycle sums of the last NsV2 launch (phase 7 = tiles)
extern "C" __attribute__((visibility("default"))) int sm_debug_nsv_trace(unsigned long long* dst, int nblocks) {
    if (nblocks > sm::NSV_TRACE_BLOCKS) nblocks = sm::NSV_TRACE_BLOCKS;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(sm::g_nsv_trace), (size_t)nblocks * 2 * sm::NSV_TRACE_PH * 8, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? nblocks : -1;
}
#endif

