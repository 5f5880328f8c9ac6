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
// Instruction budget (the sweeps are issue-bound at 2-3 waves per CU):
//  * arms are stored as two u16-pair planes per pixel, (L | R<<16) and (U | D<<16), so the
//    intersection of a pair is one v_pk_min_u16 against the uniform reference-pixel word;
//  * in horizontal sweeps the right-image arm word of lane d at position q is A1[q - d] — the
//    window shifts by one lane per step, so it lives in a register advanced with DPP wave_shr
//    (lanes with q - d < 0 keep the initial 0, which is exactly the reference's zeroed tail);
//  * ring wraps are single v_min_u32 selections; full 64-lane chunks use uniform addressing.
// Scheduling: the next tile of T positions (volume values, arm words) is loaded while the
// current tile is processed; inside a steady-state tile all ring writes precede all ring reads,
// so a tile costs one or two LDS round trips.  Rings hold 2*lag + T + 1 slots.
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
__device__ __forceinline__ uint32_t shr1_in(uint32_t v, uint32_t in) {  // lane l <- lane l-1, lane 0 <- in
    return (uint32_t)__builtin_amdgcn_update_dpp((int)in, (int)v, DPP_WAVE_SHR1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t shl1_in(uint32_t v, uint32_t in) {  // lane l <- lane l+1, lane 63 <- in
    return (uint32_t)__builtin_amdgcn_update_dpp((int)in, (int)v, DPP_WAVE_SHL1, 0xF, 0xF, false);
}

// Positions per tile and tiles prefetched ahead: the sweeps are bound by memory latency at the
// 5-6 waves per CU the LDS rings allow, so PF tiles of loads are kept in flight; the loads of PF
// tiles plus the stores of one stay below the 63 of vmcnt (V sweeps load one right-arm word per
// position and set, hence their shorter tiles).
// The normalising sweeps use T = 10 with two tiles in flight: their rings (2 lag + T + 1 slots of
// S plus a u16 area ring) then fit five waves per CU instead of four (Teddy x16, same box:
// h_norm 0.459 -> 0.425 ms, v_norm 0.505 -> 0.480 ms with the LDS-staged arm words).
// Three tiles in flight (PF = 3, 141 / 217 VGPRs for H / V norm) measured no better: h_norm
// 0.415 -> 0.416, v_norm 0.463 -> 0.469 ms (Teddy x16, same box).
// (Overridable at build time for tuning sweeps, see tools/build_variants.sh.)
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
// Arm words of a tile are staged in LDS (SM_CB_LDS_WIN): the pixel's own arm pair of position k is
// a broadcast read, and in horizontal sweeps the other image's arm pair of lane d at position k is
// read from a staged span of 64 + T - 1 words at k + 63 - d (left view) / k + d (right view).  This
// replaces per position and set a v_readlane (own) and a readlane + v_mov + DPP wave shift (other
// image) by LDS reads with immediate offsets.  0 keeps the DPP-shifted register window.
#ifndef SM_CB_LDS_WIN
#define SM_CB_LDS_WIN 1
#endif
// H sweeps keep the other image's span as a ring (SM_CB_WIN_RING): consecutive tiles' spans
// overlap in 63 words, so a tile loads only its T new words (one lane-vector load per set
// instead of 64 + T - 1 words); the ring of R = 63 + T words is mirrored (every word written at
// i and i + R), so reads at start + offset never wrap.  Probe with no window loads at all:
// h_scan 0.265 -> 0.242 ms, h_norm 0.435 -> 0.418 ms (Teddy x16); the ring itself measured
// h_norm 0.416 -> 0.409 ms, h_scan unchanged (same box).
#ifndef SM_CB_WIN_RING
#define SM_CB_WIN_RING 1
#endif
// V sweeps take the pixel's own arm pair of position k by v_readlane from the tile's lane-vector
// load instead of staging it in LDS (SM_CB_V_READLANE): their other-image words are register
// gathers, so the sweep's tile then has a single LDS round trip (the S / area rings) instead of two.
#ifndef SM_CB_V_READLANE
#define SM_CB_V_READLANE 1
#endif
#ifndef SM_CB_PROBE_NOVG
// Timing probes only (wrong results; DESIGN §5 "What the V gathers cost"): V sweeps skip the other
// image's arm gathers (1), gather row 0 every time (2), gather columns 0..63 of the right rows (3),
// gather 16 distinct words (4), skip v_norm's second-set gather (5), 5 with padded rings (6).
#define SM_CB_PROBE_NOVG 0
#endif
#ifndef SM_CB_ACC_DOT2
#define SM_CB_ACC_DOT2 1     // area prefix step as v_dot2_u32_u16 (see tile())
#endif
#ifndef SM_CB_VG_AUX
#define SM_CB_VG_AUX 0       // cache policy bits of the V sweeps' arm gathers (tuning)
#endif
// CB_NORM_SCAN sweeps (two S rings + the area ring): tile and tiles in flight.  T = 12 with three
// tiles in flight (two waves per CU by LDS, one per SIMD by VGPRs) measured fastest among T = 6-20,
// PF = 1-3 (same-process A/B, profiles/r3c, r3i): full resolution v_norm + v_scan 12.20 ms ->
// 11.09 ms fused, 1080p 16.38 -> 15.68 ms; Teddy 0.76 -> 0.82 ms (hence sm_params.fuse_norm_scan's
// auto mode: fused for volumes >= 256 MiB per pair)
#ifndef SM_CB_T_NS
#define SM_CB_T_NS 12
#endif
#ifndef SM_CB_PF_NS_H
#define SM_CB_PF_NS_H 2
#endif
#ifndef SM_CB_PF_NS_V
#define SM_CB_PF_NS_V 3
#endif
// NORM_SCAN V sweeps at the reference's lag (cbca_crossL_out = 34, a compile-time LAGC): the scan
// stage's pass intersection at position j is the norm stage's at j - lag (both are the pass pair
// of row j - 2 lag), so the sweep keeps the last four tiles' norm intersections in registers and
// drops the third set's own-arm load, readlane, pkmin and 64-word gather per position
// (SM_CB_NS_REUSE; other lags run the generic sweep).
#ifndef SM_CB_NS_REUSE
#define SM_CB_NS_REUSE 1
#endif
// Normalising sweeps decide per TILE whether a dividend can lie in (0, 2^-110), where div_area
// needs the IEEE division (SM_CB_SAFE_TILE): prefix sums of costs >= +0 never decrease along a
// line, and a difference S(h) - S(t) with S(t) >= 2^-86 is 0 or >= ulp(S(t)) >= 2^-109.  Each lane
// records per tile whether S at the tile's start reached 2^-86; a tile whose window start lies
// at least ceil(2 lag / T) tiles back in a lane that had then reached it skips the per-position
// check (the first tiles of a line, and lines of tiny costs, keep it).
#ifndef SM_CB_SAFE_TILE
#define SM_CB_SAFE_TILE 0
#endif
// Ring slots of a position's window ends as one packed u16 pair (SM_CB_PK_SLOTS): with the uniform
// slot c of position i and the intersection pair (tail | head << 16), (pair ^ 0xffff) + (c, c) is
// (c - tail - 1, c + head) modulo 2^16, and one packed add of (ring, -ring) plus a packed minimum
// wraps both ends into [0, ring) -- four VALU for both slots instead of seven.
#ifndef SM_CB_PK_SLOTS
#define SM_CB_PK_SLOTS 1
#endif
// ... and each ring address is one v_mad_u32_u16 of the pair's half (op_sel) with the ring's
// bytes per slot and the lane's byte offset (SM_CB_MAD_ADDR) instead of an extract and a shift-add
#ifndef SM_CB_MAD_ADDR
#define SM_CB_MAD_ADDR 1
#endif
template <int HI>
__device__ __forceinline__ uint32_t mad_u32_u16(uint32_t a, uint32_t b, uint32_t c) {   // a.half * b.lo + c
    uint32_t r;
    if (HI)
        asm("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    else
        asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}
__host__ __device__ constexpr int cbca_win_ring(int T) { return 63 + T; }
__host__ __device__ constexpr int cbca_tile(bool horiz, int mode) {
    return mode == CB_SCAN ? (horiz ? SM_CB_T_SCAN_H : SM_CB_T_SCAN_V)
                           : (mode == CB_NORM ? (horiz ? SM_CB_T_NORM_H : SM_CB_T_NORM_V) : SM_CB_T_NS);
}
// V sweeps as workgroups of KW waves on KW adjacent columns of one 64-disparity chunk
// (SM_CB_VGROUP): per tile the workgroup stages, for each arm set and row, the KW own-image words
// and the KW + 63 other-image words its lanes pair with (lane d of column u0 + w reads the
// other image at u0 + w - d, i.e. span index w + 63 - d) in LDS with one coalesced load per
// thread, instead of every wave gathering 64 words per row and set (the same words, shifted by
// one column, as its neighbours: full resolution, probe without the gather: v_norm 7.29 ->
// 5.5 ms, v_scan 5.56 -> 4.6-5.1 ms).  Staging is double-buffered, one barrier per tile.
// KW waves share one CU's LDS with their rings, so the normalising sweep runs T = 7 (ring 77
// slots) to fit five waves; the host falls back to KW = 1 when the rings of a larger lag do not fit.
// Measured (full resolution, same box): v_scan 5.57 -> 5.69 ms, v_norm 7.30 -> 11.07 ms — the
// extra LDS round trip for the staged words on the tile's critical path and the per-tile barrier
// of five lock-stepped waves cost more than the gathers; kept as a switch, off.
#ifndef SM_CB_VGROUP
#define SM_CB_VGROUP 0   // measured slower (see above): off
#endif
#ifndef SM_CB_KW_SCAN
#define SM_CB_KW_SCAN 6
#endif
#ifndef SM_CB_KW_NORM
#define SM_CB_KW_NORM 5
#endif
#ifndef SM_CB_T_NORM_VG
#define SM_CB_T_NORM_VG 7
#endif
__host__ __device__ constexpr int cbca_kw(bool horiz, int mode) {
    return (horiz || !SM_CB_VGROUP || mode == CB_NORM_SCAN) ? 1 : (mode == CB_SCAN ? SM_CB_KW_SCAN : SM_CB_KW_NORM);
}
// staged words per set and row: KW own + KW + 63 other
__host__ __device__ constexpr int cbca_spw(int kw) { return 2 * kw + 63; }
// V sweeps as blocks of WPB INDEPENDENT waves on WPB adjacent columns of one chunk
// (SM_CB_WPB_*_V): every wave runs the one-line sweep with its own rings and its own gathers — no
// staging and no per-tile barrier — but the waves of a block share one CU, so a row's
// other-image gathers of neighbouring columns (spans overlapping in all but one word per column)
// are served by that CU's L1 instead of each going to L2.  One block per CU (WPB rings fill its
// LDS), the same waves per CU as one-wave blocks.  Measured (full resolution, interleaved
// same-process A/B, profiles/r2l/ab_vsweeps.txt): v_norm 6.71 -> 9.56 ms at WPB = 5, v_scan
// 5.06 -> 5.86 ms at WPB = 6 — slower; off.
#ifndef SM_CB_WPB_SCAN_V
#define SM_CB_WPB_SCAN_V 1
#endif
#ifndef SM_CB_WPB_NORM_V
#define SM_CB_WPB_NORM_V 1
#endif
__host__ __device__ constexpr int cbca_wpb(bool horiz, int mode) {
    return (horiz || SM_CB_VGROUP) ? 1 : (mode == CB_SCAN ? SM_CB_WPB_SCAN_V : (mode == CB_NORM ? SM_CB_WPB_NORM_V : 1));
}
// V sweeps with CPW adjacent columns per wave (SM_CB_CPW_*_V): lane l runs column u0 + l / CW at
// disparity c + l % CW (CW = 64 / CPW disparities per chunk).  A row's other-image gather of the
// wave then reads columns u0 + cl - d of both halves, which overlap in all but one word: 33 distinct
// words (one or two 128-byte lines) instead of 64 (two or three), the effect timing probe 4 showed
// (DESIGN §5).  The rings stay one slot per lane; the volume accesses become CPW segments of
// 4 CW bytes.  The pixel's own arm pair differs between the halves: two readlanes and a select
// (SM_CB_CPW_OWN 0) or one ds_bpermute (1) per set and position instead of one readlane.
#ifndef SM_CB_CPW_SCAN_V
#define SM_CB_CPW_SCAN_V 1
#endif
#ifndef SM_CB_CPW_NORM_V
#define SM_CB_CPW_NORM_V 1
#endif
#ifndef SM_CB_CPW_OWN
#define SM_CB_CPW_OWN 0
#endif
__host__ __device__ constexpr int cbca_cpw(bool horiz, int mode, int kw, int wpb) {
    return (horiz || kw > 1 || wpb > 1 || !SM_CB_V_READLANE) ? 1 : (mode == CB_SCAN ? SM_CB_CPW_SCAN_V : (mode == CB_NORM ? SM_CB_CPW_NORM_V : 1));
}

template <bool HORIZ, int MODE, int KW = 1>
struct CbCfg {
    static constexpr int T = (KW > 1 && MODE == CB_NORM) ? SM_CB_T_NORM_VG : cbca_tile(HORIZ, MODE);
    static constexpr int PF = MODE == CB_SCAN ? (HORIZ ? SM_CB_PF_SCAN_H : SM_CB_PF_SCAN_V)
                                              : (MODE == CB_NORM ? (HORIZ ? SM_CB_PF_NORM_H : SM_CB_PF_NORM_V) : (HORIZ ? SM_CB_PF_NS_H : SM_CB_PF_NS_V));
    // arm sets: 0 = pass pair at i (= j - lag), 1 = perpendicular pair at j, 2 = pass pair at j - 2 lag
    static constexpr int NSETS = MODE == CB_SCAN ? 1 : (MODE == CB_NORM ? 2 : 3);
    static constexpr int NW = KW > 1 ? NSETS * T * cbca_spw(KW) : 0;          // staged words per tile
    static constexpr int NV = KW > 1 ? (NW + 64 * KW - 1) / (64 * KW) : 1;   // per thread
};

// ring slots: >= 2*lag + T + 1 (a whole tile is written before any of it is read) and a multiple
// of T (a tile's write slots never wrap)
__host__ __device__ inline int cbca_tile_kw(bool horiz, int mode, int kw) {
    return (kw > 1 && mode == CB_NORM) ? SM_CB_T_NORM_VG : cbca_tile(horiz, mode);
}
__host__ __device__ inline int cbca_ring(int lag, bool horiz, int mode, int kw = 1) {
    const int T = cbca_tile_kw(horiz, mode, kw);
    return (2 * lag + T + 1 + T - 1) / T * T;
}
// dynamic LDS in 4-byte words: S ring(s) of ring x 64 floats, then the u16 area ring (6 bytes
// per slot and lane; 8-byte {S, area} records were measured slower: one wave less per CU), then
// the staged arm words of one tile (SM_CB_LDS_WIN): per set T own words [+ 64 + T - 1 span words]
__host__ __device__ inline int cbca_ring_words(int lag, bool horiz, int mode, int kw = 1) {
    const int ring = cbca_ring(lag, horiz, mode, kw);
    const int floats = mode == CB_NORM_SCAN ? 2 : 1;
    const int u16s = mode == CB_SCAN ? 0 : 1;
    // (SM_CB_PROBE_NOVG == 6: timing probe, a further 2 bytes per slot and lane in normalising sweeps)
    return ring * 64 * floats + ring * 32 * u16s + (SM_CB_PROBE_NOVG == 6 && mode == CB_NORM ? ring * 32 : 0);
}
__host__ __device__ inline int cbca_win_words(bool horiz, int mode) {
    if (!SM_CB_LDS_WIN) return 0;
    if (!horiz && SM_CB_V_READLANE) return 0;   // V sweeps: own words by v_readlane, gathers in registers
    const int T = cbca_tile(horiz, mode);
    const int nsets = mode == CB_SCAN ? 1 : (mode == CB_NORM ? 2 : 3);
    return nsets * (T + (horiz ? (SM_CB_WIN_RING ? 2 * cbca_win_ring(T) : 64 + T - 1) : 0));
}
__host__ __device__ inline int cbca_smem_words(int lag, bool horiz, int mode) {
    return cbca_ring_words(lag, horiz, mode) + cbca_win_words(horiz, mode);
}
// V-group launch: KW rings, then two staging buffers
__host__ __device__ inline int cbca_smem_words_vg(int lag, int mode, int kw) {
    const int T = cbca_tile_kw(false, mode, kw);
    const int nsets = mode == CB_SCAN ? 1 : 2;
    return kw * cbca_ring_words(lag, false, mode, kw) + 2 * nsets * T * cbca_spw(kw);
}

template <bool HORIZ, int T, int NSETS, int KW, int NV>
struct CbTile {
    float x[T];                          // vm at positions j0 .. j0+T-1
    uint32_t a0[KW > 1 ? 1 : NSETS];     // lane k < T: left arm pair at position (j0 + k - off)
    uint32_t a1v[NSETS];                 // H: lane k < T: right arm pair at position (j0 + k - off)
    uint32_t a1w[SM_CB_LDS_WIN && HORIZ ? NSETS : 1][2];  // H, LDS window: the other image's span
    uint32_t a1[HORIZ || KW > 1 ? 1 : NSETS][T];   // V: right arm pair at (row j0 + k - off, u - d)
    uint32_t sv[NV];                     // V group: this thread's staged words of the tile
};

// RV: the right view's volume vm[1] (cbca_core's LOR = 1, run when Do_refine): the pixel's own
// arms are the right image's, and lane d pairs them with the LEFT image's arms at u + d
// (HVL_INTERSECTION[1], cpp:2794-2845) — zero once u + d >= W.
template <bool HORIZ, int MODE, bool FULL, bool SCALE, bool RV, int KW = 1, int CPW = 1, int LAGC = 0>
struct CbLine {
    static constexpr int CW = 64 / CPW;   // disparities per chunk (lanes per column)
    static constexpr int T = CbCfg<HORIZ, MODE, KW>::T;
    static_assert(T <= CW, "a column's own arm words of a tile are one lane each");
    static constexpr int NSETS = CbCfg<HORIZ, MODE, KW>::NSETS;
    static constexpr int NW = CbCfg<HORIZ, MODE, KW>::NW;
    static constexpr int NV = CbCfg<HORIZ, MODE, KW>::NV;
    static constexpr int SPW = cbca_spw(KW);
    using Tile = CbTile<HORIZ, T, NSETS, KW, NV>;
    // SM_CB_NS_REUSE: scan-stage intersections from the norm stage's, LAGC positions back
    static constexpr bool REUSE2 = LAGC > 0 && !HORIZ && MODE == CB_NORM_SCAN && KW == 1 && CPW == 1;
    static_assert(!REUSE2 || (CbCfg<HORIZ, MODE, KW>::PF == 3 && LAGC + T - 1 <= 4 * T),
                  "the history is the last four tiles of the four-tile loop");

    // Volume and V-sweep arm accesses are buffer instructions: the tile's first position in the
    // resource base, lane + k * stride in a loop-invariant VGPR.  Loads are not clamped: the
    // resource's range ends at the allocation's end (reads past it return 0; those positions are
    // never output) and the arm planes carry a 2 * lag row front pad for set positions < 0.
    const char* xline;        // byte address of (line, position 0, chunk's first disparity)
    const char* xend;         // end of the volume allocation
    const char* aend;         // end of the arm allocation
    uint32_t xo[T];           // lane's load offset of tile position k (lanes past D re-read D - 1)
    uint32_t ao[HORIZ ? 1 : T];  // V: lane's arm offset (column u - d) of tile position k
    uint32_t ov;              // lane's store offset (lanes past D: out of range, dropped)
    uint32_t vsb;             // bytes between consecutive positions
    int lane;
    int kk, cl;               // V, CPW > 1: lane = cl * CW + kk (column u0 + cl, chunk lane kk)
    bool colok;               // column u0 + cl < W
    __amdgpu_buffer_rsrc_t A0r[NSETS];  // left-image arm-pair plane of each set over the line
    __amdgpu_buffer_rsrc_t A1r[NSETS];  // H: right-image plane over the line
    const char* A1v[NSETS];     // V: right-image plane, row 0 (uniform)
    int pstride, line, len, lag, ring;
    int c64;                  // first disparity of the chunk
    uint32_t sh[NSETS];       // H sweeps: shifted right-arm window per set
    uint32_t* wown;           // LDS window: own arm words of the tile, T per set
    uint32_t* wspan;          // LDS window (H): the other image's span, 64 + T - 1 per set
    float S1, S2;
    uint32_t Acc;
    int ws;                   // ring slot of the tile's first position
    int wrs;                  // SM_CB_WIN_RING: span-ring slot of the current tile's first word (j0 mod R)
    float* r1;
    float* r2;
    uint16_t* ra;
    uint32_t o1, o2, oa;      // SM_CB_MAD_ADDR: LDS address of this lane's slot-0 entry in r1, r2, ra
    float scale;
    uint32_t ph[REUSE2 ? 4 : 1][REUSE2 ? T : 1];   // REUSE2: pass intersections of the last 4 tiles
    uint32_t shist;           // SM_CB_SAFE_TILE: bit m = S at the start of the tile m back >= 2^-86
    int msafe;                // tiles back to the tile holding the window start (> 31: never safe)
    // V group (KW > 1)
    int wv;                   // wave index in the workgroup = column u0 + wv
    bool active;              // column < W (the last group's spare waves only keep the barriers)
    int H;                    // rows (staged rows outside [0, H) read 0)
    uint32_t rowb;            // bytes per arm-plane row
    __amdgpu_buffer_rsrc_t Ar;   // the pair's four arm planes
    uint32_t sboff[NV];       // staged word m: plane + column byte offset
    int skoff[NV];            // staged word m: row offset from the tile's first position
    uint32_t sok;             // bit m: word m exists and its column lies inside the image
    uint32_t* stg;            // two staging buffers of NW words
    int sbuf;                 // buffer of the current tile

    __device__ __forceinline__ int set_off(int s) const { return s == 0 ? lag : (s == 1 ? 0 : 2 * lag); }
    __device__ __forceinline__ static int clampi(int k, int n) { return k < 0 ? 0 : (k >= n ? n - 1 : k); }

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
    __device__ __forceinline__ void store_tile(const __amdgpu_buffer_rsrc_t& r, int k, float v) const {
        if (KW > 1 && !active) return;
        if (FULL)
            buf_st(r, xo[k], 0, v);
        else
            buf_st(r, ov, (uint32_t)k * vsb, v);
    }

    // Tile loads: positions past the line end read the next line (or 0 past the allocation);
    // their prefix values are never read.
    __device__ __forceinline__ void load(Tile& t, int j0) const {
        const __amdgpu_buffer_rsrc_t rx = bounded_rsrc(xline + (long)j0 * (long)vsb, xend);
#pragma unroll
        for (int k = 0; k < T; k++)   // normalising sweeps: non-temporal volume loads (v_norm 0.466 -> 0.434 ms)
            t.x[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, (int)xo[k], 0, MODE == CB_SCAN ? SM_LD_AUX : 2));
        // lane-vector arm loads: positions outside the line read 0 (an out-of-range offset) --
        // for the right image's arms that is the reference's zeroed intersection when u - d < 0.
        // The offset is a select, never a wrapped negative sum: the range check does not wrap,
        // and the compiler would otherwise move constant parts of a sum into the immediate field.
        if constexpr (KW > 1) {
            // the workgroup's staged words of this tile: one coalesced dword per thread and word
#pragma unroll
            for (int m = 0; m < NV; m++) {
                const int row = j0 + skoff[m];
                const bool ok = ((sok >> m) & 1u) && (unsigned)row < (unsigned)H;
                t.sv[m] = buf_ld_u32(Ar, ok ? sboff[m] + (uint32_t)row * rowb : 0x80000000u, 0);
            }
            return;
        }
#pragma unroll
        for (int s = 0; s < NSETS; s++) {
            if (REUSE2 && s == 2) continue;
            const int base = j0 - set_off(s);
            // (only lanes k < T are read back; the others stay off the memory system, which
            // matters for the strided column loads of vertical sweeps)
            const int p0 = base + kk;
            t.a0[s] = buf_ld_u32(A0r[s], (kk < T && colok && (unsigned)p0 < (unsigned)len) ? (uint32_t)(p0 * pstride + cl) * 4u : 0x80000000u, 0);
            if (HORIZ && SM_CB_LDS_WIN) {
                // the other image's arm pairs that lanes c64 .. c64 + 63 pair with at positions
                // base .. base + T - 1: left view q = p - d in [base - c64 - 63, base - c64 + T - 1],
                // right view q = p + d in [base + c64, base + c64 + 63 + T - 1]; 0 outside the line
                const int q0 = RV ? base + c64 : base - c64 - 63;
                if (SM_CB_WIN_RING) {   // the tile's T new words q0 + 63 .. q0 + 62 + T
                    const int qn = q0 + 63 + lane;
                    t.a1w[s][0] = buf_ld_u32(A1r[s], (lane < T && (unsigned)qn < (unsigned)len) ? (uint32_t)qn * 4u : 0x80000000u, 0);
                } else {
                    const int qa = q0 + lane, qb = q0 + 64 + lane;
                    t.a1w[s][0] = buf_ld_u32(A1r[s], (unsigned)qa < (unsigned)len ? (uint32_t)qa * 4u : 0x80000000u, 0);
                    t.a1w[s][1] = buf_ld_u32(A1r[s], (lane < T - 1 && (unsigned)qb < (unsigned)len) ? (uint32_t)qb * 4u : 0x80000000u, 0);
                }
            } else if (HORIZ) {
                // H window input at position base + lane: left view — the right pixel of lane 0
                // (shifted in at lane 0); right view — the left pixel of lane 63 (shifted in there)
                const int q = RV ? base + lane + c64 + 63 : base + lane - c64;
                t.a1v[s] = buf_ld_u32(A1r[s], (lane < T && (unsigned)q < (unsigned)len) ? (uint32_t)q * 4u : 0x80000000u, 0);
            } else {
                // (SM_CB_PROBE_NOVG == 2, timing only: every gather re-reads row 0 of the plane)
                const __amdgpu_buffer_rsrc_t ra1 = bounded_rsrc(A1v[s] + (SM_CB_PROBE_NOVG == 2 ? 0L : (long)base * (long)(pstride * 4)), aend);
#pragma unroll
                for (int k = 0; k < T; k++)
                    t.a1[s][k] = SM_CB_PROBE_NOVG == 1 ? 0x00110011u
                               : ((SM_CB_PROBE_NOVG == 5 || SM_CB_PROBE_NOVG == 6) && s == 1)
                                   ? t.a1[0][k] ^ 0x00010001u   // probe: the second set's gather skipped
                                   : __builtin_amdgcn_raw_buffer_load_b32(ra1, (int)(SM_CB_PROBE_NOVG == 2 ? ao[0] : ao[k]), 0, SM_CB_VG_AUX);
            }
        }
    }

    // Advance every set's window to position j (call once per position, in order).
    __device__ __forceinline__ void advance(const Tile& t, int k, int /*j*/) {
        if (HORIZ && !SM_CB_LDS_WIN) {
#pragma unroll
            for (int s = 0; s < NSETS; s++) {
                const uint32_t in = (uint32_t)__builtin_amdgcn_readlane((int)t.a1v[s], k);
                sh[s] = RV ? shl1_in(sh[s], in) : shr1_in(sh[s], in);
            }
        }
    }

    // intersection arm pair of set s at tile position k
    __device__ __forceinline__ uint32_t isect(const Tile& t, int s, int k) const {
        if constexpr (KW > 1) {
            // own word: broadcast; other word: span index wv + 63 - d (left) / wv + d (right view)
            const uint32_t* row = stg + sbuf * NW + (s * T + k) * SPW;
            return pkmin(row[wv], row[KW + (RV ? wv + lane : wv + 63 - lane)]);
        }
        if (!HORIZ && SM_CB_V_READLANE) {
            uint32_t a0;
            if constexpr (CPW == 1) {
                a0 = (uint32_t)__builtin_amdgcn_readlane((int)t.a0[s], k);
            } else if constexpr (SM_CB_CPW_OWN == 1) {
                a0 = (uint32_t)__builtin_amdgcn_ds_bpermute((cl * CW + k) * 4, (int)t.a0[s]);
            } else {
                a0 = (uint32_t)__builtin_amdgcn_readlane((int)t.a0[s], k);
#pragma unroll
                for (int c = 1; c < CPW; c++) {
                    const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)t.a0[s], c * CW + k);
                    a0 = cl == c ? x : a0;
                }
            }
            return pkmin(a0, t.a1[s][k]);
        }
        if (SM_CB_LDS_WIN) {
            const uint32_t a0 = wown[s * T + k];   // broadcast read
            const uint32_t a1 = HORIZ ? (SM_CB_WIN_RING ? wspan[s * 2 * cbca_win_ring(T) + wrs + (RV ? k + lane : k + 63 - lane)]
                                                        : wspan[s * (64 + T - 1) + (RV ? k + lane : k + 63 - lane)])
                                      : t.a1[s][k];
            return pkmin(a0, a1);
        }
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)t.a0[s], k);
        const uint32_t a1 = HORIZ ? sh[s] : t.a1[s][k];
        return pkmin(a0, a1);
    }
    // stage the tile's arm words in LDS (one wave: its LDS accesses complete in order)
    __device__ __forceinline__ void stage(const Tile& t) {
        if constexpr (KW > 1) {
            // the other buffer was last read in the previous tile, before every wave passed that
            // tile's barrier, so one barrier per tile orders both reuse hazards
            sbuf ^= 1;
            const int tid = wv * 64 + lane;
#pragma unroll
            for (int m = 0; m < NV; m++)
                if (m * 64 * KW + tid < NW) stg[sbuf * NW + m * 64 * KW + tid] = t.sv[m];
            __syncthreads();
            return;
        }
        if (!SM_CB_LDS_WIN || (!HORIZ && SM_CB_V_READLANE)) return;
#pragma unroll
        for (int s = 0; s < NSETS; s++) {
            if (lane < T) wown[s * T + lane] = t.a0[s];
            if (HORIZ && SM_CB_WIN_RING) {
                constexpr int R = cbca_win_ring(T);
                uint32_t* sp = wspan + s * 2 * R;
                const int w = wrs + 63 + lane;           // < 2 R
                const int i = w >= R ? w - R : w;
                if (lane < T) {
                    sp[i] = t.a1w[s][0];
                    sp[i + R] = t.a1w[s][0];
                }
            } else if (HORIZ) {
                uint32_t* sp = wspan + s * (64 + T - 1);
                sp[lane] = t.a1w[s][0];
                if (lane < T - 1) sp[64 + lane] = t.a1w[s][1];
            }
        }
    }

    __device__ __forceinline__ int uwrap(int s) const {  // uniform slot, any s in (-2 ring, 3 ring)
        s = s < 0 ? s + ring : s;
        s = s < 0 ? s + ring : s;
        s = s >= ring ? s - ring : s;
        return s >= ring ? s - ring : s;
    }
    __device__ __forceinline__ int up(int s) const { return (int)min((uint32_t)s, (uint32_t)(s - ring)); }   // s in [0, 2 ring)
    __device__ __forceinline__ int dn(int s) const { return (int)min((uint32_t)s, (uint32_t)(s + ring)); }   // s in (-ring, ring)
    // SM_CB_PK_SLOTS: (tail slot | head slot << 16) of intersection pair p at uniform slot c < 2 ring
    __device__ __forceinline__ uint32_t slot_pair(uint32_t p, int c) const {
        c = c >= ring ? c - ring : c;   // c < 2 ring: then c + head < 2 ring, c - tail - 1 > -ring
        const us2 q = __builtin_bit_cast(us2, p ^ 0xffffu) + us2{(unsigned short)c, (unsigned short)c};
        const us2 w = q + us2{(unsigned short)ring, (unsigned short)(-ring)};
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(q, w));
    }
    // LDS element of a ring of 4-byte / 2-byte entries at slot s (packed half h of sp) for this lane
    // RG: 0 = r1, 1 = r2 (floats), 2 = ra (u16)
    template <int H_, int RG, typename E = typename std::conditional<RG == 2, uint16_t, float>::type>
    __device__ __forceinline__ E ring_at(uint32_t sp) const {
        if (SM_CB_MAD_ADDR) {
            const uint32_t o = RG == 2 ? oa : (RG == 1 ? o2 : o1);
            // (an integer LDS address cast to an LDS pointer: no base add in front of the read)
            typedef __attribute__((address_space(3))) const E lds_e;
            return *(lds_e*)(size_t)mad_u32_u16<H_>(sp, 64u * (uint32_t)sizeof(E), o);
        }
        const uint32_t sl = H_ ? sp >> 16 : sp & 0xffffu;
        const E* r = RG == 2 ? (const E*)ra : (const E*)(RG == 1 ? r2 : r1);
        return r[sl * 64u + (uint32_t)lane];
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
    template <bool GUARD, int R>
    __device__ __forceinline__ void tile(const Tile& t, int j0) {
        uint32_t pi[T], pi2[T];
        if (MODE != CB_SCAN && SM_CB_SAFE_TILE) shist = (shist << 1) | (S1 >= 0x1p-86f ? 1u : 0u);   // S(j0 - 1)
        // ring % T == 0 and ws % T == 0, so the tile's write slots ws .. ws+T-1 never wrap
        float* w1 = r1 + ws * 64 + lane;
        uint16_t* wa = ra + ws * 64 + lane;
        const int si0 = uwrap(ws - lag);        // slot of i = j0 - lag
        // (NORM_SCAN: r2 holds position p's S2 at slot (p + lag) mod ring, so the tile's S2 writes
        // are slots ws .. ws + T - 1 and the slot of i2 = j0 - 2 lag in r2 is si0)
        const int i0 = j0 - lag;
        const __amdgpu_buffer_rsrc_t ob = tile_rsrc(i0);
        stage(t);
        // phase A: inputs j0 .. j0+T-1 (+ arm windows)
#pragma unroll
        for (int k = 0; k < T; k++) {
            advance(t, k, j0 + k);
            S1 = S1 + t.x[k];
            w1[k * 64] = S1;
            pi[k] = isect(t, 0, k);
            if (MODE != CB_SCAN) {
                const uint32_t pp = isect(t, 1, k);
#if SM_CB_ACC_DOT2
                // only Acc mod 2^16 is ever read (u16 ring): Acc + pp + 1 adds lo + 1 (and hi << 16),
                // the dot adds lo + hi exactly; one udot2 + one add instead of shift, add, add3
                Acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, pp), us2{1, 1}, Acc, false) + 1u;
#else
                Acc = Acc + (pp & 0xffffu) + (pp >> 16) + 1u;
#endif
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
            if (SM_CB_PK_SLOTS) {
                const uint32_t sp = slot_pair(pi[k], si0 + k);   // slots of i - tail - 1, i + head
                shv[k] = ring_at<1, 0>(sp);
                stv[k] = ring_at<0, 0>(sp);
                if (MODE != CB_SCAN) {
                    ahv[k] = ring_at<1, 2>(sp);
                    atv[k] = ring_at<0, 2>(sp);
                }
                continue;
            }
            const int tl = pi[k] & 0xffff, hd = pi[k] >> 16;
            const int hs = up(si0 + k + hd);             // slot of i + head  (< 2 ring)
            const int ts = dn(hs - (hd + tl + 1));       // slot of i - tail - 1 (window < ring)
            shv[k] = r1[hs * 64 + lane];
            stv[k] = r1[ts * 64 + lane];
            if (MODE != CB_SCAN) {
                ahv[k] = ra[hs * 64 + lane];
                atv[k] = ra[ts * 64 + lane];
            }
        }
        if (MODE == CB_SCAN) {
#pragma unroll
            for (int k = 0; k < T; k++)
                if (!GUARD || (unsigned)(i0 + k) < (unsigned)len) store_tile(ob, k, shv[k] - stv[k]);
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
            // SM_CB_SAFE_TILE: every lane's window start S >= 2^-86 (see the switch) -> no check
            const bool check = !SM_CB_SAFE_TILE || msafe > 31 || __ballot(((shist >> msafe) & 1u) == 0u);
            if (check) {
                // dividends are >= +0 (prefix sums of costs >= 0; S - S = +0), so "0 < dv < 2^-110"
                // is "bits(dv) - 1 < 0x087fffff" (unsigned); the tile's minimum of bits - 1 decides it
                uint32_t tmin = 0xffffffffu;
#pragma unroll
                for (int k = 0; k < T; k++) tmin = min(tmin, __builtin_bit_cast(uint32_t, dv[k]) - 1u);
                if (__ballot(tmin < 0x087fffffu)) {
#pragma unroll
                    for (int k = 0; k < T; k++) qv[k] = dv[k] / (float)av[k];
                }
            }
#pragma unroll
            for (int k = 0; k < T; k++) {
                if (MODE == CB_NORM) {
                    if (!GUARD || (unsigned)(i0 + k) < (unsigned)len) store_tile(ob, k, finish_norm(qv[k]));
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
                if (SM_CB_PK_SLOTS) {
                    const uint32_t sp = slot_pair(pi2[k], si0 + k);
                    s2h[k] = ring_at<1, 1>(sp);
                    s2t[k] = ring_at<0, 1>(sp);
                    continue;
                }
                const int tl = pi2[k] & 0xffff, hd = pi2[k] >> 16;
                const int hs = up(si0 + k + hd);
                s2h[k] = r2[hs * 64 + lane];
                s2t[k] = r2[dn(hs - (hd + tl + 1)) * 64 + lane];
            }
            const int i20 = j0 - 2 * lag;
            const __amdgpu_buffer_rsrc_t ob2 = tile_rsrc(i20);
#pragma unroll
            for (int k = 0; k < T; k++)
                if (!GUARD || (unsigned)(i20 + k) < (unsigned)len) store_tile(ob2, k, s2h[k] - s2t[k]);
        }
        ws = (ws + T == ring) ? 0 : ws + T;
        if (SM_CB_WIN_RING) wrs = (wrs + T >= cbca_win_ring(T)) ? wrs + T - cbca_win_ring(T) : wrs + T;
    }

    template <int R = 0>   // R: the tile's slot in the four-tile loop (REUSE2 history)
    __device__ __forceinline__ void process(const Tile& t, int j0) {
        constexpr int stages = MODE == CB_NORM_SCAN ? 2 : 1;
        const int last_out = j0 + T - 1 - lag * stages;        // last output position of the tile
        if (j0 - lag >= 0 && last_out < len && (MODE != CB_NORM_SCAN || j0 - 2 * lag >= 0))
            tile<false, R>(t, j0);
        else
            tile<true, R>(t, j0);
    }
};

// Persistent V sweeps (SM_CB_PERSIST_V): the grid is the number of blocks that fit the chip at
// once and block i runs lines i, i + grid, i + 2 grid, ...  All resident waves then start their
// k-th line together, so the waves of neighbouring columns (one XCD, see xcd_swizzle) walk down
// the rows in near lockstep and share the other image's arm rows through the XCD's L2.  With one
// block per line, blocks of later dispatch waves start whenever a slot frees, neighbours drift
// apart and the 64-word arm gathers of every row miss L2.  Measured at full resolution (same
// box, FETCH_SIZE x 2 per launch): the fetched bytes did not fall (v_norm 20.8 -> 22.2 GB) and the
// sweeps got slower (v_norm 7.35 -> 7.85 ms, v_scan 5.6 -> 6.0 ms): off.
#ifndef SM_CB_PERSIST_V
#define SM_CB_PERSIST_V 0
#endif
// What did cut the gathers' misses is the block order: chunk-major V sweeps (below) put one
// chunk's consecutive columns on an XCD at a time, and neighbouring columns' other-image spans
// overlap in all but one word: v_norm fetches 20.8 -> 13.4 GB (12.3 GB of volume), v_scan 17.2 ->
// 14.2 GB; time 7.34 -> 7.20 ms and 5.60 -> 5.53 ms (full resolution, same box) — the gathers'
// remaining cost is their issue and latency on the tile's critical path (no gathers at all:
// v_norm 5.5 ms), not bytes.
#ifndef SM_CB_CHUNK_MAJOR_V
#define SM_CB_CHUNK_MAJOR_V 1
#endif

template <bool HORIZ, int MODE, bool FULL, bool SCALE, bool RV, int KW, int WPB, int LAGC>
__device__ __forceinline__ void cbca_run_line(const CbcaArgs& a, const int blk, float* smem) {
    constexpr int CPW = cbca_cpw(HORIZ, MODE, KW, WPB);
    constexpr int CW = 64 / CPW;
    CbLine<HORIZ, MODE, FULL, SCALE, RV, KW, CPW, LAGC> L;
    constexpr int T = CbCfg<HORIZ, MODE, KW>::T;
    constexpr int NSETS = CbCfg<HORIZ, MODE, KW>::NSETS;
    L.lane = (KW > 1 || WPB > 1) ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
    L.kk = L.lane % CW;
    L.cl = L.lane / CW;
    L.wv = KW > 1 ? (int)(threadIdx.x >> 6) : 0;
    const int wb = WPB > 1 ? (int)(threadIdx.x >> 6) : 0;      // independent wave of a WPB block
    const int nchunks = (a.D + CW - 1) / CW;
    const int ngroups = ((HORIZ ? a.H : a.W) + KW * WPB * CPW - 1) / (KW * WPB * CPW);   // KW = WPB = CPW = 1: one line per block
    const int per_pair = ngroups * nchunks;
    const int b = blk / per_pair;
    const int lc = blk - b * per_pair;
    // V sweeps, chunk-major (SM_CB_CHUNK_MAJOR_V): the blocks resident on one XCD are
    // consecutive columns of ONE disparity chunk, whose other-image spans [u - c64 - 63, u - c64]
    // overlap almost entirely, instead of 1/nchunks as many columns of every chunk
    const bool cmaj = !HORIZ && SM_CB_CHUNK_MAJOR_V;
    const int grp = cmaj ? lc % ngroups : lc / nchunks;
    const int chunk = cmaj ? lc / ngroups : lc - grp * nchunks;
    L.line = grp * KW * WPB * CPW + L.wv + wb;   // CPW > 1: the wave's first column u0
    L.colok = CPW == 1 || L.line + L.cl < a.W;
    // a WPB block's spare waves (past the last column) only zero their rings and pass the barrier
    const bool spare = WPB > 1 && L.line >= (HORIZ ? a.H : a.W);
    if (spare) L.line = (HORIZ ? a.H : a.W) - 1;
    L.active = true;
    if (KW > 1 && L.line >= (HORIZ ? a.H : a.W)) {   // spare wave: runs column W - 1, stores nothing
        L.active = false;
        L.line = (HORIZ ? a.H : a.W) - 1;
    }
    const size_t npix = (size_t)a.H * a.W;
    const size_t first_pix = HORIZ ? (size_t)L.line * a.W : (size_t)L.line;
    L.pstride = HORIZ ? 1 : a.W;
    L.vsb = (uint32_t)(L.pstride * a.D * 4);
    L.xline = (const char*)(a.vm + ((size_t)b * npix + first_pix) * a.D + (size_t)chunk * CW);
    const int dl = chunk * CW + L.kk;  // true disparity (also for masked lanes)
    {
        // CPW > 1: lane's element of column u0 + cl; lanes of columns past W (non-FULL launches
        // only) load column W - 1 and store nothing
        const int lc = CPW == 1 ? 0 : min(L.cl, a.W - 1 - L.line);
        const uint32_t xv = FULL ? (uint32_t)(L.cl * a.D + L.kk) * 4u : (uint32_t)(lc * a.D + min(L.kk, a.D - 1 - chunk * CW)) * 4u;
#pragma unroll
        for (int k = 0; k < T; k++) L.xo[k] = xv + (uint32_t)k * L.vsb;
        L.ov = (FULL || (dl < a.D && L.colok)) ? (uint32_t)(L.cl * a.D + L.kk) * 4u : 0x80000000u;
    }
    L.xend = (const char*)a.vm_end;
    L.aend = (const char*)a.arms_end;
    // arm planes: [b][view][plane][npix]; plane 0 = (L | R<<16), plane 1 = (U | D<<16)
    // own = this view's image, other = the image it is matched against
    const int pass_plane = HORIZ ? 0 : 1, perp_plane = HORIZ ? 1 : 0;
    const int own = RV ? 2 : 0, other = RV ? 0 : 2;
    const uint32_t* planeL = a.arms + ((size_t)b * 4) * npix + first_pix;
    const int line_bytes = (((HORIZ ? a.W : a.H) - 1) * L.pstride + CPW) * 4;   // CPW columns from u0
#pragma unroll
    for (int s = 0; s < NSETS; s++) {
        const int pl = (s == 1) ? perp_plane : pass_plane;
        L.A0r[s] = buf_rsrc(planeL + (size_t)(own + pl) * npix, line_bytes);
        L.A1r[s] = buf_rsrc(planeL + (size_t)(other + pl) * npix, line_bytes);
        L.A1v[s] = (const char*)(a.arms + ((size_t)b * 4 + other + pl) * npix);
        L.sh[s] = 0u;
    }
    if (!HORIZ) {
        // other image's column: u - d (left view) or u + d (right view); lanes whose column lies
        // outside the image get an out-of-range offset, so their gathers return the reference's
        // zeroed intersection (cpp:2794-2845) without a mask per position
        const int u = L.line + L.cl;
        bool out = RV ? u + dl >= a.W : u - dl < 0;
        uint32_t col = (uint32_t)(RV ? u + dl : u - dl) * 4u;
        if (SM_CB_PROBE_NOVG == 3) {   // timing probe: every wave gathers columns 0..63 of the right rows
            out = false;
            col = (uint32_t)L.lane * 4u;
        } else if (SM_CB_PROBE_NOVG == 4) {   // timing probe: 16 distinct words per gather (lane & 15)
            out = L.line - (chunk * 64 + (L.lane & 15)) < 0;
            col = (uint32_t)(L.line - (chunk * 64 + (L.lane & 15))) * 4u;
        }
#pragma unroll
        for (int k = 0; k < (HORIZ ? 1 : T); k++) L.ao[k] = out ? 0x80000000u : col + (uint32_t)(k * a.W * 4);
    }
    L.c64 = chunk * CW;
    L.len = HORIZ ? a.W : a.H;
    L.lag = a.lag;
    L.ring = cbca_ring(a.lag, HORIZ, MODE, KW);
    L.shist = 0u;
    L.msafe = (2 * a.lag + T - 1) / T;
    if constexpr (decltype(L)::REUSE2) {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int k = 0; k < T; k++) L.ph[r][k] = 0u;   // positions before the line: zero arms
    }
    if (HORIZ && RV && !SM_CB_LDS_WIN) {
        // right view: the window before each set's first position p0 = -off holds, in lane l, the
        // left image's arm pair at p0 - 1 + c64 + l (0 outside the line)
#pragma unroll
        for (int s = 0; s < NSETS; s++) {
            const int q = -L.set_off(s) - 1 + chunk * 64 + L.lane;
            L.sh[s] = buf_ld_u32(L.A1r[s], (unsigned)q < (unsigned)a.W ? (uint32_t)q * 4u : 0x80000000u, 0);
        }
    }
    const int ring_words = cbca_ring_words(a.lag, HORIZ, MODE, KW);
    // this wave's rings (WPB blocks: each wave's rings + window words)
    float* const mine = KW > 1 ? smem + (size_t)L.wv * ring_words
                               : (WPB > 1 ? smem + (size_t)wb * cbca_smem_words(a.lag, HORIZ, MODE) : smem);
    L.r1 = mine;
    L.r2 = mine + (size_t)L.ring * 64;
    L.ra = (uint16_t*)(mine + (size_t)L.ring * 64 * (MODE == CB_NORM_SCAN ? 2 : 1));
    {
        typedef __attribute__((address_space(3))) char lds_c;
        L.o1 = (uint32_t)(size_t)(lds_c*)L.r1 + 4u * (uint32_t)L.lane;
        L.o2 = (uint32_t)(size_t)(lds_c*)L.r2 + 4u * (uint32_t)L.lane;
        L.oa = (uint32_t)(size_t)(lds_c*)L.ra + 2u * (uint32_t)L.lane;
    }
    L.wown = (uint32_t*)((KW > 1 ? smem : mine) + ring_words);
    L.wspan = L.wown + NSETS * T;
    L.scale = a.scale;
    {   // zero the rings: reads of positions before the line start then yield S = 0, area = 0
        const int words = KW > 1 ? ring_words : cbca_smem_words(a.lag, HORIZ, MODE);
        for (int w = L.lane; w < words; w += 64) mine[w] = 0.f;
    }
    if constexpr (KW > 1) {
        // staged word idx = m * 64 KW + tid of a tile: [set s][row k][KW own | KW + 63 other]
        constexpr int SPW = cbca_spw(KW);
        constexpr int NW = CbCfg<HORIZ, MODE, KW>::NW;
        constexpr int NV = CbCfg<HORIZ, MODE, KW>::NV;
        L.stg = (uint32_t*)(smem + (size_t)KW * ring_words);
        L.sbuf = 1;
        L.H = a.H;
        L.rowb = (uint32_t)a.W * 4u;
        L.Ar = buf_rsrc(a.arms + (size_t)b * 4 * npix, (int)(4 * npix * 4));
        const int u0 = grp * KW;
        const int own = RV ? 2 : 0, other = RV ? 0 : 2;
        L.sok = 0;
#pragma unroll
        for (int m = 0; m < NV; m++) {
            const int idx = m * 64 * KW + (int)threadIdx.x;
            const int sset = idx / (T * SPW);
            const int rem = idx - sset * (T * SPW);
            const int k = rem / SPW;
            const int c = rem - k * SPW;
            const int pl = sset == 1 ? 0 : 1;   // V sweeps: pass pair = (U | D) plane 1, perpendicular = plane 0
            const int plane = (c < KW ? own : other) + pl;
            const int col = c < KW ? u0 + c : (RV ? u0 + L.c64 + (c - KW) : u0 - L.c64 - 63 + (c - KW));
            L.skoff[m] = k - (sset == 0 ? a.lag : 0);
            L.sboff[m] = ((uint32_t)plane * (uint32_t)npix + (uint32_t)(col < 0 ? 0 : col)) * 4u;
            if (idx < NW && col >= 0 && col < a.W) L.sok |= 1u << m;
        }
    }
    __syncthreads();  // orders the float ring stores before the u16 ring reads (and across waves)
    if (spare) return;   // WPB blocks have no later barrier
    L.S1 = L.S2 = 0.f;
    L.Acc = 0;
    L.ws = 0;
    L.wrs = 0;
    if constexpr (HORIZ && SM_CB_LDS_WIN && SM_CB_WIN_RING) {
        // span-ring prologue: the first tile's words q0 .. q0 + 62 of every set (the tiles add the rest)
        constexpr int R = cbca_win_ring(T);
#pragma unroll
        for (int s = 0; s < NSETS; s++) {
            const int base = -L.set_off(s);
            const int q = (RV ? base + L.c64 : base - L.c64 - 63) + L.lane;
            const uint32_t w = buf_ld_u32(L.A1r[s], (L.lane < 63 && (unsigned)q < (unsigned)L.len) ? (uint32_t)q * 4u : 0x80000000u, 0);
            if (L.lane < 63) {
                L.wspan[s * 2 * R + L.lane] = w;
                L.wspan[s * 2 * R + L.lane + R] = w;
            }
        }
    }
    const int nst = L.len + a.lag * (MODE == CB_NORM_SCAN ? 2 : 1);
    typename CbLine<HORIZ, MODE, FULL, SCALE, RV, KW, CPW, LAGC>::Tile ta, tb, tc, td;
    if constexpr (CbCfg<HORIZ, MODE, KW>::PF == 3) {
        L.load(ta, 0);
        L.load(tb, T);
        L.load(tc, 2 * T);
        for (int j0 = 0; j0 < nst; j0 += 4 * T) {
            L.load(td, j0 + 3 * T);
            L.template process<0>(ta, j0);
            if (j0 + T >= nst) break;
            L.load(ta, j0 + 4 * T);
            L.template process<1>(tb, j0 + T);
            if (j0 + 2 * T >= nst) break;
            L.load(tb, j0 + 5 * T);
            L.template process<2>(tc, j0 + 2 * T);
            if (j0 + 3 * T >= nst) break;
            L.load(tc, j0 + 6 * T);
            L.template process<3>(td, j0 + 3 * T);
        }
    } else if constexpr (CbCfg<HORIZ, MODE, KW>::PF == 2) {
        L.load(ta, 0);
        L.load(tb, T);
        for (int j0 = 0; j0 < nst; j0 += 3 * T) {
            L.load(tc, j0 + 2 * T);
            L.process(ta, j0);
            if (j0 + T >= nst) break;
            L.load(ta, j0 + 3 * T);
            L.process(tb, j0 + T);
            if (j0 + 2 * T >= nst) break;
            L.load(tb, j0 + 4 * T);
            L.process(tc, j0 + 2 * T);
        }
    } else {
        L.load(ta, 0);
        for (int j0 = 0; j0 < nst; j0 += 2 * T) {
            L.load(tb, j0 + T);
            L.process(ta, j0);
            if (j0 + T >= nst) break;
            L.load(ta, j0 + 2 * T);
            L.process(tb, j0 + T);
        }
    }
}

template <bool HORIZ, int MODE, bool FULL, bool SCALE, bool RV, int KW, bool PERSIST, int WPB, int LAGC = 0>
__global__ __launch_bounds__(64 * KW * WPB) void k_cbca(const CbcaArgs a, const int nlines) {
    extern __shared__ float smem[];
    const int slot = xcd_swizzle(blockIdx.x, gridDim.x);   // neighbouring lines on one XCD
    if (!PERSIST) {
        cbca_run_line<HORIZ, MODE, FULL, SCALE, RV, KW, WPB, LAGC>(a, slot, smem);
        return;
    }
    for (int blk = slot; blk < nlines; blk += gridDim.x) {   // every block exits after its last line
        cbca_run_line<HORIZ, MODE, FULL, SCALE, RV, KW, WPB, LAGC>(a, blk, smem);
        __syncthreads();   // the next line's ring zeroing follows this line's last ring reads
    }
}

template <bool HORIZ, int MODE, bool SCALE, int KW, int WPB = 1>
static void launch_kw(const CbcaArgs& a, int n, hipStream_t st) {
    constexpr int CPW = cbca_cpw(HORIZ, MODE, KW, WPB);
    const int nchunks = (a.D + 64 / CPW - 1) / (64 / CPW);
    const int groups = ((HORIZ ? a.H : a.W) + KW * WPB * CPW - 1) / (KW * WPB * CPW);
    const int nlines = groups * nchunks * n;
    const size_t shm = 4 * (size_t)(KW > 1 ? cbca_smem_words_vg(a.lag, MODE, KW) : WPB * cbca_smem_words(a.lag, HORIZ, MODE));
    const bool full = a.D % (64 / CPW) == 0 && (HORIZ || a.W % CPW == 0);
    constexpr bool PERSIST = !HORIZ && KW == 1 && WPB == 1 && SM_CB_PERSIST_V;
    int nblk = nlines;
    if (PERSIST) {
        // resident blocks: LDS-bound (160 KiB per CU), at most 8 waves per CU
        const int per_cu = std::max(1, std::min(8, (int)((160 * 1024) / std::max<size_t>(shm, 1))));
        nblk = std::min(nlines, per_cu * a.num_cu);
    }
    dim3 grid(nblk), block(64 * KW * WPB);
    if constexpr (!HORIZ && MODE == CB_NORM_SCAN && KW == 1 && WPB == 1 && !PERSIST && SM_CB_NS_REUSE) {
        if (a.lag == 34) {   // the reference's cbca_crossL_out (h:266)
            if (a.view == 0) {
                if (full) hipLaunchKernelGGL((k_cbca<HORIZ, MODE, true, SCALE, false, KW, PERSIST, WPB, 34>), grid, block, shm, st, a, nlines);
                else hipLaunchKernelGGL((k_cbca<HORIZ, MODE, false, SCALE, false, KW, PERSIST, WPB, 34>), grid, block, shm, st, a, nlines);
            } else {
                if (full) hipLaunchKernelGGL((k_cbca<HORIZ, MODE, true, SCALE, true, KW, PERSIST, WPB, 34>), grid, block, shm, st, a, nlines);
                else hipLaunchKernelGGL((k_cbca<HORIZ, MODE, false, SCALE, true, KW, PERSIST, WPB, 34>), grid, block, shm, st, a, nlines);
            }
            return;
        }
    }
    if (a.view == 0) {
        if (full) hipLaunchKernelGGL((k_cbca<HORIZ, MODE, true, SCALE, false, KW, PERSIST, WPB>), grid, block, shm, st, a, nlines);
        else hipLaunchKernelGGL((k_cbca<HORIZ, MODE, false, SCALE, false, KW, PERSIST, WPB>), grid, block, shm, st, a, nlines);
    } else {
        if (full) hipLaunchKernelGGL((k_cbca<HORIZ, MODE, true, SCALE, true, KW, PERSIST, WPB>), grid, block, shm, st, a, nlines);
        else hipLaunchKernelGGL((k_cbca<HORIZ, MODE, false, SCALE, true, KW, PERSIST, WPB>), grid, block, shm, st, a, nlines);
    }
}

template <bool HORIZ, int MODE, bool SCALE>
static void launch_scaled(const CbcaArgs& a, int n, hipStream_t st) {
    constexpr int KW = cbca_kw(HORIZ, MODE);
    if constexpr (KW > 1) {
        // the group's rings and staging must fit one CU's 160 KiB of LDS (lag <= 34 does)
        if (4 * (size_t)cbca_smem_words_vg(a.lag, MODE, KW) <= 160 * 1024) return launch_kw<HORIZ, MODE, SCALE, KW>(a, n, st);
    }
    constexpr int WPB = cbca_wpb(HORIZ, MODE);
    if constexpr (WPB > 1) {
        // WPB waves' rings must fit one CU's 160 KiB of LDS (else one wave per block)
        if (4 * (size_t)WPB * cbca_smem_words(a.lag, HORIZ, MODE) <= 160 * 1024) return launch_kw<HORIZ, MODE, SCALE, 1, WPB>(a, n, st);
    }
    launch_kw<HORIZ, MODE, SCALE, 1>(a, n, st);
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
