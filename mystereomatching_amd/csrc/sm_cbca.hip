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
// kept in an LDS ring of 2*lag+2 slots (lag = longest arm), so each 1-D pass is ONE read and ONE
// write of the volume (the reference: two reads, two writes and a full-volume temporary).
// Kernel modes:
//   CB_SCAN       first pass of an iteration:            vm <- diff(prefix(vm))
//   CB_NORM       last pass of an iteration:             vm <- diff(prefix(vm)) / area  [* SolveAll]
//   CB_NORM_SCAN  last pass of iteration k fused with the first pass of iteration k+1 (both run
//                 along the same direction): two S rings, one sweep instead of two.
// Areas are integers (< 2^16): after the first pass of an iteration the area of (p,d) is
// tail+head+1 of that pass's intersection arms, so the normalising pass prefix-sums that value
// modulo 2^16 next to S — no area volume is ever stored.  In CB_NORM_SCAN the same LDS word also
// carries the position's (tail, head) so the arms are gathered once per position, not per use.
//
// Latency hiding: the next tile of T steps (volume values and arm words) is loaded into registers
// while the current tile is processed (loads of step j+T are legal before the stores of step j:
// stores trail the reads by `lag` positions).  Tiles that lie wholly in the steady state take a
// branch-free path so the compiler can overlap LDS round trips of consecutive steps; lanes past D
// read and write a private dummy slot instead of being masked.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

namespace sm {

__device__ __forceinline__ uint32_t bmin4(uint32_t a, uint32_t b) {
    uint32_t r = min(a & 0xffu, b & 0xffu);
    r |= min(a & 0xff00u, b & 0xff00u);
    r |= min(a & 0xff0000u, b & 0xff0000u);
    r |= min(a & 0xff000000u, b & 0xff000000u);
    return r;
}

template <int T, int NSETS>
struct CbTile {
    float x[T];            // vm at positions j0 .. j0+T-1
    uint32_t a0[NSETS];    // lane k < T: A0 at position (j0 + k - set offset)
    uint32_t a1[NSETS][T]; // A1 at (position, u - d) for this lane
};

template <bool HORIZ, int MODE, int T>
struct CbLine {
    // set 0 = positions i (= j - lag) for SCAN/NORM; set 1 = positions j (NORM); NS uses set 0 = j
    static constexpr int NSETS = MODE == CB_NORM ? 2 : 1;
    using Tile = CbTile<T, NSETS>;

    float* lvm;               // this lane's element of the line's first pixel (or a dummy slot)
    int lstride;              // floats between consecutive positions (0 for dummy lanes)
    const uint32_t* A0l;      // A0 + first pixel of the line
    const uint32_t* A1l;      // A1 + first pixel of the line
    int pstride;              // pixels between consecutive positions
    int line, len, lag, ring, d, lane;
    float S1, S2;
    uint32_t Acc;
    int ws;
    float* r1;
    float* r2;
    uint32_t* ra;             // NORM: area prefix (low 16 bits); NS: area16 << 16 | tail << 8 | head
    int apply_scale;
    float scale;

    __device__ __forceinline__ int set_off(int s) const {
        if (MODE == CB_NORM_SCAN) return 0;
        return s == 0 ? lag : 0;
    }
    __device__ __forceinline__ static int clampi(int k, int n) { return k < 0 ? 0 : (k >= n ? n - 1 : k); }

    __device__ __forceinline__ void load(Tile& t, int j0) const {
#pragma unroll
        for (int k = 0; k < T; k++) t.x[k] = lvm[clampi(j0 + k, len) * lstride];
#pragma unroll
        for (int s = 0; s < NSETS; s++) {
            const int base = j0 - set_off(s);
            t.a0[s] = A0l[clampi(base + lane, len) * pstride];
#pragma unroll
            for (int k = 0; k < T; k++) {
                const int q = clampi(base + k, len);
                const int uq = HORIZ ? q : line;
                t.a1[s][k] = A1l[q * pstride - (uq - d >= 0 ? d : uq)];  // u - d < 0 masked at use
            }
        }
    }

    __device__ __forceinline__ uint32_t isect(const Tile& t, int s, int k, int pos) const {
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)t.a0[s], k);
        const int u = HORIZ ? pos : line;
        const uint32_t a1 = (u - d >= 0) ? t.a1[s][k] : 0u;   // genTrueHorVerArms: 0 once u - d < 0
        return bmin4(a0, a1);
    }

    __device__ __forceinline__ int wrap1(int s) const { return s < 0 ? s + ring : s; }

    static constexpr int TSH = HORIZ ? 0 : 16, HSH = HORIZ ? 8 : 24;
    static constexpr int PTS = HORIZ ? 16 : 0, PHS = HORIZ ? 24 : 8;

    // One position of the sweep.  G = guarded (boundary tiles): every range test is evaluated;
    // G = false: the caller guarantees j < len, lag <= j (and 2*lag <= j for NS).
    template <bool G>
    __device__ __forceinline__ void step(const Tile& t, int k, int j) {
        const int sj = ws;  // slot of position j
        // ---- input at j
        if (!G || j < len) {
            const float x = t.x[k];
            S1 = (G && j == 0) ? x : S1 + x;
            r1[sj * 64 + lane] = S1;
            if (MODE == CB_NORM) {
                const uint32_t is = isect(t, 1, k, j);
                const uint32_t ain = ((is >> PTS) & 0xffu) + ((is >> PHS) & 0xffu) + 1u;
                Acc = (G && j == 0) ? ain : Acc + ain;
                ra[sj * 64 + lane] = Acc;
            } else if (MODE == CB_NORM_SCAN) {
                const uint32_t is = isect(t, 0, k, j);
                const uint32_t ain = ((is >> PTS) & 0xffu) + ((is >> PHS) & 0xffu) + 1u;
                Acc = (G && j == 0) ? ain : Acc + ain;
                ra[sj * 64 + lane] = (Acc << 16) | (((is >> TSH) & 0xffu) << 8) | ((is >> HSH) & 0xffu);
            }
        }
        // ---- first-stage output at i = j - lag
        const int i = j - lag;
        if (!G || (i >= 0 && i < len)) {
            const int si = wrap1(sj - lag);
            int tl, hd;
            if (MODE == CB_NORM_SCAN) {
                const uint32_t w = ra[si * 64 + lane];
                tl = (w >> 8) & 0xff;
                hd = w & 0xff;
            } else {
                const uint32_t is = isect(t, 0, k, i);
                tl = (is >> TSH) & 0xff;
                hd = (is >> HSH) & 0xff;
            }
            const int hs2 = (si + hd >= ring) ? si + hd - ring : si + hd;  // slot of i + head
            const int ts = wrap1(si - tl - 1);
            const bool inner = i - tl - 1 >= 0;
            const float sh = r1[hs2 * 64 + lane];
            const float st = r1[ts * 64 + lane];
            float out = sh - (inner ? st : 0.f);  // == inner ? sh - st : sh  (x - +0 == x)
            if (MODE == CB_SCAN) {
                lvm[i * lstride] = out;
            } else {
                const uint32_t ah = ra[hs2 * 64 + lane], at = ra[ts * 64 + lane];
                const uint32_t sh16 = MODE == CB_NORM_SCAN ? 16 : 0;
                const uint32_t area = ((ah >> sh16) - (inner ? (at >> sh16) : 0u)) & 0xffffu;
                out = out / (float)area;
                if (MODE == CB_NORM) {
                    if (apply_scale) {
                        float sum = 0.f;
                        sum += scale * out;
                        out = sum;
                    }
                    lvm[i * lstride] = out;
                } else {
                    S2 = (G && i == 0) ? out : S2 + out;   // prefix of iteration k+1's first pass
                    r2[si * 64 + lane] = S2;
                }
            }
        }
        // ---- second-stage output at i2 = j - 2*lag (NS only)
        if (MODE == CB_NORM_SCAN) {
            const int i2 = j - 2 * lag;
            if (!G || (i2 >= 0 && i2 < len)) {
                int s2 = sj - 2 * lag;
                s2 = s2 < 0 ? s2 + ring : s2;
                const uint32_t w = ra[s2 * 64 + lane];
                const int tl = (w >> 8) & 0xff, hd = w & 0xff;
                const int hs = (s2 + hd >= ring) ? s2 + hd - ring : s2 + hd;
                const int ts = wrap1(s2 - tl - 1);
                const float sh = r2[hs * 64 + lane];
                const float st = r2[ts * 64 + lane];
                lvm[i2 * lstride] = sh - ((i2 - tl - 1 >= 0) ? st : 0.f);
            }
        }
        ws = (ws + 1 == ring) ? 0 : ws + 1;
    }

    __device__ __forceinline__ void process(const Tile& t, int j0, int nst, int fast_lo) {
        if (j0 >= fast_lo && j0 + T <= len) {
#pragma unroll
            for (int k = 0; k < T; k++) step<false>(t, k, j0 + k);
        } else {
#pragma unroll
            for (int k = 0; k < T; k++)
                if (j0 + k < nst) step<true>(t, k, j0 + k);
        }
    }
};

template <bool HORIZ, int MODE, int T>
__global__ __launch_bounds__(64) void k_cbca(const CbcaArgs a) {
    extern __shared__ float smem[];
    CbLine<HORIZ, MODE, T> L;
    L.lane = threadIdx.x;
    const int nchunks = (a.D + 63) >> 6;
    L.line = blockIdx.x / nchunks;
    const int chunk = blockIdx.x - L.line * nchunks;
    const int b = blockIdx.y;
    L.d = chunk * 64 + L.lane;
    const bool valid = L.d < a.D;
    const size_t npix = (size_t)a.H * a.W;
    const size_t first_pix = HORIZ ? (size_t)L.line * a.W : (size_t)L.line;
    L.pstride = HORIZ ? 1 : a.W;
    L.lstride = valid ? L.pstride * a.D : 0;
    L.lvm = valid ? a.vm + ((size_t)b * npix + first_pix) * a.D + L.d : a.dummy + L.lane;
    L.A0l = a.arms + (size_t)b * 2 * npix + first_pix;
    L.A1l = L.A0l + npix;
    L.len = HORIZ ? a.W : a.H;
    L.lag = a.lag;
    L.ring = a.ring;
    L.r1 = smem;
    L.r2 = smem + (size_t)a.ring * 64;
    L.ra = (uint32_t*)(smem + (size_t)a.ring * 64 * (MODE == CB_NORM_SCAN ? 2 : 1));
    L.apply_scale = a.apply_scale;
    L.scale = a.scale;
    L.S1 = L.S2 = 0.f;
    L.Acc = 0;
    L.ws = 0;
    const int nst = L.len + a.lag * (MODE == CB_NORM_SCAN ? 2 : 1);
    const int fast_lo = a.lag * (MODE == CB_NORM_SCAN ? 2 : 1);
    typename CbLine<HORIZ, MODE, T>::Tile ta, tb;
    L.load(ta, 0);
    for (int j0 = 0; j0 < nst; j0 += 2 * T) {
        L.load(tb, j0 + T);
        L.process(ta, j0, nst, fast_lo);
        L.load(ta, j0 + 2 * T);
        L.process(tb, j0 + T, nst, fast_lo);
    }
}

template <bool HORIZ, int MODE>
static void launch_mode(const CbcaArgs& a, int n, hipStream_t st) {
    const int nchunks = (a.D + 63) / 64;
    const int lines = HORIZ ? a.H : a.W;
    dim3 grid(lines * nchunks, n);
    const int nrings = MODE == CB_SCAN ? 1 : (MODE == CB_NORM ? 2 : 3);
    const size_t shm = (size_t)a.ring * 64 * 4 * nrings;
    // tile depth: loads per tile (+ the tile's stores) must stay below the 6-bit vmcnt limit
    constexpr int T = MODE == CB_NORM ? 12 : 16;
    hipLaunchKernelGGL((k_cbca<HORIZ, MODE, T>), grid, dim3(64), shm, st, a);
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
