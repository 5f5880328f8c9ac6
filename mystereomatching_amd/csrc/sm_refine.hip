// sm_refine.hip — disparity refinement (refine(), stereoMatching.cpp:1138-1511, the non-
// USE_RECONCV branch cpp:1347-1510, run by main_.cpp:165-166 when Do_refine).
//
// Default stage switches (stereoMatching.h:72-81): LR consistency check, region_vote_nums (2) x
// regionVote_my, region_vote_nums x properIpol, then a 3x3 median.  All stages work on int16
// H x W maps (2 bytes per pixel, a few MB even at full resolution), so they are cheap next to the
// W x H x D volume passes; every stage that reads neighbours is Jacobi (reads the previous map,
// writes a new one) exactly like the reference's dp_res / DpCopy / OpenCV's copied source.
//
// Mapping: one thread per pixel, 256-thread blocks over [pair][row-tile][col-tile] 64 x 4 tiles so
// a wave covers one 64-pixel row segment (coalesced int16 accesses); valid pixels exit at once,
// the holes (typically 5-20 %) do the searches.  Maps and arms are re-read from L2 / MALL.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

namespace sm {

namespace {

__device__ __forceinline__ int colour_dif(uint32_t x, uint32_t y) {  // max_c |I(x)_c - I(y)_c|
    return max(max(abs((int)(x & 0xff) - (int)(y & 0xff)), abs((int)((x >> 8) & 0xff) - (int)((y >> 8) & 0xff))),
               abs((int)((x >> 16) & 0xff) - (int)((y >> 16) & 0xff)));
}

constexpr int TX = 64, TY = 4;

struct Pix {
    int b, v, u;
    bool ok;
};

__device__ __forceinline__ Pix pixel_of(int H, int W) {
    const int tiles_x = (W + TX - 1) / TX, tiles_y = (H + TY - 1) / TY;
    const int per_pair = tiles_x * tiles_y;
    const int blk = blockIdx.x;
    Pix p;
    p.b = blk / per_pair;
    const int t = blk - p.b * per_pair;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    p.u = tx * TX + (int)(threadIdx.x & (TX - 1));
    p.v = ty * TY + (int)(threadIdx.x / TX);
    p.ok = p.u < W && p.v < H;
    return p;
}

dim3 grid_of(int n, int H, int W) { return dim3((unsigned)(n * ((W + TX - 1) / TX) * ((H + TY - 1) / TY))); }

// LRConsistencyCheck_normal (cpp:2262-2282), LOR = 0, in place: d < 0, u - d < 0 or
// |d - D2(u - d)| > LRmaxDiff  ->  -1.  The int difference is compared as a float (int > float).
__global__ __launch_bounds__(256) void k_lr_check(int16_t* __restrict__ d0, const int16_t* __restrict__ d1, int H, int W,
                                                  float maxdiff) {
    const Pix p = pixel_of(H, W);
    if (!p.ok) return;
    const size_t row = ((size_t)p.b * H + p.v) * W;
    const int d = d0[row + p.u];
    if (d < 0 || p.u - d < 0 || (float)abs(d - (int)d1[row + p.u - d]) > maxdiff) d0[row + p.u] = -1;
}

// regionVote_my (cpp:7219-7277).  A hole collects the valid disparities of its cross region:
// rows v - U .. v + D of its column (its own vertical arms), each row spanning that row's pixel's
// L/R arms (HVL[0], the left image).  With validNum > rv_s, the first most frequent value `most`
// replaces the hole when hist[most] / validNum >= rv_ratio, where the division is an INTEGER
// division (cpp:7270): its value is 1 exactly when hist[most] == validNum (every valid neighbour
// agrees) and 0 otherwise.  For 0 < rv_ratio <= 1 the condition is therefore "all valid values
// are equal", i.e. min == max over the region, and `most` is that value — no histogram needed
// (rv_ratio > 1 never fills; the C-ABI rejects rv_ratio <= 0).
__global__ __launch_bounds__(256) void k_region_vote(const int16_t* __restrict__ src, int16_t* __restrict__ dst,
                                                     const uint32_t* __restrict__ arms, int H, int W, int rv_s,
                                                     int can_fill) {
    const Pix p = pixel_of(H, W);
    if (!p.ok) return;
    const size_t npix = (size_t)H * W;
    const int16_t* dp = src + (size_t)p.b * npix;
    const size_t o = (size_t)p.v * W + p.u;
    const int cur = dp[o];
    int out = cur;
    if (cur < 0 && can_fill) {
        const uint32_t* lr = arms + (size_t)p.b * 4 * npix;  // [b][view 0][plane 0] = L | R << 16
        const uint32_t* ud = lr + npix;                       // plane 1 = U | D << 16
        const uint32_t a = ud[o];
        const int v0 = p.v - (int)(a & 0xffff), v1 = p.v + (int)(a >> 16);
        int cnt = 0, mn = 0x7fff, mx = -1;
        for (int vn = v0; vn <= v1; vn++) {
            const uint32_t h = lr[(size_t)vn * W + p.u];
            const int16_t* row = dp + (size_t)vn * W;
            const int u0 = p.u - (int)(h & 0xffff), u1 = p.u + (int)(h >> 16);
            for (int un = u0; un <= u1; un++) {
                const int q = row[un];
                if (q >= 0) {
                    cnt++;
                    mn = min(mn, q);
                    mx = max(mx, q);
                }
            }
        }
        if (cnt > rv_s && mn == mx) out = mn;
    }
    dst[(size_t)p.b * npix + o] = (int16_t)out;
}

// properIpol (cpp:7395-7490).  A hole searches 16 directions, up to 20 steps each, for the first
// valid disparity; steps alternate pw / 2 and pw - pw / 2 (C truncating division).  DISP_OCC
// holes take the smallest disparity found; other holes the disparity whose pixel's colour is
// closest (max channel |diff| of I_c[0]), first strict minimum below 255 in direction order.
//
// Holes are sparse and scattered, so a block first compacts the holes of its 64 x 4 tile into an
// LDS list; then 16 lanes serve one hole, lane k walking direction k (positions move
// monotonically, so leaving the image ends the walk exactly like the reference's break), 5
// speculative loads per round to hide the L2 latency of the dependent walk; the group's result
// is a 16-lane min of (colour difference, direction) or of the disparity.
constexpr int PI_DEPTH = 20, PI_CHUNK = 5;
__global__ __launch_bounds__(256) void k_proper_ipol(const int16_t* __restrict__ src, int16_t* __restrict__ dst,
                                                     const uint32_t* __restrict__ px, int H, int W, int disp_occ) {
    __shared__ uint32_t holes[TX * TY];
    __shared__ int nholes;
    const Pix p = pixel_of(H, W);
    const size_t npix = (size_t)H * W;
    const int16_t* dp = src + (size_t)p.b * npix;
    if (threadIdx.x == 0) nholes = 0;
    __syncthreads();
    if (p.ok) {
        const size_t o = (size_t)p.v * W + p.u;
        const int cur = dp[o];
        if (cur >= 0)
            dst[(size_t)p.b * npix + o] = (int16_t)cur;
        else
            holes[atomicAdd(&nholes, 1)] = (uint32_t)threadIdx.x;
    }
    __syncthreads();
    const int n = nholes;
    const uint32_t* col = px + (size_t)p.b * 2 * npix;  // left view's packed BGR
    const int k = threadIdx.x & 15;
    const int DW[16] = {0, 2, 2, 2, 0, -2, -2, -2, 1, 2, 2, 1, -1, -2, -2, -1};
    const int DH[16] = {2, 2, 0, -2, -2, -2, 0, 2, 2, 1, -1, -2, -2, -1, 1, 2};
    const int pw = DW[k], ph = DH[k];
    const int sw0 = pw / 2, sh0 = ph / 2, sw1 = pw - pw / 2, sh1 = ph - ph / 2;
    // tile origin of this block (pixel_of maps threadIdx -> (u, v) inside it)
    const int u_org = p.u - (int)(threadIdx.x & (TX - 1)), v_org = p.v - (int)(threadIdx.x / TX);
    for (int base = 0; base < n; base += 16) {   // uniform trip count: every lane joins the shuffles
        const int hi = base + (int)(threadIdx.x >> 4);
        const bool act = hi < n;
        const uint32_t t = act ? holes[hi] : 0u;
        const int u = u_org + (int)(t & (TX - 1)), v = v_org + (int)(t / TX);
        const int cur = act ? (int)dp[(size_t)v * W + u] : 0;
        int found = -1, fu = 0, fv = 0;
        for (int t0 = 0; act && t0 < PI_DEPTH && found < 0; t0 += PI_CHUNK) {
            int q[PI_CHUNK], qu[PI_CHUNK], qv[PI_CHUNK];
#pragma unroll
            for (int j = 0; j < PI_CHUNK; j++) {
                const int st = t0 + j;
                const int n0 = (st + 2) >> 1, n1 = (st + 1) >> 1;   // even / odd steps taken
                qu[j] = u + n0 * sw0 + n1 * sw1;
                qv[j] = v + n0 * sh0 + n1 * sh1;
                const bool in = qu[j] >= 0 && qu[j] < W && qv[j] >= 0 && qv[j] < H;
                q[j] = in ? (int)dp[(size_t)qv[j] * W + qu[j]] : -32768;   // outside (ends the walk; sm_create
                                                                              // rejects DISP_OCC = -32768)
            }
#pragma unroll
            for (int j = PI_CHUNK - 1; j >= 0; j--)   // first valid step of the chunk before any exit
                if (q[j] >= 0) {
                    found = q[j];
                    fu = qu[j];
                    fv = qv[j];
                }
            // positions are monotone: after the first outside step every later one is outside, so
            // a valid step of the chunk always precedes the exit
            if (q[PI_CHUNK - 1] == -32768) break;
        }
        const bool occ = cur == disp_occ;
        // keys: occ -> the disparity; else (colour diff < 255) -> diff * 16 + direction
        uint32_t key = 0xffffffffu;
        if (found >= 0) {
            if (occ) {
                key = (uint32_t)found;
            } else {
                const int cd = colour_dif(col[(size_t)v * W + u], col[(size_t)fv * W + fu]);
                if (cd < 255) key = (uint32_t)(cd * 16 + k);
            }
        }
#pragma unroll
        for (int m = 8; m >= 1; m >>= 1) key = min(key, (uint32_t)__shfl_xor((int)key, m, 16));
        const int fsel = __shfl(found, (int)(key & 15), 16);   // all lanes take part
        const int res = key == 0xffffffffu ? cur : (occ ? (int)key : fsel);
        if (act && k == 0) dst[(size_t)p.b * npix + (size_t)v * W + u] = (int16_t)res;
    }
}

__device__ __forceinline__ void cswap(int& a, int& b) {
    const int lo = min(a, b), hi = max(a, b);
    a = lo;
    b = hi;
}

// cv::medianBlur(DP[0], DP[0], 3) (cpp:1497-1505): 3x3 median with replicated borders (OpenCV's
// sorting-network path; in place it filters a copy).  The median of 9 values is unique, so any
// exact selection network reproduces it: this is the 19-exchange median-of-9 network.
__global__ __launch_bounds__(256) void k_median3(const int16_t* __restrict__ src, int16_t* __restrict__ dst, int H, int W) {
    const Pix p = pixel_of(H, W);
    if (!p.ok) return;
    const size_t npix = (size_t)H * W;
    const int16_t* s = src + (size_t)p.b * npix;
    const int r0 = max(p.v - 1, 0) * W, r1 = p.v * W, r2 = min(p.v + 1, H - 1) * W;
    const int c0 = max(p.u - 1, 0), c1 = p.u, c2 = min(p.u + 1, W - 1);
    int x0 = s[r0 + c0], x1 = s[r0 + c1], x2 = s[r0 + c2];
    int x3 = s[r1 + c0], x4 = s[r1 + c1], x5 = s[r1 + c2];
    int x6 = s[r2 + c0], x7 = s[r2 + c1], x8 = s[r2 + c2];
    cswap(x1, x2); cswap(x4, x5); cswap(x7, x8);
    cswap(x0, x1); cswap(x3, x4); cswap(x6, x7);
    cswap(x1, x2); cswap(x4, x5); cswap(x7, x8);
    cswap(x0, x3); cswap(x5, x8); cswap(x4, x7);
    cswap(x3, x6); cswap(x1, x4); cswap(x2, x5);
    cswap(x4, x7); cswap(x4, x2); cswap(x6, x4);
    cswap(x4, x2);
    dst[(size_t)p.b * npix + (size_t)p.v * W + p.u] = (int16_t)x4;
}

}  // namespace

void launch_lr_check(int16_t* d0, const int16_t* d1, int n, int H, int W, float maxdiff, hipStream_t st) {
    hipLaunchKernelGGL(k_lr_check, grid_of(n, H, W), dim3(256), 0, st, d0, d1, H, W, maxdiff);
}

void launch_region_vote(const int16_t* src, int16_t* dst, const uint32_t* arms, int n, int H, int W, int rv_s,
                        float rv_ratio, hipStream_t st) {
    // hist/validNum is 0 or 1; 1 >= rv_ratio decides whether a unanimous region fills the hole
    const int can_fill = 1.0f >= rv_ratio ? 1 : 0;
    hipLaunchKernelGGL(k_region_vote, grid_of(n, H, W), dim3(256), 0, st, src, dst, arms, H, W, rv_s, can_fill);
}

void launch_proper_ipol(const int16_t* src, int16_t* dst, const uint32_t* px, int n, int H, int W, int disp_occ,
                        hipStream_t st) {
    hipLaunchKernelGGL(k_proper_ipol, grid_of(n, H, W), dim3(256), 0, st, src, dst, px, H, W, disp_occ);
}

void launch_median3(const int16_t* src, int16_t* dst, int n, int H, int W, hipStream_t st) {
    hipLaunchKernelGGL(k_median3, grid_of(n, H, W), dim3(256), 0, st, src, dst, H, W);
}

}  // namespace sm
