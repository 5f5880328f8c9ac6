// sm_pyramid.hip — the cross-scale pyramid of main_.cpp:131-158 (PY_LEV > 1).
//
//   pyrDown   cv::pyrDown on the u8 colour / gray inputs (main_.cpp:145-148): 5x5 binomial
//             1-4-6-4-1 filter, BORDER_REFLECT_101, (sum + 128) >> 8, every second row / column.
//   SolveAll  (stereoMatching.cpp:2142-2208) for PY_LVL levels: level 0's volume becomes
//             sum_s invWgt[s] * vm_s(y >> s, x >> s, d_s), d_s = (d_{s-1} + 1) / 2, summed in level
//             order from 0.f (the host computes invWgt with OpenCV's small-matrix invert).
// Both are bandwidth-trivial next to the per-level cost / CBCA passes: pyrDown touches each input
// byte ~2x (cached), SolveAll reads level 0 (4 B / element) plus the coarse levels (1/8, 1/64 of
// that, mostly from L2) and writes level 0 once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

namespace sm {

namespace {

// one thread per destination pixel x channel; the 5 x 5 integer sum is exact, so any summation
// order equals OpenCV's separable row-then-column evaluation
__global__ __launch_bounds__(256) void k_pyr_down(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int rows,
                                                  int cols, int ch) {
    const int dr = (rows + 1) / 2, dc = (cols + 1) / 2;
    const size_t total = (size_t)dr * dc * ch;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % ch);
        const size_t px = i / ch;
        const int x = (int)(px % dc), y = (int)(px / dc);
        const int k[5] = {1, 4, 6, 4, 1};
        int cx[5];
#pragma unroll
        for (int j = 0; j < 5; j++) cx[j] = reflect101(2 * x + j - 2, cols);
        int sum = 0;
#pragma unroll
        for (int r = 0; r < 5; r++) {
            const uint8_t* row = src + (size_t)reflect101(2 * y + r - 2, rows) * cols * ch + c;
            int rs = 0;
#pragma unroll
            for (int j = 0; j < 5; j++) rs += k[j] * (int)row[(size_t)cx[j] * ch];
            sum += k[r] * rs;
        }
        dst[i] = (uint8_t)((sum + 128) >> 8);
    }
}

// cv::pyrDown on a 1-channel f32 image (main_.cpp:149: the ground truth DT goes down the pyramid
// with the inputs).  OpenCV's scalar pyrDown_ (FltCast<float, 8>) order, restated: the row pass
// r = s0*6 + (s-1 + s+1)*4 + s-2 + s+2 (left to right), the column pass the same over the five row
// sums, then * (1/256) (exact: a power of two).  OpenCV's SIMD rows may fuse multiply-adds, so the
// last bit is unpinned; only the evaluator reads DT, never the disparity path.
__global__ __launch_bounds__(256) void k_pyr_down_f32(const float* __restrict__ src, float* __restrict__ dst, int rows,
                                                      int cols) {
    const int dr = (rows + 1) / 2, dc = (cols + 1) / 2;
    const size_t total = (size_t)dr * dc;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % dc), y = (int)(i / dc);
        int cx[5];
#pragma unroll
        for (int j = 0; j < 5; j++) cx[j] = reflect101(2 * x + j - 2, cols);
        float r[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const float* row = src + (size_t)reflect101(2 * y + k - 2, rows) * cols;
            r[k] = row[cx[2]] * 6.f + (row[cx[1]] + row[cx[3]]) * 4.f + row[cx[0]] + row[cx[4]];
        }
        dst[i] = (r[2] * 6.f + (r[1] + r[3]) * 4.f + r[0] + r[4]) * (1.f / 256.f);
    }
}

// one wave per level-0 pixel (grid-stride), lanes over disparities; levels read in order
__global__ __launch_bounds__(256) void k_solve_all_pyr(const PyrArgs a) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const int H0 = a.H[0], W0 = a.W[0], D0 = a.D[0];
    const size_t npix0 = (size_t)H0 * W0;
    const size_t total = npix0 * (size_t)a.n;
    for (size_t q = wave; q < total; q += nwaves) {
        const size_t b = q / npix0, p = q - b * npix0;
        const int y = (int)(p / W0), x = (int)(p - (size_t)y * W0);
        for (int d = lane; d < D0; d += 64) {
            int cy = y, cx = x, cd = d;
            float sum = 0.f;
            for (int s = 0; s < a.levels; s++) {
                const size_t npix = (size_t)a.H[s] * a.W[s];
                const float cur = a.vm[s][(b * npix + (size_t)cy * a.W[s] + cx) * a.D[s] + cd];
                sum += a.w[s] * cur;
                cy >>= 1;
                cx >>= 1;
                cd = (cd + 1) >> 1;
            }
            a.vm[0][(b * npix0 + p) * D0 + d] = sum;
        }
    }
}

}  // namespace

void launch_pyr_down(const uint8_t* src, uint8_t* dst, int rows, int cols, int ch, hipStream_t st) {
    const size_t total = (size_t)((rows + 1) / 2) * ((cols + 1) / 2) * ch;
    size_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_pyr_down, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, rows, cols, ch);
}

void launch_pyr_down_f32(const float* src, float* dst, int rows, int cols, hipStream_t st) {
    const size_t total = (size_t)((rows + 1) / 2) * ((cols + 1) / 2);
    size_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_pyr_down_f32, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, rows, cols);
}

void launch_solve_all_pyr(const PyrArgs& a, hipStream_t st) {
    const size_t waves = (size_t)a.H[0] * a.W[0] * a.n;
    size_t blocks = (waves + 3) / 4;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_solve_all_pyr, dim3((unsigned)blocks), dim3(256), 0, st, a);
}

}  // namespace sm
