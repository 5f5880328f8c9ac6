// Microbenchmark: the CBCA line-sweep memory pattern without the ring arithmetic.
// One 64-lane wave per line, lane = disparity, sequential positions, T positions per tile,
// PF tiles prefetched; dynamic LDS throttles occupancy like the real rings do.
// build: hipcc --offload-arch=gfx950 -O3 -o ubench_stream ubench_stream.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int T>
struct Tile {
    float x[T];
};

template <int T, int PF>
__global__ __launch_bounds__(64) void k_stream(const float* __restrict__ in, float* __restrict__ out, int len, int D,
                                               size_t stride_line, int vstride) {
    extern __shared__ float sm[];
    const int lane = threadIdx.x;
    const float* ib = in + blockIdx.x * stride_line + lane;
    float* ob = out + blockIdx.x * stride_line + lane;
    if (lane == 0 && len < 0) sm[0] = 1;  // keep the LDS allocation
    float S = 0.f;
    Tile<T> t[PF + 1];
    auto load = [&](Tile<T>& tt, int j0) {
#pragma unroll
        for (int k = 0; k < T; k++) tt.x[k] = ib[(size_t)min(j0 + k, len - 1) * vstride];
    };
    auto proc = [&](const Tile<T>& tt, int j0) {
#pragma unroll
        for (int k = 0; k < T; k++) {
            S += tt.x[k];
            if (j0 + k < len) ob[(size_t)(j0 + k) * vstride] = S;
        }
    };
#pragma unroll
    for (int p = 0; p < PF; p++) load(t[p], p * T);
    for (int j0 = 0; j0 < len; j0 += (PF + 1) * T) {
#pragma unroll
        for (int p = 0; p <= PF; p++) {
            load(t[(p + PF) % (PF + 1)], j0 + (p + PF) * T);
            proc(t[p], j0 + p * T);
        }
    }
}

template <int T, int PF>
static float run(const float* in, float* out, int lines, int len, int D, bool horiz, size_t shm, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const size_t stride_line = horiz ? (size_t)len * D : (size_t)D;
    const int vstride = horiz ? D : lines * D;
    for (int r = 0; r < 2; r++)
        hipLaunchKernelGGL((k_stream<T, PF>), dim3(lines), dim3(64), shm, 0, in, out, len, D, stride_line, vstride);
    hipEventRecord(a);
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL((k_stream<T, PF>), dim3(lines), dim3(64), shm, 0, in, out, len, D, stride_line, vstride);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const int pairs = 16, H = 375, W = 450, D = 64;
    const size_t n = (size_t)pairs * H * W * D;
    float *in, *out;
    hipMalloc(&in, n * 4);
    hipMalloc(&out, n * 4);
    hipMemset(in, 0, n * 4);
    const double bytes = 2.0 * n * 4;
    const size_t shms[] = {0, 16384, 24576, 32768};
    for (size_t shm : shms) {
        // H sweep: lines = pairs*H rows of W positions
        float t1 = run<16, 1>(in, out, pairs * H, W, D, true, shm, 10);
        float t2 = run<16, 2>(in, out, pairs * H, W, D, true, shm, 10);
        float t3 = run<8, 3>(in, out, pairs * H, W, D, true, shm, 10);
        float t4 = run<32, 1>(in, out, pairs * H, W, D, true, shm, 10);
        printf("H shm %6zu  T16PF1 %.3f ms %.0f GB/s | T16PF2 %.3f %.0f | T8PF3 %.3f %.0f | T32PF1 %.3f %.0f\n", shm, t1,
               bytes / t1 / 1e6, t2, bytes / t2 / 1e6, t3, bytes / t3 / 1e6, t4, bytes / t4 / 1e6);
        // V sweep (one pair-stack treated as W*pairs columns of H positions)
        float v1 = run<16, 1>(in, out, pairs * W, H, D, false, shm, 10);
        float v2 = run<16, 2>(in, out, pairs * W, H, D, false, shm, 10);
        printf("V shm %6zu  T16PF1 %.3f ms %.0f GB/s | T16PF2 %.3f %.0f\n", shm, v1, bytes / v1 / 1e6, v2, bytes / v2 / 1e6);
    }
    hipFree(in);
    hipFree(out);
    return 0;
}
