// Microbenchmark: the HBM write ceiling the cost-volume kernel is measured against.
// Pure stores (dword / dwordx4 per lane, default and non-temporal), a float4 read stream and a
// float4 copy, over buffers far larger than the 256 MB Infinity Cache.
// build: hipcc --offload-arch=gfx950 -O3 -o ubench_write ubench_write.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int NT>
__global__ __launch_bounds__(256) void k_st1(float* __restrict__ out, size_t n, float v) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        if (NT) __builtin_nontemporal_store(v, out + i);
        else out[i] = v;
    }
}
typedef float f4v __attribute__((ext_vector_type(4)));
template <int NT>
__global__ __launch_bounds__(256) void k_st4(f4v* __restrict__ out, size_t n4, float v) {
    const size_t stride = (size_t)gridDim.x * 256;
    const f4v x = {v, v, v, v};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        if (NT) __builtin_nontemporal_store(x, out + i);
        else out[i] = x;
    }
}
// one block writes a contiguous 32 KB segment (the cost kernel's shape: 128 pixels x 64 d x 4 B)
__global__ __launch_bounds__(256) void k_seg(float* __restrict__ out, float v) {
    float* o = out + (size_t)blockIdx.x * 8192;
    for (int i = threadIdx.x; i < 8192; i += 256) o[i] = v;
}
__global__ __launch_bounds__(256) void k_rd4(const float4* __restrict__ in, size_t n4, float* sink) {
    const size_t stride = (size_t)gridDim.x * 256;
    float acc = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        const float4 x = in[i];
        acc += x.x + x.y + x.z + x.w;
    }
    if (acc == 1234.5f) sink[0] = acc;
}
__global__ __launch_bounds__(256) void k_cp4(const float4* __restrict__ in, float4* __restrict__ out, size_t n4) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) out[i] = in[i];
}

#define TIME(label, bytes, launch)                                                                \
    do {                                                                                          \
        for (int r = 0; r < 2; r++) launch;                                                       \
        hipEventRecord(a);                                                                        \
        for (int r = 0; r < reps; r++) launch;                                                    \
        hipEventRecord(b);                                                                        \
        hipEventSynchronize(b);                                                                   \
        float ms;                                                                                 \
        hipEventElapsedTime(&ms, a, b);                                                           \
        ms /= reps;                                                                               \
        printf("%-28s %8.1f MB  %8.4f ms  %6.2f TB/s\n", label, (bytes) / 1e6, ms, (bytes) / ms / 1e9); \
    } while (0)

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? (size_t)atoll(argv[1]) : 691;
    const size_t bytes = mb * 1000000 / 32768 * 32768;
    const size_t n = bytes / 4, n4 = bytes / 16;
    float *x, *y;
    if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&y, bytes) != hipSuccess) return 1;
    hipMemset(x, 0, bytes);
    hipMemset(y, 0, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int reps = 10;
    for (int g : {2048, 8192, 32768}) {
        char l[64];
        snprintf(l, sizeof l, "store dword   grid %d", g);
        TIME(l, (double)bytes, hipLaunchKernelGGL(k_st1<0>, dim3(g), dim3(256), 0, 0, x, n, 1.f));
        snprintf(l, sizeof l, "store dword nt grid %d", g);
        TIME(l, (double)bytes, hipLaunchKernelGGL(k_st1<1>, dim3(g), dim3(256), 0, 0, x, n, 1.f));
        snprintf(l, sizeof l, "store x4      grid %d", g);
        TIME(l, (double)bytes, hipLaunchKernelGGL(k_st4<0>, dim3(g), dim3(256), 0, 0, (f4v*)x, n4, 1.f));
        snprintf(l, sizeof l, "store x4 nt   grid %d", g);
        TIME(l, (double)bytes, hipLaunchKernelGGL(k_st4<1>, dim3(g), dim3(256), 0, 0, (f4v*)x, n4, 1.f));
        snprintf(l, sizeof l, "read x4       grid %d", g);
        TIME(l, (double)bytes, hipLaunchKernelGGL(k_rd4, dim3(g), dim3(256), 0, 0, (const float4*)x, n4, y));
        snprintf(l, sizeof l, "copy x4 (R+W) grid %d", g);
        TIME(l, 2.0 * bytes, hipLaunchKernelGGL(k_cp4, dim3(g), dim3(256), 0, 0, (const float4*)x, (float4*)y, n4));
    }
    TIME("32KB segments/block", (double)bytes, hipLaunchKernelGGL(k_seg, dim3((unsigned)(bytes / 32768)), dim3(256), 0, 0, x, 1.f));
    hipFree(x);
    hipFree(y);
    return 0;
}
