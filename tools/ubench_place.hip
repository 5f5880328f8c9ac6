// ubench_place.hip — does a plain line sweep see the "fast / slow placement" of a volume
// allocation?  Allocates NB volumes of the full-resolution batch size (2 pairs x
// 3000 x 2000 x 256 floats = 12.3 GB) and times, interleaved, a sweep with the CBCA H scan's
// access shape on each: one wave per (row, 64-disparity chunk), position by position along the
// row (stride D floats), reading and writing 256 bytes per position, a running prefix in registers.
// usage: ubench_place [NB] [rounds]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(64) void k_sweep(float* vm, int H, int W, int D, int n) {
    const int chunks = D / 64;
    const long blk = blockIdx.x;
    const int lane = threadIdx.x;
    const long per_pair = (long)H * chunks;
    const long b = blk / per_pair, r = blk % per_pair;
    const int row = (int)(r / chunks), ch = (int)(r % chunks);
    float* p = vm + (((size_t)b * H + row) * W) * D + ch * 64 + lane;
    float s = 0.f;
    float x0 = __builtin_nontemporal_load(p);
    for (int j = 0; j < W; j++) {
        const float x1 = j + 1 < W ? __builtin_nontemporal_load(p + (size_t)(j + 1) * D) : 0.f;
        s += x0;
        __builtin_nontemporal_store(s, p + (size_t)j * D);
        x0 = x1;
    }
}

int main(int argc, char** argv) {
    const int NB = argc > 1 ? atoi(argv[1]) : 4, rounds = argc > 2 ? atoi(argv[2]) : 3;
    const int H = 2000, W = 3000, D = 256, n = 2;
    const size_t elems = (size_t)n * H * W * D;
    std::vector<float*> bufs(NB);
    for (int i = 0; i < NB; i++) {
        CK(hipMalloc(&bufs[i], elems * 4));
        CK(hipMemset(bufs[i], 0, elems * 4));
        printf("buf %d at %p\n", i, (void*)bufs[i]);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 grid((unsigned)((long)n * H * (D / 64))), block(64);
    std::vector<std::vector<float>> t(NB);
    for (int r = 0; r < rounds; r++)
        for (int i = 0; i < NB; i++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_sweep, grid, block, 0, 0, bufs[i], H, W, D, n);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms);
        }
    for (int i = 0; i < NB; i++) {
        printf("buf %d:", i);
        for (float x : t[i]) printf(" %.3f", x);
        printf(" ms\n");
    }
    for (float* b : bufs) CK(hipFree(b));
    return 0;
}
