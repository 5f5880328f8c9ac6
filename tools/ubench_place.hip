// ubench_place.hip — does a plain line sweep see the "fast / slow placement" of a volume
// allocation, and does a row pitch that is not a multiple of 1 MiB remove it?
// Allocates NB volumes of the full-resolution batch size (2 pairs x 3000 x 2000 x 256 floats =
// 12.3 GB, plus room for the largest row pad) and times, interleaved, a sweep with the CBCA H
// scan's access shape on each: one wave per (row, 64-disparity chunk), position by position along
// the row (stride D floats), reading and writing 256 bytes per position, a running prefix in
// registers.  Rows start every W * D + pad floats (pad 0: the dense layout, whose row starts are
// all 0 or 1 MiB modulo the 2 MiB page, so the waves in flight differ only in physical page bits).
// usage: ubench_place [NB] [rounds] [pad,pad,...]   (pads in floats)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(64) void k_sweep(float* vm, int H, int W, int D, size_t pitch) {
    const int chunks = D / 64;
    const long blk = blockIdx.x;
    const int lane = threadIdx.x;
    const long per_pair = (long)H * chunks;
    const long b = blk / per_pair, r = blk % per_pair;
    const int row = (int)(r / chunks), ch = (int)(r % chunks);
    float* p = vm + ((size_t)b * H + row) * pitch + ch * 64 + lane;
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
    std::vector<long> pads;
    if (argc > 3) {
        char* s = strdup(argv[3]);
        for (char* t = strtok(s, ","); t; t = strtok(nullptr, ",")) pads.push_back(atol(t));
        free(s);
    } else {
        pads.push_back(0);
    }
    long maxpad = 0;
    for (long p : pads) maxpad = p > maxpad ? p : maxpad;
    const int H = 2000, W = 3000, D = 256, n = 2;
    const size_t elems = (size_t)n * H * ((size_t)W * D + maxpad);
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
    std::vector<std::vector<std::vector<float>>> t(NB, std::vector<std::vector<float>>(pads.size()));
    for (int r = 0; r < rounds; r++)
        for (int i = 0; i < NB; i++)
            for (size_t q = 0; q < pads.size(); q++) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_sweep, grid, block, 0, 0, bufs[i], H, W, D, (size_t)W * D + pads[q]);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                t[i][q].push_back(ms);
            }
    for (int i = 0; i < NB; i++)
        for (size_t q = 0; q < pads.size(); q++) {
            printf("buf %d pad %6ld:", i, pads[q]);
            for (float x : t[i][q]) printf(" %.3f", x);
            printf(" ms\n");
        }
    for (float* b : bufs) CK(hipFree(b));
    return 0;
}
