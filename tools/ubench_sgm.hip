// Microbenchmark: the SGM path-sweep memory pattern (read C, read acc, write acc) without the
// recurrence, against a flat elementwise acc += C over the same buffers.
//   k_lines: one wave per group of LPW lines, 64/LPW lanes per line, float4 chunks, T steps per
//            tile, two tiles in flight (the k_sgm_rows / k_sgm structure)
//   k_flat : grid-stride float4 acc += C (the streaming ceiling for these 3 passes)
// build: hipcc --offload-arch=gfx950 -O3 -o ubench_sgm ubench_sgm.hip
// usage: ./ubench_sgm H W D npairs
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int KV, int T, int LPW>
__global__ __launch_bounds__(256) void k_lines(const float* vm, float* acc, int H, int W, int D, int vert, int n) {
    constexpr int LL = 64 / LPW;  // lanes per line
    const int lane = threadIdx.x & 63, row = lane / LL, ll = lane % LL;
    const int nl = vert ? W : H, steps = vert ? H : W;
    const int wpp = (nl + LPW - 1) / LPW;
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256 + threadIdx.x) >> 6));
    const int b = wave / wpp;
    if (b >= n) return;
    const int w = wave - b * wpp;
    const int line = min(w * LPW + row, nl - 1);
    const size_t npix = (size_t)H * W;
    const float* vb = vm + (size_t)b * npix * D;
    float* ab = acc + (size_t)b * npix * D;
    const bool ok = ll * 4 * KV < D;
    auto addr = [&](int j, int c) -> size_t {
        const size_t p = vert ? (size_t)j * W + line : (size_t)line * W + j;
        return p * D + (size_t)(ll * KV + c) * 4;
    };
    float4 tc[2][T][KV], ta[2][T][KV];
    float4 run = make_float4(0, 0, 0, 0);
    auto load = [&](int buf, int j0) {
#pragma unroll
        for (int s = 0; s < T; s++)
#pragma unroll
            for (int c = 0; c < KV; c++) {
                const size_t o = addr(min(j0 + s, steps - 1), c);
                tc[buf][s][c] = *(const float4*)(vb + o);
                ta[buf][s][c] = *(const float4*)(ab + o);
            }
    };
    auto proc = [&](int buf, int j0) {
#pragma unroll
        for (int s = 0; s < T; s++) {
            if (j0 + s >= steps) break;
#pragma unroll
            for (int c = 0; c < KV; c++) {
                float4 v = tc[buf][s][c];
                run.x = fminf(run.x + v.x, 1e30f);
                run.y = fminf(run.y + v.y, 1e30f);
                run.z = fminf(run.z + v.z, 1e30f);
                run.w = fminf(run.w + v.w, 1e30f);
                float4 q = ta[buf][s][c];
                q.x += run.x; q.y += run.y; q.z += run.z; q.w += run.w;
                if (ok) *(float4*)(ab + addr(j0 + s, c)) = q;
            }
        }
    };
    load(0, 0);
    for (int j0 = 0; j0 < steps; j0 += 2 * T) {
        load(1, j0 + T);
        proc(0, j0);
        load(0, j0 + 2 * T);
        proc(1, j0 + T);
    }
}

__global__ __launch_bounds__(256) void k_flat(const float4* vm, float4* acc, size_t n4) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        float4 a = acc[i], v = vm[i];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        acc[i] = a;
    }
}

template <typename F>
static float timeit(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    f();
    hipEventRecord(a);
    for (int r = 0; r < reps; r++) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

template <int KV, int T, int LPW>
static void lines(const float* vm, float* acc, int H, int W, int D, int n, double bytes) {
    for (int vert = 0; vert < 2; vert++) {
        const int nl = vert ? W : H;
        const int waves = (nl + LPW - 1) / LPW * n;
        const float ms = timeit([&] { hipLaunchKernelGGL((k_lines<KV, T, LPW>), dim3((waves + 3) / 4), dim3(256), 0, 0, vm, acc, H, W, D, vert, n); }, 5);
        printf("lines KV=%d T=%d LPW=%d %s waves=%6d  %.3f ms  %.0f GB/s\n", KV, T, LPW, vert ? "vert " : "horiz", waves, ms, bytes / ms / 1e6);
    }
}

int main(int argc, char** argv) {
    const int H = atoi(argv[1]), W = atoi(argv[2]), D = atoi(argv[3]), n = atoi(argv[4]);
    const size_t elems = (size_t)n * H * W * D;
    float *vm, *acc;
    hipMalloc(&vm, elems * 4 + 65536);
    hipMalloc(&acc, elems * 4 + 65536);
    hipMemset(vm, 0, elems * 4);
    hipMemset(acc, 0, elems * 4);
    const double bytes = 3.0 * elems * 4;
    for (int g : {1024, 2048, 4096, 16384}) {
        const float ms = timeit([&] { hipLaunchKernelGGL(k_flat, dim3(g), dim3(256), 0, 0, (const float4*)vm, (float4*)acc, elems / 4); }, 5);
        printf("flat grid=%5d  %.3f ms  %.0f GB/s\n", g, ms, bytes / ms / 1e6);
    }
    if (D == 64) {
        lines<1, 8, 4>(vm, acc, H, W, D, n, bytes);
        lines<1, 8, 1>(vm, acc, H, W, D, n, bytes);
    } else if (D == 192) {
        lines<3, 2, 4>(vm, acc, H, W, D, n, bytes);
        lines<3, 4, 4>(vm, acc, H, W, D, n, bytes);
        lines<1, 4, 1>(vm, acc, H, W, D, n, bytes);
        lines<1, 8, 1>(vm, acc, H, W, D, n, bytes);
        lines<3, 4, 2>(vm, acc, H, W, D, n, bytes);
    } else {
        lines<4, 2, 4>(vm, acc, H, W, D, n, bytes);
        lines<4, 4, 4>(vm, acc, H, W, D, n, bytes);
        lines<1, 4, 1>(vm, acc, H, W, D, n, bytes);
        lines<1, 8, 1>(vm, acc, H, W, D, n, bytes);
        lines<2, 4, 2>(vm, acc, H, W, D, n, bytes);
    }
    return 0;
}
