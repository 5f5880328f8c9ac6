// Probe: which SIMD of which CU each wave of a workgroup lands on, for the launch shapes of the
// two-wave V NORM_SCAN sweep (k_cbca_nsv2: 128 threads, 53,120 B of dynamic LDS, 252 VGPRs, so
// three workgroups per CU) and of a 6-wave workgroup holding three lines (384 threads, the three
// lines' LDS in one workgroup).  Each wave reads HW_ID / XCC_ID (s_getreg, read only), spins
// ~30 us so that the workgroups of one dispatch round are co-resident, and stores one record with
// a vector store.  The host tallies, per co-resident CU, whether the second waves of different
// workgroups share a SIMD.
// build: hipcc --offload-arch=gfx950 -O2 -o build/simd_place simd_place.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <map>
#include <vector>
#include <tuple>

__global__ __launch_bounds__(384) void k_probe(uint32_t* out, int spin_ticks, int lds_words) {
    extern __shared__ float smem[];
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int w = threadIdx.x; w < lds_words; w += blockDim.x) smem[w] = 0.f;
    while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < spin_ticks) __builtin_amdgcn_s_sleep(2);
    asm volatile("" ::: "v250", "v251");   // occupy the register file like the sweep (252 VGPRs)
    const int wave = threadIdx.x >> 6;
    const int waves = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        uint32_t* r = out + ((size_t)blockIdx.x * waves + wave) * 4;
        r[0] = hw;
        r[1] = xcc;
        r[2] = (uint32_t)t0;
        r[3] = (uint32_t)(t0 >> 32);
    }
}

static void run(const char* name, int blocks, int threads, int lds_bytes) {
    const int waves = threads / 64;
    uint32_t* d;
    hipMalloc(&d, (size_t)blocks * waves * 16);
    hipMemset(d, 0, (size_t)blocks * waves * 16);
    hipFuncSetAttribute((const void*)k_probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(threads), lds_bytes, 0, d, 3000, lds_bytes / 4);
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) { printf("%s: %s\n", name, hipGetErrorString(e)); return; }
    std::vector<uint32_t> h((size_t)blocks * waves * 4);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    // first dispatch round: the earliest start of each CU's workgroups (within 10 us of the first)
    uint64_t tmin = ~0ull;
    for (int b = 0; b < blocks; b++) {
        const uint64_t t = h[(size_t)b * waves * 4 + 2] | ((uint64_t)h[(size_t)b * waves * 4 + 3] << 32);
        if (t < tmin) tmin = t;
    }
    typedef std::tuple<int, int, int, int> Cu;   // xcc, se, sh, cu
    std::map<Cu, std::vector<std::vector<int>>> round1;   // per CU: per workgroup, SIMD of each wave
    std::map<int, int> simd_hist[8];
    for (int b = 0; b < blocks; b++) {
        const uint32_t* r = &h[(size_t)b * waves * 4];
        const uint64_t t = r[2] | ((uint64_t)r[3] << 32);
        std::vector<int> simds;
        for (int w = 0; w < waves; w++) {
            const uint32_t hw = r[w * 4];
            simds.push_back((hw >> 4) & 3);
            simd_hist[w][(hw >> 4) & 3]++;
        }
        if (t - tmin < 1000) {   // 100 MHz counter: 10 us
            const uint32_t hw = r[0];
            Cu cu{(int)(r[1] & 0xf), (int)((hw >> 13) & 7), (int)((hw >> 12) & 1), (int)((hw >> 8) & 0xf)};
            round1[cu].push_back(simds);
        }
    }
    int cus = 0, shared_w1 = 0, per_cu_hist[8] = {0};
    std::map<std::vector<int>, int> patterns;
    for (auto& kv : round1) {
        cus++;
        per_cu_hist[std::min<int>(7, kv.second.size())]++;
        int cnt[4] = {0};
        for (auto& s : kv.second) {
            if (waves >= 2) cnt[s[1]]++;
            patterns[s]++;
        }
        for (int i = 0; i < 4; i++)
            if (cnt[i] > 1) { shared_w1++; break; }
    }
    printf("%s: %d blocks x %d threads, LDS %d B; first-round CUs %d (workgroups per CU:", name, blocks, threads,
           lds_bytes, cus);
    for (int i = 1; i < 8; i++) if (per_cu_hist[i]) printf(" %d:%d", i, per_cu_hist[i]);
    printf("), CUs where two wave-1s share a SIMD: %d\n", shared_w1);
    for (int w = 0; w < waves; w++) {
        printf("  wave %d SIMD histogram:", w);
        for (auto& kv : simd_hist[w]) printf(" simd%d:%d", kv.first, kv.second);
        printf("\n");
    }
    int shown = 0;
    for (auto& kv : patterns) {
        if (shown++ >= 12) break;
        printf("  pattern");
        for (int s : kv.first) printf(" %d", s);
        printf(" : %d\n", kv.second);
    }
    // the SIMD patterns of the first 6 CUs' workgroups
    shown = 0;
    for (auto& kv : round1) {
        if (shown++ >= 6) break;
        printf("  cu(xcc %d se %d sh %d cu %d):", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first),
               std::get<3>(kv.first));
        for (auto& s : kv.second) {
            printf(" [");
            for (int x : s) printf("%d", x);
            printf("]");
        }
        printf("\n");
    }
}

int main() {
    run("nsv2 shape (128 thr, 53120 B)", 768, 128, 53120);
    run("nsv2 shape, full grid", 24000, 128, 53120);
    run("three lines per workgroup (384 thr, 159360 B)", 256, 384, 159360);
    run("two lines per workgroup (256 thr, 106240 B)", 512, 256, 106240);
    return 0;
}
