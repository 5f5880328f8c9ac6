// Probe: what do raw buffer loads return for offsets outside num_records on this GPU?
// Every probed address stays inside one 1 MiB allocation, so the probe cannot fault even if
// range checking were absent.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(const uint32_t* buf, uint32_t* out, int n, int nrec) {
    auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(buf + 131072), (short)0, nrec, 0x00020000);
    const int offs[8] = {0, 60, 64, 128, 1024, -4, -256, 4096};
    if (threadIdx.x < 8) {
        out[threadIdx.x] = __builtin_amdgcn_raw_buffer_load_b32(r, offs[threadIdx.x], 0, 0);
        out[8 + threadIdx.x] = __builtin_amdgcn_raw_buffer_load_b32(r, 0, offs[threadIdx.x] >= 0 ? offs[threadIdx.x] : 0, 0);
    }
}
int main() {
    uint32_t *buf, *out;
    hipMalloc(&buf, 1 << 20);
    hipMalloc(&out, 64);
    uint32_t* h = (uint32_t*)malloc(1 << 20);
    for (int i = 0; i < 262144; i++) h[i] = 0x10000000u + i;
    hipMemcpy(buf, h, 1 << 20, hipMemcpyHostToDevice);
    for (int nrec : {64, 0x7fffffff}) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, buf, out, 0, nrec);
        uint32_t o[16];
        hipMemcpy(o, out, 64, hipMemcpyDeviceToHost);
        printf("num_records=%d\n  voffset: ", nrec);
        const int offs[8] = {0, 60, 64, 128, 1024, -4, -256, 4096};
        for (int i = 0; i < 8; i++) printf("[%d]=%08x ", offs[i], o[i]);
        printf("\n  soffset: ");
        for (int i = 0; i < 8; i++) printf("[%d]=%08x ", offs[i] >= 0 ? offs[i] : 0, o[8 + i]);
        printf("\n");
    }
    return 0;
}
