// Probe 2: range-check granularity of raw dword buffer loads (num_records not a multiple of 16).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(const uint32_t* buf, uint32_t* out, int nrec, int baseoff) {
    auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(buf + 131072 + baseoff), (short)0, nrec, 0x00020000);
    out[threadIdx.x] = __builtin_amdgcn_raw_buffer_load_b32(r, threadIdx.x * 4, 0, 0);
}
int main() {
    uint32_t *buf, *out;
    (void)hipMalloc(&buf, 1 << 20);
    (void)hipMalloc(&out, 256);
    uint32_t* h = (uint32_t*)malloc(1 << 20);
    for (int i = 0; i < 262144; i++) h[i] = 0x10000000u + i;
    (void)hipMemcpy(buf, h, 1 << 20, hipMemcpyHostToDevice);
    for (int baseoff : {0, 1, 3})
        for (int nrec : {112, 100, 104, 108, 116, 120, 52}) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, buf, out, nrec, baseoff);
            uint32_t o[64];
            (void)hipMemcpy(o, out, 256, hipMemcpyDeviceToHost);
            int last = -1;
            for (int i = 0; i < 64; i++)
                if (o[i] != 0) last = i;
            int bad = 0;
            for (int i = 0; i <= last; i++) bad += o[i] != 0x10000000u + 131072 + baseoff + i;
            printf("base+%d*4 nrec=%3d: lanes returning data 0..%d (expected 0..%d), wrong values %d\n", baseoff, nrec, last,
                   nrec / 4 - 1, bad);
        }
    return 0;
}
