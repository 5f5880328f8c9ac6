// Probe 3: does an out-of-range buffer load write 0 to its destination, or leave it unchanged?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(const uint32_t* buf, uint32_t* out, int nrec) {
    auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(buf + 131072), (short)0, nrec, 0x00020000);
    uint32_t x;
    const uint32_t voff = threadIdx.x * 4;
    asm volatile(
        "v_mov_b32 %0, 0xdeadbeef\n\t"
        "buffer_load_dword %0, %1, %2, 0 offen\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(x)
        : "v"(voff), "s"(r)
        : "memory");
    out[threadIdx.x] = x;
}
int main() {
    uint32_t *buf, *out;
    (void)hipMalloc(&buf, 1 << 20);
    (void)hipMalloc(&out, 256);
    uint32_t* h = (uint32_t*)malloc(1 << 20);
    for (int i = 0; i < 262144; i++) h[i] = 0x10000000u + i;
    (void)hipMemcpy(buf, h, 1 << 20, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, buf, out, 40);
    uint32_t o[64];
    (void)hipMemcpy(o, out, 256, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; i++) printf("lane %2d: %08x\n", i, o[i]);
    return 0;
}
