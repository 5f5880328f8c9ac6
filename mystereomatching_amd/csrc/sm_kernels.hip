// sm_kernels.hip — hand-written gfx950 kernels for the census / CBCA / SGM / WTA hot path.
//
// Layout in HBM (per pair b, all packed):
//   bgr   [b][view][H][W][3] u8  gray [b][view][H][W] u8   (view 0 = left, 1 = right)
//   code  [b][view][H][W] ulonglong2   (census words 0,1; genCensusCode_NC_Sur h:867-934)
//   gx,gy [b][view][H][W] f32    (calGrad / calGrad_y cpp:271-386)
//   arms  [b][view][H][W] u8x4   (L,R,U,D; calHorVerDis cpp:2959-3050)
//   vm    [b][H][W][D] f32       (d innermost, as the reference's CV_32FC(D), cpp:2080)
//   acc   [b][H][W][D] f32       (SGM path sum in path order, gen_sgm_vm cpp:2031-2056)
//   disp  [b][H][W] i16          (DP[0], gen_dispFromVm cpp:3928-3967)
// Every float op below is written in the reference's evaluation order and the file is compiled
// with -ffp-contract=off, so results are bit-identical to the scalar CPU path.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_device.h"
#include "sm_kernels.h"

namespace sm {

__constant__ uint64_t c_exp_tab[32] = SM_EXPF_TABLE;
__constant__ float c_lut_a[1024];   // expf(-x/lam) for integer-valued costs (census / AD)
__constant__ float c_lut_b[1024];

__device__ inline float dev_expf(float x) { return expf_glibc(x, c_exp_tab); }

// ---------------------------------------------------------------------------------------
// K0a: census codes + x/y gradients for both views of every pair; one thread per pixel.
// genCensusCode_NC_Sur (h:867-934): MSB-first bit stream, flush when step > 63.
// calGrad / calGrad_y single-channel branches (cpp:271-287, 320-350).
// ---------------------------------------------------------------------------------------
__global__ void k_census_grad(const uint8_t* __restrict__ gray, ulonglong2* __restrict__ code,
                              float* __restrict__ gx, float* __restrict__ gy, int H, int W, int rv,
                              int ru, int ring, int views_per_pair) {
    const int npix = H * W;
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= npix) return;
    const int view = blockIdx.y;  // 0 left, 1 right
    const int b = blockIdx.z;
    const uint8_t* I = gray + ((size_t)b * 2 + view) * npix;
    const int v = pix / W, u = pix - v * W;
    const int c = I[pix];
    uint64_t w[2] = {0, 0};
    uint64_t cs = 0;
    int step = 0, dep = 0;
    for (int dv = -rv; dv <= rv; dv++) {
        const uint8_t* row = I + (size_t)reflect101(v + dv, H) * W;
        for (int du = -ru; du <= ru; du++) {
            if (step > 63) {
                w[dep & 1] = cs;
                cs = 0;
                step = 0;
                dep++;
            }
            cs <<= 1;
            if (c - (int)row[reflect101(u + du, W)] < 0) cs++;
            step++;
        }
    }
    if (ring) {
        const int dvs[9] = {-1, -1, -1, 0, 1, 1, 1, 0, -1};
        const int dus[9] = {-1, 0, 1, 1, 1, 0, -1, -1, -1};
        for (int i = 0; i < 8; i++) {
            int pre = I[(size_t)reflect101(v + dvs[i], H) * W + reflect101(u + dus[i], W)];
            int aft = I[(size_t)reflect101(v + dvs[i + 1], H) * W + reflect101(u + dus[i + 1], W)];
            if (step > 63) {
                w[dep & 1] = cs;
                cs = 0;
                step = 0;
                dep++;
            }
            cs <<= 1;
            if (pre - aft < 0) cs++;
            step++;
        }
    }
    if (step > 0) w[dep & 1] = cs;
    const size_t o = ((size_t)b * views_per_pair + view) * npix + pix;
    code[o] = make_ulonglong2(w[0], w[1]);
    // gradients (edges: full difference; interior: 0.5 * central difference, exact in f32)
    const uint8_t* r = I + (size_t)v * W;
    float g;
    if (u == 0)
        g = (float)(r[1] - r[0]);
    else if (u == W - 1)
        g = (float)(r[W - 1] - r[W - 2]);
    else
        g = 0.5f * (float)(r[u + 1] - r[u - 1]);
    gx[o] = g;
    if (v == 0)
        g = (float)(I[W + u] - I[u]);
    else if (v == H - 1)
        g = (float)(I[(size_t)(H - 1) * W + u] - I[(size_t)(H - 2) * W + u]);
    else
        g = 0.5f * (float)(I[(size_t)(v + 1) * W + u] - I[(size_t)(v - 1) * W + u]);
    gy[o] = g;
}

// ---------------------------------------------------------------------------------------
// K0b: cross arms (calHorVerDis 7-arg, cpp:2959-3050); one thread per (pixel, direction).
// ---------------------------------------------------------------------------------------
__device__ inline bool color_ok(const uint8_t* a, const uint8_t* b, int t) {
    return abs((int)a[0] - (int)b[0]) <= t && abs((int)a[1] - (int)b[1]) <= t && abs((int)a[2] - (int)b[2]) <= t;
}

__global__ void k_arms(const uint8_t* __restrict__ bgr, uint8_t* __restrict__ arms, int H, int W, int L,
                       int L_out, int C_D, int C_D_out, int minL) {
    const int npix = H * W;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npix * 4) return;
    const int pix = t >> 2, direc = t & 3;
    const int view = blockIdx.y, b = blockIdx.z;
    const uint8_t* I = bgr + ((size_t)b * 2 + view) * npix * 3;
    const int v = pix / W, u = pix - v * W;
    const int du = direc == 0 ? -1 : (direc == 1 ? 1 : 0);
    const int dv = direc == 2 ? -1 : (direc == 3 ? 1 : 0);
    const uint8_t* IPtr = I + (size_t)pix * 3;
    int arm = 1;
    for (; arm <= L_out; arm++) {
        int va = v + arm * dv, ua = u + arm * du;
        if (va < 0 || va >= H || ua < 0 || ua >= W) break;
        const uint8_t* ap = I + ((size_t)va * W + ua) * 3;
        const uint8_t* pp = ap - (dv * W + du) * 3;
        bool nb = color_ok(ap, pp, C_D);
        bool ip = color_ok(IPtr, ap, arm <= L ? C_D : C_D_out);
        if (!nb || !ip) break;
    }
    int out = 0;
    if (--arm >= minL)
        out = arm;
    else {
        for (int len = minL; len >= 0; len--)
            if (u + len * du >= 0 && u + len * du <= W - 1 && v + len * dv >= 0 && v + len * dv <= H - 1) {
                out = len;
                break;
            }
    }
    arms[(((size_t)b * 2 + view) * npix + pix) * 4 + direc] = (uint8_t)out;
}

// ---------------------------------------------------------------------------------------
// K1: cost volume.  One thread per (pixel, d) element; consecutive threads = consecutive d, so
// the f32 volume write is fully coalesced.  view 0: pairs (u, u-d); view 1: (u+d, u).
//   census  gen_cenVM_XOR (h:936-981); grad calgradvm (cpp:388-455);
//   AD      gen_ad_sd_vm (cpp:2468-2509);   fusion gen_vm_from2vm_exp (cpp:3566-3590).
// The census term exp(-C/lam) (C integer 0..71) and the AD term exp(-AD/lam) (AD = s/3,
// s integer 0..765) come from host-built LUTs of libm expf; only the gradient term needs
// sm::dev_expf.
// ---------------------------------------------------------------------------------------
template <int METHOD>
__global__ void k_cost(const CostArgs a) {
    const size_t nvol = (size_t)a.H * a.W * a.D;
    const int b = blockIdx.y;
    const size_t npix = (size_t)a.H * a.W;
    float* out = a.vm + (size_t)b * nvol;
    const int lc = a.view == 1 ? 1 : 0, rc = a.view == 1 ? 0 : 1;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < nvol; e += (size_t)gridDim.x * blockDim.x) {
        const int pix = (int)(e / a.D);
        const int d = (int)(e - (size_t)pix * a.D);
        const int v = pix / a.W, u = pix - v * a.W;
        const int lp = u + d * lc, rp = u - d * rc;
        const bool oor = lp >= a.W || rp < 0;
        const size_t rowb = (size_t)v * a.W;
        float cen = 0.f;
        if (METHOD != SM_M_AD) {
            if (oor)
                cen = a.census_default;
            else {
                const ulonglong2 cl = a.code[((size_t)b * 2 + 0) * npix + rowb + lp];
                const ulonglong2 cr = a.code[((size_t)b * 2 + 1) * npix + rowb + rp];
                float cost = 0;
                cost += (float)__popcll(cl.x ^ cr.x);
                if (a.nwords > 1) cost += (float)__popcll(cl.y ^ cr.y);
                cen = fminf(cost, a.census_default);
            }
        }
        float res;
        if (METHOD == SM_M_CENSUS) {
            res = cen;
        } else if (METHOD == SM_M_CENSUS_GRAD) {
            float g;
            if (oor)
                g = a.grad_oor;
            else {
                const uint8_t* arm = a.arms + (((size_t)b * 2 + a.view) * npix + pix) * 4;
                float sH = (float)min(arm[0], arm[1]);
                float sV = (float)min(arm[2], arm[3]);
                if (sH == 0) sH = 1;
                if (sV == 0) sV = 1;
                const float wa = sH / (sH + sV);
                const size_t o0 = ((size_t)b * 2 + 0) * npix + rowb + lp;
                const size_t o1 = ((size_t)b * 2 + 1) * npix + rowb + rp;
                const float dx = fminf(fabsf(a.gx[o0] - a.gx[o1]), a.grad_trunc);
                const float dy = fminf(fabsf(a.gy[o0] - a.gy[o1]), a.grad_trunc);
                if (a.grad_adaptive) {
                    const float t1 = wa * dx;
                    const float t2 = (1.0f - wa) * dy;
                    g = t1 + t2;
                } else {
                    g = dx + dy;
                }
            }
            const float e0 = c_lut_a[(int)cen];                 // expf(-C / lamCen)
            const float e1 = dev_expf(-g / a.lam2);             // expf(-G / lamG)
            const float t = 2.0f - e0;
            res = t - e1;
        } else {  // AD-based: AD = min(s/3, trunc), s = sum_c |L_c - R_c| (integer)
            int s = 0;
            if (!oor) {
                const uint8_t* L = a.bgr + (((size_t)b * 2 + 0) * npix + rowb + lp) * 3;
                const uint8_t* R = a.bgr + (((size_t)b * 2 + 1) * npix + rowb + rp) * 3;
                s = abs((int)L[0] - (int)R[0]) + abs((int)L[1] - (int)R[1]) + abs((int)L[2] - (int)R[2]);
            }
            if (METHOD == SM_M_AD) {
                res = oor ? a.ad_trunc : fminf((float)s / 3.0f, a.ad_trunc);
            } else {  // ADCensus: 2 - exp(-AD/lamAD) - exp(-C/lamC); AD trunc 1000 > 255 never binds
                const float e0 = oor ? a.ad_oor_exp : c_lut_b[s];
                const float e1 = c_lut_a[(int)cen];
                const float t = 2.0f - e0;
                res = t - e1;
            }
        }
        out[e] = res;
    }
}

// SolveAll with PY_LVL = 1 as a standalone pass (used by the reference-ordered API):
// vm = 0 + invWgt * vm (cpp:2189-2201).
__global__ void k_scale(float* __restrict__ vm, size_t n, float w) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float sum = 0.f;
        sum += w * vm[i];
        vm[i] = sum;
    }
}

// WTA alone (optimization == "" / aggregation-only runs): one wave per pixel.
template <int K>
__global__ __launch_bounds__(256) void k_wta(const float* __restrict__ vm, int16_t* __restrict__ disp, int H, int W, int D) {
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const size_t npix = (size_t)H * W;
    const int b = blockIdx.y;
    if ((size_t)wave >= npix) return;
    const float* f = vm + ((size_t)b * npix + wave) * D;
    const int d0 = lane * K;
    float bm = FLT_MAX;
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < K; k++)
        if (d0 + k < D && bm > f[d0 + k]) {
            bm = f[d0 + k];
            bi = d0 + k;
        }
    const float wm = wave_min(bm);
    const int widx = wave_min_i(bm == wm ? bi : 0x7fffffff);
    if (lane == 0) disp[(size_t)b * npix + wave] = (int16_t)((wm < FLT_MAX) ? widx : -1);
}

__global__ void k_expf_range(uint32_t first, uint32_t n, float* __restrict__ out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[i] = dev_expf(__builtin_bit_cast(float, first + i));
}

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
hipError_t upload_luts(const float* lut_a, const float* lut_b, hipStream_t st) {
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_lut_a), lut_a, sizeof(float) * 1024, 0, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_lut_b), lut_b, sizeof(float) * 1024, 0, hipMemcpyHostToDevice, st);
}

void launch_census_grad(const uint8_t* gray, ulonglong2* code, float* gx, float* gy, int n, int H, int W, int rv,
                        int ru, int ring, hipStream_t st) {
    dim3 grid((H * W + 255) / 256, 2, n);
    hipLaunchKernelGGL(k_census_grad, grid, dim3(256), 0, st, gray, code, gx, gy, H, W, rv, ru, ring, 2);
}

void launch_arms(const uint8_t* bgr, uint8_t* arms, int n, int H, int W, int L, int L_out, int C_D, int C_D_out,
                 int minL, hipStream_t st) {
    dim3 grid((H * W * 4 + 255) / 256, 2, n);
    hipLaunchKernelGGL(k_arms, grid, dim3(256), 0, st, bgr, arms, H, W, L, L_out, C_D, C_D_out, minL);
}

void launch_cost(const CostArgs& a, int method, int n, hipStream_t st) {
    const size_t nvol = (size_t)a.H * a.W * a.D;
    size_t blocks = (nvol + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    dim3 grid((unsigned)blocks, n);
    switch (method) {
        case SM_M_CENSUS_GRAD: hipLaunchKernelGGL(k_cost<SM_M_CENSUS_GRAD>, grid, dim3(256), 0, st, a); break;
        case SM_M_CENSUS: hipLaunchKernelGGL(k_cost<SM_M_CENSUS>, grid, dim3(256), 0, st, a); break;
        case SM_M_AD_CENSUS: hipLaunchKernelGGL(k_cost<SM_M_AD_CENSUS>, grid, dim3(256), 0, st, a); break;
        default: hipLaunchKernelGGL(k_cost<SM_M_AD>, grid, dim3(256), 0, st, a); break;
    }
}

void launch_scale(float* vm, size_t n, float w, hipStream_t st) {
    size_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_scale, dim3((unsigned)blocks), dim3(256), 0, st, vm, n, w);
}

int sgm_k_for(int D) {
    const int k = (D + 63) / 64;
    if (k <= 4) return k;
    if (k <= 6) return 6;
    if (k <= 8) return 8;
    if (k <= 12) return 12;
    return 16;
}

void launch_wta(const float* vm, int16_t* disp, int n, int H, int W, int D, hipStream_t st) {
    const size_t npix = (size_t)H * W;
    dim3 grid((unsigned)((npix + 3) / 4), n);
    switch (sgm_k_for(D)) {
        case 1: hipLaunchKernelGGL(k_wta<1>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 2: hipLaunchKernelGGL(k_wta<2>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 3: hipLaunchKernelGGL(k_wta<3>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 4: hipLaunchKernelGGL(k_wta<4>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 6: hipLaunchKernelGGL(k_wta<6>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 8: hipLaunchKernelGGL(k_wta<8>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        case 12: hipLaunchKernelGGL(k_wta<12>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
        default: hipLaunchKernelGGL(k_wta<16>, grid, dim3(256), 0, st, vm, disp, H, W, D); break;
    }
}

void launch_expf_range(uint32_t first, uint32_t n, float* out, hipStream_t st) {
    hipLaunchKernelGGL(k_expf_range, dim3(4096), dim3(256), 0, st, first, n, out);
}

float expf_host(float x) {
    static const uint64_t tab[32] = SM_EXPF_TABLE;
    return expf_glibc(x, tab);
}

}  // namespace sm
