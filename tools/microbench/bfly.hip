// VALU ceiling of the NTT butterfly the kernels use (fhs_modarith.h shoup_lazy + lazy add/sub,
// fhs_ntt.h LAZY forward form), with operands in registers: no LDS, no memory, no barriers.
// bench.py prices k_modup's butterfly rate against this number (ntt_valu_roofline.peak).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../fhe-spear_amd/csrc/fhs_modarith.h"
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)

__global__ void k_bfly(u64* out, const u64* tw, u64 q, int iters) {
    u64 x[16];
    for (int k = 0; k < 16; ++k) x[k] = (threadIdx.x * 16 + k + blockIdx.x) % q;
    const u64 q2 = 2 * q;
    u64 w[8], wp[8];
    for (int k = 0; k < 8; ++k) { w[k] = tw[2 * k]; wp[k] = tw[2 * k + 1]; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {   // 8 butterflies per iteration, lazy forward form
            const u64 t = shoup_lazy(x[k + 8], w[k], wp[k], q);
            const u64 X = x[k] >= 8 * q ? x[k] - 8 * q : x[k];   // keep the loop bounded (one csub / 2 bfly)
            x[k] = X + t;
            x[k + 8] = X + (q2 - t);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) { const u64 s = x[k]; x[k] = x[k + 8]; x[k + 8] = s; }
    }
    u64 s = 0;
    for (int k = 0; k < 16; ++k) s ^= x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const u64 q = 576460752303415297ull;   // a 59-bit NTT prime (2^59 - 2^13 * 1 + 1 form not required)
    u64 htw[16];
    for (int k = 0; k < 8; ++k) {
        htw[2 * k] = (123456789ull * (k + 1)) % q;
        htw[2 * k + 1] = (u64)(((unsigned __int128)htw[2 * k] << 64) / q);
    }
    u64 *d, *dtw;
    CK(hipMalloc(&d, 64 << 20));
    CK(hipMalloc(&dtw, sizeof(htw)));
    CK(hipMemcpy(dtw, htw, sizeof(htw), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 256 * 8, threads = 256, iters = 2000;
    for (int rep = 0; rep < 3; ++rep) {
        float ms;
        hipEventRecord(a);
        hipLaunchKernelGGL(k_bfly, dim3(blocks), dim3(threads), 0, 0, d, dtw, q, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        const double bf = (double)blocks * threads * iters * 8;
        printf("lazy butterfly (registers): %.1f G/s (%.3f ms)\n", bf / ms / 1e6, ms);
    }
    return 0;
}
