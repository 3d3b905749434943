// LDS-DMA variant of tools/microbench/diagread.hip: can k_bsgs_inner's diagonal stream
// run faster through a per-wave LDS ring filled by global_load_lds_dwordx4 than through the 8 x 16-byte
// register loads in flight it uses today (6.3 TB/s for the bare access shape)?  Same grid, 16 waves, 94 KB of
// LDS for the baby-step slice; each wave owns a private ring of RS 1-KB slots (one diagonal's 128
// coefficients of limb i per slot) after the slice.  A wave issues RS pieces ahead; before it reads slot s it
// waits until at most RS - 1 of its later pieces are outstanding (s_waitcnt vmcnt(RS - 1): the issuing wave's
// covering vmcnt orders its own ds_read, MI355X_MICROARCH.md item 7), reads the slot (ds_read_b128), waits
// for the read, refills the slot with the diagonal RS ahead.  The pieces are issued by inline asm (the
// compiler then inserts no conservative vmcnt(0) before the LDS reads) and the waits are explicit.
//   Build: hipcc -O3 --offload-arch=gfx950 diagread_dma.hip -o diagread_dma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N = 16384, L = 36, D = 2048, G = 46, B = 45, W = 128, NB = N / W, WAVES = 16;

__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_base) {
    // one 1-KB piece: lane k's 16 bytes from its own global address land at lds_base + 16 k
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_base)
                 : "memory");
}

// the 32-bit LDS byte address of a __shared__ object (generic -> address space 3 is the LDS offset)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <int RS>
__device__ __forceinline__ void wait_ring() {
    if constexpr (RS == 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (RS == 3) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (RS == 2) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int RS>
__global__ void __launch_bounds__(64 * WAVES) k_read_dma(const uint64_t* base, uint64_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sb[];
    const int blk = blockIdx.x, i = blockIdx.y, lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 64) sb[threadIdx.x] = 0;
    const uint32_t ring = lds_addr(sb + G * 2 * W) + (uint32_t)wave * RS * 1024;
    uint32_t acc = 0;
    // this wave's diagonals in order: groups g = wave, wave + WAVES, ...; all of each group
    int gq[4], nq = 0;
    for (int g = wave; g < B; g += WAVES) gq[nq++] = g;
    int total = 0;
    for (int q = 0; q < nq; ++q) total += min(G, D - gq[q] * G);
    auto diag = [&](int t) {   // t-th diagonal of this wave -> global index
        int q = 0;
        while (t >= min(G, D - gq[q] * G)) { t -= min(G, D - gq[q] * G); ++q; }
        return gq[q] * G + t;
    };
    auto src = [&](int k) { return (const void*)(base + (size_t)k * L * N + (size_t)i * N + (size_t)blk * W + lane * 2); };
    for (int t = 0; t < RS && t < total; ++t) dma16(src(diag(t)), ring + t * 1024);
    for (int t = 0; t < total; ++t) {
        const int s = t % RS;
        if (t + RS <= total) wait_ring<RS>();
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t v[4];
        const uint32_t a = ring + s * 1024 + lane * 16;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(*(__attribute__((ext_vector_type(4))) uint32_t*)v) : "v"(a) : "memory");
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
        if (t + RS < total) dma16(src(diag(t + RS)), ring + s * 1024);
    }
    out[((size_t)i * NB + blk) * 64 * WAVES + threadIdx.x] = acc + sb[lane & 63];
}

int main() {
    const size_t words = (size_t)D * L * N;
    uint64_t* base = nullptr;
    uint64_t* out = nullptr;
    if (hipMalloc(&base, words * 8) != hipSuccess || hipMalloc(&out, (size_t)L * NB * 64 * WAVES * 8) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(base, 0x5a, words * 8);
    const double bytes = (double)D * L * N * 8;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, int rs) {
        const size_t lds = (size_t)G * 2 * W * 8 + (size_t)WAVES * rs * 1024;
        if (lds > 160 * 1024) { printf("RS=%d: %zu bytes of LDS do not fit\n", rs, lds); return; }
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        for (int rep = 0; rep < 3; ++rep) {
            const int iters = 10;
            hipEventRecord(e0);
            for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(kern, dim3(NB, L), dim3(64 * WAVES), lds, 0, base, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("dma ring RS=%d  %.3f ms per pass, %.2f TB/s (all %d diagonals)\n", rs, ms / iters,
                   bytes / (ms / iters * 1e-3) / 1e12, D);
        }
    };
    run(k_read_dma<4>, 4);
    run(k_read_dma<3>, 3);
    run(k_read_dma<2>, 2);
    hipFree(base);
    hipFree(out);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
