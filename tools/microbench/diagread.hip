// Read rate of the Hadamard's diagonal stream (k_bsgs_inner's access shape, cfg2: D = 2048 diagonals of
// l = 36 limbs x N = 16384 words, 9.66 GB) in two layouts:
//   separate  -- each diagonal its own l x N plaintext (today's layout): a wave's 8 loads in flight hit
//                8 different 4.7 MB plaintexts, 1 KB each
//   packed    -- [limb][128-coefficient block][diagonal][128]: the same 1 KB pieces, a giant group's
//                diagonals adjacent (46 KB contiguous per group and slice)
// Same grid, waves, 16-byte non-temporal buffer loads, 8 in flight per lane and 94 KB of LDS (one
// workgroup per CU) as k_bsgs_inner; the loaded words are folded into one XOR per lane (written out so
// nothing is elided).  Build: hipcc -O3 --offload-arch=gfx950 diagread.hip -o diagread
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int N = 16384, L = 36, D = 2048, G = 46, B = 45, W = 128, NB = N / W, WAVES = 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <bool PACKED>
__global__ void __launch_bounds__(64 * WAVES) k_read(const uint64_t* base, uint64_t* out) {
    extern __shared__ uint64_t sb[];
    const int blk = blockIdx.x, i = blockIdx.y, lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 64) sb[threadIdx.x] = 0;   // touch the LDS (occupancy as the real kernel)
    uint32_t acc = 0;
    for (int g = wave; g < B; g += WAVES) {
        const int bmax = min(G, D - g * G);
        for (int b = 0; b + 8 <= bmax; b += 8) {
            uint32_t v[8][4];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = g * G + b + u;
                __amdgpu_buffer_rsrc_t r;
                int soff;
                if (PACKED) {
                    r = rsrc(base + ((size_t)i * NB + blk) * D * W, D * W * 8);
                    soff = k * W * 8;
                } else {
                    r = rsrc(base + (size_t)k * L * N + (size_t)i * N, N * 8);
                    soff = blk * W * 8;
                }
                const auto t = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, soff, 2);
                v[u][0] = t[0]; v[u][1] = t[1]; v[u][2] = t[2]; v[u][3] = t[3];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
        }
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
    const size_t lds = (size_t)G * 2 * W * 8;   // 94 KB, as k_bsgs_inner
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_read<false>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_read<true>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // bytes actually read: whole batches of 8 only (the kernel skips the < 8 tail, like a lower bound)
    size_t loads = 0;
    for (int g = 0; g < B; ++g) loads += (size_t)(std::min(G, D - g * G) / 8) * 8;
    const double bytes = (double)loads * L * N * 8;
    for (int rep = 0; rep < 3; ++rep) {
        for (int packed = 0; packed < 2; ++packed) {
            const int iters = 10;
            hipEventRecord(e0);
            for (int it = 0; it < iters; ++it) {
                if (packed)
                    hipLaunchKernelGGL(k_read<true>, dim3(NB, L), dim3(64 * WAVES), lds, 0, base, out);
                else
                    hipLaunchKernelGGL(k_read<false>, dim3(NB, L), dim3(64 * WAVES), lds, 0, base, out);
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("%-8s %.3f ms per pass, %.2f TB/s\n", packed ? "packed" : "separate", ms / iters,
                   bytes / (ms / iters * 1e-3) / 1e12);
        }
    }
    hipFree(base);
    hipFree(out);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
