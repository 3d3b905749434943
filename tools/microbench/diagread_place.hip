// Placement sweep of the Hadamard's diagonal stream (round 6; companion of tools/debug/alloc_spread.py, which found
// k_bsgs_inner 1.75-2.02 ms across re-allocations of the same slab in one process, while a plain streaming read
// varied 5 %).  The 9.66 GB slab of cfg2's 2048 diagonals (36 limbs x 16384 words each) is re-allocated TRIALS
// times after a spacer allocation of a different size; per trial three access orders with k_bsgs_inner's grid,
// 16 waves, 16-byte non-temporal buffer loads, 8 in flight per lane and 94 KB of LDS:
//   groups   -- today's: wave w takes giant groups w, w+16, w+32, 8 diagonals of its group at a time (the
//               workgroup's 128 loads in flight hit 16 groups' diagonals, spread over the whole slab);
//   consec   -- wave w takes diagonals [8 w + 128 j, +8): the workgroup's 128 loads in flight hit 128 consecutive
//               diagonals (what a kernel splitting each group over waves, with an LDS reduction, would read);
//   packed   -- the packed layout [limb][128-block][diagonal][128] read in the groups order (a reference point:
//               each workgroup streams one contiguous 2 MB region).
// Build: hipcc -O3 --offload-arch=gfx950 diagread_place.hip -o diagread_place;  run: ./diagread_place [TRIALS]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <algorithm>

constexpr int N = 16384, L = 36, D = 2048, G = 46, B = 45, W = 128, NB = N / W, WAVES = 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int MODE>   // 0 groups, 1 consec, 2 packed
__global__ void __launch_bounds__(64 * WAVES) k_read(const uint64_t* base, uint64_t* out) {
    extern __shared__ uint64_t sb[];
    const int blk = blockIdx.x, i = blockIdx.y, lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 64) sb[threadIdx.x] = 0;
    uint32_t acc = 0;
    auto batch = [&](int k0) {
        uint32_t v[8][4];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int k = k0 + u;
            __amdgpu_buffer_rsrc_t r;
            int soff;
            if (MODE == 2) {
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
    };
    if (MODE == 1) {
        for (int k0 = wave * 8; k0 + 8 <= D; k0 += 8 * WAVES) batch(k0);
    } else {
        for (int g = wave; g < B; g += WAVES) {
            const int bmax = min(G, D - g * G);
            for (int b = 0; b + 8 <= bmax; b += 8) batch(g * G + b);
        }
    }
    out[((size_t)i * NB + blk) * 64 * WAVES + threadIdx.x] = acc + sb[lane & 63];
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 8;
    const size_t words = (size_t)D * L * N;
    uint64_t* out = nullptr;
    if (hipMalloc(&out, (size_t)L * NB * 64 * WAVES * 8) != hipSuccess) return 1;
    const size_t lds = (size_t)G * 2 * W * 8;
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_read<0>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_read<1>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_read<2>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    size_t loads_g = 0;
    for (int g = 0; g < B; ++g) loads_g += (size_t)(std::min(G, D - g * G) / 8) * 8;
    const double bytes_g = (double)loads_g * L * N * 8, bytes_c = (double)D * L * N * 8;
    double lo[3] = {1e9, 1e9, 1e9}, hi[3] = {0, 0, 0};
    for (int t = 0; t < trials; ++t) {
        void* spacer = nullptr;
        const size_t sp = (size_t)((0.5 + 1.7 * t) * (1 << 30));
        if (hipMalloc(&spacer, sp) != hipSuccess) return 1;
        uint64_t* base = nullptr;
        if (hipMalloc(&base, words * 8) != hipSuccess) return 1;
        hipMemset(base, 0x5a, words * 8);
        printf("trial %d (spacer %.1f GiB):", t, sp / double(1 << 30));
        for (int mode = 0; mode < 3; ++mode) {
            auto launch = [&] {
                if (mode == 0) hipLaunchKernelGGL(k_read<0>, dim3(NB, L), dim3(64 * WAVES), lds, 0, base, out);
                else if (mode == 1) hipLaunchKernelGGL(k_read<1>, dim3(NB, L), dim3(64 * WAVES), lds, 0, base, out);
                else hipLaunchKernelGGL(k_read<2>, dim3(NB, L), dim3(64 * WAVES), lds, 0, base, out);
            };
            launch();
            const int iters = 8;
            hipEventRecord(e0);
            for (int it = 0; it < iters; ++it) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double tbs = (mode == 1 ? bytes_c : bytes_g) / (ms / iters * 1e-3) / 1e12;
            lo[mode] = std::min(lo[mode], tbs);
            hi[mode] = std::max(hi[mode], tbs);
            printf("  %s %.2f TB/s", mode == 0 ? "groups" : mode == 1 ? "consec" : "packed", tbs);
        }
        printf("\n");
        fflush(stdout);
        hipFree(base);
        hipFree(spacer);
    }
    for (int mode = 0; mode < 3; ++mode)
        printf("%s: %.2f - %.2f TB/s over %d placements\n", mode == 0 ? "groups" : mode == 1 ? "consec" : "packed",
               lo[mode], hi[mode], trials);
    hipFree(out);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
