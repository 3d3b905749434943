// fhs_buffer.h -- buffer-descriptor loads / stores for the gfx950 kernels (fhs_kernels.hip only).
#pragma once
#include "fhs_modarith.h"

// Buffer loads / stores through a wave-uniform descriptor (base + byte size): the per-lane byte offset
// goes in voffset, every wave-uniform offset (limb, chunk, row) in soffset, so a strided access costs
// no 64-bit address arithmetic on the VALU (MI355X guide T8/T20).  Build descriptors only from
// wave-uniform values.
typedef unsigned int fhs_u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* base, uint32_t bytes) {
    // readfirstlane on the inputs makes their uniformity provable to the compiler (otherwise every
    // buffer op is wrapped in a waterfall loop)
    const u64 p = reinterpret_cast<u64>(base);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((u64)hi << 32) | lo), 0, nb, 0x00020000);
}
__device__ __forceinline__ u64 bload64(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ void bstore64(u64 v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(fhs_u32x2, v), r, voff, soff, 0);
}
// the same with the cache-policy bits (2: non-temporal -- streamed results that L2 need not keep)
template <int AUX>
__device__ __forceinline__ void bstore64_aux(u64 v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(fhs_u32x2, v), r, voff, soff, AUX);
}
