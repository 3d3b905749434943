// Host shim so the device arithmetic headers (fhs_modarith.h, fhs_ntt.h) compile with g++ for
// CPU emulation tests (tests/test_cpu.py::test_device_ntt_emulated_matches_oracle).
#pragma once
#include <stdint.h>
#include <string.h>
#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __shared__
struct ulonglong2 { unsigned long long x, y; };
static inline uint64_t __umul64hi(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }
static inline unsigned __umulhi(unsigned a, unsigned b) { return (unsigned)(((uint64_t)a * b) >> 32); }
#define __builtin_amdgcn_readfirstlane(x) (x)
static inline void __syncthreads() {}
static inline void __builtin_amdgcn_wave_barrier() {}
#define __builtin_amdgcn_fence(order, scope) ((void)0)
static inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
