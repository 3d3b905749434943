// fhs_modarith.h -- 64-bit modular arithmetic for gfx950 (CDNA4) device code.
//
// CDNA4 has no 64x64->128 multiplier: a 64-bit product is built from v_mad_u64_u32 /
// v_mul_hi_u32 (quarter-rate integer multiplies, measured 2.2e12 Shoup mulmod/s chip-wide,
// tools/microbench/mulrate.hip).  Everything here is written to minimise those multiplies:
//   * Shoup multiply for fixed operands (twiddles, base-conversion constants): 1 mulhi + 2 mullo;
//   * lazy 128-bit accumulation + one Barrett reduction for sums of products (Hadamard, ModUp);
//   * Harvey lazy butterflies keep NTT values in [0, 4q) so most conditional subtractions vanish.
// All primes are < 2^61 (reference uses 59-bit, fhe_rwkv_inference.py uses 40/60-bit).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint64_t u64;

struct u128 {
    u64 lo, hi;
};

__device__ __forceinline__ u64 mulhi64(u64 a, u64 b) { return __umul64hi(a, b); }

__device__ __forceinline__ void mac128(u128& acc, u64 a, u64 b) {
    u64 lo = a * b, hi = __umul64hi(a, b);
    acc.lo += lo;
    acc.hi += hi + (acc.lo < lo);
}

__device__ __forceinline__ u64 csub(u64 a, u64 q) { return a >= q ? a - q : a; }

// Shoup: w * a mod q given wp = floor(w 2^64 / q); result in [0, 2q) for any 64-bit a.
__device__ __forceinline__ u64 shoup_lazy(u64 a, u64 w, u64 wp, u64 q) {
    u64 qh = __umul64hi(a, wp);
    return a * w - qh * q;
}
__device__ __forceinline__ u64 shoup(u64 a, u64 w, u64 wp, u64 q) { return csub(shoup_lazy(a, w, wp, q), q); }

// Barrett reduction of a 128-bit value with r = floor(2^128 / q) = (r1:r0).  The quotient
// estimate is short by at most 2, so two corrections give the canonical residue in [0, q).
__device__ __forceinline__ u64 barrett128(u64 lo, u64 hi, u64 q, u64 r0, u64 r1) {
    u64 c = __umul64hi(lo, r0);
    u64 a_lo = lo * r1, a_hi = __umul64hi(lo, r1);
    u64 t1 = a_lo + c;
    u64 t3 = a_hi + (t1 < c);
    u64 b_lo = hi * r0, b_hi = __umul64hi(hi, r0);
    u64 s = t1 + b_lo;
    u64 carry = b_hi + (s < t1);
    u64 qest = hi * r1 + t3 + carry;
    u64 r = lo - qest * q;
    r = csub(r, q);
    return csub(r, q);
}
__device__ __forceinline__ u64 barrett64(u64 a, u64 q, u64 r0, u64 r1) { return barrett128(a, 0, q, r0, r1); }

__device__ __forceinline__ u64 mulmod(u64 a, u64 b, u64 q, u64 r0, u64 r1) {
    return barrett128(a * b, __umul64hi(a, b), q, r0, r1);
}
__device__ __forceinline__ u64 addmod(u64 a, u64 b, u64 q) { return csub(a + b, q); }
__device__ __forceinline__ u64 submod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }

// Per-prime constants, 64 B, kept in a device table indexed by key-level prime index.
struct PrimeK {
    u64 q;
    u64 r0, r1;       // Barrett floor(2^128/q)
    u64 ninv, ninv_s; // N^-1 and Shoup companion
    u64 w1ninv, w1ninv_s;  // psi_rev_inv[1] * N^-1 (last GS stage)
    u64 pad;
};
