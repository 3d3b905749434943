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

__host__ __device__ __forceinline__ u64 csub(u64 a, u64 q) { return a >= q ? a - q : a; }

// 64x64 products spelled out in 32-bit halves: gfx950 issues v_mad_u64_u32 / v_mul_lo_u32 /
// v_mul_hi_u32 at about the rate of a 64-bit add (tools/microbench/instrate.hip), so what counts is
// the instruction total; this form lets the compiler fold the carries into the mad accumulators.
__host__ __device__ __forceinline__ u64 mul32w(uint32_t a, uint32_t b) { return (u64)a * b; }
__device__ __forceinline__ u64 mulhi64x(u64 a, u64 b) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const u64 t = mul32w(a1, b0) + __umulhi(a0, b0);
    const u64 s = mul32w(a0, b1) + (uint32_t)t;
    return mul32w(a1, b1) + (t >> 32) + (s >> 32);
}
__device__ __forceinline__ u64 mullo64x(u64 a, u64 b) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const u64 p = mul32w(a0, b0);
    const uint32_t hi = (uint32_t)(p >> 32) + a1 * b0 + a0 * b1;
    return ((u64)hi << 32) | (uint32_t)p;
}
// FHS_ASM_SHOUP (default 1): Shoup products with the mad carry-out and an opaque add3, written as
// one-instruction asm statements (the compiler still allocates registers and schedules around
// them): 7.7 % fewer VALU instructions in k_modup_h, 15 % in k_ks_intt_h, k_modup 2.72 -> 2.64 ms per
// cfg2 step, limbs unchanged (profiles/r02/ab_asm_shoup.txt).  0 keeps the plain C form.
#ifndef FHS_ASM_SHOUP
#define FHS_ASM_SHOUP 1
#endif
#if FHS_ASM_SHOUP
// v_mad_u64_u32 with its carry-out (the lane mask of the 64-bit accumulate's overflow)
__device__ __forceinline__ u64 mad_cc(uint32_t a, uint32_t b, u64 c, u64& cc) {
    u64 r;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t addc_lane(uint32_t x, u64 cc) {
    uint32_t r;
    asm("v_addc_co_u32 %0, vcc, %1, 0, %2" : "=v"(r) : "v"(x), "s"(cc) : "vcc");
    return r;
}
__device__ __forceinline__ uint32_t add3_opaque(uint32_t x, uint32_t y, uint32_t z) {
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    return r;
}
// hi64(a b): the middle sum's carry taken from the mad's carry-out instead of zero-extended halves
__device__ __forceinline__ u64 mulhi64a(u64 a, u64 b) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const u64 t = mul32w(a1, b0) + __umulhi(a0, b0);   // < 2^64
    u64 cc;
    const u64 s = mad_cc(a0, b1, t, cc);               // a0 b1 + t mod 2^64, cc = overflow
    const u64 r = mul32w(a1, b1) + (s >> 32);
    return ((u64)addc_lane((uint32_t)(r >> 32), cc) << 32) | (uint32_t)r;
}
// low 64 bits of a w + b v
__device__ __forceinline__ u64 mullo64a2(u64 a, u64 w, u64 b, u64 v) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32), v0 = (uint32_t)v, v1 = (uint32_t)(v >> 32);
    const u64 p = mul32w(a0, w0) + mul32w(b0, v0);
    const uint32_t h = add3_opaque((uint32_t)(p >> 32), a1 * w0 + a0 * w1, b1 * v0 + b0 * v1);
    return ((u64)h << 32) | (uint32_t)p;
}
#endif
// Shoup: w * a mod q given wp = floor(w 2^64 / q); result in [0, 2q) for any 64-bit a.
__device__ __forceinline__ u64 shoup_lazy(u64 a, u64 w, u64 wp, u64 q) {
#if FHS_ASM_SHOUP   // a w - qh q = a w + qh (2^64 - q) mod 2^64
    const u64 qh = mulhi64a(a, wp);
    return mullo64a2(a, w, qh, 0 - q);
#else
    const u64 qh = mulhi64x(a, wp);
    return mullo64x(a, w) - mullo64x(qh, q);
#endif
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

// Pseudo-Mersenne reduction for q = 2^b - d (d < 2^32): x = x_h 2^b + x_l == x_h d + x_l (mod q).
// Three folds take any 128-bit x below 2q; the host (pm_eligible in fhs_host.hip) proves the
// fold bounds for each prime before enabling this path.  SEAL-style Create() primes sit just
// below 2^b, so d is small (< 2^27 for the reference's 59-bit chain).  Six 32x32->64 multiplies
// against ~23 for barrett128.
__host__ __device__ __forceinline__ u64 pm_reduce128(u64 lo, u64 hi, u64 q, unsigned b, unsigned d) {
    const u64 mask = (1ull << b) - 1;
    const unsigned sb = 64 - b;
    // fold 1: x_h = top 2^64 + mid, top < 2^(64-b)
    const u64 top = hi >> b;
    const u64 mid = (hi << sb) | (lo >> b);
    const u64 p0 = (u64)(uint32_t)mid * d;
    const u64 p1 = (u64)(uint32_t)(mid >> 32) * d;
    u64 s_lo = p0 + (p1 << 32);
    u64 s_hi = (p1 >> 32) + (u64)(uint32_t)top * d + (s_lo < p0);
    const u64 xl = lo & mask;
    s_lo += xl;
    s_hi += (s_lo < xl);
    // fold 2: x_h < 2^64
    const u64 h2 = (s_hi << sb) | (s_lo >> b);
    const u64 q0 = (u64)(uint32_t)h2 * d;
    const u64 q1 = (u64)(uint32_t)(h2 >> 32) * d;
    u64 t_lo = q0 + (q1 << 32);
    u64 t_hi = (q1 >> 32) + (t_lo < q0);
    const u64 yl = s_lo & mask;
    t_lo += yl;
    t_hi += (t_lo < yl);
    // fold 3: x_h < 2^32
    const u64 h3 = (t_hi << sb) | (t_lo >> b);
    return csub((u64)(uint32_t)h3 * d + (t_lo & mask), q);
}
__device__ __forceinline__ u64 addmod(u64 a, u64 b, u64 q) { return csub(a + b, q); }
__device__ __forceinline__ u64 submod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }

// Split-30 lazy accumulation of sums of 64x64 products for residues < 2^60 (every context prime
// is < 2^60): x = x1 2^30 + x0 with x0, x1 < 2^30, so each partial product is < 2^60 and a plain
// v_mad_u64_u32 accumulates it in 64 bits.  L, H take one partial per product, M two, so up to 8
// products fit before acc3_fold must move the sums into a 128-bit accumulator: 4 multiply-adds per
// product instead of a full 128-bit product and carry chain (~15 instructions).
struct Acc3 {
    u64 L, M, H;
};
struct Split30 {
    uint32_t lo, hi;
};
__device__ __forceinline__ Split30 split30(u64 x) { return Split30{(uint32_t)x & 0x3FFFFFFFu, (uint32_t)(x >> 30)}; }
__host__ __device__ __forceinline__ u64 pack30(u64 x) { return (u64)(((uint32_t)x) & 0x3FFFFFFFu) | ((x >> 30) << 32); }
__host__ __device__ __forceinline__ Split30 unpack30(u64 p) { return Split30{(uint32_t)p, (uint32_t)(p >> 32)}; }
// The compiler forms M's two partials separately and adds their sum (a v_lshl_add_u64 more per product);
// forcing the chain -- one v_mad_u64_u32 per partial as inline asm, or an empty asm between M's two mads --
// measured slower on MI355X (r04c: key inner products 1.62 -> 1.90 ms/step, Hadamard 1.93 -> 1.96-1.98;
// the asm blocks unrolling and adds hazard nops), so the plain expression stays.
__device__ __forceinline__ void acc3_mac(Acc3& a, Split30 x, Split30 y) {
    a.L += mul32w(x.lo, y.lo);
    a.M += mul32w(x.lo, y.hi);
    a.M += mul32w(x.hi, y.lo);
    a.H += mul32w(x.hi, y.hi);
}
// (L + M 2^30 + H 2^60) mod q, result in [0, 2q), for q = 2^b - d: the split-30 sums are cut at
// bit b (A = L + (M mod 2^(b-30)) 2^30, B = M >> (b-30) + H 2^(60-b), x == A + B d) and folded once
// more.  Valid when the host's conv_pm_ok bounds hold (PrimeK.pm bit 40); ~23 instructions against
// ~37 for acc3_fold + pm_reduce128.
__host__ __device__ __forceinline__ u64 acc3_reduce_pm(u64 L, u64 M, u64 H, unsigned b, unsigned d) {
    const unsigned sh = b - 30;
    const u64 A = L + ((M & ((1ull << sh) - 1)) << 30);
    const u64 B = (M >> sh) + (H << (60 - b));
    const u64 p0 = (u64)(uint32_t)B * d, p1 = (u64)(uint32_t)(B >> 32) * d;
    u64 lo = A + p0;
    u64 hi = (lo < p0);
    const u64 p1l = p1 << 32;
    lo += p1l;
    hi += (lo < p1l) + (p1 >> 32);
    const u64 Sh = (hi << (64 - b)) | (lo >> b);
    return (lo & ((1ull << b) - 1)) + (u64)(uint32_t)Sh * d;
}
// ---- X form of the centred base extension of a full 3-limb digit (DESIGN.md §3 "ModUp X form";
// k_centered_x / modup_convert3x in fhs_kernels.hip, the host tables in fhs_host.hip
// modup_xform_tables).  D = the digit's 32-word table: Q_S/q_u (2 words each, u < 3), the rounding
// thresholds ((2k - 1) Q_S + 1)/2 (k = 1..3) and 2^179 - v Q_S (v = 0..3), 3 words each.
typedef unsigned __int128 u128x;
__host__ __device__ __forceinline__ bool ge192(const u64 s[3], const u64* t) {
    return s[2] != t[2] ? s[2] > t[2] : (s[1] != t[1] ? s[1] > t[1] : s[0] >= t[0]);
}
// y[u] (< q_u) -> U = X + 2^179 as base-2^60 words (V0 plain, V1 and V2 split-30 packed), X = S - v Q_S the centred digit
// value: S = sum_u y_u Q_S/q_u < 3 Q_S, v = round(S/Q_S) (never a tie: Q_S is odd), |X| < Q_S/2 < 2^179 (primes < 2^60)
__host__ __device__ __forceinline__ void centered_x_pack(const u64 y[3], const u64* D, u64 out[3]) {
    u128x lo = 0;   // S below 2^128
    u64 s2 = 0;     // S >> 128
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const u128x a = (u128x)y[k] * D[2 * k], b = (u128x)y[k] * D[2 * k + 1];   // y H = a + b 2^64
        const u128x t = lo + a;
        s2 += (u64)(t < a);
        const u128x bl = b << 64;
        lo = t + bl;
        s2 += (u64)(b >> 64) + (u64)(lo < bl);
    }
    const u64 s[3] = {(u64)lo, (u64)(lo >> 64), s2};
    const int v = (int)ge192(s, D + 6) + (int)ge192(s, D + 9) + (int)ge192(s, D + 12);
    const u64* C = D + 15 + 3 * v;
    const u128x c01 = (u128x)C[0] | ((u128x)C[1] << 64);
    const u128x u01 = lo + c01;
    const u64 u2 = s2 + C[2] + (u64)(u01 < c01);
    const u64 u0 = (u64)u01, u1 = (u64)(u01 >> 64);
    constexpr u64 M60 = (1ull << 60) - 1;
    out[0] = u0 & M60;   // plain: the conversions add it whole (convert3x_b59) or split it (convert3x_value)
    out[1] = pack30(((u0 >> 60) | (u1 << 4)) & M60);
    out[2] = pack30((u1 >> 56) | (u2 << 8));
}
// X mod m in [0, 2m) from the packed words: V0 + V1 e1 + V2 e2 + c3 with xt = {2^60 mod m (< 2^30: the
// host requires it -- 2d or d for the usual 59/60-bit q = 2^b - d), pack30(2^120 mod m), -2^179 mod m};
// the split-30 sums stay inside the 3-product bounds conv_pm_ok proves for m (L < 2 p30^2 + 2^30 + m,
// M < 3 p30^2 + 2^30, H < p30^2, p30 = 2^30 - 1)
__host__ __device__ __forceinline__ u64 convert3x_value(u64 p0, u64 p1, u64 p2, uint32_t e1, Split30 e2, u64 c3,
                                                        unsigned b, unsigned d) {
    const Split30 a = {(uint32_t)p0 & 0x3FFFFFFFu, (uint32_t)(p0 >> 30)}, v1 = unpack30(p1), v2 = unpack30(p2);
    const u64 L = (u64)a.lo + c3 + mul32w(v1.lo, e1) + mul32w(v2.lo, e2.lo);
    const u64 M = (u64)a.hi + mul32w(v1.hi, e1) + mul32w(v2.lo, e2.hi) + mul32w(v2.hi, e2.lo);
    const u64 H = mul32w(v2.hi, e2.hi);
    return acc3_reduce_pm(L, M, H, b, d);
}

// The same value for a 59-bit target m = 2^59 - d with d < 2^27 (DevTables::conv_b59: every prime of the
// chain), where 2^59 == d makes every fold a 32 x 32 product and the sums stay below 2^63:
//   L = V0 + c3 + v1.lo e1 + v2.lo e2.lo < 2^60 + 2^59 + 2^60 + 2^60,  M = v1.hi e1 + v2.lo e2.hi + v2.hi e2.lo
//   < 2^58 + 2^59 + 2^60 (e1 = 2d < 2^28, e2 < 2^59),  H = v2.hi e2.hi < 2^59;
//   x == L + M 2^30 + H 2^60 == A + B d,  A = L + (M mod 2^29) 2^30 < 2^62 + 2^59,  B = (M >> 29) + 2H < 2^32 + 2^60;
//   B d = B0 d + B1 d 2^32 (B0 < 2^32, B1 < 2^29), and with B1 d = h 2^27 + r:  B1 d 2^32 == h d + r 2^32;
//   s = A + B0 d + r 2^32 + h d < 2^62 + 3 * 2^59 + 2^55 < 2^63.
// canon: one more fold, s mod 2^59 + (s >> 59) d < 2^59 + 2^4 d < 2m (the NTT's added inputs); otherwise s
// itself (any 64-bit value congruent to x: the inputs the first butterfly multiplies by a twiddle).
// About 18 instructions without the fold, against ~34 for convert3x_value with a run-time b.
__host__ __device__ __forceinline__ u64 convert3x_b59(u64 V0, u64 p1, u64 p2, uint32_t e1, Split30 e2, u64 c3,
                                                      uint32_t d, bool canon) {
    const Split30 v1 = unpack30(p1), v2 = unpack30(p2);
    const u64 L = V0 + c3 + mul32w(v1.lo, e1) + mul32w(v2.lo, e2.lo);
    const u64 M = mul32w(v1.hi, e1) + mul32w(v2.lo, e2.hi) + mul32w(v2.hi, e2.lo);
    const u64 H = mul32w(v2.hi, e2.hi);
    const u64 A = L + ((M & ((1ull << 29) - 1)) << 30);
    const u64 B = (M >> 29) + (H << 1);
    const u64 b1d = mul32w((uint32_t)(B >> 32), d);
    u64 sv = A + mul32w((uint32_t)B, d);
    sv += (b1d & ((1ull << 27) - 1)) << 32;
    sv += mul32w((uint32_t)(b1d >> 27), d);
    if (!canon) return sv;
    return (sv & ((1ull << 59) - 1)) + mul32w((uint32_t)(sv >> 59), d);
}

// c += L + M 2^30 + H 2^60 (< 2^123 for 8 products), then clear
__device__ __forceinline__ void acc3_fold(u128& c, Acc3& a) {
    u64 lo = a.L, hi = 0;
    u64 t = a.M << 30;
    lo += t;
    hi += (lo < t) + (a.M >> 34);
    t = a.H << 60;
    lo += t;
    hi += (lo < t) + (a.H >> 4);
    c.lo += lo;
    c.hi += hi + (c.lo < lo);
    a = Acc3{0, 0, 0};
}

// ---- secret randomness: ChaCha20 (RFC 8439 §2.3) as a PRF keyed by a 256-bit secret (DESIGN.md
// §Sampling; shared with oracle/ckks_oracle.c ock_chacha20_block).  Stream `sid` (a 64-bit domain
// label: kind, Galois element, digit, encryption counter) is the 96-bit nonce (lo32, hi32, "FHS1"),
// the block counter indexes the coefficient.  Everything secret (s, errors, encryption masks) and
// every public value derived from the secret key (the switching keys' a_j seeds, the public key's
// a) is a PRF output, so publishing it reveals nothing about the key.
struct PrfKey {
    uint32_t k[8];
};
#define FHS_ROTL32(v, n) (((v) << (n)) | ((v) >> (32 - (n))))
#define FHS_QR(a, b, c, d)                  \
    a += b; d ^= a; d = FHS_ROTL32(d, 16);  \
    c += d; b ^= c; b = FHS_ROTL32(b, 12);  \
    a += b; d ^= a; d = FHS_ROTL32(d, 8);   \
    c += d; b ^= c; b = FHS_ROTL32(b, 7);
__host__ __device__ __forceinline__ void chacha20_block(const PrfKey& K, uint32_t ctr, uint32_t n0, uint32_t n1,
                                                         uint32_t n2, uint32_t out[16]) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, K.k[0], K.k[1], K.k[2], K.k[3],
                      K.k[4],      K.k[5],      K.k[6],      K.k[7],      ctr,    n0,     n1,     n2};
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = s[i];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        FHS_QR(x[0], x[4], x[8], x[12]) FHS_QR(x[1], x[5], x[9], x[13])
        FHS_QR(x[2], x[6], x[10], x[14]) FHS_QR(x[3], x[7], x[11], x[15])
        FHS_QR(x[0], x[5], x[10], x[15]) FHS_QR(x[1], x[6], x[11], x[12])
        FHS_QR(x[2], x[7], x[8], x[13]) FHS_QR(x[3], x[4], x[9], x[14])
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}
#undef FHS_QR
#undef FHS_ROTL32
constexpr uint32_t kPrfTag = 0x31534846u;   // "FHS1"
// first two 64-bit words of block `ctr` of stream `sid`
__host__ __device__ __forceinline__ void prf128(const PrfKey& K, u64 sid, uint32_t ctr, u64& w0, u64& w1) {
    uint32_t o[16];
    chacha20_block(K, ctr, (uint32_t)sid, (uint32_t)(sid >> 32), kPrfTag, o);
    w0 = (u64)o[0] | ((u64)o[1] << 32);
    w1 = (u64)o[2] | ((u64)o[3] << 32);
}

// SplitMix64 (the sampling spec shared with oracle/ckks_oracle.c ock_splitmix64): public
// expansion of a switching key's a_j from its seed (regenerated inside the key inner product, where
// a ChaCha block per coefficient would cost more than the key bytes it saves) and test data.
__host__ __device__ __forceinline__ u64 sm64(u64 x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
// Seeded uniform residue (switching-key `a` components): the top `bits`
// bits of sm64(key + ctr * gamma), ctr = m 2^40 | prime 2^20 | n, accepted when < q (rejection
// sampling: exactly uniform; for SEAL-style primes a retry has probability (2^bits - q) / 2^bits <
// 2^-32).  `kx` = key + (prime 2^20 | n) * gamma is hoisted by callers that vary only the key.
__host__ __device__ __forceinline__ u64 seeded_uniform_x(u64 kx, u64 q, unsigned bits) {
    const u64 v0 = sm64(kx) >> (64 - bits);
    if (__builtin_expect(v0 < q, 1)) return v0;
    for (u64 m = 1;; ++m) {   // taken with probability < 2^-32 per draw for SEAL-style primes
        const u64 v = sm64(kx + (m << 40) * 0x9E3779B97F4A7C15ULL) >> (64 - bits);
        if (v < q) return v;
    }
}
__host__ __device__ __forceinline__ u64 seeded_ctr_mix(int prime, int n) {
    return (((u64)prime << 20) | (u64)n) * 0x9E3779B97F4A7C15ULL;
}

// Per-prime constants, 64 B, kept in a device table indexed by key-level prime index.
struct PrimeK {
    u64 q;
    u64 r0, r1;       // Barrett floor(2^128/q)
    u64 ninv, ninv_s; // N^-1 and Shoup companion
    u64 w1ninv, w1ninv_s;  // psi_rev_inv[1] * N^-1 (last GS stage)
    u64 pm;           // (d << 8) | lazy << 7 | b when q = 2^b - d passes the pm_reduce128 bounds, else 0;
                      // lazy: q (4 + 2 logN) < 2^64, so forward-NTT values never leave 64 bits
};

__device__ __forceinline__ u64 reduce128(u64 lo, u64 hi, const PrimeK& P) {
    if (P.pm) return pm_reduce128(lo, hi, P.q, (unsigned)(P.pm & 127), (unsigned)((P.pm >> 8) & 0xFFFFFFFFu));
    return barrett128(lo, hi, P.q, P.r0, P.r1);
}
// Wave-uniform view of a prime's reduction constants (SGPRs): kernels whose prime is uniform per
// wave use it so the pseudo-Mersenne / Barrett choice is a scalar branch, not a divergent one.
__device__ __forceinline__ u64 rfl64(u64 x) {
    // the builtin is int -> int: widen through uint32_t so the low word is not sign-extended
    return ((u64)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32) |
           (u64)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}
struct RedU {
    u64 q, r0, r1;
    unsigned b, d;
    bool lazy;   // forward NTT may skip Harvey's conditional subtraction (PrimeK.pm bit 7)
    bool cpm;    // ModUp conversion may use acc3_reduce_pm (PrimeK.pm bit 40)
};
__device__ __forceinline__ RedU redu(const PrimeK& P) {
    const u64 pm = rfl64(P.pm);
    return RedU{rfl64(P.q), rfl64(P.r0), rfl64(P.r1), (unsigned)(pm & 127), (unsigned)((pm >> 8) & 0xFFFFFFFFu),
                (pm & 128) != 0, ((pm >> 40) & 1) != 0};
}
__device__ __forceinline__ u64 reduce128(u64 lo, u64 hi, const RedU& R) {
    if (R.b) return pm_reduce128(lo, hi, R.q, R.b, R.d);
    return barrett128(lo, hi, R.q, R.r0, R.r1);
}
// Any 64-bit value of a pseudo-Mersenne prime (b >= 41) to [0, q): one fold, one subtraction.
__device__ __forceinline__ u64 pm_fold64(u64 x, const RedU& R) {
    const u64 h = x >> R.b;
    return csub((x & ((1ull << R.b) - 1)) + (u64)(uint32_t)h * R.d, R.q);
}
// A lazy forward-NTT output (< (4 + 2 logN) q < 2^64; lazy implies q = 2^b - d on the fold, b >= 41) folded
// once: < 2^b + 2^(64-b) 2^32 < 2^60 and congruent to x, but not canonical -- for consumers that take any
// value below 2^60 (the key inner products' split-30 sums read ModUp's extended limbs)
__device__ __forceinline__ u64 pm_fold_lt60(u64 x, const RedU& R) {
    return (x & ((1ull << R.b) - 1)) + (u64)(uint32_t)(x >> R.b) * R.d;
}
// Any 64-bit x for a 59-bit prime q = 2^59 - d, d < 2^27 (DevTables::conv_b59): one fold to
// < 2^59 + 2^5 d < 2q, congruent to x -- a forward-NTT output (lazy or Harvey) ready for a + 2q - x
__device__ __forceinline__ u64 fold59(u64 x, uint32_t d) {
    return (x & ((1ull << 59) - 1)) + mul32w((uint32_t)(x >> 59), d);
}
// Canonical residue of a forward-NTT output: lazy outputs are < (4 + 2 logN) q, Harvey ones < 4q.
__device__ __forceinline__ u64 fwd_canon(u64 x, const RedU& R) {
    if (R.lazy) return pm_fold64(x, R);
    return csub(csub(x, 2 * R.q), R.q);
}
__device__ __forceinline__ u64 reduce64(u64 a, const PrimeK& P) { return reduce128(a, 0, P); }
__device__ __forceinline__ u64 mulmod(u64 a, u64 b, const PrimeK& P) { return reduce128(a * b, __umul64hi(a, b), P); }
