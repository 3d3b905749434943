// fhs_kernels.hip -- hand-written gfx950 kernels for the CKKS BSGS hot path.
//
// Kernel map:
//   k_ntt_fwd / k_ntt_inv          batched per-limb negacyclic NTT (one limb per workgroup, LDS-resident)
//   k_eltwise / k_tensor           ct add/sub/negate, ct x pt Hadamard (pb:167, 181), ct x ct tensor (pb:177)
//   k_rescale_*                    divide-and-round by q_last (pb:185, bg:484)
//   k_ks_intt / k_modup_ip /       hybrid key-switch: automorphism+INTT, fused ModUp+NTT+key inner product,
//   k_ks_special_intt / k_moddown  ModDown (pb:203 rotate, pb:183 relinearize)
//   k_bsgs_inner                   sum_b baby[b] (.) pt[gG+b] for every giant group g (bg:465-476)
//   k_giant_sum / k_giant_final    giant-step rotations summed exactly in the extended basis (bg:478-483)
//   k_sample / k_swk / ...         deterministic key generation and encryption helpers
// Every integer result is reduced to [0, q): limbs are bit-identical to oracle/ckks_oracle.c.
#include "fhs_kernels.h"
typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
#ifndef FHS_MODUP_STORE_AUX
#define FHS_MODUP_STORE_AUX 2   // k_modup_h output stores non-temporal: L2 keeps the digits the next
                                // targets convert (reads 3.14 -> 2.49 GB/step, profiles/r03/ab/*_modup_nt.json)
#endif
#ifndef FHS_KSIP_UNROLL
#define FHS_KSIP_UNROLL 4   // digits of the key inner product unrolled together (4 since the buffer loads: profiles/r03/ab/ksip_ch_summary.txt)
#endif
#include "fhs_ntt.h"
#include "fhs_buffer.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

// Tuning constants (each chosen by an A/B on the cfg2 bench, limbs unchanged; the rejected
// alternatives and their records are listed in DESIGN.md and profiles/r0*/ab_*).
#define FHS_INNER_WAVES 16     // waves per k_bsgs_inner workgroup sharing one LDS baby-step slice
#define FHS_INNER_VEC 2        // consecutive coefficients per lane in k_bsgs_inner (16-byte loads)
#define FHS_MODDOWN_HALF 1     // k_moddown_h: half-limb LDS
#define FHS_INTT_HALF 1        // k_ks_intt_h: half-limb LDS inverse NTT
#ifndef FHS_MODUP_QUADPAIR
#define FHS_MODUP_QUADPAIR 1   // k_modup_h block decode: 1 = xcd_quadpair (inputs read by 4 XCDs), 0 = xcd_tinner
#endif
#ifndef FHS_MODUPH_CH
#define FHS_MODUPH_CH 2        // k_modup_h: coefficient pairs per conversion chunk
#endif
#ifndef FHS_MODUPH_RL
#define FHS_MODUPH_RL 3        // k_modup_h: radix (log2) of the NTT register passes
#endif
#define FHS_MODUP_CH 4         // k_modup (full-limb form): coefficients per conversion chunk
#define FHS_MODUP_RL 4         // k_modup (full-limb form): radix (log2) of the NTT register passes
#define FHS_NTT_RL 3           // radix (log2) for the other NTT kernels
#ifndef FHS_FWD_FIRST3
#define FHS_FWD_FIRST3 1       // half-limb forward transforms at N = 32768: global stages 0-2 in registers
#endif
#ifndef FHS_KSIP_HALVES
#define FHS_KSIP_HALVES 1      // k_ks_ip (hoisted): coefficient halves outermost (L2 reuse of the extension)
#endif

namespace fhs {

#define FHS_DISPATCH_LOGN(logN, ...)                   \
    switch (logN) {                                    \
        case 8: { constexpr int LOGN = 8; __VA_ARGS__; } break;   \
        case 9: { constexpr int LOGN = 9; __VA_ARGS__; } break;   \
        case 10: { constexpr int LOGN = 10; __VA_ARGS__; } break; \
        case 11: { constexpr int LOGN = 11; __VA_ARGS__; } break; \
        case 12: { constexpr int LOGN = 12; __VA_ARGS__; } break; \
        case 13: { constexpr int LOGN = 13; __VA_ARGS__; } break; \
        case 14: { constexpr int LOGN = 14; __VA_ARGS__; } break; \
        case 15: { constexpr int LOGN = 15; __VA_ARGS__; } break; \
        default: return hipErrorInvalidValue;          \
    }

__device__ __forceinline__ const PrimeK& PK(const DevTables& T, int i) {
    return reinterpret_cast<const PrimeK*>(T.primes)[i];
}

// XCD-aware block decode.  Workgroups are dealt round-robin over the 8 XCDs (observed placement,
// MI355X_MICROARCH.md "Workgroup dispatch"; speed only, never correctness), so block b runs on the
// XCD shared by all blocks b' == b (mod 8).  Giving XCD x only the limbs t == x (mod 8) keeps that
// XCD's L2 (4 MiB) holding ~E/8 primes' twiddle tables instead of all E (10 MiB at E = 39).
// Grid = 8 * ceil(E/8) * M blocks; returns false for the padding blocks.
//   t-inner: an XCD cycles its primes fastest (blocks sharing an input m = (digit, input) run together)
//   t-outer: an XCD finishes one limb t across all m before the next (shared per-limb data stays hot)
__host__ __device__ __forceinline__ int xcd_grid(int E, int M) { return 8 * ((E + 7) / 8) * M; }
__device__ __forceinline__ bool xcd_tinner(int E, int M, int& t, int& m) {
    const int b = blockIdx.x, x = b & 7, k = b >> 3, nx = (E - x + 7) >> 3;
    if (nx <= 0 || k >= nx * M) return false;
    t = x + 8 * (k % nx);
    m = k / nx;
    return true;
}
// m-major: XCD x takes the inputs m == x (mod 8), all limbs t of one m back to back
__device__ __forceinline__ bool xcd_mmajor(int E, int M, int& t, int& m) {
    const int b = blockIdx.x, x = b & 7, k = b >> 3, nm = (M - x + 7) >> 3;
    if (nm <= 0 || k >= nm * E) return false;
    m = x + 8 * (k / E);
    t = k % E;
    return true;
}
// quad-pair: XCD x takes the limbs t == x (mod 4) of the inputs m == x / 4 (mod 2) -- ~E/4 primes' twiddle
// tables per XCD L2 (2.5 MiB at E = 39) and each input read by 4 XCDs instead of all 8 (t-inner as
// xcd_tinner).  Grid = 8 * ceil(E/4) * ceil(M/2).
__host__ __device__ __forceinline__ int xcd_grid_q(int E, int M) { return 8 * ((E + 3) / 4) * ((M + 1) / 2); }
__device__ __forceinline__ bool xcd_quadpair(int E, int M, int& t, int& m) {
    const int b = blockIdx.x, x = b & 7, k = b >> 3, pg = x & 3, mh = x >> 2;
    const int nx = (E - pg + 3) >> 2, nm = (M - mh + 1) >> 1;
    if (nx <= 0 || nm <= 0 || k >= nx * nm) return false;
    t = pg + 4 * (k % nx);
    m = mh + 2 * (k / nx);
    return true;
}
__host__ __device__ __forceinline__ int xcd_grid_m(int E, int M) { return 8 * ((M + 7) / 8) * E; }
// plain: blockIdx.x = t + E * m (t fastest)
__device__ __forceinline__ bool plain_tm(int E, int M, int& t, int& m) {
    t = blockIdx.x % E;
    m = blockIdx.x / E;
    return m < M;
}
__device__ __forceinline__ bool xcd_touter(int E, int M, int& t, int& m) {
    const int b = blockIdx.x, x = b & 7, k = b >> 3, nx = (E - x + 7) >> 3;
    if (nx <= 0 || k >= nx * M) return false;
    t = x + 8 * (k / M);
    m = k % M;
    return true;
}
__device__ __forceinline__ int limb_prime(int b, int l_split, int L0) { return b < l_split ? b : L0 + (b - l_split); }

// NTT-domain automorphism X -> X^elt: output slot e reads input slot galois_src(e)
__device__ __forceinline__ int galois_src(int e, u64 elt, int logN) {
    if (elt == 1) return e;
    const unsigned r = __brev((unsigned)e) >> (32 - logN);
    const u64 m = (u64)2 << logN;
    const u64 e2 = ((2 * (u64)r + 1) * elt) & (m - 1);
    return (int)(__brev((unsigned)((e2 - 1) >> 1)) >> (32 - logN));
}

// The forward NTT may skip Harvey's conditional subtraction (RedU::lazy: q (4 + 2 log N) < 2^64).  Every
// prime of a B59 context is below 2^59, so for N <= 16384 that holds for all of them: the kernels'
// B59 instantiations drop the non-lazy code at compile time (same values -- lazy is true at run time too)
template <int LOGN, bool B59>
__device__ __forceinline__ bool lazy_of(const RedU& R) { return (B59 && LOGN <= 14) || R.lazy; }

template <int LOGN>
constexpr size_t lds_bytes() { return (size_t)((1 << LOGN) + (1 << LOGN) / 16) * 8; }

// ---- one-limb transforms, full limb in LDS (N <= 16384: 136 KiB) or half a limb (N = 32768):
// the half form does the global first forward stage / last inverse stage, which pairs e with
// e + N/2, in registers and transforms each half in LDS (k_modup_h explains the scheme).
// FHS_NTT_HALF_MIN (fhs_kernels.h): A/B at N = 16384, 2048-diagonal encode + matvec 18.64 -> 18.12 ms, bench unchanged
template <int LOGN> constexpr bool ntt_half() { return LOGN >= FHS_NTT_HALF_MIN; }
template <int LOGN, bool H = ntt_half<LOGN>()> constexpr int ntt_threads() { return H ? (1 << LOGN) / 32 : (1 << LOGN) / 16; }
template <int LOGN, bool H = ntt_half<LOGN>()> constexpr int ntt_lds_words() {
    return H ? (1 << (LOGN - 1)) + (1 << (LOGN - 1)) / 16 : (1 << LOGN) + (1 << LOGN) / 16;
}
// Launches with fewer workgroups than CUs (one transform per workgroup: the key switch's special
// limbs, rescale, the giant-step tail) are latency-bound: there the full-limb form (both halves in
// LDS at once, 1024 threads at N = 16384) finishes a transform in about half the time of the
// half-limb form, which transforms its two halves one after the other.  Same values.
#ifndef FHS_FULL_FORM_MAX_WG
#define FHS_FULL_FORM_MAX_WG 256
#endif
#define FHS_NTT_LAUNCH(K, nwg, grid, st, ...)                                                          \
    do {                                                                                               \
        constexpr bool FH_ = (LOGN > 14);   /* the full-limb form needs N <= 16384 */                   \
        if ((nwg) < FHS_FULL_FORM_MAX_WG && !FH_)                                                      \
            hipLaunchKernelGGL((K<LOGN, FH_>), grid, dim3(ntt_threads<LOGN, FH_>()), 0, st, __VA_ARGS__); \
        else                                                                                           \
            hipLaunchKernelGGL((K<LOGN>), grid, dim3(ntt_threads<LOGN>()), 0, st, __VA_ARGS__);        \
    } while (0)
// Radix-4 first stages: the half-limb forward transforms of ModUp / ModDown do global stages 0 and 1 in
// registers while converting -- a thread's rows c and c + 8 are N/4 apart, so it converts the quad
// (e, e + N/4, e + N/2, e + 3N/4) and applies a radix-4 butterfly (stage 0 twiddle psi^rev(1); stage 1
// psi^rev(2) on the lower half, psi^rev(3) on the upper).  Each half's LDS transform then starts at its
// local stage 1: 12 stages = four radix-8 passes, no radix-2 pass.  Same butterflies, same values
// (A/B on the cfg2 bench: k_modup 2.04 -> 1.98 ms, k_moddown 0.46 -> 0.44 ms per step,
// profiles/r03/ab/r4*.json).
struct Tw4 {
    u64 w1, w1p, w2, w2p, w3, w3p;
};
__device__ __forceinline__ Tw4 ld_tw4(const u64* __restrict__ tw) {
    Tw4 t;
    ld_tw(tw, 1, t.w1, t.w1p);
    ld_tw(tw, 2, t.w2, t.w2p);
    ld_tw(tw, 3, t.w3, t.w3p);
    return t;
}
// x = {row c lower, row c + 8 lower, row c upper, row c + 8 upper}, each < 2q: lower-half results to LDS
// rows c, c + 8, upper-half results to hi[c], hi[c + 8] (values as the LDS passes would leave them)
template <int TH>
__device__ __forceinline__ void fwd_quad_first2(u64 x[4], const Tw4& w, u64 q, bool lazy, u64* lds, int tid, int c,
                                                u64 hi[16]) {
    const u64 q2 = 2 * q;
#pragma unroll
    for (int k = 0; k < 2; ++k) {   // global stage 0: (e, e + N/2); outputs < 4q
        const u64 tt = shoup_lazy(x[2 + k], w.w1, w.w1p, q);
        const u64 X = x[k];
        x[k] = X + tt;
        x[2 + k] = X + (q2 - tt);
    }
    if (!lazy) {   // Harvey form: the next butterfly's unmultiplied inputs back below 2q
        x[0] = x[0] >= q2 ? x[0] - q2 : x[0];
        x[2] = x[2] >= q2 ? x[2] - q2 : x[2];
    }
    const u64 ta = shoup_lazy(x[1], w.w2, w.w2p, q), tb = shoup_lazy(x[3], w.w3, w.w3p, q);   // global stage 1
    lds[row_pad<TH>(tid, c)] = x[0] + ta;
    lds[row_pad<TH>(tid, c + 8)] = x[0] + (q2 - ta);
    hi[c] = x[2] + tb;
    hi[c + 8] = x[2] + (q2 - tb);
}
// Radix-8 first stages (N = 32768): the half transforms have 14 stages, which start-at-1 splits 3+3+3+3+1 (a
// radix-2 pass, and no wave-local exit); with global stages 0-2 in registers they start at local stage 2: four
// radix-8 passes, the last three wave-local.  x[k] = element e + k N/8 (e = tid + c TH, c < 4: rows c + 4k of
// the lower half for k < 4, of the upper half for k >= 4), each < 2q; stage s twiddle psi^rev(2^s + block).
// Lower-half results to LDS rows c, c + 4, c + 8, c + 12, upper-half results to hi[] at the same rows.
template <int TH>
__device__ __forceinline__ void fwd_oct_first3(u64 x[8], const u64* __restrict__ tw, u64 q, bool lazy, u64* lds,
                                               int tid, int c, u64 hi[16]) {
    const u64 q2 = 2 * q;
    auto bfly = [&](int a, int b, int wi) {
        u64 w, wp;
        ld_tw(tw, wi, w, wp);
        u64 X = x[a];
        if (!lazy) X = X >= q2 ? X - q2 : X;
        const u64 t = shoup_lazy(x[b], w, wp, q);
        x[a] = X + t;
        x[b] = X + (q2 - t);
    };
#pragma unroll
    for (int k = 0; k < 4; ++k) bfly(k, k + 4, 1);   // global stage 0: (e, e + N/2)
#pragma unroll
    for (int k = 0; k < 8; k += 4) {                  // stage 1: (e, e + N/4) in each half
        bfly(k, k + 2, 2 + k / 4);
        bfly(k + 1, k + 3, 2 + k / 4);
    }
#pragma unroll
    for (int k = 0; k < 8; k += 2) bfly(k, k + 1, 4 + k / 2);   // stage 2: (e, e + N/8) in each quarter
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        lds[row_pad<TH>(tid, c + 4 * k)] = x[k];
        hi[c + 4 * k] = x[4 + k];
    }
}
// radix-8 first stages where they leave the half transforms whole radix-8 passes and radix-4 would not
template <int LOGN>
constexpr bool fwd_first3() { return (LOGN - 2) % 3 != 0 && (LOGN - 3) % 3 == 0; }

// The inverse counterpart: the last two stages of a half-limb inverse in registers.  x = {half 0 row c,
// half 0 row c + 8, half 1 row c, half 1 row c + 8} (each < 2q, after the halves' LDS passes from local
// stage 1 on): the halves' local stage 0 (twiddle psi^-rev(2) / psi^-rev(3)), then the global stage 0
// with (s0, s1) = N^-1 times any per-limb constant folded in.  Out: {row c, row c + 8} of the lower half,
// then of the upper half, each < 2q.
__device__ __forceinline__ void inv_quad_last2(u64 x[4], const u64* __restrict__ tw, u64 q, u64 s0, u64 s0s, u64 s1,
                                               u64 s1s) {
    const u64 q2 = 2 * q;
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
        u64 w, wp;
        ld_tw(tw, 2 + k / 2, w, wp);
        const u64 X = x[k], Y = x[k + 1], S = X + Y;
        x[k] = S >= q2 ? S - q2 : S;
        x[k + 1] = shoup_lazy(X - Y + q2, w, wp, q);
    }
    const u64 a = x[0], b = x[1], c = x[2], d = x[3];
    x[0] = shoup_lazy(a + c, s0, s0s, q);
    x[1] = shoup_lazy(b + d, s0, s0s, q);
    x[2] = shoup_lazy(a - c + q2, s1, s1s, q);
    x[3] = shoup_lazy(b - d + q2, s1, s1s, q);
}
// forward: load(e) < 2q for every e < N; store(e, v) receives the canonical NTT value
template <int LOGN, int RL, bool H = ntt_half<LOGN>(), class Load, class Store>
__device__ __forceinline__ void fwd_limb(u64* lds, int tid, const u64* __restrict__ tw, const RedU& R, Load load,
                                         Store store) {
    constexpr int N = 1 << LOGN;
    if constexpr (!H) {
        constexpr int TH = N / 16;
#pragma unroll
        for (int c = 0; c < 16; ++c) lds[row_pad<TH>(tid, c)] = load(tid + c * TH);
        __syncthreads();
        ntt_fwd_lds<LOGN, RL>(lds, tid, tw, R.q, R.lazy);
#pragma unroll
        for (int c = 0; c < 16; ++c) store(tid + c * TH, fwd_canon(lds[row_pad<TH>(tid, c)], R));
    } else {
        constexpr int NH = N / 2, TH = N / 32;
        constexpr bool F3 = FHS_FWD_FIRST3 && fwd_first3<LOGN>();
        constexpr int S0 = F3 ? 2 : 1;
        u64 hi[16];
        if constexpr (F3) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {   // rows c + 4k of both halves: global stages 0-2 in registers
                u64 x[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) x[k] = load(tid + (c + 4 * k) * TH);
                fwd_oct_first3<TH>(x, tw, R.q, R.lazy, lds, tid, c, hi);
            }
        } else {
            const Tw4 w4 = ld_tw4(tw);
#pragma unroll
            for (int c = 0; c < 8; ++c) {   // rows c, c + 8 of both halves: global stages 0-1 in registers
                const int e = tid + c * TH;
                u64 x[4] = {load(e), load(e + 8 * TH), load(e + NH), load(e + NH + 8 * TH)};
                fwd_quad_first2<TH>(x, w4, R.q, R.lazy, lds, tid, c, hi);
            }
        }
#pragma unroll 1
        for (int h = 0; h < 2; ++h) {
            if (h) {
                __syncthreads();
#pragma unroll
                for (int c = 0; c < 16; ++c) lds[row_pad<TH>(tid, c)] = hi[c];
            }
            __syncthreads();
            constexpr bool WLX = FHS_NTT_WAVELOCAL && fwd_exit_wave_local<LOGN - 1, 3, S0>();
            ntt_fwd_lds<LOGN - 1, 3, 16, S0, WLX>(lds, tid, tw, R.q, R.lazy, 1 + h);
            if constexpr (WLX) {   // this wave's own outputs (wave-local tail, fhs_ntt.h)
                const int wb = wl_base<LOGN - 1, 16, 8>(tid), wp = lds_pad(wb);
#pragma unroll
                for (int c = 0; c < 16; ++c) {
                    const int off = wl_off<LOGN - 1, 16, 8>(c);
                    store(h * NH + wb + off, fwd_canon(lds[wp + off + off / 16], R));
                }
            } else {
#pragma unroll
                for (int c = 0; c < 16; ++c) store(h * NH + tid + c * TH, fwd_canon(lds[row_pad<TH>(tid, c)], R));
            }
        }
    }
}
// inverse with the last stage scaled by (s0, s1) (N^-1 and any per-limb constant folded in);
// load(e) < 2q; store(e, v) receives the canonical coefficient
template <int LOGN, int RL, bool H = ntt_half<LOGN>(), class Load, class Store>
__device__ __forceinline__ void inv_limb(u64* lds, int tid, const u64* __restrict__ tw, u64 q, u64 s0, u64 s0s,
                                         u64 s1, u64 s1s, Load load, Store store) {
    constexpr int N = 1 << LOGN;
    if constexpr (!H) {
        constexpr int TH = N / 16;
#pragma unroll
        for (int c = 0; c < 16; ++c) lds[row_pad<TH>(tid, c)] = load(tid + c * TH);
        __syncthreads();
        ntt_inv_lds<LOGN, RL>(lds, tid, tw, q, s0, s0s, s1, s1s);
#pragma unroll
        for (int c = 0; c < 16; ++c) store(tid + c * TH, csub(lds[row_pad<TH>(tid, c)], q));
    } else {
        constexpr int NH = N / 2, TH = N / 32;
        u64 lo[16];
#pragma unroll 1
        for (int h = 0; h < 2; ++h) {
            if (h) __syncthreads();
            constexpr bool WLI = FHS_NTT_WAVELOCAL && (LOGN - 2) % 3 == 0;
            if constexpr (WLI) {   // wave-local head: each wave loads the blocks its deep passes transform
                const int wb = wl_base<LOGN - 1, 16, 8>(tid), wp = lds_pad(wb);
#pragma unroll
                for (int c = 0; c < 16; ++c) {
                    const int off = wl_off<LOGN - 1, 16, 8>(c);
                    lds[wp + off + off / 16] = load(h * NH + wb + off);
                }
            } else {
#pragma unroll
                for (int c = 0; c < 16; ++c) lds[row_pad<TH>(tid, c)] = load(h * NH + tid + c * TH);
                __syncthreads();
            }
            ntt_inv_half_lds<LOGN - 1, 3, 16, 1, WLI>(lds, tid, tw, q, 1 + h);   // local stage 0: inv_quad_last2
            if (h == 0) {
#pragma unroll
                for (int c = 0; c < 16; ++c) lo[c] = lds[row_pad<TH>(tid, c)];
            }
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            u64 x[4] = {lo[c], lo[c + 8], lds[row_pad<TH>(tid, c)], lds[row_pad<TH>(tid, c + 8)]};
            inv_quad_last2(x, tw, q, s0, s0s, s1, s1s);
#pragma unroll
            for (int k = 0; k < 4; ++k) store((k >> 1) * NH + tid + (c + 8 * (k & 1)) * TH, csub(x[k], q));
        }
    }
}

// ============================================================================ plain NTT
template <int LOGN>
__global__ void __launch_bounds__(ntt_threads<LOGN>()) k_ntt_fwd(DevTables T, u64* data, int limbs, int l_split,
                                                                 size_t poly_stride) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN>()];
    const int b = blockIdx.x;
    const int pi = limb_prime(b, l_split, T.L0);
    const RedU R = redu(PK(T, pi));
    u64* p = data + blockIdx.y * poly_stride + (size_t)b * N;
    fwd_limb<LOGN, FHS_NTT_RL>(lds, threadIdx.x, T.tw_fwd + (size_t)pi * N * 2, R, [&](int e) { return p[e]; },
                               [&](int e, u64 v) { p[e] = v; });
}

template <int LOGN>
__global__ void __launch_bounds__(ntt_threads<LOGN>()) k_ntt_inv(DevTables T, u64* data, int limbs, int l_split,
                                                                 size_t poly_stride) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN>()];
    const int b = blockIdx.x;
    const int pi = limb_prime(b, l_split, T.L0);
    const PrimeK& P = PK(T, pi);
    u64* p = data + blockIdx.y * poly_stride + (size_t)b * N;
    inv_limb<LOGN, FHS_NTT_RL>(lds, threadIdx.x, T.tw_inv + (size_t)pi * N * 2, P.q, P.ninv, P.ninv_s, P.w1ninv,
                               P.w1ninv_s, [&](int e) { return p[e]; }, [&](int e, u64 v) { p[e] = v; });
}

hipError_t launch_ntt_fwd(const DevTables& T, u64* data, int limbs, int l_split, int npoly, size_t poly_stride,
                          hipStream_t st) {
    if (limbs <= 0 || npoly <= 0) return hipSuccess;
    FHS_DISPATCH_LOGN(T.logN, {
        hipLaunchKernelGGL((k_ntt_fwd<LOGN>), dim3(limbs, npoly), dim3(ntt_threads<LOGN>()), 0, st, T,
                           data, limbs, l_split, poly_stride);
    });
    return hipGetLastError();
}
hipError_t launch_ntt_inv(const DevTables& T, u64* data, int limbs, int l_split, int npoly, size_t poly_stride,
                          hipStream_t st) {
    if (limbs <= 0 || npoly <= 0) return hipSuccess;
    FHS_DISPATCH_LOGN(T.logN, {
        hipLaunchKernelGGL((k_ntt_inv<LOGN>), dim3(limbs, npoly), dim3(ntt_threads<LOGN>()), 0, st, T,
                           data, limbs, l_split, poly_stride);
    });
    return hipGetLastError();
}

// ============================================================================ element-wise
// a: ncomp x l x N (component stride a_cs); b: component stride b_cs (0 = plaintext broadcast)
__global__ void k_eltwise(DevTables T, int op, const u64* __restrict__ a, const u64* __restrict__ b,
                          u64* __restrict__ out, int ncomp, int l, size_t a_cs, size_t b_cs) {
    const int N = T.N;
    const size_t half = (size_t)N / 2;
    const size_t total = (size_t)ncomp * l * half;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        const size_t n2 = idx % half;
        const size_t li = idx / half;
        const int i = (int)(li % l), comp = (int)(li / l);
        const PrimeK& P = PK(T, i);
        const u64 q = P.q;
        const size_t off = (size_t)i * N + 2 * n2;
        const ulonglong2 av = *reinterpret_cast<const ulonglong2*>(a + comp * a_cs + off);
        ulonglong2 bv = make_ulonglong2(0, 0);
        if (op != OP_NEG) bv = *reinterpret_cast<const ulonglong2*>(b + comp * b_cs + off);
        u64 r0, r1;
        switch (op) {
            case OP_ADD: r0 = addmod(av.x, bv.x, q); r1 = addmod(av.y, bv.y, q); break;
            case OP_SUB: r0 = submod(av.x, bv.x, q); r1 = submod(av.y, bv.y, q); break;
            case OP_SUBNEG: r0 = submod(bv.x, av.x, q); r1 = submod(bv.y, av.y, q); break;
            case OP_NEG: r0 = av.x ? q - av.x : 0; r1 = av.y ? q - av.y : 0; break;
            case OP_MULP: r0 = mulmod(av.x, bv.x, P); r1 = mulmod(av.y, bv.y, P); break;
            case OP_ADDP:
                if (comp == 0) { r0 = addmod(av.x, bv.x, q); r1 = addmod(av.y, bv.y, q); }
                else { r0 = av.x; r1 = av.y; }
                break;
            case OP_SUBP:
                if (comp == 0) { r0 = submod(av.x, bv.x, q); r1 = submod(av.y, bv.y, q); }
                else { r0 = av.x; r1 = av.y; }
                break;
            default: r0 = r1 = 0;
        }
        *reinterpret_cast<ulonglong2*>(out + (size_t)comp * l * N + off) = make_ulonglong2(r0, r1);
    }
}

static inline int eltwise_grid(size_t work) {
    size_t g = (work + 255) / 256;
    if (g > 8192) g = 8192;
    return (int)(g ? g : 1);
}

hipError_t launch_eltwise(const DevTables& T, int op, const u64* a, const u64* b, u64* out, int ncomp, int l,
                          size_t a_cs, size_t b_cs, hipStream_t st) {
    const size_t work = (size_t)ncomp * l * T.N / 2;
    hipLaunchKernelGGL(k_eltwise, dim3(eltwise_grid(work)), dim3(256), 0, st, T, op, a, b, out, ncomp, l, a_cs, b_cs);
    return hipGetLastError();
}

// (a0 b0, a0 b1 + a1 b0, a1 b1)  -- pb:177 multiply
__global__ void k_tensor(DevTables T, const u64* __restrict__ a, const u64* __restrict__ b, u64* __restrict__ out,
                         int l) {
    const int N = T.N;
    const size_t S = (size_t)l * N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(idx / N);
        const PrimeK& P = PK(T, i);
        const u64 a0 = a[idx], a1 = a[S + idx], b0 = b[idx], b1 = b[S + idx];
        out[idx] = mulmod(a0, b0, P);
        u128 m = {0, 0};
        mac128(m, a0, b1);
        mac128(m, a1, b0);
        out[S + idx] = reduce128(m.lo, m.hi, P);
        out[2 * S + idx] = mulmod(a1, b1, P);
    }
}
hipError_t launch_tensor(const DevTables& T, const u64* a, const u64* b, u64* out3, int l, hipStream_t st) {
    hipLaunchKernelGGL(k_tensor, dim3(eltwise_grid((size_t)l * T.N)), dim3(256), 0, st, T, a, b, out3, l);
    return hipGetLastError();
}

// product of two K-limb polynomials (key material: s^2)
__global__ void k_key_prod(DevTables T, const u64* a, const u64* b, u64* out, int limbs) {
    const size_t S = (size_t)limbs * T.N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const PrimeK& P = PK(T, (int)(idx / T.N));
        out[idx] = mulmod(a[idx], b[idx], P);
    }
}
hipError_t launch_key_prod(const DevTables& T, const u64* a, const u64* b, u64* out, int limbs, hipStream_t st) {
    hipLaunchKernelGGL(k_key_prod, dim3(eltwise_grid((size_t)limbs * T.N)), dim3(256), 0, st, T, a, b, out, limbs);
    return hipGetLastError();
}

__global__ void k_galois_perm(DevTables T, const u64* in, u64* out, int limbs, u64 elt) {
    const size_t S = (size_t)limbs * T.N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const size_t base = idx - idx % T.N;
        out[idx] = in[base + galois_src((int)(idx % T.N), elt, T.logN)];
    }
}
hipError_t launch_galois_perm(const DevTables& T, const u64* in, u64* out, int limbs, u64 elt, hipStream_t st) {
    hipLaunchKernelGGL(k_galois_perm, dim3(eltwise_grid((size_t)limbs * T.N)), dim3(256), 0, st, T, in, out, limbs,
                       elt);
    return hipGetLastError();
}

// ============================================================================ rescale (pb:185)
// 1) last limb of each component -> coefficient form (scratch[comp])
template <int LOGN, bool H = ntt_half<LOGN>()>
__global__ void __launch_bounds__((ntt_threads<LOGN, H>())) k_rescale_intt(DevTables T, const u64* in, u64* scratch, int l) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN, H>()];
    const int comp = blockIdx.x, pi = l - 1;
    const PrimeK& P = PK(T, pi);
    const u64* src = in + ((size_t)comp * l + pi) * N;
    u64* dst = scratch + (size_t)comp * N;
    const u64 half = P.q >> 1, q = P.q;
    inv_limb<LOGN, FHS_NTT_RL, H>(lds, threadIdx.x, T.tw_inv + (size_t)pi * N * 2, q, P.ninv, P.ninv_s, P.w1ninv,
                               P.w1ninv_s, [&](int e) { return src[e]; },
                               [&](int e, u64 v) { dst[e] = addmod(v, half, q); });
}
// 2) per (i < l-1, comp): NTT_i([v mod q_i] - [half mod q_i]) and combine (a_i - t) * q_last^-1
template <int LOGN, bool H = ntt_half<LOGN>()>
__global__ void __launch_bounds__((ntt_threads<LOGN, H>())) k_rescale_ntt(DevTables T, const u64* in, const u64* scratch,
                                                                     u64* out, int l) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN, H>()];
    const int i = blockIdx.x, comp = blockIdx.y;
    const PrimeK& P = PK(T, i);
    const RedU RU = redu(P);
    const u64* rs = T.rescale + ((size_t)l * T.L0 + i) * 4;   // inv, inv_s, half mod q_i
    const u64 inv = rs[0], inv_s = rs[1], hq = rs[2], q = RU.q;
    const u64* src = scratch + (size_t)comp * N;
    const u64* a = in + ((size_t)comp * l + i) * N;
    u64* o = out + ((size_t)comp * (l - 1) + i) * N;
    fwd_limb<LOGN, FHS_NTT_RL, H>(lds, threadIdx.x, T.tw_fwd + (size_t)i * N * 2, RU,
                               [&](int e) { return submod(reduce64(src[e], P), hq, q); },
                               [&](int e, u64 t) { o[e] = shoup(submod(a[e], t, q), inv, inv_s, q); });
}
// N = 32768: a rescale is two latency-bound launches (2 and 2 (l - 1) workgroups, each transforming a whole limb as
// two halves in turn).  Here every half gets its own workgroup -- twice the workgroups, half the serial work each:
// (a) k_rescale_intt_hs: the last limb's INTT up to its final two stages, per half (inv_limb's iteration h), the
//     thread's 16 rows to `pre` ([comp][half][row][thread]: the scratch's 2 N words);
// (b) k_rescale_ntt_hs, per (target limb, comp, half): for the thread's column the INTT's last two stages
//     (inv_quad_last2, as inv_limb), k_rescale_intt's + floor(q_last/2) and k_rescale_ntt's conversion, the forward
//     NTT's first three stages (fwd_oct_first3, as fwd_limb: its row groups c, c+4, c+8, c+12 are the INTT quads c and
//     c+4), then only this half's LDS passes and stores.  The same operations on the same values: identical limbs.
template <int LOGN>
__global__ void __launch_bounds__((ntt_threads<LOGN, true>())) k_rescale_intt_hs(DevTables T, const u64* in, u64* pre,
                                                                             int l) {
    constexpr int N = 1 << LOGN, TH = N / 32;
    static_assert(!(FHS_NTT_WAVELOCAL && (LOGN - 2) % 3 == 0), "plain half loads (inv_limb's non-wave-local head)");
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN, true>()];
    const int h = blockIdx.x, comp = blockIdx.y, pi = l - 1, tid = threadIdx.x;
    const PrimeK& P = PK(T, pi);
    const u64* src = in + ((size_t)comp * l + pi) * N + (size_t)h * (N / 2);
#pragma unroll
    for (int c = 0; c < 16; ++c) lds[row_pad<TH>(tid, c)] = src[tid + c * TH];
    __syncthreads();
    ntt_inv_half_lds<LOGN - 1, 3, 16, 1, false>(lds, tid, T.tw_inv + (size_t)pi * N * 2, P.q, 1 + h);
    u64* o = pre + ((size_t)comp * 2 + h) * 16 * TH + tid;
#pragma unroll
    for (int c = 0; c < 16; ++c) o[(size_t)c * TH] = lds[row_pad<TH>(tid, c)];
}
template <int LOGN>
__global__ void __launch_bounds__((ntt_threads<LOGN, true>())) k_rescale_ntt_hs(DevTables T, const u64* in, const u64* pre,
                                                                            u64* out, int l) {
    static_assert(FHS_FWD_FIRST3 && fwd_first3<LOGN>(), "the column's forward first stages in radix-8 groups");
    constexpr int N = 1 << LOGN, NH = N / 2, TH = N / 32;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN, true>()];
    const int i = blockIdx.x, comp = blockIdx.y, g = blockIdx.z, tid = threadIdx.x;
    const PrimeK& P = PK(T, i);
    const RedU RU = redu(P);
    const u64* rs = T.rescale + ((size_t)l * T.L0 + i) * 4;   // inv, inv_s, half mod q_i
    const u64 inv = rs[0], inv_s = rs[1], hq = rs[2], q = RU.q;
    const PrimeK& PL = PK(T, l - 1);
    const u64 qL = PL.q, halfL = qL >> 1;
    const u64* twL = T.tw_inv + (size_t)(l - 1) * N * 2;
    const u64* tw = T.tw_fwd + (size_t)i * N * 2;
    const u64* pr = pre + (size_t)comp * 2 * 16 * TH + tid;
    auto conv = [&](u64 y) { return submod(reduce64(addmod(csub(y, qL), halfL, qL), P), hq, q); };
    u64 hi[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        u64 x[8];   // x[m] = half 0 row c + 4m, x[4 + m] = half 1 row c + 4m (fwd_limb's F3 loads)
#pragma unroll
        for (int j = 0; j < 2; ++j) {   // INTT quad r = c + 4j: rows r, r + 8 of both halves
            const int r = c + 4 * j;
            u64 y[4] = {pr[(size_t)r * TH], pr[(size_t)(r + 8) * TH], pr[(size_t)(16 + r) * TH], pr[(size_t)(24 + r) * TH]};
            inv_quad_last2(y, twL, qL, PL.ninv, PL.ninv_s, PL.w1ninv, PL.w1ninv_s);
            x[j] = conv(y[0]);
            x[j + 2] = conv(y[1]);
            x[4 + j] = conv(y[2]);
            x[6 + j] = conv(y[3]);
        }
        fwd_oct_first3<TH>(x, tw, q, RU.lazy, lds, tid, c, hi);
    }
    if (g) {   // the upper half's rows from registers (each thread overwrites only its own rows)
#pragma unroll
        for (int c = 0; c < 16; ++c) lds[row_pad<TH>(tid, c)] = hi[c];
    }
    __syncthreads();
    const u64* a = in + ((size_t)comp * l + i) * N;
    u64* o = out + ((size_t)comp * (l - 1) + i) * N;
    constexpr bool WLX = FHS_NTT_WAVELOCAL && fwd_exit_wave_local<LOGN - 1, 3, 2>();
    ntt_fwd_lds<LOGN - 1, 3, 16, 2, WLX>(lds, tid, tw, q, RU.lazy, 1 + g);
    if constexpr (WLX) {
        const int wb = wl_base<LOGN - 1, 16, 8>(tid), wp = lds_pad(wb);
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            const int off = wl_off<LOGN - 1, 16, 8>(c);
            const int e = g * NH + wb + off;
            o[e] = shoup(submod(a[e], fwd_canon(lds[wp + off + off / 16], RU), q), inv, inv_s, q);
        }
    } else {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            const int e = g * NH + tid + c * TH;
            o[e] = shoup(submod(a[e], fwd_canon(lds[row_pad<TH>(tid, c)], RU), q), inv, inv_s, q);
        }
    }
}
#ifndef FHS_SPLIT_MAX_WG
#define FHS_SPLIT_MAX_WG 256   // below this many workgroups a launch is latency-bound: one workgroup per half-limb
#endif
#ifndef FHS_RESCALE_SPLIT
#define FHS_RESCALE_SPLIT 1   // 0: the one-workgroup-per-limb rescale at N = 32768 too (A/B and test knob)
#endif
hipError_t launch_rescale(const DevTables& T, const u64* in, u64* out, u64* scratch, int ncomp, int l,
                          hipStream_t st, const KTimer* tm) {
    FHS_TMARK(tm, KID_RESCALE, 1, st);
    static const bool split_off = getenv("FHESPEAR_RESCALE_UNSPLIT") != nullptr;
    FHS_DISPATCH_LOGN(T.logN, {
        if constexpr (LOGN == 15 && FHS_RESCALE_SPLIT) {
            if (!split_off && ncomp <= 2) {
                hipLaunchKernelGGL((k_rescale_intt_hs<LOGN>), dim3(2, ncomp), dim3(ntt_threads<LOGN, true>()), 0, st, T,
                                   in, scratch, l);
                hipLaunchKernelGGL((k_rescale_ntt_hs<LOGN>), dim3(l - 1, ncomp, 2), dim3(ntt_threads<LOGN, true>()), 0, st,
                                   T, in, scratch, out, l);
                break;
            }
        }
        FHS_NTT_LAUNCH(k_rescale_intt, ncomp, dim3(ncomp), st, T, in, scratch, l);
        FHS_NTT_LAUNCH(k_rescale_ntt, (l - 1) * ncomp, dim3(l - 1, ncomp), st, T, in, scratch, out, l);
    });
    FHS_TMARK(tm, KID_RESCALE, 0, st);
    return hipGetLastError();
}

// ============================================================================ key-switch
// (a) y = INTT(a) * inv_hat(digit) per data limb of every distinct input (inv_hat folded into
// the N^-1 stage).  No automorphism here: it is applied after the (hoisted) ModUp.
template <int LOGN>
__global__ void __launch_bounds__((1 << LOGN) / 16) k_ks_intt(DevTables T, const u64* const* uniq, u64* acoef, int l, int U) {
    constexpr int N = 1 << LOGN, TH = N / 16;
    __shared__ __attribute__((aligned(16))) u64 lds[LOGN > 14 ? 1 : (1 << LOGN) + (1 << LOGN) / 16];
    if constexpr (LOGN <= 14) {   // full-limb form: N <= 16384 only (small launches, ks_intt_half())
    const int tid = threadIdx.x;
    int i, u;
    if (!plain_tm(l, U, i, u)) return;
    const PrimeK& P = PK(T, i);
    const u64* src = uniq[u] + (size_t)i * N;
#pragma unroll
    for (int c = 0; c < 16; ++c) lds[row_pad<TH>(tid, c)] = src[tid + c * TH];
    __syncthreads();
    const u64* cst = T.modup_intt + ((size_t)l * T.L0 + i) * 4;
    ntt_inv_lds<LOGN, FHS_NTT_RL>(lds, tid, T.tw_inv + (size_t)i * N * 2, P.q, cst[0], cst[1], cst[2], cst[3]);
    u64* dst = acoef + ((size_t)u * l + i) * N;
#pragma unroll
    for (int k = 0; k < 16; ++k) dst[tid + k * TH] = csub(lds[row_pad<TH>(tid, k)], P.q);
    }
}

// k_ks_intt with half the limb in LDS (two workgroups per CU, co-resident with the half-limb ModUp
// and the Hadamard): each half runs every inverse stage but the last two, which are done in registers
// as a radix-4 (rows c, c + 8 of both halves: the halves' (e, e + N/4) stage, then the global (e, e + N/2)
// one with the N^-1 and ModUp scaling folded in) -- four radix-8 LDS passes per half, no radix-2 pass.
// Same values.
template <int LOGN>
__global__ void __launch_bounds__((1 << LOGN) / 32, 4) k_ks_intt_h(DevTables T, const u64* const* uniq, u64* acoef,
                                                                   int l, int U) {
    constexpr int N = 1 << LOGN, NH = N / 2, TH = N / 32;
    __shared__ __attribute__((aligned(16))) u64 lds[(1 << (LOGN - 1)) + (1 << (LOGN - 1)) / 16];
    const int tid = threadIdx.x;
    int i, u;
    if (!plain_tm(l, U, i, u)) return;
    const PrimeK& P = PK(T, i);
    const u64 q = P.q;
    // buffer loads / stores: per-lane offset tid in voffset, the half / row offsets in soffset
    const __amdgpu_buffer_rsrc_t rs = brsrc(uniq[u] + (size_t)i * N, N * 8);
    const u64* tw = T.tw_inv + (size_t)i * N * 2;
    u64 lo[16];
    // wave-local head (fhs_ntt.h inv_from): each wave loads the blocks its deep passes transform, so no barrier
    // before them and none between them
    constexpr bool WLI = FHS_NTT_WAVELOCAL && (LOGN - 2) % FHS_NTT_RL == 0;
    constexpr int GS = 1 << FHS_NTT_RL;
    const int tb = WLI ? wl_base<LOGN - 1, 16, GS>(tid) : tid;
    auto eoff = [&](int c) { return WLI ? wl_off<LOGN - 1, 16, GS>(c) : c * TH; };
    auto lidx = [&](int c) { return WLI ? lds_pad(tb) + eoff(c) + eoff(c) / 16 : row_pad<TH>(tid, c); };
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
        if (h) __syncthreads();
        u64 v[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) v[c] = bload64(rs, tb * 8, (h * NH + eoff(c)) * 8);
#pragma unroll
        for (int c = 0; c < 16; ++c) lds[lidx(c)] = v[c];
        if constexpr (!WLI) __syncthreads();
        // every stage of the half but its local stage 0 (rows c, c + 8: done below in registers)
        ntt_inv_half_lds<LOGN - 1, FHS_NTT_RL, 16, 1, WLI>(lds, tid, tw, q, 1 + h);
        if (h == 0) {
#pragma unroll
            for (int c = 0; c < 16; ++c) lo[c] = lds[row_pad<TH>(tid, c)];
        }
    }
    const u64* cst = T.modup_intt + ((size_t)l * T.L0 + i) * 4;
    const u64 s0 = cst[0], s0s = cst[1], s1 = cst[2], s1s = cst[3];
    const __amdgpu_buffer_rsrc_t rd = brsrc(acoef + ((size_t)u * l + i) * N, N * 8);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        u64 x[4] = {lo[c], lo[c + 8], lds[row_pad<TH>(tid, c)], lds[row_pad<TH>(tid, c + 8)]};
        inv_quad_last2(x, tw, q, s0, s0s, s1, s1s);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            bstore64(csub(x[k], q), rd, tid * 8, ((k >> 1) * NH + (c + 8 * (k & 1)) * TH) * 8);
    }
}

// k_ks_intt_h (half limb, two workgroups per CU) unless the launch has fewer workgroups than CUs
// (e.g. the baby-step input alone, l workgroups): then the full-limb k_ks_intt halves the latency.
template <int LOGN>
static bool ks_intt_half(int nwg) {
    if (LOGN <= 14 && nwg < FHS_FULL_FORM_MAX_WG) return false;
    return (FHS_INTT_HALF && LOGN >= 9) || ntt_half<LOGN>();
}

// Exact centred-extension count, slow path (|frac - 1/2| < 2^-58; never seen on random data
// but required for exactness): v = carry + [2X >= (2 carry + 1) Q_S], X = sum_u y_u Q_S/q_u.
__device__ __noinline__ int centered_exact(const u64* y, const u64* qs, int ns, int carry) {
    u64 X[10], Q[10], t[10];
    for (int w = 0; w < 10; ++w) { X[w] = 0; Q[w] = 0; }
    Q[0] = 1;
    for (int u = 0; u < ns; ++u) {
        u64 cy = 0;
        for (int w = 0; w < 10; ++w) {
            const u64 lo = Q[w] * qs[u], hi = __umul64hi(Q[w], qs[u]);
            const u64 z = lo + cy;
            cy = hi + (z < lo);
            Q[w] = z;
        }
    }
    for (int u = 0; u < ns; ++u) {
        for (int w = 0; w < 10; ++w) t[w] = 0;
        t[0] = y[u];
        for (int v = 0; v < ns; ++v) {
            if (v == u) continue;
            u64 cy = 0;
            for (int w = 0; w < 10; ++w) {
                const u64 lo = t[w] * qs[v], hi = __umul64hi(t[w], qs[v]);
                const u64 z = lo + cy;
                cy = hi + (z < lo);
                t[w] = z;
            }
        }
        u64 cy = 0;
        for (int w = 0; w < 10; ++w) {
            const u64 z1 = X[w] + t[w];
            const u64 c1 = z1 < X[w];
            const u64 z2 = z1 + cy;
            cy = c1 + (z2 < z1);
            X[w] = z2;
        }
    }
    // compare 2X with (2 carry + 1) Q from the top word down
    const u64 mlt = (u64)(2 * carry + 1);
    u64 L[10], Rr[10], cl = 0, cr = 0;
    for (int w = 0; w < 10; ++w) {
        L[w] = (X[w] << 1) | cl;
        cl = X[w] >> 63;
        const u64 lo = Q[w] * mlt, hi = __umul64hi(Q[w], mlt);
        const u64 z = lo + cr;
        cr = hi + (z < lo);
        Rr[w] = z;
    }
    for (int w = 9; w >= 0; --w)
        if (L[w] != Rr[w]) return carry + (L[w] > Rr[w] ? 1 : 0);
    return carry + 1;
}

// (a2) v[u][j][n] = round(sum_{u in digit j} y_u / q_u): fixed-point fast path (error < 2 ns ulp
// of 2^-64), exact fallback within 64 ulp of a half (oracle: ock_centered_count).
__global__ void k_centered(DevTables T, const u64* acoef, unsigned char* vout, int l, int U, unsigned* zflag) {
    // grid (N / 256, U dn): the (input, digit) pair is per workgroup, so no 64-bit index division
    const int N = T.N, P_ = T.P, dn = (l + P_ - 1) / P_;
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y % dn, u = blockIdx.y / dn;
    if (n >= N || u >= U) return;
    const size_t idx = ((size_t)u * dn + j) * N + n;
    {
        const int s0 = j * P_, ns = min(s0 + P_, l) - s0;
        const u64* yb = acoef + ((size_t)u * l + s0) * N + n;
        int v;
        if (ns == 1) {   // SEAL: the limb's residue in [0, q) is lifted as is
            const u64 y0 = yb[0];
            v = T.ks_seal ? 0 : (y0 > (PK(T, s0).q >> 1) ? 1 : 0);
            if (zflag && y0 == 0) atomicOr(zflag, 1u);   // hoisted SEAL rotations: SealHoist
        } else {
            // fixed-point fast path in registers (a guarded unrolled loop: no private arrays, so no
            // scratch traffic); the exact path re-reads the digit into its own arrays
            const u64* R = T.modup_R + (((size_t)l * T.dnum + j) * P_) * 2;
            constexpr int PMAX = 8;   // digit size P (context_create limit)
            u64 y[PMAX];
#pragma unroll
            for (int k = 0; k < PMAX; ++k) y[k] = k < ns ? yb[(size_t)k * N] : 0;
            u64 lo = 0;
            int carry = 0;
#pragma unroll
            for (int k = 0; k < PMAX; ++k) {
                if (k < ns) {
                    const u64 F = y[k] * R[2 * k + 1] + __umul64hi(y[k], R[2 * k]);
                    lo += F;
                    carry += lo < F;
                }
            }
            const u64 half = 1ULL << 63;
            const u64 d = lo >= half ? lo - half : half - lo;
            if (d > 64) {
                v = carry + (lo >= half ? 1 : 0);
            } else {
                u64 ys[PMAX], qs[PMAX];
                for (int k = 0; k < ns; ++k) {
                    ys[k] = yb[(size_t)k * N];
                    qs[k] = PK(T, s0 + k).q;
                }
                v = centered_exact(ys, qs, ns, carry);
            }
        }
        vout[idx] = (unsigned char)v;
    }
}
// (a2') X form of the centred extension (full 3-limb digits, modup_xform): the exact centred digit value
// X = S - v Q_S, S = sum_u y_u Q_S/q_u, v = round(S / Q_S) (|X| < Q_S/2; S/Q_S is never a half: Q_S is
// odd), computed once per coefficient and digit instead of once per target limb, and stored in place of
// the digit's three residues as U = X + 2^179 in base-2^60 words V0, V1, V2, each split-30 packed.
// modup_convert3x reduces V0 + V1 (2^60 mod m) + V2 (2^120 mod m) - 2^179 mod m = X mod m: the same
// residue the count form gives (it is the same integer), with two split-30 products per target instead
// of three plus the count term, and no count bytes.
__global__ void k_centered_x(DevTables T, u64* acoef, int l, int U) {
    const int N = T.N, dn = l / 3;
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y % dn, u = blockIdx.y / dn;
    if (n >= N || u >= U) return;
    u64* yb = acoef + ((size_t)u * l + 3 * j) * N + n;
    const u64 y[3] = {yb[0], yb[N], yb[2 * (size_t)N]};
    u64 w[3];
    centered_x_pack(y, T.modup_xd + (size_t)j * 32, w);
    yb[0] = w[0];
    yb[N] = w[1];
    yb[2 * (size_t)N] = w[2];
}

static void launch_centered(const DevTables& T, u64* acoef, unsigned char* vout, int l, int U, hipStream_t st,
                            unsigned* zflag = nullptr) {
    const int dn = (l + T.P - 1) / T.P;
    if (modup_xform(T, l))
        hipLaunchKernelGGL(k_centered_x, dim3((T.N + 255) / 256, U * dn), dim3(256), 0, st, T, acoef, l, U);
    else
        hipLaunchKernelGGL(k_centered, dim3((T.N + 255) / 256, U * dn), dim3(256), 0, st, T, acoef, vout, l, U, zflag);
}

// (b1) ModUp + NTT: ext[u][j][t] = NTT_t(centred conv_{digit j -> t}(y_u)) for t outside digit
// j, and a copy of the input limb t for t inside digit j.
template <int LOGN>
__global__ void __launch_bounds__((1 << LOGN) / 16) k_modup(DevTables T, const u64* const* uniq, const u64* acoef,
                                                            const unsigned char* vcnt, u64* ext, int l, int U) {
    constexpr int N = 1 << LOGN, TH = N / 16;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_half<LOGN>() ? 1 : (1 << LOGN) + (1 << LOGN) / 16];
    if constexpr (!ntt_half<LOGN>()) {   // full-limb form: N <= 16384 only
    const int tid = threadIdx.x;
    const int P_ = T.P, K = T.K, E = l + P_, dn = (l + P_ - 1) / P_;
    int t, mi;
    if (!xcd_tinner(E, dn * U, t, mi)) return;
    const int j = mi % dn, u = mi / dn;
    const int s0 = j * P_, s1 = min(s0 + P_, l), ns = s1 - s0;
    u64* o = ext + (((size_t)u * dn + j) * E + t) * N;
    if (t >= s0 && t < s1) return;   // own limb: k_ks_ip reads it from the input itself
    const int pt = t < l ? t : T.L0 + (t - l);
    const PrimeK& PM = PK(T, pt);
    const u64 m = PM.q;
    const u64* yb = acoef + ((size_t)u * l + s0) * N;
    const u64* hat = T.modup_hat + (((size_t)l * T.dnum + j) * P_) * K + pt;
    const u64* qv = T.modup_Q + (((size_t)l * T.dnum + j) * K + pt) * 2;
    const u64 Qm = qv[0], nsQm = qv[1];
    const unsigned char* vb = vcnt + ((size_t)u * dn + j) * N;
    const RedU R = redu(PM);
    constexpr int CH = FHS_MODUP_CH;
    // CH outputs per thread at a time; the digit's ns input limbs stream through a runtime loop so
    // the CH loads of one limb are issued together (no per-element guards between loads).
#pragma unroll 1
    for (int half = 0; half < 16 / CH; ++half) {
        u128 acc[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) acc[k] = u128{0, 0};
        Acc3 a3[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) a3[k] = Acc3{0, 0, 0};
#pragma unroll 1
        for (int w = 0; w < ns; ++w) {   // ns <= 8 products per Acc3
            const Split30 hw = split30(hat[(size_t)w * K]);
            const u64* yw = yb + (size_t)w * N + half * CH * TH + tid;
            u64 y[CH];
#pragma unroll
            for (int k = 0; k < CH; ++k) y[k] = yw[k * TH];
#pragma unroll
            for (int k = 0; k < CH; ++k) acc3_mac(a3[k], split30(y[k]), hw);
        }
#pragma unroll
        for (int k = 0; k < CH; ++k) acc3_fold(acc[k], a3[k]);
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int e = tid + (half * CH + k) * TH;
            mac128(acc[k], (u64)(ns - vb[e]), Qm);   // + (ns - v) Q_S, then - ns Q_S below
            lds[lds_pad(e)] = submod(reduce128(acc[k].lo, acc[k].hi, R), nsQm, m);
        }
    }
    __syncthreads();
    ntt_fwd_lds<LOGN, FHS_MODUP_RL>(lds, tid, T.tw_fwd + (size_t)pt * N * 2, m, R.lazy);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const int e = tid + c * TH;
        o[e] = fwd_canon(lds[row_pad<TH>(tid, c)], R);
    }
    }
}

// ModUp conversion of a full 3-limb digit from its X form (k_centered_x) into target limb `m`
// (pseudo-Mersenne fold, PrimeK.pm bit 40), radix-4 first stages (fwd_quad_first2), buffer loads:
// x = V0 + V1 e1 + V2 e2 + c3 (e1 = 2^60, e2 = 2^120, c3 = -2^179 mod m) as split-30 sums (each within
// the 3-product bounds conv_pm_ok proves for this prime), folded by acc3_reduce_pm to [0, 2m).
template <int LOGN, bool B59>
__device__ __forceinline__ void modup_convert3x(const u64* yb, const u64* xt, const RedU& R, const u64* tw, int tid,
                                                u64* lds, u64 hi[16]) {
    constexpr int N = 1 << LOGN, NH = N / 2, TH = N / 32, CH = FHS_MODUPH_CH;
    const __amdgpu_buffer_rsrc_t ry = brsrc(yb, 3 * N * 8);
    const uint32_t e1 = (uint32_t)xt[0];
    const Split30 e2 = unpack30(xt[1]);
    const u64 c3 = xt[2], m = R.q, q2 = 2 * m;
    const int vo = tid * 8;
    const Tw4 w4 = ld_tw4(tw);
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {
        u64 V[3][4];   // k: rows ch (k = 0, 2) and ch + 8 (k = 1, 3), lower (k < 2) / upper half
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = (ch + 8 * (k & 1)) * TH + (k >= 2 ? NH : 0);   // coefficient index minus tid
#pragma unroll
            for (int w = 0; w < 3; ++w) V[w][k] = bload64(ry, vo, (w * N + e) * 8);
        }
        u64 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)   // B59: the upper half (k >= 2) is multiplied by the stage-0 twiddle first,
                                      // so any congruent 64-bit value will do (no final fold)
            x[k] = B59 ? convert3x_b59(V[0][k], V[1][k], V[2][k], e1, e2, c3, R.d, k < 2)
                       : convert3x_value(V[0][k], V[1][k], V[2][k], e1, e2, c3, R.b, R.d);
        fwd_quad_first2<TH>(x, w4, m, lazy_of<LOGN, B59>(R), lds, tid, ch, hi);
    }
}

// ModUp of a one-limb digit (P = 1: SEAL's convention, fhe_rwkv_inference's ring): Q_S = q_u, so the
// hat factor is 1 and the conversion is y - v q_u mod m = y + v (m - q_u mod m): below q_u + m <= 4 m
// when q_u <= 3 m (the caller checks), inside the forward NTT's input bound, so no product and no
// reduction.
template <int LOGN>
__device__ __forceinline__ void modup_convert1(const u64* yb, const unsigned char* vb, u64 negQ, u64 m, u64 w0,
                                               u64 w0p, int tid, u64* lds, u64 hi[16]) {
    constexpr int N = 1 << LOGN, NH = N / 2, TH = N / 32;
    const __amdgpu_buffer_rsrc_t ry = brsrc(yb, N * 8), rv = brsrc(vb, N);
    const u64 q2 = 2 * m;
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
        u64 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = (ch * 4 + (k & 3)) * TH + (k >= 4 ? NH : 0);
            const u64 y = bload64(ry, tid * 8, e * 8);
            const uint32_t v = __builtin_amdgcn_raw_buffer_load_b8(rv, tid, e, 0);
            x[k] = y + (v ? negQ : 0);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // global stage 0: (e, e + N/2), twiddle psi^rev(1)
            const u64 tt = shoup_lazy(x[4 + k], w0, w0p, m);
            lds[row_pad<TH>(tid, ch * 4 + k)] = x[k] + tt;
            hi[ch * 4 + k] = x[k] + (q2 - tt);
        }
    }
}

// The same with global stages 0 and 1 as a register radix-4 (fwd_quad_first2), so the half transforms start at
// their local stage 1 (four radix-8 passes, no radix-2 pass, wave-local tail): B59 chains only, where every
// prime is within 2^27 of 2^59, so y < q_u < 2 m and y + v negQ < 3 m; one conditional subtraction of 2 m
// gives fwd_quad_first2's input bound (< 2 m) for the lazy and the Harvey form alike.  SEAL's convention (P = 1).
template <int LOGN>
__device__ __forceinline__ void modup_convert1_r4(const u64* yb, const unsigned char* vb, u64 negQ, u64 m,
                                                  bool lazy, const u64* tw, int tid, u64* lds, u64 hi[16]) {
    constexpr int N = 1 << LOGN, NH = N / 2, TH = N / 32;
    const __amdgpu_buffer_rsrc_t ry = brsrc(yb, N * 8), rv = brsrc(vb, N);
    const Tw4 w4 = ld_tw4(tw);
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {
        u64 x[4];   // rows ch (k = 0, 2) and ch + 8 (k = 1, 3) of the lower (k < 2) / upper half
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = (ch + 8 * (k & 1)) * TH + (k >= 2 ? NH : 0);
            const u64 y = bload64(ry, tid * 8, e * 8);
            const uint32_t v = __builtin_amdgcn_raw_buffer_load_b8(rv, tid, e, 0);
            const u64 t = y + (v ? negQ : 0);
            x[k] = t >= 2 * m ? t - 2 * m : t;
        }
        fwd_quad_first2<TH>(x, w4, m, lazy, lds, tid, ch, hi);
    }
}

// (b1') ModUp + NTT with half the limb in LDS (68 KiB at N = 16384): two workgroups share a CU,
// so one's loads and base conversion overlap the other's NTT.  Stage 0 of the forward NTT pairs
// coefficient e with e + N/2; each thread converts both, applies that butterfly in registers, keeps
// the upper half in registers while the lower half is transformed in LDS, then transforms it.
// Same values as k_modup (same butterflies, same lazy bounds: < q + 2 q log N).
template <int LOGN>
constexpr int modup_h_lds_words() { return (1 << (LOGN - 1)) + (1 << (LOGN - 1)) / 16; }
// one workgroup's share: target limb t of digit j = mi % dn of input u = mi / dn
// DP: the digit size with a specialised conversion compiled in (3: modup_convert3x, 1: modup_convert1,
// 0: the generic loop only) -- one instantiation per context shape, so the rarely used paths cost the
// usual one no registers
template <int LOGN, int DP, bool B59>
__device__ __forceinline__ void modup_h_body(const DevTables& T, const u64* acoef, const unsigned char* vcnt, u64* ext,
                                             int l, int t, int mi, int tid, u64* lds) {
    constexpr int N = 1 << LOGN, NH = N / 2, TH = N / 32;   // 16 coefficient pairs per thread
    const int P_ = T.P, K = T.K, E = l + P_, dn = (l + P_ - 1) / P_;
    const int j = mi % dn, u = mi / dn;
    const int s0 = j * P_, s1 = min(s0 + P_, l), ns = s1 - s0;
    u64* o = ext + (((size_t)u * dn + j) * E + t) * N;
    if (t >= s0 && t < s1) return;   // own limb: k_ks_ip reads it from the input itself
    const int pt = t < l ? t : T.L0 + (t - l);
    const PrimeK& PM = PK(T, pt);
    const u64 m = PM.q;
    const u64* yb = acoef + ((size_t)u * l + s0) * N;
    const u64* hat = T.modup_hat + (((size_t)l * T.dnum + j) * P_) * K + pt;
    const u64* qv = T.modup_Q + (((size_t)l * T.dnum + j) * K + pt) * 2;
    const u64 Qm = qv[0], nsQm = qv[1], negQ = Qm ? m - Qm : 0;
    const unsigned char* vb = vcnt + ((size_t)u * dn + j) * N;
    const RedU R = redu(PM);
    const u64* tw = T.tw_fwd + (size_t)pt * N * 2;
    u64 w0, w0p;
    ld_tw(tw, 1, w0, w0p);
    const u64 q2 = 2 * m;
    u64 hi[16];
    if constexpr (DP == 3) {   // every digit 3 limbs, every target on the fold (launch_modup checks)
        // the usual digit (P = 3 limbs, pseudo-Mersenne target): compile-time digit size, buffer loads
        // whose limb / chunk offsets are scalar (no per-load address arithmetic on the VALU)
        modup_convert3x<LOGN, B59>(yb, T.modup_xt + (size_t)pt * 4, R, tw, tid, lds, hi);
    } else if (DP == 1 && B59) {   // one-limb digits on a 59-bit chain: radix-4 first stages
        modup_convert1_r4<LOGN>(yb, vb, negQ, m, lazy_of<LOGN, B59>(R), tw, tid, lds, hi);
    } else if (DP == 1 && ns == 1 && PK(T, s0).q <= 3 * m) {   // y + v negQ < q_u + m <= 4 m: the NTT's input bound
        modup_convert1<LOGN>(yb, vb, negQ, m, w0, w0p, tid, lds, hi);
    } else {
    constexpr int CH = FHS_MODUPH_CH;   // coefficient pairs per conversion chunk
#pragma unroll
    for (int ch = 0; ch < 16 / CH; ++ch) {
        Acc3 a3[2 * CH];
#pragma unroll
        for (int k = 0; k < 2 * CH; ++k) a3[k] = Acc3{0, 0, 0};
        // the centred counts of this chunk, loaded together up front (one latency, not one per element)
        uint32_t vv[2 * CH];
#pragma unroll
        for (int k = 0; k < 2 * CH; ++k) vv[k] = vb[tid + (ch * CH + (k % CH)) * TH + (k >= CH ? NH : 0)];
#pragma unroll 1
        for (int w = 0; w < ns; ++w) {   // ns <= 8 products per Acc3
            const Split30 hw = split30(hat[(size_t)w * K]);
            const u64* yw = yb + (size_t)w * N + tid;
            u64 y[2 * CH];
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                y[k] = yw[(ch * CH + k) * TH];
                y[CH + k] = yw[(ch * CH + k) * TH + NH];
            }
#pragma unroll
            for (int k = 0; k < 2 * CH; ++k) acc3_mac(a3[k], split30(y[k]), hw);
        }
        u64 x[2 * CH];
        if (R.cpm) {   // - v Q_S folded into L as v (m - Q_S mod m); result in [0, 2q)
#pragma unroll
            for (int k = 0; k < 2 * CH; ++k) {
                const uint32_t v = vv[k];
                const u64 vq = mul32w(v, (uint32_t)negQ) + ((u64)(v * (uint32_t)(negQ >> 32)) << 32);
                x[k] = acc3_reduce_pm(a3[k].L + vq, a3[k].M, a3[k].H, R.b, R.d);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 2 * CH; ++k) {
                u128 acc = {0, 0};
                acc3_fold(acc, a3[k]);
                mac128(acc, (u64)(ns - vv[k]), Qm);   // + (ns - v) Q_S, then - ns Q_S below
                x[k] = submod(reduce128(acc.lo, acc.hi, R), nsQm, m);
            }
        }
#pragma unroll
        for (int k = 0; k < CH; ++k) {   // global stage 0: (e, e + N/2), twiddle psi^rev(1)
            const int e = tid + (ch * CH + k) * TH;
            const u64 tt = shoup_lazy(x[CH + k], w0, w0p, m);
            lds[row_pad<TH>(tid, ch * CH + k)] = x[k] + tt;
            hi[ch * CH + k] = x[k] + (q2 - tt);
        }
    }
    }
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
        if (h) {   // lower half written out: the upper half moves from registers into LDS
            __syncthreads();
#pragma unroll
            for (int c = 0; c < 16; ++c) lds[row_pad<TH>(tid, c)] = hi[c];
        }
        __syncthreads();
        // the radix-4 conversion (modup_convert3x, FHS_MODUP_R4) did each half's local stage 0 already
        constexpr int S0 = (DP == 3 || (DP == 1 && B59)) ? 1 : 0;
        // wave-local tail: no barriers between the passes with TL <= 64, none before the stores
        constexpr bool WLX = FHS_NTT_WAVELOCAL && fwd_exit_wave_local<LOGN - 1, FHS_MODUPH_RL, S0>();
        ntt_fwd_lds<LOGN - 1, FHS_MODUPH_RL, 16, S0, WLX>(lds, tid, tw, m, lazy_of<LOGN, B59>(R), 1 + h);
        // buffer stores: per-lane offset tid, the half / row offset in soffset.  The extended limbs feed only
        // the key inner products, whose split-30 sums take any value < 2^60: lazy outputs are folded once
        // (pm_fold_lt60), without fwd_canon's final subtraction.  The wave-uniform lazy choice is made once
        // per sweep, outside the unrolled loop, so its 16 LDS reads issue together (a choice per element
        // split the loop into blocks, each waiting for its own read)
        const __amdgpu_buffer_rsrc_t ro = brsrc(o, N * 8);
        if constexpr (WLX) {   // this wave's own outputs (wl_base + wl_off): rows of 64 consecutive elements
            constexpr int GS = 1 << FHS_MODUPH_RL;
            const int wb = wl_base<LOGN - 1, 16, GS>(tid), wp = lds_pad(wb);
            if (lazy_of<LOGN, B59>(R)) {
#pragma unroll
                for (int c = 0; c < 16; ++c) {
                    const int off = wl_off<LOGN - 1, 16, GS>(c);
                    bstore64_aux<FHS_MODUP_STORE_AUX>(pm_fold_lt60(lds[wp + off + off / 16], R), ro, wb * 8,
                                                      (h * NH + off) * 8);
                }
            } else {
#pragma unroll
                for (int c = 0; c < 16; ++c) {
                    const int off = wl_off<LOGN - 1, 16, GS>(c);
                    bstore64_aux<FHS_MODUP_STORE_AUX>(fwd_canon(lds[wp + off + off / 16], R), ro, wb * 8,
                                                      (h * NH + off) * 8);
                }
            }
        } else if (lazy_of<LOGN, B59>(R)) {
#pragma unroll
            for (int c = 0; c < 16; ++c)
                bstore64_aux<FHS_MODUP_STORE_AUX>(pm_fold_lt60(lds[row_pad<TH>(tid, c)], R), ro, tid * 8,
                                                  (h * NH + c * TH) * 8);
        } else {
#pragma unroll
            for (int c = 0; c < 16; ++c)
                bstore64_aux<FHS_MODUP_STORE_AUX>(fwd_canon(lds[row_pad<TH>(tid, c)], R), ro, tid * 8,
                                                  (h * NH + c * TH) * 8);
        }
    }
}
template <int LOGN, int DP, bool B59>
__global__ void __launch_bounds__((1 << LOGN) / 32, 4) k_modup_h(DevTables T, const u64* const* uniq,
                                                                 const u64* acoef, const unsigned char* vcnt, u64* ext,
                                                                 int l, int U) {
    __shared__ __attribute__((aligned(16))) u64 lds[modup_h_lds_words<LOGN>()];
    const int E = l + T.P, dn = (l + T.P - 1) / T.P;
    int t, mi;
    if (!(FHS_MODUP_QUADPAIR ? xcd_quadpair(E, dn * U, t, mi) : xcd_tinner(E, dn * U, t, mi))) return;
    modup_h_body<LOGN, DP, B59>(T, acoef, vcnt, ext, l, t, mi, threadIdx.x, lds);
}

template <int LOGN>
static void launch_modup(const DevTables& T, const u64* const* uniq, const u64* acoef, const unsigned char* vcnt,
                         u64* ext, int l, int U, hipStream_t st) {
    const int E = l + T.P, dn = (l + T.P - 1) / T.P;
    const int mgrid = xcd_grid(E, dn * U);
    const dim3 g(FHS_MODUP_QUADPAIR ? xcd_grid_q(E, dn * U) : mgrid), b((1 << LOGN) / 32);
    static_assert(modup_uses_half(LOGN) || !ntt_half<LOGN>(), "the full-limb ModUp needs N <= 16384");
    if (!modup_uses_half(LOGN))   // residues + counts (launch_centered wrote no X form: modup_xform is false)
        hipLaunchKernelGGL((k_modup<LOGN>), dim3(mgrid), dim3((1 << LOGN) / 16), 0, st, T, uniq, acoef, vcnt, ext, l, U);
    else if (modup_xform(T, l) && T.conv_b59)   // every digit full (3 limbs), X form, 59-bit primes
        hipLaunchKernelGGL((k_modup_h<LOGN, 3, true>), g, b, 0, st, T, uniq, acoef, vcnt, ext, l, U);
    else if (modup_xform(T, l))   // every digit of this level full (3 limbs), X form (launch_centered)
        hipLaunchKernelGGL((k_modup_h<LOGN, 3, false>), g, b, 0, st, T, uniq, acoef, vcnt, ext, l, U);
    else if (T.modup_dp == 1)
        if (T.all_b59)   // SEAL's 59-bit chains: compile-time lazy NTT and folded stores
            hipLaunchKernelGGL((k_modup_h<LOGN, 1, true>), g, b, 0, st, T, uniq, acoef, vcnt, ext, l, U);
        else
            hipLaunchKernelGGL((k_modup_h<LOGN, 1, false>), g, b, 0, st, T, uniq, acoef, vcnt, ext, l, U);
    else
        hipLaunchKernelGGL((k_modup_h<LOGN, 0, false>), g, b, 0, st, T, uniq, acoef, vcnt, ext, l, U);
}

// (b2) key inner product with the automorphism applied on the fly, lazy 128-bit over digits:
// acc[r][c][t][n] = sum_j ext[src][j][t][galois_src(n)] * key_j[c][t][n].
// The NTT-domain automorphism maps every aligned run of 64 slots onto an aligned run of 64 slots
// (bit-reversed order: the low 6 bits of the slot index are the top 6 bits of the evaluation
// exponent, which k * (.) permutes among themselves), so each wave's gather touches exactly one
// 512-byte region: four whole cache lines, no amplification.
// Limbs t >= t0 only (the giant-step path sums limbs t < l over rotations in k_ks_ip_sum).  A digit's
// own limbs were not extended (k_modup skips them): they are read from the input itself.
// Operands of one (rotation, target limb) key inner product as buffer descriptors built from
// wave-uniform pointers: the per-lane offsets (gathered source slot sn, key slot n) go in voffset, the
// digit strides in soffset -- global loads without 64-bit address arithmetic on the VALU, and (unlike
// the flat loads the generic pointers produced) counted on vmcnt alone, so the digits' loads overlap.
struct KsOps {
    __amdgpu_buffer_rsrc_t ext, own, key, akey;
    int sn8, n8;      // per-lane byte offsets: gathered source slot, key slot
    int per_r8, kn8;  // digit strides in bytes: ext (E N), key (K N)
    int jown;         // the digit whose own limb t is (read from the input, not extended); -1 if none
};
__device__ __forceinline__ KsOps ks_ops(const DevTables& T, const KsItem& it, const u64* const* uniq, const u64* ext,
                                        int t, int pt, int l, int n, int sn) {
    const int N = T.N, P_ = T.P, E = l + P_, dn = (l + P_ - 1) / P_, K = T.K;
    KsOps o;
    o.ext = brsrc(ext + ((size_t)it.src * dn * E + t) * N, (uint32_t)((size_t)dn * E * N * 8));
    o.own = brsrc(uniq[it.src] + (size_t)t * N, (uint32_t)N * 8);
    o.key = brsrc(it.key + (size_t)pt * N, (uint32_t)((size_t)T.dnum * K * N * 8));
    o.akey = brsrc(it.akey ? it.akey + (size_t)pt * N : it.key, (uint32_t)((size_t)T.dnum * K * N * 8));
    o.sn8 = sn * 8;
    o.n8 = n * 8;
    o.per_r8 = E * N * 8;
    o.kn8 = K * N * 8;
    o.jown = t < l ? t / P_ : -1;
    return o;
}
constexpr int kBufNT = 2;   // buffer aux: non-temporal (streamed once: the switching keys)
// sum_j ext_j[t][sigma(n)] (b_j, a_j)[t][n] as two lazy 128-bit sums; a_j regenerated from the key's
// seeds, or read from an imported key's explicit a (akey, a separate instantiation: the choice is
// per item, so the digit loop carries no branch)
typedef const __attribute__((address_space(4))) u64* cu64p;   // constant address space: scalar loads
#ifndef FHS_KSIP_V6
#define FHS_KSIP_V6 0   // 1: own digit first, the other digits branch-free -- measured slower, kept off (profiles/r06/ab_ksip_v6)
#endif
template <bool EXPLICIT_A>
__device__ __forceinline__ void ks_digit(const KsOps& o, u64 x, int j, u64 seed, u64 cx, const RedU& RD, unsigned qb,
                                         Acc3& a0, Acc3& a1) {
    const Split30 v = split30(x);
    acc3_mac(a0, v, split30(__builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(o.key, o.n8, j * o.kn8,
                                                                                         kBufNT))));
    if constexpr (EXPLICIT_A)
        acc3_mac(a1, v, split30(__builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(o.akey, o.n8, j * o.kn8,
                                                                                             kBufNT))));
    else
        acc3_mac(a1, v, split30(seeded_uniform_x(seed + cx, RD.q, qb)));
}
template <bool EXPLICIT_A>
__device__ __forceinline__ void ks_digits(const KsOps& o, const u64* seeds_g, u64 cx, const RedU& RD, unsigned qb,
                                          int dn, u128& c0, u128& c1) {
    // the seeds are wave-uniform and read-only: scalar loads instead of flat vector loads
    const cu64p seeds = (cu64p)seeds_g;
    Acc3 a0 = {0, 0, 0}, a1 = {0, 0, 0};
#if FHS_KSIP_V6
    // The digit whose limb t is the input's own (read from the input, not extended) first, then the others as
    // j = k + (k >= jown): the unrolled body has no per-digit branch between the input and the extension, so the
    // scheduler can issue a group's seed loads and buffer loads together (round 5: a diamond per digit and a
    // scalar load waited on at once -- 0.61 SALU per VALU, 46 % of wave cycles ready but not issued).  The sums
    // are exact integers, so the order of the products does not change them.
    // wave-uniform by construction (readfirstlane: the own digit's sampler loop must not make them look divergent,
    // which turns every digit's soffset into a waterfall loop)
    const int jo = __builtin_amdgcn_readfirstlane(o.jown >= 0 ? o.jown : dn);
    const int nd = __builtin_amdgcn_readfirstlane(o.jown >= 0 ? dn - 1 : dn);
    if (o.jown >= 0) {
        ks_digit<EXPLICIT_A>(o, bload64(o.own, o.sn8, 0), o.jown, seeds[o.jown], cx, RD, qb, a0, a1);
        acc3_fold(c0, a0);
        acc3_fold(c1, a1);
    }
    int k = 0;
    for (; k + 4 <= nd; k += 4) {   // groups of 4 digits: the 4 seed loads issued together, then the products
        int jj[4];
        u64 sd[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            jj[u] = __builtin_amdgcn_readfirstlane(k + u + (k + u >= jo ? 1 : 0));
            sd[u] = seeds[jj[u]];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            ks_digit<EXPLICIT_A>(o, bload64(o.ext, o.sn8, jj[u] * o.per_r8), jj[u], sd[u], cx, RD, qb, a0, a1);
        if (k & 4) {   // Acc3 holds 8 products; 128-bit sums stay < 2^128 for any dnum <= 8 * 32
            acc3_fold(c0, a0);
            acc3_fold(c1, a1);
        }
    }
    for (; k < nd; ++k) {   // < 4 left (at most 7 products since the last fold)
        const int j = __builtin_amdgcn_readfirstlane(k + (k >= jo ? 1 : 0));
        ks_digit<EXPLICIT_A>(o, bload64(o.ext, o.sn8, j * o.per_r8), j, seeds[j], cx, RD, qb, a0, a1);
    }
#else
#pragma unroll FHS_KSIP_UNROLL
    for (int j = 0; j < dn; ++j) {
        const bool own = j == o.jown;
        const u64 x = own ? bload64(o.own, o.sn8, 0) : bload64(o.ext, o.sn8, j * o.per_r8);
        ks_digit<EXPLICIT_A>(o, x, j, seeds[j], cx, RD, qb, a0, a1);
        if ((j & 7) == 7) {   // Acc3 holds 8 products; 128-bit sums stay < 2^128 for any dnum <= 8 * 32
            acc3_fold(c0, a0);
            acc3_fold(c1, a1);
        }
    }
#endif
    acc3_fold(c0, a0);
    acc3_fold(c1, a1);
}
__global__ void __launch_bounds__(256) k_ks_ip(DevTables T, const KsItem* items, const u64* const* uniq, const u64* ext,
                                                u64* acc, int l, int R, int t0) {
    const int N = T.N, P_ = T.P, K = T.K, E = l + P_, dn = (l + P_ - 1) / P_;
    const int NB = N >> 8;
    int t, m;
    // t0 == 0 (hoisted rotations of one input): the rotations of one limb t run together on one XCD, so
    // their shared extension stays in its L2.  t0 > 0 (the giant steps' special limbs): every rotation has
    // its own input, so nothing is shared and a plain map keeps all 8 XCDs busy (an XCD map over P = 3
    // limbs would leave 5 of them idle)
    if (!(t0 > 0 ? plain_tm(E - t0, R * NB, t, m) : xcd_touter(E - t0, R * NB, t, m))) return;
    t += t0;
    int r, nb;
    if (FHS_KSIP_HALVES && t0 == 0 && NB >= 2 && (size_t)dn * N * 8 > ((size_t)3 << 20)) {
        // half-major: every rotation's lower coefficient half, then every rotation's upper half.  A rotation
        // X -> X^(5^g) maps NTT slot exponents 2 rev(n) + 1 = 1 mod 4 (n < N/2) to 1 mod 4 again, so each half
        // reads only its own half of the shared extension: the limb's working set on its XCD halves (SEAL's
        // convention: 36 one-limb digits x 128 KiB = 4.6 MiB per limb, over the 4 MiB L2; 2.3 MiB per half).
        // Only where the limb's extension would not fit the L2 anyway: the default convention's 12 digits
        // (1.5 MiB) measured 2 % slower half-major (profiles/r05/ab_seal_perm_halves)
        const int hb = NB >> 1, h = m / (R * hb), k = m % (R * hb);
        r = k / hb;
        nb = h * hb + k % hb;
    } else {
        r = m / NB;
        nb = m % NB;
    }
    const int n = (nb << 8) + threadIdx.x;
    const int pt = t < l ? t : T.L0 + (t - l);
    const RedU RD = redu(PK(T, pt));
    const KsItem it = items[r];
    const int sn = galois_src(n, it.elt, T.logN);
    const KsOps o = ks_ops(T, it, uniq, ext, t, pt, l, n, sn);
    const u64* seeds = it.key + (size_t)T.dnum * K * N;
    const u64 cx = seeded_ctr_mix(pt, n);
    const unsigned qb = 64 - __clzll(RD.q);
    u128 c0 = {0, 0}, c1 = {0, 0};
    if (it.akey)
        ks_digits<true>(o, seeds, cx, RD, qb, dn, c0, c1);
    else
        ks_digits<false>(o, seeds, cx, RD, qb, dn, c0, c1);
    u64 v0 = reduce128(c0.lo, c0.hi, RD), v1 = reduce128(c1.lo, c1.hi, RD);
    if (it.corr) {   // hoisted SEAL convention: the item's correction (SealHoist)
        v0 = addmod(v0, it.corr[(size_t)t * N + n], RD.q);
        v1 = addmod(v1, it.corr[((size_t)E + t) * N + n], RD.q);
    }
    acc[(((size_t)r * 2 + 0) * E + t) * N + n] = v0;
    acc[(((size_t)r * 2 + 1) * E + t) * N + n] = v1;
}

// Giant steps, limbs t < l: the key inner products of all R rotations summed in place, already
// scaled by P^-1 and with the rotated c0's added (comp 0) -- the t < l part of
// sum_r ModDown(acc_r) + sigma_r(c0_r) (k_giant_sum adds the special-limb conversion).  Writes
// bpart[c][t][n] into the r = 0 slot of acc (acc[0][c][t], t < l), which nothing else uses.
__global__ void __launch_bounds__(256) k_ks_ip_sum(DevTables T, const KsItem* items, const u64* const* uniq,
                                                    const u64* ext, u64* acc, int l, int R) {
    const int N = T.N, P_ = T.P, K = T.K, E = l + P_, dn = (l + P_ - 1) / P_;
    const int NB = N >> 8;
    int t, m;
    if (!xcd_touter(l, NB, t, m)) return;
    const int n = (m << 8) + threadIdx.x;
    const RedU RD = redu(PK(T, t));
    const u64 q = RD.q;
    const u64 cx = seeded_ctr_mix(t, n);
    const unsigned qb = 64 - __clzll(q);
    u64 s0 = 0, s1 = 0, sadd = 0;
    for (int r = 0; r < R; ++r) {
        const KsItem it = items[r];
        const int sn = galois_src(n, it.elt, T.logN);
        const KsOps o = ks_ops(T, it, uniq, ext, t, t, l, n, sn);
        const u64* seeds = it.key + (size_t)T.dnum * K * N;
        u128 c0 = {0, 0}, c1 = {0, 0};
        if (it.akey)
            ks_digits<true>(o, seeds, cx, RD, qb, dn, c0, c1);
        else
            ks_digits<false>(o, seeds, cx, RD, qb, dn, c0, c1);
        s0 = addmod(s0, reduce128(c0.lo, c0.hi, RD), q);
        s1 = addmod(s1, reduce128(c1.lo, c1.hi, RD), q);
        if (it.corr) {   // hoisted SEAL convention (SealHoist)
            s0 = addmod(s0, it.corr[(size_t)t * N + n], q);
            s1 = addmod(s1, it.corr[((size_t)E + t) * N + n], q);
        }
        sadd = addmod(sadd, bload64(brsrc(it.add0 + (size_t)t * N, (uint32_t)N * 8), o.sn8, 0), q);
    }
    const u64 pinv = T.md_pinv[2 * t], pinv_s = T.md_pinv[2 * t + 1];
    acc[((size_t)0 * E + t) * N + n] = addmod(shoup(s0, pinv, pinv_s, q), sadd, q);
    acc[((size_t)1 * E + t) * N + n] = shoup(s1, pinv, pinv_s, q);
}

// (c) special limbs of the accumulator -> coefficient form, scaled by inv(P / p_k)
template <int LOGN, bool H = ntt_half<LOGN>()>
__global__ void __launch_bounds__((ntt_threads<LOGN, H>())) k_ks_special_intt(DevTables T, const u64* acc, u64* ycoef, int l,
                                                                         int R) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN, H>()];
    const int k = blockIdx.x, comp = blockIdx.y, r = blockIdx.z;
    const int P_ = T.P, E = l + P_, pi = T.L0 + k;
    const PrimeK& P = PK(T, pi);
    const u64* src = acc + (((size_t)r * 2 + comp) * E + l + k) * N;
    u64* dst = ycoef + (((size_t)r * 2 + comp) * P_ + k) * N;
    const u64* cst = T.md_intt + (size_t)k * 4;
    const u64 p = P.q, half = T.ks_seal ? p >> 1 : 0;   // SEAL: + floor(p/2) turns the floor into rounding
    inv_limb<LOGN, FHS_NTT_RL, H>(lds, threadIdx.x, T.tw_inv + (size_t)pi * N * 2, P.q, cst[0], cst[1], cst[2], cst[3],
                               [&](int e) { return src[e]; }, [&](int e, u64 v) { dst[e] = csub(csub(v, p) + half, p); });
}

// (c') ModDown's special digit in X form (T.md_xform): Y = sum_k y_k (P/p_k) (< 3P < 2^179, the fast
// base conversion's integer, no centring) once per coefficient, stored in place of the three special
// residues as base-2^60 words (centered_x_pack with md_xd) -- each of the l targets then reduces it with
// two split-30 products (moddown_convert3x) instead of three: the same integer, the same residues
__global__ void k_special_x(DevTables T, u64* ycoef, int R2) {
    const int N = T.N, n = blockIdx.x * blockDim.x + threadIdx.x, rc = blockIdx.y;
    if (n >= N || rc >= R2) return;
    u64* yb = ycoef + (size_t)rc * 3 * N + n;
    const u64 y[3] = {yb[0], yb[N], yb[2 * (size_t)N]};
    u64 w[3];
    centered_x_pack(y, T.md_xd, w);
    yb[0] = w[0];
    yb[N] = w[1];
    yb[2 * (size_t)N] = w[2];
}

// (d) ModDown: out_c[i] = (acc_c[i] - NTT(conv_P->q_i(y_c))) * P^-1 (+ add_c)
template <int LOGN>
__global__ void __launch_bounds__((1 << LOGN) / 16) k_moddown(DevTables T, const KsItem* items, const u64* acc,
                                                              const u64* ycoef, int l, int R) {
    constexpr int N = 1 << LOGN, TH = N / 16;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_half<LOGN>() ? 1 : (1 << LOGN) + (1 << LOGN) / 16];
    if constexpr (!ntt_half<LOGN>()) {   // full-limb form: N <= 16384 only
    const int tid = threadIdx.x;
    const int P_ = T.P, E = l + P_;
    int i, m;
    if (!plain_tm(l, 2 * R, i, m)) return;
    const int comp = m & 1, r = m >> 1;
    const PrimeK& P = PK(T, i);
    const u64 q = P.q;
    const KsItem it = items[r];
    const u64* y = ycoef + ((size_t)r * 2 + comp) * P_ * N;
    const u64 halfq = T.ks_seal ? T.md_pinv[3 * T.L0 + i] : 0;   // SEAL rounding: - floor(p/2) mod q_i
#pragma unroll 4
    for (int kk = 0; kk < 16; ++kk) {
        const int e = tid + kk * TH;
        u128 s = {0, 0};
        for (int k = 0; k < P_; ++k) mac128(s, y[(size_t)k * N + e], T.md_hat[(size_t)k * T.L0 + i]);
        lds[row_pad<TH>(tid, kk)] = submod(reduce128(s.lo, s.hi, P), halfq, q);
    }
    __syncthreads();
    const RedU RU = redu(P);
    ntt_fwd_lds<LOGN, FHS_NTT_RL>(lds, tid, T.tw_fwd + (size_t)i * N * 2, q, RU.lazy);
    const u64 pinv = T.md_pinv[2 * i], pinv_s = T.md_pinv[2 * i + 1];
    const u64* add = comp == 0 ? it.add0 : it.add1;
    const u64 aelt = comp == 0 ? it.elt : 1;
    u64* o = (comp == 0 ? it.out0 : it.out1) + (size_t)i * N;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const int e = tid + c * TH;
        const u64 v = fwd_canon(lds[row_pad<TH>(tid, c)], RU);
        const u64 a = acc[(((size_t)r * 2 + comp) * E + i) * N + e];
        u64 res = shoup(submod(a, v, q), pinv, pinv_s, q);
        if (add) res = addmod(res, add[(size_t)i * N + galois_src(e, aelt, LOGN)], q);
        o[e] = res;
    }
    }
}

// ModDown conversion of the P = 3 special limbs (coefficient form, already scaled by inv(P/p_k)) into
// data limb i (pseudo-Mersenne fold), half-limb form as modup_convert3x: x = sum_k y_k (P/p_k) mod q_i,
// global stages 0 and 1 in registers (fwd_quad_first2), lower results to LDS, upper ones kept in hi[].
template <int LOGN>
__device__ __forceinline__ void moddown_convert3(const u64* y, const u64* hat, int L0, const RedU& R, const u64* tw,
                                                 int tid, u64* lds, u64 hi[16]) {
    constexpr int N = 1 << LOGN, NH = N / 2, TH = N / 32;
    const __amdgpu_buffer_rsrc_t ry = brsrc(y, 3 * N * 8);
    const Split30 h0 = split30(hat[0]), h1 = split30(hat[L0]), h2 = split30(hat[2 * L0]);
    const u64 m = R.q;
    const int vo = tid * 8;
    const Tw4 w4 = ld_tw4(tw);
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {
        u64 v[3][4];   // k: rows ch (k = 0, 2) and ch + 8 (k = 1, 3), lower (k < 2) / upper half
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = (ch + 8 * (k & 1)) * TH + (k >= 2 ? NH : 0);
#pragma unroll
            for (int w = 0; w < 3; ++w) v[w][k] = bload64(ry, vo, (w * N + e) * 8);
        }
        u64 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            Acc3 a = {0, 0, 0};
            acc3_mac(a, split30(v[0][k]), h0);
            acc3_mac(a, split30(v[1][k]), h1);
            acc3_mac(a, split30(v[2][k]), h2);
            x[k] = acc3_reduce_pm(a.L, a.M, a.H, R.b, R.d);
        }
        fwd_quad_first2<TH>(x, w4, m, R.lazy, lds, tid, ch, hi);
    }
}

// moddown_convert3 from the X form (k_special_x): x = V0 + V1 (2^60 mod q_i) + V2 (2^120 mod q_i)
template <int LOGN, bool B59>
__device__ __forceinline__ void moddown_convert3x(const u64* y, const u64* xt, const RedU& R, const u64* tw, int tid,
                                                  u64* lds, u64 hi[16]) {
    constexpr int N = 1 << LOGN, NH = N / 2, TH = N / 32;
    const __amdgpu_buffer_rsrc_t ry = brsrc(y, 3 * N * 8);
    const uint32_t e1 = (uint32_t)xt[0];
    const Split30 e2 = unpack30(xt[1]);
    const int vo = tid * 8;
    const Tw4 w4 = ld_tw4(tw);
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {
        u64 v[3][4];   // k: rows ch (k = 0, 2) and ch + 8 (k = 1, 3), lower (k < 2) / upper half
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = (ch + 8 * (k & 1)) * TH + (k >= 2 ? NH : 0);
#pragma unroll
            for (int w = 0; w < 3; ++w) v[w][k] = bload64(ry, vo, (w * N + e) * 8);
        }
        u64 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)   // B59: upper half unfolded, as modup_convert3x
            x[k] = B59 ? convert3x_b59(v[0][k], v[1][k], v[2][k], e1, e2, 0, R.d, k < 2)
                       : convert3x_value(v[0][k], v[1][k], v[2][k], e1, e2, 0, R.b, R.d);
        fwd_quad_first2<TH>(x, w4, R.q, lazy_of<LOGN, B59>(R), lds, tid, ch, hi);
    }
}

// k_moddown with half the limb in LDS (see k_modup_h): conversion of both coefficients of each
// (e, e + N/2) pair, global NTT stage 0 in registers, then each half transformed in LDS and finished
// ((acc - conv) P^-1 + sigma(c0)).  Same values as k_moddown.  SPLIT (launches with few workgroups: a single key
// switch's ModDown, latency-bound): two workgroups per (limb, component, item), each converting the whole column
// and transforming and finishing one half -- twice the workgroups, half the serial work each (as k_rescale_ntt_hs).
template <int LOGN, bool MX, bool B59 = false, bool SPLIT = false>
__global__ void __launch_bounds__((1 << LOGN) / 32, 4) k_moddown_h(DevTables T, const KsItem* items, const u64* acc,
                                                                   const u64* ycoef, int l, int R) {
    constexpr int N = 1 << LOGN, NH = N / 2, TH = N / 32;
    __shared__ __attribute__((aligned(16))) u64 lds[(1 << (LOGN - 1)) + (1 << (LOGN - 1)) / 16];
    const int tid = threadIdx.x;
    const int P_ = T.P, E = l + P_;
    const int bx = SPLIT ? (int)(blockIdx.x >> 1) : (int)blockIdx.x, hg = SPLIT ? (int)(blockIdx.x & 1) : 0;
    const int i = bx % l, mm = bx / l;
    if (mm >= 2 * R) return;
    const int comp = mm & 1, r = mm >> 1;
    const PrimeK& P = PK(T, i);
    const RedU RU = redu(P);
    const u64 q = RU.q, q2 = 2 * q;
    const KsItem it = items[r];
    const u64* y = ycoef + ((size_t)r * 2 + comp) * P_ * N;
    const u64* tw = T.tw_fwd + (size_t)i * N * 2;
    const u64 halfq = T.ks_seal ? T.md_pinv[3 * T.L0 + i] : 0;
    u64 hi[16];
    if constexpr (MX) {   // T.md_xform: y holds the special digit's X form
        moddown_convert3x<LOGN, B59>(y, T.modup_xt + (size_t)i * 4, RU, tw, tid, lds, hi);
    } else if (P_ == 3 && RU.cpm && !T.ks_seal) {
        moddown_convert3<LOGN>(y, T.md_hat + i, T.L0, RU, tw, tid, lds, hi);
    } else {
    const Tw4 w4 = ld_tw4(tw);
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {   // rows ch and ch + 8 of both halves per chunk
        Acc3 a3[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) a3[k] = Acc3{0, 0, 0};
#pragma unroll 1
        for (int k = 0; k < P_; ++k) {   // P <= 7 products per Acc3
            const Split30 hk = split30(T.md_hat[(size_t)k * T.L0 + i]);
            const u64* yk = y + (size_t)k * N + tid;
            u64 v[4];
            v[0] = yk[ch * TH];
            v[1] = yk[(ch + 8) * TH];
            v[2] = yk[ch * TH + NH];
            v[3] = yk[(ch + 8) * TH + NH];
#pragma unroll
            for (int z = 0; z < 4; ++z) acc3_mac(a3[z], split30(v[z]), hk);
        }
        u64 x[4];
#pragma unroll
        for (int z = 0; z < 4; ++z) {
            if (RU.cpm) {
                x[z] = acc3_reduce_pm(a3[z].L, a3[z].M, a3[z].H, RU.b, RU.d);
            } else {
                u128 s = {0, 0};
                acc3_fold(s, a3[z]);
                x[z] = reduce128(s.lo, s.hi, RU);
            }
            if (T.ks_seal) x[z] = submod(csub(x[z], q), halfq, q);   // SEAL rounding: - floor(p/2) mod q_i
        }
        fwd_quad_first2<TH>(x, w4, q, lazy_of<LOGN, B59>(RU), lds, tid, ch, hi);
    }
    }
    const u64 pinv = T.md_pinv[2 * i], pinv_s = T.md_pinv[2 * i + 1];
    const u64* add = comp == 0 ? it.add0 : it.add1;
    const u64 aelt = comp == 0 ? it.elt : 1;
    u64* o = (comp == 0 ? it.out0 : it.out1) + (size_t)i * N;
    const u64* ac = acc + (((size_t)r * 2 + comp) * E + i) * N;
#pragma unroll 1
    for (int h = hg; h < (SPLIT ? hg + 1 : 2); ++h) {
        if (h) {   // (SPLIT, upper half: each thread overwrites only its own rows; the barrier is harmless)
            __syncthreads();
#pragma unroll
            for (int c = 0; c < 16; ++c) lds[row_pad<TH>(tid, c)] = hi[c];
        }
        __syncthreads();
        // wave-local tail (fhs_ntt.h): the outputs are read by the wave that made them, no exit barrier; element
        // of output c: tb + eoff(c) (tb = wl_base or tid), LDS word lb + loff(c)
        constexpr bool WLX = FHS_NTT_WAVELOCAL && fwd_exit_wave_local<LOGN - 1, FHS_MODUPH_RL, 1>();
        constexpr int GS = 1 << FHS_MODUPH_RL;
        ntt_fwd_lds<LOGN - 1, FHS_MODUPH_RL, 16, 1, WLX>(lds, tid, tw, q, lazy_of<LOGN, B59>(RU), 1 + h);
        const int tb = WLX ? wl_base<LOGN - 1, 16, GS>(tid) : tid, lb = lds_pad(tb);
        auto eoff = [&](int c) { return WLX ? wl_off<LOGN - 1, 16, GS>(c) : c * TH; };
        auto lidx = [&](int c) { return WLX ? lb + eoff(c) + eoff(c) / 16 : row_pad<TH>(tid, c); };
        // outputs in batches of 4 whose accumulator (and rotated c0) loads are issued together, with
        // the add / no-add choice outside the loop (one latency per batch, not one per coefficient);
        // buffer loads / stores with the row offsets in soffset
        const __amdgpu_buffer_rsrc_t rac = brsrc(ac, N * 8), ro = brsrc(o, N * 8);
        if (add) {
            const __amdgpu_buffer_rsrc_t rad = brsrc(add + (size_t)i * N, N * 8);
            // galois_src(e) for e = tid + c TH + h NH: rev(e) = rev(tid) + rev(c TH + h NH) (disjoint bits),
            // so the exponent (2 rev(e) + 1) elt mod 2N is a per-thread base plus a wave-uniform term
            const unsigned rt = __brev((unsigned)tb) >> (32 - LOGN);
            const u64 ebase = ((2 * (u64)rt + 1) * aelt) & (2 * (u64)N - 1);
#pragma unroll
            for (int c0 = 0; c0 < 16; c0 += 4) {
                u64 av[4], dv[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int eo = h * NH + eoff(c0 + k);
                    av[k] = bload64(rac, tb * 8, eo * 8);
                    const u64 ec = (2 * (u64)(__brev((unsigned)eo) >> (32 - LOGN)) * aelt) & (2 * (u64)N - 1);
                    const u64 e2 = (ebase + ec) & (2 * (u64)N - 1);
                    const int src = (int)(__brev((unsigned)((e2 - 1) >> 1)) >> (32 - LOGN));
                    dv[k] = bload64(rad, src * 8, 0);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    // B59: the NTT output folded once (< 2q) and a + 2q - v handed to the Shoup product
                    // (any 64-bit input) -- no run-time lazy choice per element, no canonicalisation
                    const u64 x = lds[lidx(c0 + k)];
                    const u64 dif = B59 ? av[k] + q2 - fold59(x, RU.d) : submod(av[k], fwd_canon(x, RU), q);
                    bstore64(addmod(shoup(dif, pinv, pinv_s, q), dv[k], q), ro, tb * 8, (h * NH + eoff(c0 + k)) * 8);
                }
            }
        } else {
#pragma unroll
            for (int c0 = 0; c0 < 16; c0 += 4) {
                u64 av[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) av[k] = bload64(rac, tb * 8, (h * NH + eoff(c0 + k)) * 8);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const u64 x = lds[lidx(c0 + k)];
                    const u64 dif = B59 ? av[k] + q2 - fold59(x, RU.d) : submod(av[k], fwd_canon(x, RU), q);
                    bstore64(shoup(dif, pinv, pinv_s, q), ro, tb * 8, (h * NH + eoff(c0 + k)) * 8);
                }
            }
        }
    }
}

static size_t ks_core_bytes(const DevTables& T, int R, int U, int l) {
    const size_t N = T.N, E = l + T.P, dn = (l + T.P - 1) / T.P;
    // acoef | ext | acc | ycoef | centred counts (bytes, rounded up to words)
    return 8 * N * ((size_t)U * l + (size_t)U * dn * E + (size_t)R * 2 * E + (size_t)R * 2 * T.P) +
           ((size_t)U * dn * N + 7) / 8 * 8;
}
// SEAL convention: every item's input gets its own decomposition (U = R) and the permuted
// ciphertexts [R][2][l][N] follow the core workspace
size_t keyswitch_workspace_bytes(const DevTables& T, int R, int U, int l) {
    if (!T.ks_seal) return ks_core_bytes(T, R, U, l);
    return ks_core_bytes(T, R, R, l) + 8 * (size_t)R * 2 * l * T.N;
}
// SEAL's switch_key_inplace decomposes the automorphed ciphertext (the lift without centring does
// not commute with the automorphism, so nothing is hoisted): items with elt != 1 are rewritten to
// read galois_elt(c0), galois_elt(c1) materialised in `perm`, with elt = 1 and an input each.
// seal_rewrite changes the host items; seal_permute (enqueued once the inputs exist) fills `perm`.
static void seal_rewrite(const DevTables& T, KsItem* items, int R, const u64** uniq, int l, u64* perm) {
    const size_t S = (size_t)l * T.N;
    for (int r = 0; r < R; ++r) {
        KsItem& it = items[r];
        if (it.elt != 1) {
            u64* pc = perm + (size_t)r * 2 * S;
            it.a = pc + S;
            if (it.add0) it.add0 = pc;
            it.elt = 1;
        }
        it.corr = nullptr;   // the automorphed input is decomposed itself: nothing to correct
        uniq[r] = it.a;
        it.src = (u64)r;
    }
}
// up to kPermBatch permutations per launch, passed by value (one launch per 32 polynomials instead of one each:
// the giant steps' 2 (B - 1) permutations were 88 launches of ~5 us at cfg2)
constexpr int kPermBatch = 32;
struct PermBatch {
    const u64* in[kPermBatch];
    u64* out[kPermBatch];
    u64 elt[kPermBatch];
};
__global__ void __launch_bounds__(256) k_galois_perm_batch(DevTables T, PermBatch pb, int limbs) {
    const int y = blockIdx.y;
    const u64* in = pb.in[y];
    u64* out = pb.out[y];
    const u64 elt = pb.elt[y];
    const size_t S = (size_t)limbs * T.N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const size_t base = idx - idx % T.N;
        out[idx] = in[base + galois_src((int)(idx % T.N), elt, T.logN)];
    }
}
static hipError_t seal_permute(const DevTables& T, const KsItem* orig, int R, int l, u64* perm, hipStream_t st) {
    const size_t S = (size_t)l * T.N;
    PermBatch pb;
    int n = 0;
    const int gx = std::max(1, eltwise_grid(S) / 8);
    auto flush = [&]() -> hipError_t {
        if (!n) return hipSuccess;
        hipLaunchKernelGGL(k_galois_perm_batch, dim3(gx, n), dim3(256), 0, st, T, pb, l);
        n = 0;
        return hipGetLastError();
    };
    for (int r = 0; r < R; ++r) {
        const KsItem& it = orig[r];
        if (it.elt == 1) continue;
        u64* pc = perm + (size_t)r * 2 * S;
        for (int c = 1; c >= 0; --c) {
            const u64* src = c ? it.a : it.add0;
            if (!src) continue;
            pb.in[n] = src;
            pb.out[n] = pc + (c ? S : 0);
            pb.elt[n] = it.elt;
            if (++n == kPermBatch) {
                hipError_t e = flush();
                if (e != hipSuccess) return e;
            }
        }
    }
    return flush();
}

// key-switch workspace carve: acoef | ext | acc | ycoef | centred counts (ks_core_bytes)
struct KsBufs {
    u64 *acoef, *ext, *acc, *ycoef;
    unsigned char* vcnt;
};
static KsBufs ks_carve(const DevTables& T, u64* ws, int R, int U, int l) {
    const size_t N = T.N, E = l + T.P, dn = (l + T.P - 1) / T.P;
    KsBufs b;
    b.acoef = ws;
    b.ext = b.acoef + (size_t)U * l * N;
    b.acc = b.ext + (size_t)U * dn * E * N;
    b.ycoef = b.acc + (size_t)R * 2 * E * N;
    b.vcnt = reinterpret_cast<unsigned char*>(b.ycoef + (size_t)R * 2 * T.P * N);
    return b;
}
// INTT + centred ModUp per distinct input, then key inner product and special-limb INTT per item;
// leaves acc [R][2][E][N] and ycoef [R][2][P][N]
template <int LOGN>
static void ks_front(const DevTables& T, const KsItem* it, const u64* const* uniq, int R, int U, int l, u64* ws,
                     hipStream_t st, const KTimer* tm, u64** acc_out, u64** ycoef_out) {
    const size_t N = T.N, E = l + T.P, dn = (l + T.P - 1) / T.P;
    u64* acoef = ws;
    u64* ext = acoef + (size_t)U * l * N;
    u64* acc = ext + (size_t)U * dn * E * N;
    u64* ycoef = acc + (size_t)R * 2 * E * N;
    unsigned char* vcnt = reinterpret_cast<unsigned char*>(ycoef + (size_t)R * 2 * T.P * N);
    const dim3 blk((1 << LOGN) / 16);
    FHS_TMARK(tm, KID_KS_INTT, 1, st);
    if (ks_intt_half<LOGN>(l * U))
        hipLaunchKernelGGL((k_ks_intt_h<LOGN>), dim3(l * U), dim3((1 << LOGN) / 32), 0, st, T, uniq, acoef, l, U);
    else
        hipLaunchKernelGGL((k_ks_intt<LOGN>), dim3(l * U), blk, 0, st, T, uniq, acoef, l, U);
    launch_centered(T, acoef, vcnt, l, U, st);
    FHS_TMARK(tm, KID_KS_INTT, 0, st);
    FHS_TMARK(tm, KID_MODUP, 1, st);
    launch_modup<LOGN>(T, uniq, acoef, vcnt, ext, l, U, st);
    FHS_TMARK(tm, KID_MODUP, 0, st);
    FHS_TMARK(tm, KID_KS_IP, 1, st);
    hipLaunchKernelGGL(k_ks_ip, dim3(xcd_grid((int)E, R * (int)(N >> 8))), dim3(256), 0, st, T, it, uniq, ext, acc, l, R,
                       0);
    FHS_TMARK(tm, KID_KS_IP, 0, st);
    FHS_TMARK(tm, KID_SPECIAL_INTT, 1, st);
    FHS_NTT_LAUNCH(k_ks_special_intt, T.P * 2 * R, dim3(T.P, 2, R), st, T, acc, ycoef, l, R);
    FHS_TMARK(tm, KID_SPECIAL_INTT, 0, st);
    *acc_out = acc;
    *ycoef_out = ycoef;
}

// ModDown of the R accumulators (acc, ycoef from ks_front) into the items' outputs
template <int LOGN>
static hipError_t launch_moddown(const DevTables& T, const KsItem* it, u64* acc, u64* ycoef, int l, int R, hipStream_t st,
                                 const KTimer* tm) {
    FHS_TMARK(tm, KID_MODDOWN, 1, st);
    // a single key switch's ModDown at N = 32768 (few workgroups): one workgroup per half (SPLIT)
    static const bool split_off = getenv("FHESPEAR_MODDOWN_UNSPLIT") != nullptr;
    const bool split = LOGN == 15 && !split_off && l * 2 * R < FHS_SPLIT_MAX_WG;
    if ((FHS_MODDOWN_HALF && LOGN >= 9) || ntt_half<LOGN>()) {
        if (T.md_xform) {   // the special digit to its X form, then the two-product conversion
            hipLaunchKernelGGL(k_special_x, dim3((T.N + 255) / 256, 2 * R), dim3(256), 0, st, T, ycoef, 2 * R);
            if (T.conv_b59 && split)
                hipLaunchKernelGGL((k_moddown_h<LOGN, true, true, true>), dim3(2 * l * 2 * R), dim3((1 << LOGN) / 32), 0,
                                   st, T, it, acc, ycoef, l, R);
            else if (T.conv_b59)
                hipLaunchKernelGGL((k_moddown_h<LOGN, true, true>), dim3(l * 2 * R), dim3((1 << LOGN) / 32), 0, st, T,
                                   it, acc, ycoef, l, R);
            else
                hipLaunchKernelGGL((k_moddown_h<LOGN, true>), dim3(l * 2 * R), dim3((1 << LOGN) / 32), 0, st, T, it, acc,
                                   ycoef, l, R);
        } else {
            if (T.all_b59)
                hipLaunchKernelGGL((k_moddown_h<LOGN, false, true>), dim3(l * 2 * R), dim3((1 << LOGN) / 32), 0, st, T,
                                   it, acc, ycoef, l, R);
            else
                hipLaunchKernelGGL((k_moddown_h<LOGN, false>), dim3(l * 2 * R), dim3((1 << LOGN) / 32), 0, st, T, it,
                                   acc, ycoef, l, R);
        }
    } else {
        hipLaunchKernelGGL((k_moddown<LOGN>), dim3(l * 2 * R), dim3((1 << LOGN) / 16), 0, st, T, it, acc, ycoef, l, R);
    }
    FHS_TMARK(tm, KID_MODDOWN, 0, st);
    return hipGetLastError();
}

static hipError_t upload_items(const KsItem* items, int R, const u64* const* uniq, int U, void* dev, const Stager& sg,
                               const KsItem** it_dev, const u64* const** uniq_dev) {
    // one staged copy: [R items][U pointers]
    static thread_local std::vector<unsigned char> buf;
    buf.resize(sizeof(KsItem) * R + sizeof(u64*) * U);
    memcpy(buf.data(), items, sizeof(KsItem) * R);
    memcpy(buf.data() + sizeof(KsItem) * R, uniq, sizeof(u64*) * U);
    hipError_t e = sg.h2d(sg.user, dev, buf.data(), buf.size());
    *it_dev = reinterpret_cast<const KsItem*>(dev);
    *uniq_dev = reinterpret_cast<const u64* const*>(static_cast<unsigned char*>(dev) + sizeof(KsItem) * R);
    return e;
}

// ---- SEAL-convention hoisting (fhs_kernels.h SealHoist)
// mask_sigma in coefficient form, replicated over the K primes: coefficient i of a moves to i elt mod 2N,
// negated when that lands in [N, 2N) -- mask[k] = 1 exactly where sigma(a)[k] = -a_i
__global__ void k_seal_mask(DevTables T, u64 elt, u64* out) {
    const int N = T.N, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const u64 j = ((u64)i * elt) & (2 * (u64)N - 1);
    const u64 v = j >> T.logN;
    const size_t k = j & (N - 1);
    for (int t = 0; t < T.K; ++t) out[(size_t)t * N + k] = v;
}
// corr_c[t][n] = M_t[n] sum_{j < l, j != t} (q_j mod p_t) key_j[c][t][n], M_t = NTT_t(mask_sigma), t over the
// level's data limbs then the special primes (one-limb digits: P = 1 in SEAL's convention); key_j[1] is
// a_j, regenerated from the seeds as the key inner product does, or read from an imported key
__global__ void __launch_bounds__(256) k_seal_corr(DevTables T, const u64* key, const u64* akey, const u64* M,
                                                    int l, u64* out) {
    const int N = T.N, K = T.K, E = l + T.P;
    const int n = blockIdx.x * blockDim.x + threadIdx.x, t = blockIdx.y;
    if (n >= N || t >= E) return;
    const int pt = t < l ? t : T.L0 + (t - l);
    const RedU RD = redu(PK(T, pt));
    const u64 p = RD.q;
    const unsigned qb = 64 - __clzll(p);
    const u64* seeds = key + (size_t)T.dnum * K * N;
    const u64 cx = seeded_ctr_mix(pt, n);
    u128 s0 = {0, 0}, s1 = {0, 0};
    for (int j = 0; j < l; ++j) {
        if (j == t) continue;   // the digit's own limb is not lifted (k_ks_ip reads the input itself)
        const u64 qj = reduce128(PK(T, j).q, 0, RD);
        const size_t kx = ((size_t)j * K + pt) * N + n;
        const u64 a = akey ? akey[kx] : seeded_uniform_x(seeds[j] + cx, p, qb);
        mac128(s0, key[kx], qj);
        mac128(s1, a, qj);
        if ((j & 7) == 7) {   // < 2^120 per product: fold every 8
            s0 = u128{reduce128(s0.lo, s0.hi, RD), 0};
            s1 = u128{reduce128(s1.lo, s1.hi, RD), 0};
        }
    }
    const u64 m = M[(size_t)pt * N + n];
    const u64 r0 = reduce128(s0.lo, s0.hi, RD), r1 = reduce128(s1.lo, s1.hi, RD);
    out[(size_t)t * N + n] = reduce128(r0 * m, __umul64hi(r0, m), RD);
    out[((size_t)E + t) * N + n] = reduce128(r1 * m, __umul64hi(r1, m), RD);
}
hipError_t launch_seal_corr(const DevTables& T, const u64* key, const u64* akey, u64 elt, int l, u64* mask_scratch,
                            u64* out, hipStream_t st) {
    if (T.P != 1 || l < 1 || l > T.L0 || !key || !out || !mask_scratch) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_seal_mask, dim3((T.N + 255) / 256), dim3(256), 0, st, T, elt, mask_scratch);
    hipError_t e = launch_ntt_fwd(T, mask_scratch, T.K, T.L0, 1, 0, st);   // limb t at prime t: l_split = L0
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_seal_corr, dim3((T.N + 255) / 256, l + T.P), dim3(256), 0, st, T, key, akey, mask_scratch,
                       l, out);
    return hipGetLastError();
}

hipError_t launch_keyswitch(const DevTables& T, const KsItem* items_host, int R, const u64* const* uniq_host, int U,
                            int l, u64* ws, size_t ws_bytes, void* items_dev, const Stager& sg, hipStream_t st,
                            const KTimer* tm, SealHoist* sh) {
    if (keyswitch_workspace_bytes(T, R, U, l) > ws_bytes) return hipErrorInvalidValue;
    const KsItem* it;
    const u64* const* uq;
    std::vector<KsItem> sitems;
    std::vector<const u64*> suniq;
    // SEAL convention: hoist only when some input is shared (U < R) and every rotated item has its correction
    bool hoist = T.ks_seal && sh && U < R;
    for (int r = 0; hoist && r < R; ++r) hoist = items_host[r].elt == 1 || items_host[r].corr;
    if (hoist) {
        hipError_t e = upload_items(items_host, R, uniq_host, U, items_dev, sg, &it, &uq);
        if (e == hipSuccess) e = hipMemsetAsync(sh->zflag_dev, 0, sizeof(unsigned), st);
        if (e != hipSuccess) return e;
        const KsBufs b = ks_carve(T, ws, R, U, l);
        FHS_DISPATCH_LOGN(T.logN, {
            FHS_TMARK(tm, KID_KS_INTT, 1, st);
            if (ks_intt_half<LOGN>(l * U))
                hipLaunchKernelGGL((k_ks_intt_h<LOGN>), dim3(l * U), dim3((1 << LOGN) / 32), 0, st, T, uq, b.acoef, l, U);
            else
                hipLaunchKernelGGL((k_ks_intt<LOGN>), dim3(l * U), dim3((1 << LOGN) / 16), 0, st, T, uq, b.acoef, l, U);
            launch_centered(T, b.acoef, b.vcnt, l, U, st, sh->zflag_dev);
            FHS_TMARK(tm, KID_KS_INTT, 0, st);
        });
        e = hipMemcpyAsync(sh->zflag_host, sh->zflag_dev, sizeof(unsigned), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        if (*(volatile unsigned*)sh->zflag_host) {   // a zero digit coefficient: SEAL's own per-rotation path
            ++sh->fallback;
            return launch_keyswitch(T, items_host, R, uniq_host, U, l, ws, ws_bytes, items_dev, sg, st, tm, nullptr);
        }
        ++sh->hoisted;
        FHS_DISPATCH_LOGN(T.logN, {
            FHS_TMARK(tm, KID_MODUP, 1, st);
            launch_modup<LOGN>(T, uq, b.acoef, b.vcnt, b.ext, l, U, st);
            FHS_TMARK(tm, KID_MODUP, 0, st);
            FHS_TMARK(tm, KID_KS_IP, 1, st);
            hipLaunchKernelGGL(k_ks_ip, dim3(xcd_grid(l + T.P, R * (int)(T.N >> 8))), dim3(256), 0, st, T, it, uq, b.ext,
                               b.acc, l, R, 0);
            FHS_TMARK(tm, KID_KS_IP, 0, st);
            FHS_TMARK(tm, KID_SPECIAL_INTT, 1, st);
            FHS_NTT_LAUNCH(k_ks_special_intt, T.P * 2 * R, dim3(T.P, 2, R), st, T, b.acc, b.ycoef, l, R);
            FHS_TMARK(tm, KID_SPECIAL_INTT, 0, st);
            e = launch_moddown<LOGN>(T, it, b.acc, b.ycoef, l, R, st, tm);
        });
        if (e != hipSuccess) return e;
        return hipGetLastError();
    }
    if (T.ks_seal) {
        sitems.assign(items_host, items_host + R);
        suniq.resize(R);
        u64* perm = ws + ks_core_bytes(T, R, R, l) / 8;
        seal_rewrite(T, sitems.data(), R, suniq.data(), l, perm);
        hipError_t pe = seal_permute(T, items_host, R, l, perm, st);
        if (pe != hipSuccess) return pe;
        items_host = sitems.data();
        uniq_host = suniq.data();
        U = R;
    }
    hipError_t e = upload_items(items_host, R, uniq_host, U, items_dev, sg, &it, &uq);
    if (e != hipSuccess) return e;
    hipError_t me = hipSuccess;
    FHS_DISPATCH_LOGN(T.logN, {
        u64 *acc, *ycoef;
        ks_front<LOGN>(T, it, uq, R, U, l, ws, st, tm, &acc, &ycoef);
        me = launch_moddown<LOGN>(T, it, acc, ycoef, l, R, st, tm);
    });
    if (me != hipSuccess) return me;
    return hipGetLastError();
}

// ============================================================================ BSGS
// inner[g] = sum_{b < G, gG+b < D} baby[b] (.) pts[gG+b]        (bg:465-476)
// Block = 4 waves sharing one 64-coefficient slice of limb i: the slice of all G baby steps
// (both components) is staged once in LDS, each wave then streams the diagonals of its giant
// groups (g = wave, wave+4, ...) from HBM with lazy 128-bit accumulation.
// diagonal words of plaintext `p` (limb base p + i N) at this lane's coefficients: a non-temporal buffer
// load (the limb offset and the slice offset n0 are wave-uniform: descriptor base and soffset), so no
// 64-bit address arithmetic and no flat load (which would also wait on the LDS counter)
// TL > 0: a compact diagonal (the periodic plaintexts' shadow, fhs_host.hip encode_rows_dev): word e >> TL of the
// limb holds dense word e, so a lane's VEC = 2 coefficients share one 8-byte word (voff, soff already shifted)
template <int VEC, int TL = 0>
__device__ __forceinline__ void ld_diag(const u64* limb, int voff, int soff, u64* out) {
    const __amdgpu_buffer_rsrc_t r = brsrc(limb, 0x7ffffff0);
    if constexpr (TL > 0) {
        static_assert(VEC == 2, "compact diagonals: two coefficients per lane");
        out[0] = out[1] = __builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, kBufNT));
    } else if constexpr (VEC == 2) {
        const auto t = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, kBufNT);
        out[0] = ((u64)t[1] << 32) | t[0];
        out[1] = ((u64)t[3] << 32) | t[2];
    } else {
        out[0] = __builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, kBufNT));
    }
}
// FOLD: products per Acc3 before its fold into the 128-bit sums -- 8 for any prime < 2^60, 16 when every
// prime is < 2^59 (T.max_qbits <= 59): then the split-30 high halves are < 2^29, so L and M gain < 2^60
// and H < 2^58 per product and 16 products stay below 2^64
// Baby-step window (G > 64: the slice of every baby step no longer fits LDS): this launch covers baby steps
// [b0, b0 + Gw) -- `baby` and `pts` arrive offset by b0 (pts keeps its row stride G), D is the caller's D - b0 --
// and ACC adds its sums to the previous windows' reduced inner products (one extra read of `inner` per window).
// TL > 0: compact diagonals (ld_diag) -- the same products, 2^-TL of the diagonal bytes
template <int VEC, int WAVES, int FOLD, bool ACC, int TL = 0>
__global__ void __launch_bounds__(64 * WAVES) k_bsgs_inner(DevTables T, const u64* const* __restrict__ baby,
                                                    const u64* const* __restrict__ pts, int G, int Gw, int g0, int g1,
                                                    int D, int l, u64* __restrict__ inner) {
    extern __shared__ __attribute__((aligned(16))) u64 sb[];   // [Gw][2][W], split-30 packed
    constexpr int W = 64 * VEC;
    const int N = T.N;
    const int i = blockIdx.y, n0 = blockIdx.x * W, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: the diagonal pointers come by scalar loads
    const size_t S = (size_t)l * N;
    const size_t off = (size_t)i * N + n0 + lane * VEC;
    const size_t dlimb = (size_t)i * (N >> TL);                   // limb i of a (compact) diagonal
    const int dvoff = ((lane * VEC) >> TL) * 8, dsoff = (n0 >> TL) * 8;
    // Rolling refill: within a giant group a wave keeps 8 diagonal loads in flight at every moment --
    // slot u is reloaded with the next batch's diagonal u as soon as its product is formed, so the loads
    // do not drain while the wave computes (they drain once per group, at its tail and stores).  The first
    // batch is requested before the baby-step slice is staged, so the staging and its barrier overlap the
    // stream too.
    u64 p[8][VEC];
    const int gcur = g0 + wave;
    auto full_batches = [&](int g) { return g < g1 ? max(0, min(Gw, D - g * G)) / 8 : 0; };
    int gf = gcur;   // the wave's first group with a full batch
    while (gf < g1 && full_batches(gf) == 0) gf += WAVES;
    if (gf < g1) {
        const u64* const* pg0 = pts + (size_t)gf * G;
#pragma unroll
        for (int u = 0; u < 8; ++u) ld_diag<VEC, TL>(pg0[u] + dlimb, dvoff, dsoff, p[u]);
    }
    for (int idx = tid; idx < Gw * 2 * W; idx += 64 * WAVES) {
        const int b = idx / (2 * W), comp = (idx / W) & 1, c = idx % W;
        sb[idx] = pack30(baby[b][comp * S + (size_t)i * N + n0 + c]);
    }
    __syncthreads();
    const RedU R = redu(PK(T, i));
    for (int g = gcur; g < g1; g += WAVES) {
        const int bmax = min(Gw, D - g * G);
        if (bmax <= 0) continue;
        u128 c0[VEC], c1[VEC];
        Acc3 a0[VEC], a1[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
            c0[v] = c1[v] = u128{0, 0};
            a0[v] = a1[v] = Acc3{0, 0, 0};
        }
        const u64* const* pg = pts + (size_t)g * G;
        const int nb = bmax / 8;
        // the wave's next group with a full batch (its first batch is what the last batch here refills)
        int gn = g + WAVES;
        while (gn < g1 && full_batches(gn) == 0) gn += WAVES;
        int b = 0;
        for (int bi = 0; bi < nb; ++bi, b += 8) {
            // slot u's refill: this group's next batch (none after the last: the tail, folds and stores
            // below run with the slots dead, and the next group's first batch is requested after them).
            // FOLD == 8 (a prime >= 2^59) keeps batch-at-a-time loads: its extra folds leave no registers
            // for live refills (spills)
            constexpr bool ROLL = FOLD == 16;
            if (!ROLL && bi > 0) {
#pragma unroll
                for (int u = 0; u < 8; ++u) ld_diag<VEC, TL>(pg[b + u] + dlimb, dvoff, dsoff, p[u]);
            }
            const u64* const* nxt = ROLL && bi + 1 < nb ? pg + b + 8 : nullptr;
#pragma unroll
            for (int h = 0; h < 8; h += 4) {   // half a batch at a time: products, then that half's refill
#pragma unroll
                for (int u = h; u < h + 4; ++u)
#pragma unroll
                    for (int v = 0; v < VEC; ++v) {
                        const Split30 y = split30(p[u][v]);
                        acc3_mac(a0[v], unpack30(sb[((b + u) * 2 + 0) * W + lane * VEC + v]), y);
                        acc3_mac(a1[v], unpack30(sb[((b + u) * 2 + 1) * W + lane * VEC + v]), y);
                    }
                if (h == 4 && (FOLD == 8 || (b & 15) == 8)) {   // fold after every FOLD products (b is the
#pragma unroll                                                       // batch's first index), before the refill
                    for (int v = 0; v < VEC; ++v) {
                        acc3_fold(c0[v], a0[v]);
                        acc3_fold(c1[v], a1[v]);
                    }
                }
                if (nxt) {
#pragma unroll
                    for (int u = h; u < h + 4; ++u) ld_diag<VEC, TL>(nxt[u] + dlimb, dvoff, dsoff, p[u]);
                }
            }
        }
        for (; b < bmax; ++b) {   // < 8 left: at most FOLD - 1 products since the last fold
            u64 q1[VEC];
            ld_diag<VEC, TL>(pg[b] + dlimb, dvoff, dsoff, q1);
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
                const Split30 y = split30(q1[v]);
                acc3_mac(a0[v], unpack30(sb[(b * 2 + 0) * W + lane * VEC + v]), y);
                acc3_mac(a1[v], unpack30(sb[(b * 2 + 1) * W + lane * VEC + v]), y);
            }
        }
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
            acc3_fold(c0[v], a0[v]);
            acc3_fold(c1[v], a1[v]);
        }
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
            u64* o0 = inner + (size_t)g * 2 * S + off + v;
            u64 r0 = reduce128(c0[v].lo, c0[v].hi, R), r1 = reduce128(c1[v].lo, c1[v].hi, R);
            if constexpr (ACC) {
                r0 = addmod(r0, o0[0], R.q);
                r1 = addmod(r1, o0[S], R.q);
            }
            o0[0] = r0;
            o0[S] = r1;
        }
        if (gn < g1) {
            const u64* const* pgn = pts + (size_t)gn * G;
#pragma unroll
            for (int u = 0; u < 8; ++u) ld_diag<VEC, TL>(pgn[u] + dlimb, dvoff, dsoff, p[u]);
        }
    }
}

// Giant steps.  Exactness: every output limb is a sum of exact residues, so
//   sum_r ModDown(acc_r) = (sum_r acc_r - NTT(sum_r conv(y_r))) * P^-1   (mod q_i)
// is bit-identical to rotating and adding one giant step at a time (bg:478-483).
// base_c = (sum_r acc_r,c) P^-1 + [c==0] sum_r galois_r(inner_r.c0) + inner_0.c ;  convsum_c = sum_r conv(y_r,c)
// Grid (N / 256, 2 components, ceil(l / FHS_GSUM_ICH) target-limb chunks).  The conversion is linear
// in the rotations, so sum_r sum_k y_rk hat_ki = sum_k hat_ki (sum_r y_rk): each thread sums its
// coefficient's R P special values once as exact 128-bit integers (< R 2^60) and reduces those P sums
// into each target limb of its chunk -- the same residues as converting rotation by rotation, with
// the special values read once per chunk instead of once per target limb.
#ifndef FHS_GSUM_ICH
#define FHS_GSUM_ICH 4
#endif
__global__ void __launch_bounds__(256) k_giant_sum(DevTables T, const u64* bpart, const u64* ycoef, const u64* inner0,
                                                   u64* base, u64* convsum, int l, int R) {
    const int N = T.N, P_ = T.P, E = l + P_;
    const int n = blockIdx.x * blockDim.x + threadIdx.x, comp = blockIdx.y;
    if (n >= N) return;
    const int i0 = blockIdx.z * FHS_GSUM_ICH, i1 = min(i0 + FHS_GSUM_ICH, l);
    const size_t S = (size_t)l * N;
    constexpr int PMAX = 8;   // special primes per context (context_create limit)
    u64 ylo[PMAX], yhi[PMAX];
#pragma unroll
    for (int k = 0; k < PMAX; ++k) ylo[k] = yhi[k] = 0;
    for (int r = 0; r < R; ++r) {
        const u64* y = ycoef + ((size_t)r * 2 + comp) * P_ * N + n;
#pragma unroll
        for (int k = 0; k < PMAX; ++k) {
            if (k < P_) {
                const u64 v = y[(size_t)k * N];
                ylo[k] += v;
                yhi[k] += ylo[k] < v;
            }
        }
    }
    for (int i = i0; i < i1; ++i) {
        const PrimeK& P = PK(T, i);
        const u64 q = P.q;
        u128 cs = {0, 0};
#pragma unroll
        for (int k = 0; k < PMAX; ++k)
            if (k < P_) mac128(cs, reduce128(ylo[k], yhi[k], P), T.md_hat[(size_t)k * T.L0 + i]);
        if (T.ks_seal) {   // SEAL rounding: each of the R conversions carries - floor(p/2) mod q_i
            u128 h = {0, 0};
            mac128(h, (u64)R, T.md_pinv[3 * T.L0 + i]);
            const u64 rh = reduce128(h.lo, h.hi, P);
            cs.lo = reduce128(cs.lo, cs.hi, P);
            cs.hi = 0;
            cs.lo = submod(cs.lo, rh, q);
        }
        u64 cv = reduce128(cs.lo, cs.hi, P);
        const size_t idx = (size_t)comp * S + (size_t)i * N + n;
        const u64 bv = addmod(bpart[((size_t)comp * E + i) * N + n], inner0[idx], q);
        convsum[idx] = cv;
        base[idx] = bv;
    }
}
template <int LOGN, bool H = ntt_half<LOGN>()>
__global__ void __launch_bounds__((ntt_threads<LOGN, H>())) k_giant_final(DevTables T, const u64* base, const u64* convsum,
                                                                     u64* out, int l) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN, H>()];
    const int i = blockIdx.x, comp = blockIdx.y;
    const PrimeK& P = PK(T, i);
    const RedU RU = redu(P);
    const size_t off = ((size_t)comp * l + i) * N;
    const u64 pinv = T.md_pinv[2 * i], pinv_s = T.md_pinv[2 * i + 1], q = RU.q;
    fwd_limb<LOGN, FHS_NTT_RL, H>(lds, threadIdx.x, T.tw_fwd + (size_t)i * N * 2, RU,
                               [&](int e) { return convsum[off + e]; },
                               [&](int e, u64 v) { out[off + e] = submod(base[off + e], shoup(v, pinv, pinv_s, q), q); });
}

// ---- key-switch stages of the BSGS giant steps
template <int LOGN>
static void ks_modup_stage(const DevTables& T, const u64* const* uniq, int U, int l, const KsBufs& b, hipStream_t st,
                           const KTimer* tm) {
    FHS_TMARK(tm, KID_KS_INTT, 1, st);
    if (ks_intt_half<LOGN>(l * U))
        hipLaunchKernelGGL((k_ks_intt_h<LOGN>), dim3(l * U), dim3((1 << LOGN) / 32), 0, st, T, uniq, b.acoef, l, U);
    else
        hipLaunchKernelGGL((k_ks_intt<LOGN>), dim3(l * U), dim3((1 << LOGN) / 16), 0, st, T, uniq, b.acoef, l, U);
    launch_centered(T, b.acoef, b.vcnt, l, U, st);
    FHS_TMARK(tm, KID_KS_INTT, 0, st);
    FHS_TMARK(tm, KID_MODUP, 1, st);
    launch_modup<LOGN>(T, uniq, b.acoef, b.vcnt, b.ext, l, U, st);
    FHS_TMARK(tm, KID_MODUP, 0, st);
}
template <int LOGN>
static void giant_ip_stage(const DevTables& T, const KsItem* it, const u64* const* uniq, int R, int l, const KsBufs& b,
                           hipStream_t st, const KTimer* tm) {
    const int NB = T.N >> 8;
    FHS_TMARK(tm, KID_KS_IP, 1, st);
    hipLaunchKernelGGL(k_ks_ip, dim3(T.P * R * NB), dim3(256), 0, st, T, it, uniq, b.ext, b.acc, l, R, l);
    hipLaunchKernelGGL(k_ks_ip_sum, dim3(xcd_grid(l, NB)), dim3(256), 0, st, T, it, uniq, b.ext, b.acc, l, R);
    FHS_TMARK(tm, KID_KS_IP, 0, st);
    FHS_TMARK(tm, KID_SPECIAL_INTT, 1, st);
    FHS_NTT_LAUNCH(k_ks_special_intt, T.P * 2 * R, dim3(T.P, 2, R), st, T, b.acc, b.ycoef, l, R);
    FHS_TMARK(tm, KID_SPECIAL_INTT, 0, st);
}

// core key-switch workspace of the R giant rotations, then base | convsum (2 ciphertexts)
size_t bsgs_workspace_bytes(const DevTables& T, int R, int l) {
    return keyswitch_workspace_bytes(T, R, R, l) + 8 * (size_t)T.N * 4 * l;
}

constexpr int kInnerWindow = 64;   // baby steps per k_bsgs_inner launch: [64][2][128] words = 128 KiB of LDS
// compact diagonals (tlog 1..3; 59-bit chains: the FOLD = 16 kernels)
template <int VEC, int WAVES, int TL>
static void launch_inner_compact(dim3 grid, dim3 block, size_t lds, hipStream_t st, const DevTables& T,
                                 const u64* const* baby, const u64* const* pts, int G, int Gw, int g0, int g1, int Dw,
                                 int l, u64* inner, bool acc) {
    if (acc)
        hipLaunchKernelGGL((k_bsgs_inner<VEC, WAVES, 16, true, TL>), grid, block, lds, st, T, baby, pts, G, Gw, g0, g1,
                           Dw, l, inner);
    else
        hipLaunchKernelGGL((k_bsgs_inner<VEC, WAVES, 16, false, TL>), grid, block, lds, st, T, baby, pts, G, Gw, g0, g1,
                           Dw, l, inner);
}
template <int VEC, int WAVES>
static hipError_t launch_inner_t(const DevTables& T, const u64* const* baby, const u64* const* pts, int G, int g0,
                                 int g1, int D, int l, u64* inner, hipStream_t st, int ptl) {
    constexpr int W = 64 * VEC;
    static bool attr = false;
    if (!attr) {   // dynamic LDS above 64 KiB must be opted into
        for (const void* k : {reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 8, false>),
                              reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 16, false>),
                              reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 8, true>),
                              reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 16, true>),
                              reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 16, false, 1>),
                              reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 16, true, 1>),
                              reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 16, false, 2>),
                              reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 16, true, 2>),
                              reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 16, false, 3>),
                              reinterpret_cast<const void*>(&k_bsgs_inner<VEC, WAVES, 16, true, 3>)}) {
            hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)(kInnerWindow * 2 * W * 8));
            if (e != hipSuccess) return e;
        }
        attr = true;
    }
    if (ptl < 0 || ptl > 3 || (ptl > 0 && (T.max_qbits > 59 || VEC != 2))) return hipErrorInvalidValue;
    // G <= 64: one launch over every baby step; else windows of 64, each adding to the previous ones' sums
    for (int b0 = 0; b0 < G; b0 += kInnerWindow) {
        const int Gw = std::min(kInnerWindow, G - b0), Dw = D - b0;
        const size_t lds = (size_t)Gw * 2 * W * 8;
        const dim3 grid(T.N / W, l), block(64 * WAVES);
        if (ptl == 1) {
            launch_inner_compact<VEC, WAVES, 1>(grid, block, lds, st, T, baby + b0, pts + b0, G, Gw, g0, g1, Dw, l, inner,
                                                b0 > 0);
        } else if (ptl == 2) {
            launch_inner_compact<VEC, WAVES, 2>(grid, block, lds, st, T, baby + b0, pts + b0, G, Gw, g0, g1, Dw, l, inner,
                                                b0 > 0);
        } else if (ptl == 3) {
            launch_inner_compact<VEC, WAVES, 3>(grid, block, lds, st, T, baby + b0, pts + b0, G, Gw, g0, g1, Dw, l, inner,
                                                b0 > 0);
        } else if (T.max_qbits <= 59) {
            if (b0)
                hipLaunchKernelGGL((k_bsgs_inner<VEC, WAVES, 16, true>), grid, block, lds, st, T, baby + b0, pts + b0, G, Gw,
                                   g0, g1, Dw, l, inner);
            else
                hipLaunchKernelGGL((k_bsgs_inner<VEC, WAVES, 16, false>), grid, block, lds, st, T, baby, pts, G, Gw, g0, g1,
                                   Dw, l, inner);
        } else {
            if (b0)
                hipLaunchKernelGGL((k_bsgs_inner<VEC, WAVES, 8, true>), grid, block, lds, st, T, baby + b0, pts + b0, G, Gw,
                                   g0, g1, Dw, l, inner);
            else
                hipLaunchKernelGGL((k_bsgs_inner<VEC, WAVES, 8, false>), grid, block, lds, st, T, baby, pts, G, Gw, g0, g1,
                                   Dw, l, inner);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_bsgs_inner(const DevTables& T, const u64* const* baby_dev, const u64* const* pts_dev, int G, int g0,
                             int g1, int D, int l, u64* inner, hipStream_t st, int ptl) {
    if (T.N % 128 || G < 1) return hipErrorInvalidValue;
    return launch_inner_t<FHS_INNER_VEC, FHS_INNER_WAVES>(T, baby_dev, pts_dev, G, g0, g1, D, l, inner, st, ptl);
}

// Hadamard (every giant group's inner product; skipped when pts_dev is null and `inner` already holds
// them), then the giant steps: INTT + centred ModUp + NTT of
// the B - 1 inner products (one ModUp each), key inner products with the automorphism applied on the
// fly, special-limb INTT, the giant sum before ModDown (k_giant_sum) and one ModDown NTT per output
// limb (k_giant_final).  One stream, serial: the limbs are those of the reference loop bg:464-485.
hipError_t launch_bsgs(const DevTables& T, const u64* const* baby_dev, const u64* const* pts_dev, int G, int B, int D,
                       int l, const u64* const* keys_host, const u64* const* akeys_host, const u64* giant_elts, u64* inner,
                       u64* out, u64* ws, size_t ws_bytes, void* items_dev, const Stager& sg, hipStream_t st,
                       const KTimer* tm, int ptl) {
    const int R = B - 1;
    const size_t N = T.N, S = (size_t)l * N;
    if (T.N % 128 || G < 1 || R > 512) return hipErrorInvalidValue;
    if (R > 0 && bsgs_workspace_bytes(T, R, l) > ws_bytes) return hipErrorInvalidValue;
    KsItem items[512];
    const u64* uniq[512];
    for (int r = 0; r < R; ++r) {
        const int g = r + 1;
        const u64* ct = inner + (size_t)g * 2 * S;
        u64 elt = 1;
        if (giant_elts) elt = giant_elts[g];
        else
            for (int s2 = 0; s2 < g * G; ++s2) elt = (elt * 5) & (2 * N - 1);   // 5^(g G) mod 2N
        items[r] = KsItem{ct + S, ct, nullptr, keys_host[g], nullptr, nullptr, elt, (u64)r,
                          akeys_host ? akeys_host[g] : nullptr};
        uniq[r] = ct + S;
    }
    // SEAL convention: each giant input is automorphed before its decomposition (the permutations
    // are enqueued after the Hadamard that produces the inputs)
    std::vector<KsItem> seal_orig;
    u64* seal_perm = ws + ks_core_bytes(T, R, R, l) / 8;
    if (T.ks_seal && R > 0) {
        seal_orig.assign(items, items + R);
        seal_rewrite(T, items, R, uniq, l, seal_perm);
    }
    const KsItem* it = nullptr;
    const u64* const* uq = nullptr;
    if (R > 0) {
        hipError_t e = upload_items(items, R, uniq, R, items_dev, sg, &it, &uq);
        if (e != hipSuccess) return e;
    }
    hipError_t he = hipSuccess;
    if (pts_dev) {   // null: the B inner products are already in `inner` (giant steps only)
        FHS_TMARK(tm, KID_BSGS_INNER, 1, st);
        he = launch_inner_t<FHS_INNER_VEC, FHS_INNER_WAVES>(T, baby_dev, pts_dev, G, 0, B, D, l, inner, st, ptl);
        FHS_TMARK(tm, KID_BSGS_INNER, 0, st);
        if (he != hipSuccess) return he;
    }
    if (R <= 0) return hipMemcpyAsync(out, inner, 8 * 2 * S, hipMemcpyDeviceToDevice, st);
    if (!seal_orig.empty()) {
        he = seal_permute(T, seal_orig.data(), R, l, seal_perm, st);
        if (he != hipSuccess) return he;
    }
    u64* base = ws + keyswitch_workspace_bytes(T, R, R, l) / 8;
    u64* convsum = base + 2 * S;
    FHS_DISPATCH_LOGN(T.logN, {
        const KsBufs b = ks_carve(T, ws, R, R, l);
        ks_modup_stage<LOGN>(T, uq, R, l, b, st, tm);
        giant_ip_stage<LOGN>(T, it, uq, R, l, b, st, tm);
        FHS_TMARK(tm, KID_GIANT_SUM, 1, st);
        hipLaunchKernelGGL(k_giant_sum, dim3((T.N + 255) / 256, 2, (l + FHS_GSUM_ICH - 1) / FHS_GSUM_ICH), dim3(256), 0,
                           st, T, b.acc, b.ycoef, inner, base, convsum, l, R);
        FHS_TMARK(tm, KID_GIANT_SUM, 0, st);
        FHS_TMARK(tm, KID_GIANT_FINAL, 1, st);
        FHS_NTT_LAUNCH(k_giant_final, l * 2, dim3(l, 2), st, T, base, convsum, out, l);
        FHS_TMARK(tm, KID_GIANT_FINAL, 0, st);
    });
    return hipGetLastError();
}



// ============================================================================ sampling / keys
__device__ __forceinline__ u64 rnd_testdata(u64 key, u64 ctr) { return sm64(key ^ sm64(ctr ^ 0xD1B54A32D192ED03ULL)); }

// SAMPLE_UNIFORM: uniform mod q_i in the NTT domain from 128 PRF bits (block i N + n, bias < 2^-67);
// SAMPLE_TERNARY / SAMPLE_CBD: one small value per coefficient (block n), replicated over the limbs
// in coefficient form (the caller runs the forward NTT); SAMPLE_SEEDED: public a_j expansion of the
// seed `sid`; SAMPLE_TESTDATA: SplitMix64 uniform (random_plaintexts, not secret)
// Polynomial blockIdx.y of a batch: stream sid + y sid_step, written to outs[y] (outs null: out + y l N).
__global__ void k_sample(DevTables T, int mode, PrfKey K, u64 sid, u64* out, int l, u64 sid_step, u64* const* outs) {
    const int N = T.N;
    const size_t S = (size_t)l * N;
    sid += blockIdx.y * sid_step;
    out = outs ? outs[blockIdx.y] : out + blockIdx.y * S;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(idx / N), n = (int)(idx % N);
        const PrimeK& P = PK(T, i);
        u64 v;
        if (mode == SAMPLE_UNIFORM) {
            u64 hi, lo;
            prf128(K, sid, (uint32_t)idx, hi, lo);
            v = reduce128(lo, hi, P);
        } else if (mode == SAMPLE_SEEDED) {
            v = seeded_uniform_x(sid + seeded_ctr_mix(i, n), P.q, 64 - __clzll(P.q));
        } else if (mode == SAMPLE_TESTDATA) {
            const u64 ctr = 2 * ((u64)i * N + n);
            v = reduce128(rnd_testdata(sid, ctr + 1), rnd_testdata(sid, ctr), P);
        } else {
            u64 r, unused;
            prf128(K, sid, (uint32_t)n, r, unused);
            long long s;
            if (mode == SAMPLE_TERNARY) {
                const u64 t = r % 3;
                s = t == 2 ? -1 : (long long)t;
            } else {
                s = (long long)__popcll(r & 0x1FFFFFULL) - (long long)__popcll((r >> 21) & 0x1FFFFFULL);
            }
            v = s >= 0 ? (u64)s : P.q - (u64)(-s);
        }
        out[idx] = v;
    }
}
hipError_t launch_sample(const DevTables& T, int mode, const PrfKey& K, u64 sid, u64* out, int l, hipStream_t st,
                         int npoly, u64 sid_step, u64* const* outs_dev) {
    if (npoly < 1) return hipSuccess;
    const int g1 = eltwise_grid((size_t)l * T.N) / npoly, gx = g1 > 0 ? g1 : 1;
    hipLaunchKernelGGL(k_sample, dim3(gx, npoly), dim3(256), 0, st, T, mode, K, sid, out, l, sid_step, outs_dev);
    return hipGetLastError();
}

// key_j[0] = e - a s + [i in digit j] (P mod q_i) s_new ; key_j[1] = a (already in place)
__global__ void k_swk(DevTables T, u64* b_out, const u64* a, const u64* e, const u64* s, const u64* snew, int j) {
    const int N = T.N, K = T.K;
    const size_t S = (size_t)K * N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(idx / N);
        const PrimeK& P = PK(T, i);
        u64 v = submod(e[idx], mulmod(a[idx], s[idx], P), P.q);
        if (i < T.L0 && i / T.P == j) {
            const u64 pm = T.md_pinv[2 * T.L0 + i];   // P mod q_i stored after the inverses
            v = addmod(v, mulmod(pm, snew[idx], P), P.q);
        }
        b_out[idx] = v;
    }
}
hipError_t launch_switch_key_assemble(const DevTables& T, u64* b_out, const u64* a, const u64* e_ntt, const u64* s_ntt,
                                      const u64* snew_ntt, int digit, hipStream_t st) {
    hipLaunchKernelGGL(k_swk, dim3(eltwise_grid((size_t)T.K * T.N)), dim3(256), 0, st, T, b_out, a, e_ntt, s_ntt,
                       snew_ntt, digit);
    return hipGetLastError();
}

// mode 0 (symmetric): c0 = e0 - c1 s + pt (c1 holds the uniform a); mode 1 (public key):
// c0 = u pk0 + e0 + pt, c1 = u pk1 + e1.  pk limbs are at the top level (stride L0 N).
__global__ void k_encrypt(DevTables T, int mode, u64* c0, u64* c1, const u64* s_or_pk0, const u64* pk1, const u64* u,
                          const u64* e0, const u64* e1, const u64* pt, int l) {
    const int N = T.N;
    const size_t S = (size_t)l * N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(idx / N);
        const PrimeK& P = PK(T, i);
        const u64 q = P.q;
        const u64 m = pt ? pt[idx] : 0;
        if (mode == 0) {
            c0[idx] = addmod(submod(e0[idx], mulmod(c1[idx], s_or_pk0[idx], P), q), m, q);
        } else {
            c0[idx] = addmod(addmod(mulmod(u[idx], s_or_pk0[idx], P), e0[idx], q), m, q);
            c1[idx] = addmod(mulmod(u[idx], pk1[idx], P), e1[idx], q);
        }
    }
}
// ---- batched symmetric encryption (launch_encrypt_sym_batch): the error's small value drawn once per
// coefficient (k_sample did it once per coefficient AND limb: the same PRF block l times), its forward NTT
// reading those values straight into the transform, and the mask a drawn inside the combine -- three
// launches for the whole batch, the same values as k_sample + NTT + k_encrypt per ciphertext.
__global__ void k_sample_small(int mode, PrfKey K, u64 sid, u64 sid_step, int N, signed char* out) {
    sid += blockIdx.y * sid_step;
    out += (size_t)blockIdx.y * N;
    for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < N; n += gridDim.x * blockDim.x) {
        u64 r, unused;
        prf128(K, sid, (uint32_t)n, r, unused);
        int v;
        if (mode == SAMPLE_TERNARY) {
            const u64 t = r % 3;
            v = t == 2 ? -1 : (int)t;
        } else {
            v = __popcll(r & 0x1FFFFFULL) - __popcll((r >> 21) & 0x1FFFFFULL);
        }
        out[n] = (signed char)v;
    }
}
template <int LOGN>
__global__ void __launch_bounds__(ntt_threads<LOGN>()) k_ntt_fwd_small(DevTables T, const signed char* small, u64* out,
                                                                      int limbs) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN>()];
    const int b = blockIdx.x;
    const RedU R = redu(PK(T, b));
    const signed char* sm = small + (size_t)blockIdx.y * N;
    u64* p = out + ((size_t)blockIdx.y * limbs + b) * N;
    const u64 q = R.q;
    fwd_limb<LOGN, FHS_NTT_RL>(lds, threadIdx.x, T.tw_fwd + (size_t)b * N * 2, R,
                               [&](int e) { const int v = sm[e]; return v >= 0 ? (u64)v : q - (u64)(-v); },
                               [&](int e, u64 v) { p[e] = v; });
}
// The limb's reduction of a 64-bit integer: on the pseudo-Mersenne fold one fold and one subtraction when
// 2^b + (2^(64-b) - 1) d < 2q (every 59-bit chain: d < 2^27), else reduce64's three folds or Barrett -- the
// same canonical residue either way.  The encoder's NTT loads reduce one rounded coefficient per element per
// limb with it (k_ntt_fwd_from_dbl: ~12 % of the N = 32768 encode's VALU instructions were this reduction).
struct DblMod {
    const PrimeK* P;
    const u64* pow2;   // 2^k mod q of this limb (DevTables::pow2 row)
    u64 q, mask;
    unsigned b, d;
    bool fold1;
};
__device__ __forceinline__ DblMod dbl_mod_of(const DevTables& T, int i) {
    const PrimeK& P = PK(T, i);
    const u64 pm = P.pm, q = P.q;   // i may vary per lane (k_encode_reduce): no readfirstlane
    const unsigned b = (unsigned)(pm & 127), d = (unsigned)((pm >> 8) & 0xFFFFFFFFu);
    const bool fold1 = b != 0 && ((u64)d << (64 - b)) + (1ull << b) < 2 * q;
    return DblMod{&P, T.pow2 + (size_t)i * 1088, q, b ? (1ull << b) - 1 : 0, b, d, fold1};
}
__device__ __forceinline__ u64 dbl_mod(const DblMod& M, double v) {
    const bool neg = v < 0;
    const double a = neg ? -v : v;
    u64 r;
    if (a < 9.2e18) {
        const u64 x = (u64)a;
        r = M.fold1 ? csub((x & M.mask) + mul32w((uint32_t)(x >> M.b), M.d), M.q) : reduce64(x, *M.P);
    } else {
        const PrimeK& P = *M.P;
        const u64 bits = (u64)__double_as_longlong(a);
        const int ex = (int)((bits >> 52) & 0x7FF) - 1075;
        const u64 mant = (bits & ((1ULL << 52) - 1)) | (1ULL << 52);
        r = mulmod(reduce64(mant, P), M.pow2[ex], P);
    }
    return (neg && r) ? M.q - r : r;
}
__device__ __forceinline__ u64 dbl_mod(const DevTables& T, double d, int i) { return dbl_mod(dbl_mod_of(T, i), d); }
// The encoder's forward NTTs start from inputs below 2q (a reduced coefficient, plus a small error when fused
// with encryption), not the 4q the context's lazy bit assumes: every stage adds < 2q, so 15 lazy stages stay
// below 2q + 30 q = 32 q <= 2^64 for q < 2^59 -- lazy at N = 32768 too, where the 4q bound (34 q) is not, with
// the one-fold canonicalisation (pm_fold64 via fwd_canon) valid under DblMod::fold1.  Same canonical values.
__device__ __forceinline__ RedU enc_lazy(RedU R, const DblMod& M) {
    if (M.fold1 && R.q < (1ull << 59)) R.lazy = true;
    return R;
}
// encode + encrypt fused: NTT(m + e) of the rounded message coefficients (coef, doubles; k_encode's
// coef_out, reduced per limb by dbl_mod as k_ntt_fwd_from_dbl does) plus the small error -- the NTT is
// linear and its outputs canonical, so the limbs equal NTT(m) + NTT(e) mod q, i.e. encode then encrypt
template <int LOGN>
__global__ void __launch_bounds__(ntt_threads<LOGN>()) k_ntt_fwd_msg_err(DevTables T, const double* coef,
                                                                        const signed char* small, u64* out, int limbs) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN>()];
    const int b = blockIdx.x;
    const RedU R = redu(PK(T, b));
    const double* cf = coef + (size_t)blockIdx.y * N;
    const signed char* sm = small + (size_t)blockIdx.y * N;
    u64* p = out + ((size_t)blockIdx.y * limbs + b) * N;
    const u64 q = R.q;
    const DblMod M = dbl_mod_of(T, b);
    fwd_limb<LOGN, FHS_NTT_RL>(lds, threadIdx.x, T.tw_fwd + (size_t)b * N * 2, enc_lazy(R, M),
                               [&](int e) {   // < 2q: inside the forward NTT's input bound
                                   const int v = sm[e];
                                   return dbl_mod(M, cf[e]) + (v >= 0 ? (u64)v : q - (u64)(-v));
                               },
                               [&](int e, u64 v) { p[e] = v; });
}
// ciphertext y of the batch: c1 = the uniform mask (k_sample SAMPLE_UNIFORM of stream sid + y sid_step),
// c0 = e - c1 s + m (k_encrypt mode 0)
__global__ void k_encrypt_sym(DevTables T, PrfKey K, u64 sid, u64 sid_step, u64* const* cts, const u64* s,
                              const u64* eb, const u64* const* pts, int l) {
    const int N = T.N;
    const size_t S = (size_t)l * N;
    sid += blockIdx.y * sid_step;
    u64* c0 = cts[blockIdx.y];
    u64* c1 = c0 + S;
    const u64* e = eb + blockIdx.y * S;
    const u64* m = pts ? pts[blockIdx.y] : nullptr;   // null: the message is already inside eb
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const PrimeK& P = PK(T, (int)(idx / N));
        const u64 q = P.q;
        u64 hi, lo;
        prf128(K, sid, (uint32_t)idx, hi, lo);
        const u64 a = reduce128(lo, hi, P);
        c1[idx] = a;
        const u64 c = submod(e[idx], mulmod(a, s[idx], P), q);
        c0[idx] = m ? addmod(c, m[idx], q) : c;
    }
}
hipError_t launch_encrypt_sym_batch(const DevTables& T, const PrfKey& K, u64 sid_mask, u64 sid_err, u64 sid_step,
                                    u64* const* cts_dev, const u64* s, const u64* const* pts_dev, int count, int l,
                                    signed char* small, u64* eb, hipStream_t st, const double* coef) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sample_small, dim3((T.N + 255) / 256, count), dim3(256), 0, st, (int)SAMPLE_CBD, K, sid_err,
                       sid_step, T.N, small);
    FHS_DISPATCH_LOGN(T.logN, {
        if (coef)
            hipLaunchKernelGGL((k_ntt_fwd_msg_err<LOGN>), dim3(l, count), dim3(ntt_threads<LOGN>()), 0, st, T, coef,
                               static_cast<const signed char*>(small), eb, l);
        else
            hipLaunchKernelGGL((k_ntt_fwd_small<LOGN>), dim3(l, count), dim3(ntt_threads<LOGN>()), 0, st, T,
                               static_cast<const signed char*>(small), eb, l);
    });
    const int g1 = eltwise_grid((size_t)l * T.N) / count, gx = g1 > 0 ? g1 : 1;
    hipLaunchKernelGGL(k_encrypt_sym, dim3(gx, count), dim3(256), 0, st, T, K, sid_mask, sid_step, cts_dev, s,
                       static_cast<const u64*>(eb), pts_dev, l);
    return hipGetLastError();
}
hipError_t launch_encrypt_combine(const DevTables& T, int mode, u64* c0, u64* c1, const u64* s_or_pk0, const u64* pk1,
                                  const u64* u_ntt, const u64* e0, const u64* e1, const u64* pt, int l, hipStream_t st) {
    hipLaunchKernelGGL(k_encrypt, dim3(eltwise_grid((size_t)l * T.N)), dim3(256), 0, st, T, mode, c0, c1, s_or_pk0,
                       pk1, u_ntt, e0, e1, pt, l);
    return hipGetLastError();
}

// m = c0 + c1 s + c2 s^2 (s at key level: limb i of s is at i*N)
__global__ void k_decrypt(DevTables T, const u64* ct, int ncomp, const u64* s, u64* out, int l) {
    const int N = T.N;
    const size_t S = (size_t)l * N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(idx / N);
        const PrimeK& P = PK(T, i);
        const u64 sv = s[idx];
        u64 v = ct[idx], sp = sv;
        for (int k = 1; k < ncomp; ++k) {
            v = addmod(v, mulmod(ct[k * S + idx], sp, P), P.q);
            sp = mulmod(sp, sv, P);
        }
        out[idx] = v;
    }
}
// ciphertext blockIdx.y of cts (device pointer array, all with ncomp components at l limbs) -> out + y out_stride
__global__ void k_decrypt_many(DevTables T, const u64* const* cts, int ncomp, const u64* s, u64* out, size_t out_stride,
                               int l) {
    const int N = T.N;
    const size_t S = (size_t)l * N;
    const u64* ct = cts[blockIdx.y];
    u64* o = out + blockIdx.y * out_stride;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < S; idx += (size_t)gridDim.x * blockDim.x) {
        const PrimeK& P = PK(T, (int)(idx / N));
        const u64 sv = s[idx];
        u64 v = ct[idx], sp = sv;
        for (int k = 1; k < ncomp; ++k) {
            v = addmod(v, mulmod(ct[k * S + idx], sp, P), P.q);
            sp = mulmod(sp, sv, P);
        }
        o[idx] = v;
    }
}
hipError_t launch_decrypt_many(const DevTables& T, const u64* const* cts_dev, int count, int ncomp, const u64* s, u64* out,
                               size_t out_stride, int l, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    const int g1 = eltwise_grid((size_t)l * T.N) / count, gx = g1 > 0 ? g1 : 1;
    hipLaunchKernelGGL(k_decrypt_many, dim3(gx, count), dim3(256), 0, st, T, cts_dev, ncomp, s, out, out_stride, l);
    return hipGetLastError();
}
hipError_t launch_decrypt(const DevTables& T, const u64* ct, int ncomp, const u64* s, u64* out, int l, hipStream_t st) {
    hipLaunchKernelGGL(k_decrypt, dim3(eltwise_grid((size_t)l * T.N)), dim3(256), 0, st, T, ct, ncomp, s, out, l);
    return hipGetLastError();
}

// exact residue of integral doubles: coef [count][N] -> out [count][l][N] (coefficient form)
// exact residue of an integral double (any magnitude) mod prime i

__global__ void k_encode_reduce(DevTables T, const double* coef, int count, u64* out, int l) {
    const int N = T.N;
    const size_t total = (size_t)count * l * N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        const int n = (int)(idx % N);
        const size_t rest = idx / N;
        const int i = (int)(rest % l);
        const size_t v = rest / l;
        out[idx] = dbl_mod(T, coef[v * N + n], i);
    }
}

// ---- CKKS encoder (pb:138-156, bg:382, 423 encode_*_vector_batch) ----
// Canonical embedding inverse with an N/2-point FFT: z_j = m(zeta^{5^j}), 5^j = 4 s_j + 1, so
// c_k = m_k + i m_{k+N/2} = (2/N) zeta^-k sum_j z_j omega^{-s_j k}, omega = zeta^4.  One workgroup
// per vector: z_j is scattered to LDS slot rev(s_j) (bit-reversed input), a radix-2 DIT FFT runs in
// LDS (f64), then each coefficient is scaled, rounded (half away from zero, as the host decoder's
// inverse) and reduced exactly mod every limb's prime.  The NTT follows (k_ntt_fwd_ptrs).
// radix-2 DIT over n_pts = 2^log_pts points in LDS, bit-reversed in, natural out; twiddles of the full
// 2^logh-point transform (a sub-FFT uses the same ones).  Stages go in pairs through registers (each
// thread takes the quad i0, i0 + h, i0 + 2h, i0 + 3h and applies stage s then s + 1 to it -- the same
// butterflies in the same order, half the LDS round trips and barriers); an odd last stage alone.
// bf(x, y, w): x, y <- x + w y, x - w y.
template <class BF>
__device__ __forceinline__ void fft_dit_stages(double2* a, int tid, int TH, int n_pts, int log_pts, const double2* W,
                                               int logh, BF bf) {
    int s = 0;
    for (; s + 1 < log_pts; s += 2) {
        const int half = 1 << s;
        for (int g = tid; g < n_pts / 4; g += TH) {
            const int k = g & (half - 1);
            const int i0 = ((g >> s) << (s + 2)) + k;
            double2 x0 = a[i0], x1 = a[i0 + half], x2 = a[i0 + 2 * half], x3 = a[i0 + 3 * half];
            const double2 w = W[(size_t)k << (logh - 1 - s)];
            bf(x0, x1, w);
            bf(x2, x3, w);
            bf(x0, x2, W[(size_t)k << (logh - 2 - s)]);
            bf(x1, x3, W[(size_t)(k + half) << (logh - 2 - s)]);
            a[i0] = x0;
            a[i0 + half] = x1;
            a[i0 + 2 * half] = x2;
            a[i0 + 3 * half] = x3;
        }
        __syncthreads();
    }
    if (s < log_pts) {
        const int half = 1 << s;
        for (int b = tid; b < n_pts / 2; b += TH) {
            const int k = b & (half - 1);
            const int i = ((b >> s) << (s + 1)) + k;
            double2 x = a[i], y = a[i + half];
            bf(x, y, W[(size_t)k << (logh - 1 - s)]);
            a[i] = x;
            a[i + half] = y;
        }
        __syncthreads();
    }
}
struct FftBfly {   // the encoder's butterfly (contraction as the compiler likes)
    __device__ __forceinline__ void operator()(double2& x, double2& y, const double2 w) const {
        const double2 t = {y.x * w.x - y.y * w.y, y.x * w.y + y.y * w.x};
        y = double2{x.x - t.x, x.y - t.y};
        x = double2{x.x + t.x, x.y + t.y};
    }
};
template <int LOGN>
__device__ __forceinline__ void enc_fft_stages(double2* a, int tid, int TH, int n_pts, int log_pts, const double2* W,
                                               int logh) {
    fft_dit_stages(a, tid, TH, n_pts, log_pts, W, logh, FftBfly{});
}
template <int LOGN>
__device__ __forceinline__ void enc_finish(const DevTables& T, double2 v, int k, double scale, u64* out, int l,
                                           double* dout) {
    constexpr int N = 1 << LOGN, H = N / 2;
    const double2 z = reinterpret_cast<const double2*>(T.enc_twist)[k];
    const double lo = round((v.x * z.x - v.y * z.y) * scale);
    const double hi = round((v.x * z.y + v.y * z.x) * scale);
    if (dout) {   // fused path: the rounded coefficients; k_ntt_fwd_from_dbl reduces them per limb
        dout[k] = lo;
        dout[H + k] = hi;
        return;
    }
    for (int i = 0; i < l; ++i) {
        out[(size_t)i * N + k] = dbl_mod(T, lo, i);
        out[(size_t)i * N + H + k] = dbl_mod(T, hi, i);
    }
}
// ---- periodic rows.  The reference's callers encode tiled vectors (np.tile of a d-vector: the BSGS diagonals,
// bg:361-378 / tf:48, and encrypt_replicated's input, bg:53-58).  A slot vector with z_{j+d} = z_j, d = (N/2) / t, is
// the encoding of m(X) = p(X^t): its coefficients vanish off the multiples of t, and p is the encoding of the first d
// slots in the ring of dimension M = N / t (X -> X^t carries that ring's slot group onto this one's: 5^j mod 2M has
// period d).  The encoder then runs the d-point FFT of one period instead of the N/2-point FFT of the whole vector
// (slot j of the first period goes to bin enc_pos[j] >> log t, twist t * enc_twist[t k]), and every limb's forward
// NTT is the M-point NTT of p with the first M twiddles of the limb's own N-point table (psi^rev_N(i) = (psi^t)^rev_M(i)
// for i < M), each output repeated t times (bit-reversed order: slot j of the N-point NTT holds slot j >> log t of
// the M-point one).  The NTT side is exact -- the N-point NTT of the spread coefficients gives the same canonical
// residues (FHESPEAR_ENCODE_UNFUSED runs it: tests/test_gpu_parity.py) -- and the coefficients off the multiples of t
// are exact zeros instead of the dense FFT's float64 rounding noise, so the limbs differ from a dense encode of the
// same vector by that noise, well inside the encoder's precision.  t <= 8, M >= 256; FHESPEAR_ENCODE_DENSE=1 turns
// it off.  k_enc_period: per row the largest s <= smax with z_{j + (N/2 >> s)} = z_j for every j (bit patterns).
constexpr int kEncSparseMaxLog = 3, kEncSparseMinLogM = 8;
__global__ void __launch_bounds__(256) k_enc_period(const double* vals, size_t n, size_t stride, int is_real, int smax,
                                                    unsigned char* tlog) {
    __shared__ unsigned bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(vals + (size_t)blockIdx.x * stride);
    const size_t words = is_real ? n : 2 * n;
    unsigned b = 0;
    for (size_t j = threadIdx.x; j < words; j += blockDim.x) {
        const unsigned long long x = w[j];
        for (int s = 1; s <= smax; ++s) {
            const size_t p = words >> s;
            if (j >= p && x != w[j - p]) b |= 1u << s;
        }
    }
    if (b) atomicOr(&bad, b);
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
        while (s < smax && !(bad & (2u << s))) ++s;
        tlog[blockIdx.x] = (unsigned char)s;
    }
}
// coefficient k < d of a periodic row's first period (bin k of its d-point FFT): compact (the M-ring coefficients
// p_k, p_{d+k} at k, d + k: k_ntt_fwd_from_dbl_sp reads them), or spread over the N-ring (m_{tk}, m_{N/2+tk}, zeros
// between) into the coefficient scratch or straight into every limb
template <int LOGN>
__device__ __forceinline__ void enc_finish_sparse(const DevTables& T, double2 v, int k, int sp, double scale, u64* out,
                                                  int l, double* dout, bool compact) {
    constexpr int N = 1 << LOGN, H = N / 2;
    const int t = 1 << sp;
    const double2 z0 = reinterpret_cast<const double2*>(T.enc_twist)[k << sp];
    const double2 z = {z0.x * t, z0.y * t};   // (2/M) zeta_M^-k = t (2/N) zeta^-tk, a power-of-two scaling: exact
    const double lo = round((v.x * z.x - v.y * z.y) * scale);
    const double hi = round((v.x * z.y + v.y * z.x) * scale);
    if (dout && compact) {
        dout[k] = lo;
        dout[(H >> sp) + k] = hi;
        return;
    }
    const int e0 = k << sp, e1 = H + (k << sp);
    if (dout) {
        dout[e0] = lo;
        dout[e1] = hi;
        for (int r = 1; r < t; ++r) dout[e0 + r] = dout[e1 + r] = 0.0;
        return;
    }
    for (int i = 0; i < l; ++i) {
        u64* o = out + (size_t)i * N;
        o[e0] = dbl_mod(T, lo, i);
        o[e1] = dbl_mod(T, hi, i);
        for (int r = 1; r < t; ++r) o[e0 + r] = o[e1 + r] = 0;
    }
}
template <int LOGN>
__global__ void __launch_bounds__(((1 << LOGN) / 16) < 1024 ? ((1 << LOGN) / 16) : 1024)
    k_encode(DevTables T, const double* vals, size_t n, size_t stride, int is_real, double scale, u64* const* outs,
             int l, double* coef_out, const unsigned char* tlog, int compact) {
    constexpr int N = 1 << LOGN, H = N / 2, LOGH = LOGN - 1;
    constexpr int TH = (N / 16) < 1024 ? (N / 16) : 1024;
    constexpr bool SPLIT = LOGN > 14;   // N = 32768: the H-point FFT as two H/2-point halves + a final stage
    __shared__ double2 a[SPLIT ? H / 2 : H];
    const int tid = threadIdx.x;
    const double* src = vals + (size_t)blockIdx.x * stride;
    const double2* W = reinterpret_cast<const double2*>(T.enc_w);
    u64* out = outs ? outs[blockIdx.x] : nullptr;   // null: coefficients to coef_out only
    double* dout = coef_out ? coef_out + (size_t)blockIdx.x * N : nullptr;
    const int sp = tlog ? tlog[blockIdx.x] : 0;
    if (sp) {   // a periodic row (k_enc_period, n = N/2): the (N/2 >> sp)-point FFT of its first period
        const int HM = H >> sp;
        for (int j = tid; j < HM; j += TH)
            a[T.enc_pos[j] >> sp] = is_real ? double2{src[j], 0.0} : double2{src[2 * j], src[2 * j + 1]};
        __syncthreads();
        enc_fft_stages<LOGN>(a, tid, TH, HM, LOGH - sp, W, LOGH);
        for (int k = tid; k < HM; k += TH) enc_finish_sparse<LOGN>(T, a[k], k, sp, scale, out, l, dout, compact != 0);
        return;
    }
    if constexpr (!SPLIT) {
        for (int j = tid; j < H; j += TH) {
            double2 z = {0.0, 0.0};
            if ((size_t)j < n) z = is_real ? double2{src[j], 0.0} : double2{src[2 * j], src[2 * j + 1]};
            a[T.enc_pos[j]] = z;
        }
        __syncthreads();
        enc_fft_stages<LOGN>(a, tid, TH, H, LOGH, W, LOGH);
        for (int k = tid; k < H; k += TH) enc_finish<LOGN>(T, a[k], k, scale, out, l, dout);
    } else {
        // bit-reversed input: slots with rev(s_j) < H/2 form the first half's sub-FFT
        constexpr int HH = H / 2, PER = HH / TH;
        double2 lo[PER];
        for (int h = 0; h < 2; ++h) {
            if (h) __syncthreads();
            for (int j = tid; j < H; j += TH) {
                const unsigned pos = T.enc_pos[j];
                if ((int)(pos / HH) != h) continue;
                double2 z = {0.0, 0.0};
                if ((size_t)j < n) z = is_real ? double2{src[j], 0.0} : double2{src[2 * j], src[2 * j + 1]};
                a[pos - h * HH] = z;
            }
            __syncthreads();
            enc_fft_stages<LOGN>(a, tid, TH, HH, LOGH - 1, W, LOGH);
            if (h == 0) {
#pragma unroll
                for (int c = 0; c < PER; ++c) lo[c] = a[tid + c * TH];
            }
        }
#pragma unroll
        for (int c = 0; c < PER; ++c) {   // last stage: pairs (k, k + H/2), twiddle omega^-k
            const int k = tid + c * TH;
            const double2 x = lo[c], y = a[k], w = W[k];
            const double2 t = {y.x * w.x - y.y * w.y, y.x * w.y + y.y * w.x};
            enc_finish<LOGN>(T, double2{x.x + t.x, x.y + t.y}, k, scale, out, l, dout);
            enc_finish<LOGN>(T, double2{x.x - t.x, x.y - t.y}, k + HH, scale, out, l, dout);
        }
    }
}

// ---- decoder FFT (launch_decode_slots).  fp contraction is off throughout: the host decoder's
// fft_inplace / decode_slots evaluate these products and sums unfused (x86-64 without FMA), and the GPU
// must round the same way to give the same doubles.
struct DecBfly {   // the host decoder's butterfly, unfused (decode_slots / fft_inplace round the same way)
    __device__ __forceinline__ void operator()(double2& x, double2& y, const double2 w) const {
#pragma clang fp contract(off)
        const double vr = y.x * w.x - y.y * w.y, vi = y.x * w.y + y.y * w.x;
        y = double2{x.x - vr, x.y - vi};
        x = double2{x.x + vr, x.y + vi};
    }
};
__device__ __forceinline__ void dec_fft_stages(double2* a, int tid, int TH, int n_pts, int log_pts, const double2* W,
                                               int logh) {
    fft_dit_stages(a, tid, TH, n_pts, log_pts, W, logh, DecBfly{});
}
template <int LOGN>
constexpr int dec_threads() {
    constexpr int PTS = LOGN > 14 ? (1 << (LOGN - 2)) : (1 << (LOGN - 1));
    return PTS / 2 < 1024 ? PTS / 2 : 1024;
}
// one workgroup per vector: twist + bit-reversed scatter into LDS, the N/2-point FFT (N = 2^15: two
// N/4-point halves, the last stage from registers), the spectrum to spec
template <int LOGN>
__global__ void __launch_bounds__(dec_threads<LOGN>())
    k_decode_fft(DevTables T, const double* m, const double* scales, double2* spec) {
#pragma clang fp contract(off)
    constexpr int N = 1 << LOGN, H = N / 2, LOGH = LOGN - 1;
    constexpr bool SPLIT = LOGN > 14;
    constexpr int PTS = SPLIT ? H / 2 : H, TH = dec_threads<LOGN>();
    __shared__ double2 a[PTS];
    const int tid = threadIdx.x;
    const double* src = m + (size_t)blockIdx.x * N;
    const double scale = scales[blockIdx.x];
    const double2* W = reinterpret_cast<const double2*>(T.dec_w);
    const double2* Z = reinterpret_cast<const double2*>(T.dec_twist);
    double2* out = spec + (size_t)blockIdx.x * H;
    double2 lo[SPLIT ? PTS / TH : 1];
    for (int h = 0; h < (SPLIT ? 2 : 1); ++h) {
        if (h) __syncthreads();
        for (int k = tid; k < H; k += TH) {
            const unsigned pos = __brev((unsigned)k) >> (32 - LOGH);
            if (SPLIT && (int)(pos / PTS) != h) continue;
            const double x = src[k] / scale, y = src[k + H] / scale;
            const double2 z = Z[k];
            a[pos - h * PTS] = double2{x * z.x - y * z.y, x * z.y + y * z.x};
        }
        __syncthreads();
        dec_fft_stages(a, tid, TH, PTS, SPLIT ? LOGH - 1 : LOGH, W, LOGH);
        if constexpr (!SPLIT) {
            for (int k = tid; k < H; k += TH) out[k] = a[k];
        } else if (h == 0) {
#pragma unroll
            for (int c = 0; c < PTS / TH; ++c) lo[c] = a[tid + c * TH];
        }
    }
    if constexpr (SPLIT) {
#pragma unroll
        for (int c = 0; c < PTS / TH; ++c) {   // last stage: pairs (k, k + N/4), twiddle omega^k
            const int k = tid + c * TH;
            const double2 u = lo[c], v = a[k], w = W[k];
            const double vr = v.x * w.x - v.y * w.y, vi = v.x * w.y + v.y * w.x;
            out[k] = double2{u.x + vr, u.y + vi};
            out[k + PTS] = double2{u.x - vr, u.y - vi};
        }
    }
}
// slot j of vector i: spectrum bin dec_pos[j]
__global__ void k_decode_gather(DevTables T, const double2* spec, int count, int nslots, double2* out) {
    const size_t H = (size_t)T.N / 2, total = (size_t)count * nslots;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const size_t i = e / nslots, j = e - i * nslots;
        out[e] = spec[i * H + T.dec_pos[j]];
    }
}
hipError_t launch_decode_slots(const DevTables& T, const double* m, const double* scales, int count, double* spec,
                               int nslots, double* out, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    if (nslots < 1 || nslots > T.N / 2) return hipErrorInvalidValue;
    FHS_DISPATCH_LOGN(T.logN, {
        hipLaunchKernelGGL((k_decode_fft<LOGN>), dim3(count), dim3(dec_threads<LOGN>()), 0, st, T, m, scales,
                           reinterpret_cast<double2*>(spec));
    });
    hipLaunchKernelGGL(k_decode_gather, dim3(eltwise_grid((size_t)count * nslots)), dim3(256), 0, st, T,
                       reinterpret_cast<const double2*>(spec), count, nslots, reinterpret_cast<double2*>(out));
    return hipGetLastError();
}

// forward NTT of `limbs` limbs of each polynomial ptrs[blockIdx.y] (plaintext batches)
template <int LOGN>
__global__ void __launch_bounds__(ntt_threads<LOGN>()) k_ntt_fwd_ptrs(DevTables T, u64* const* ptrs, int limbs) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN>()];
    const int b = blockIdx.x;
    const RedU R = redu(PK(T, b));
    u64* p = ptrs[blockIdx.y] + (size_t)b * N;
    fwd_limb<LOGN, FHS_NTT_RL>(lds, threadIdx.x, T.tw_fwd + (size_t)b * N * 2, R, [&](int e) { return p[e]; },
                               [&](int e, u64 v) { p[e] = v; });
}

// fused exact reduction + forward NTT: limb blockIdx.x of plaintext blockIdx.y from its rounded
// double coefficients (the same dbl_mod as enc_finish, so the same residues): the l limbs are
// written once instead of written, read and rewritten
template <int LOGN>
__global__ void __launch_bounds__(ntt_threads<LOGN>()) k_ntt_fwd_from_dbl(DevTables T, const double* coef,
                                                                         u64* const* ptrs, int limbs,
                                                                         const unsigned char* tlog) {
    constexpr int N = 1 << LOGN;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGN>()];
    if (tlog && tlog[blockIdx.y]) return;   // a periodic row: k_ntt_fwd_from_dbl_sp
    const int b = blockIdx.x;
    const RedU R = redu(PK(T, b));
    const double* cf = coef + (size_t)blockIdx.y * N;
    u64* p = ptrs[blockIdx.y] + (size_t)b * N;
    const DblMod M = dbl_mod_of(T, b);
    fwd_limb<LOGN, FHS_NTT_RL>(lds, threadIdx.x, T.tw_fwd + (size_t)b * N * 2, enc_lazy(R, M),
                               [&](int e) { return dbl_mod(M, cf[e]); }, [&](int e, u64 v) { p[e] = v; });
}
// the same for the rows with tlog = S (see k_enc_period): the 2^(LOGN-S)-point NTT of the compact coefficients,
// each value stored 2^S times (16-byte stores of two copies)
// couts (ss <= S): the compact shadow as well, 2^(S - ss) copies per value in limbs of N >> ss words
template <int LOGN, int S>
__global__ void __launch_bounds__(ntt_threads<LOGN - S>()) k_ntt_fwd_from_dbl_sp(DevTables T, const double* coef,
                                                                                u64* const* ptrs, int limbs,
                                                                                const unsigned char* tlog,
                                                                                u64* const* couts, int ss) {
    constexpr int N = 1 << LOGN, LOGM = LOGN - S;
    __shared__ __attribute__((aligned(16))) u64 lds[ntt_lds_words<LOGM>()];
    if (tlog[blockIdx.y] != S) return;
    const int b = blockIdx.x;
    const RedU R = redu(PK(T, b));
    const double* cf = coef + (size_t)blockIdx.y * N;
    u64* p = ptrs[blockIdx.y] ? ptrs[blockIdx.y] + (size_t)b * N : nullptr;   // null: a compact-only plaintext
    u64* pc = couts ? couts[blockIdx.y] + (size_t)b * (N >> ss) : nullptr;
    const int cs = S - ss;   // log2 of the copies per value in the shadow (wave-uniform)
    const DblMod M = dbl_mod_of(T, b);
    fwd_limb<LOGM, FHS_NTT_RL>(lds, threadIdx.x, T.tw_fwd + (size_t)b * N * 2, enc_lazy(R, M),
                               [&](int e) { return dbl_mod(M, cf[e]); },
                               [&](int e, u64 v) {
                                   if (p) {
                                       ulonglong2* d = reinterpret_cast<ulonglong2*>(p + ((size_t)e << S));
#pragma unroll
                                       for (int r = 0; r < (1 << S) / 2; ++r) d[r] = ulonglong2{v, v};
                                   }
                                   if (pc) {
                                       u64* c = pc + ((size_t)e << cs);
                                       if (cs == 0) {
                                           c[0] = v;
                                       } else {
                                           for (int r = 0; r < (1 << cs) / 2; ++r)
                                               reinterpret_cast<ulonglong2*>(c)[r] = ulonglong2{v, v};
                                       }
                                   }
                               });
}
template <int LOGN>
static void launch_ntt_fwd_sparse(const DevTables& T, const double* coef, u64* const* outs, int l, int count,
                                  const unsigned char* tlog, u64* const* couts, int ss, hipStream_t st) {
    static_assert(kEncSparseMaxLog == 3, "one launch per sparse factor below");
    if constexpr (LOGN - 1 >= kEncSparseMinLogM)
        if (ss <= 1)
            hipLaunchKernelGGL((k_ntt_fwd_from_dbl_sp<LOGN, 1>), dim3(l, count), dim3(ntt_threads<LOGN - 1>()), 0, st,
                               T, coef, outs, l, tlog, couts, ss);
    if constexpr (LOGN - 2 >= kEncSparseMinLogM)
        if (ss <= 2)
            hipLaunchKernelGGL((k_ntt_fwd_from_dbl_sp<LOGN, 2>), dim3(l, count), dim3(ntt_threads<LOGN - 2>()), 0, st,
                               T, coef, outs, l, tlog, couts, ss);
    if constexpr (LOGN - 3 >= kEncSparseMinLogM)
        hipLaunchKernelGGL((k_ntt_fwd_from_dbl_sp<LOGN, 3>), dim3(l, count), dim3(ntt_threads<LOGN - 3>()), 0, st, T,
                           coef, outs, l, tlog, couts, ss);
}
// dense limbs of a compact plaintext (fhs_host.hip pt_dense): d[i N + e] = dc[i (N >> tl) + (e >> tl)]
__global__ void k_expand_compact(const u64* __restrict__ dc, u64* __restrict__ d, int l, int N, int tl) {
    const size_t total = (size_t)l * N;
    const int Nc = N >> tl;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
        const size_t i = idx / N;
        const int e = (int)(idx - i * N);
        d[idx] = dc[i * Nc + (e >> tl)];
    }
}
hipError_t launch_expand_compact(const u64* dc, u64* d, int l, int N, int tl, hipStream_t st) {
    if (tl < 1 || tl > kEncSparseMaxLog || l < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_expand_compact, dim3(eltwise_grid((size_t)l * N)), dim3(256), 0, st, dc, d, l, N, tl);
    return hipGetLastError();
}
int encode_sparse_max_log(int logN) { return std::max(0, std::min(kEncSparseMaxLog, logN - kEncSparseMinLogM)); }
hipError_t launch_enc_period(const double* vals, int count, size_t n, size_t stride, bool is_real, int smax,
                             unsigned char* tlog, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_enc_period, dim3(count), dim3(256), 0, st, vals, n, stride, is_real ? 1 : 0, smax, tlog);
    return hipGetLastError();
}

hipError_t launch_encode_coef(const DevTables& T, const double* vals, int count, size_t n, size_t stride, bool is_real,
                              double scale, double* coef, hipStream_t st, const unsigned char* tlog) {
    if (count <= 0) return hipSuccess;
    FHS_DISPATCH_LOGN(T.logN, {
        constexpr int TH = ((1 << LOGN) / 16) < 1024 ? ((1 << LOGN) / 16) : 1024;
        hipLaunchKernelGGL((k_encode<LOGN>), dim3(count), dim3(TH), 0, st, T, vals, n, stride, is_real ? 1 : 0, scale,
                           static_cast<u64* const*>(nullptr), 0, coef, tlog, 0);
    });
    return hipGetLastError();
}
hipError_t launch_encode(const DevTables& T, const double* vals, int count, size_t n, size_t stride, bool is_real,
                         double scale, u64* const* outs_dev, int l, hipStream_t st, double* coef_scratch,
                         const unsigned char* tlog, u64* const* couts_dev, int ss) {
    if (count <= 0) return hipSuccess;
    if (couts_dev && (!coef_scratch || !tlog || ss < 1 || ss > kEncSparseMaxLog)) return hipErrorInvalidValue;
    if (!couts_dev) ss = 0;
    FHS_DISPATCH_LOGN(T.logN, {
        constexpr int TH = ((1 << LOGN) / 16) < 1024 ? ((1 << LOGN) / 16) : 1024;
        hipLaunchKernelGGL((k_encode<LOGN>), dim3(count), dim3(TH), 0, st, T, vals, n, stride, is_real ? 1 : 0, scale,
                           outs_dev, l, coef_scratch, tlog, coef_scratch ? 1 : 0);
        if (coef_scratch) {
            hipLaunchKernelGGL((k_ntt_fwd_from_dbl<LOGN>), dim3(l, count), dim3(ntt_threads<LOGN>()), 0, st, T,
                               static_cast<const double*>(coef_scratch), outs_dev, l, tlog);
            if (tlog) launch_ntt_fwd_sparse<LOGN>(T, coef_scratch, outs_dev, l, count, tlog, couts_dev, ss, st);
        } else {   // unfused: the spread coefficients in every limb, the N-point NTT in place
            hipLaunchKernelGGL((k_ntt_fwd_ptrs<LOGN>), dim3(l, count), dim3(ntt_threads<LOGN>()), 0, st, T, outs_dev, l);
        }
    });
    return hipGetLastError();
}

// Diagonal extraction + giant-group roll + tiling on the device (bg:198-203 _extract_diagonals and
// bg:361-378 / 394-421 _batch_encode_diags_*): row k of the encoder input, slot j, is
//   d_k[m'] = M[m', (m' + k) mod D],  m' = (j mod D - g G) mod D,  g = k / G
// (np.roll of group g's rows by g G, then np.tile / the remainder columns -- both are j mod D).
// Complex (M2 != null): re = M1, im = M2, interleaved as the complex encoder reads them.
__global__ void k_diag_gather(const double* __restrict__ M1, const double* __restrict__ M2, int D, int G, int n,
                              int k0, int rows, int trans, double* __restrict__ out) {
    const size_t total = (size_t)rows * n;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(idx / n), j = (int)(idx % n), k = k0 + r;
        const int shift = (k / G) * G % D;
        int m = j % D - shift;
        if (m < 0) m += D;
        int col = m + k % D;
        if (col >= D) col -= D;
        const size_t src = trans ? (size_t)col * D + m : (size_t)m * D + col;   // trans: M^T stored
        if (M2) {
            out[2 * idx] = M1[src];
            out[2 * idx + 1] = M2[src];
        } else {
            out[idx] = M1[src];
        }
    }
}
hipError_t launch_diag_gather(const double* M1, const double* M2, int D, int G, int n, int k0, int rows, int trans,
                              double* out, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_diag_gather, dim3(eltwise_grid((size_t)rows * n)), dim3(256), 0, st, M1, M2, D, G, n, k0,
                       rows, trans, out);
    return hipGetLastError();
}

hipError_t launch_encode_reduce(const DevTables& T, const double* coef, int count, u64* out, int l, hipStream_t st) {
    hipLaunchKernelGGL(k_encode_reduce, dim3(eltwise_grid((size_t)count * l * T.N)), dim3(256), 0, st, T, coef, count,
                       out, l);
    return hipGetLastError();
}

// ============================================================================ decode: centred CRT
constexpr int kCrtCheckPer = 4;   // extra limbs checked per grid row
__device__ __forceinline__ void crt_compose_body(const CrtConsts& K, const u64* __restrict__ limbs, double* __restrict__ out,
                                                 int N, const u64* __restrict__ extra, int nx,
                                                 const u64* __restrict__ vtab, unsigned* flag) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const int l = K.l, W = K.W;
    u64 x[kCrtMaxL + 2];
#pragma unroll
    for (int w = 0; w < kCrtMaxL + 2; ++w) x[w] = 0;
    for (int i = 0; i < l; ++i) {
        const u64 a = limbs[(size_t)i * N + n], qi = K.q[i];
        const u64 qh = __umul64hi(a, K.ihat_s[i]);
        u64 y = a * K.ihat[i] - qh * qi;
        if (y >= qi) y -= qi;
        u64 carry = 0;   // x += hat_i * y over W words (each partial < 2^128: hi word + carries fit)
        for (int w = 0; w < W; ++w) {
            const u64 lo = K.hat[i][w] * y, hi = __umul64hi(K.hat[i][w], y);
            const u64 s1 = lo + x[w];
            const u64 c1 = s1 < lo;
            const u64 s2 = s1 + carry;
            const u64 c2 = s2 < s1;
            x[w] = s2;
            carry = hi + c1 + c2;
        }
        x[W] += carry;
        for (;;) {   // x < 2Q: at most one subtraction
            bool ge = x[W] != 0;
            if (!ge) {
                ge = true;
                for (int w = W - 1; w >= 0; --w)
                    if (x[w] != K.Q[w]) { ge = x[w] > K.Q[w]; break; }
            }
            if (!ge) break;
            u64 br = 0;
            for (int w = 0; w < W; ++w) {
                const u64 qa = K.Q[w] + br;
                const u64 nb = (qa < br) || (x[w] < qa);
                x[w] -= qa;
                br = nb;
            }
            x[W] -= br;
        }
    }
    bool neg = false;
    for (int w = W - 1; w >= 0; --w)
        if (x[w] != K.halfQ[w]) { neg = x[w] > K.halfQ[w]; break; }
    if (neg) {
        u64 br = 0;
        for (int w = 0; w < W; ++w) {
            const u64 xa = x[w] + br;
            const u64 nb = (xa < br) || (K.Q[w] < xa);
            x[w] = K.Q[w] - xa;
            br = nb;
        }
    }
    if (blockIdx.y == 0) {
        double v = 0;   // v 2^64 is exact, so one rounding per step as on the host
        for (int w = W - 1; w >= 0; --w) v = __dadd_rn(__dmul_rn(v, 18446744073709551616.0), (double)x[w]);
        out[n] = neg ? -v : v;
    }
    // the composition is the true coefficient only if it also matches every limb not composed: row y of
    // the grid checks limbs [y kCrtCheckPer, (y + 1) kCrtCheckPer) (the composition above is a few
    // multiply-adds per limb; the check is the long part, serial in one thread it left the kernel
    // latency-bound at N / 256 workgroups)
    bool bad = false;
    const int e1 = min(nx, (int)(blockIdx.y + 1) * kCrtCheckPer);
    for (int e = blockIdx.y * kCrtCheckPer; e < e1; ++e) {
        const u64* vt = vtab + (size_t)e * kCrtVtabWords;
        const u64 q = vt[0];
        u64 lo = 0, hi = 0;   // sum_w x[w] (2^64w mod q) < W 2^123: no overflow
        for (int w = 0; w < W; ++w) {
            const u64 p = x[w] * vt[3 + w], ph = __umul64hi(x[w], vt[3 + w]);
            lo += p;
            hi += ph + (lo < p);
        }
        u64 r = barrett128(lo, hi, q, vt[1], vt[2]);
        if (neg && r) r = q - r;
        bad |= r != extra[(size_t)e * N + n];
    }
    if (bad) atomicOr(flag, 1u);
}
__global__ void k_crt_compose(CrtConsts K, const u64* __restrict__ limbs, double* __restrict__ out, int N,
                              const u64* __restrict__ extra, int nx, const u64* __restrict__ vtab, unsigned* flag) {
    crt_compose_body(K, limbs, out, N, extra, nx, vtab, flag);
}
// a batch of compositions (one decode call's plaintexts): job blockIdx.z, its check rows up to its own nx
__global__ void k_crt_compose_jobs(const CrtJob* __restrict__ jobs, int N) {
    const CrtJob& J = jobs[blockIdx.z];
    if (blockIdx.y > 0 && (int)blockIdx.y * kCrtCheckPer >= J.nx) return;
    crt_compose_body(J.K, J.limbs, J.out, N, J.extra, J.nx, J.vtab, J.flag);
}
hipError_t launch_crt_compose_jobs(const CrtJob* jobs_dev, int count, int max_nx, int N, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    const int rows = max_nx > 0 ? (max_nx + kCrtCheckPer - 1) / kCrtCheckPer : 1;
    hipLaunchKernelGGL(k_crt_compose_jobs, dim3((N + 255) / 256, rows, count), dim3(256), 0, st, jobs_dev, N);
    return hipGetLastError();
}
hipError_t launch_crt_compose(const CrtConsts& K, const u64* limbs, double* out, int N, hipStream_t st, const u64* extra,
                              int nx, const u64* vtab, unsigned* flag) {
    if (K.l < 1 || K.l > kCrtMaxL || K.W != K.l + 1) return hipErrorInvalidValue;
    if (nx > 0 && (!extra || !vtab || !flag)) return hipErrorInvalidValue;
    const int rows = nx > 0 ? (nx + kCrtCheckPer - 1) / kCrtCheckPer : 1;
    hipLaunchKernelGGL(k_crt_compose, dim3((N + 255) / 256, rows), dim3(256), 0, st, K, limbs, out, N, extra, nx, vtab,
                       flag);
    return hipGetLastError();
}

// ============================================================================ bootstrapping primitives
// Constant products / sums (ckks_bootstrapper: pre-scale, EvalMod's Chebyshev coefficients and
// constants, scale alignment).  A constant polynomial c has NTT image c in every slot, so both ops
// are slot-wise: MULC multiplies every component by c_i (Shoup), ADDC adds c_i to component 0.
__global__ void k_scalar(DevTables T, int op, const u64* __restrict__ a, u64* __restrict__ out, int ncomp, int l,
                         ScalarConsts K) {
    const int N = T.N;
    const size_t total = (size_t)ncomp * l * N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        const size_t li = idx / N;
        const int i = (int)(li % l), comp = (int)(li / l);
        const u64 q = PK(T, i).q, x = a[idx];
        u64 r;
        if (op == SCALAR_MUL) r = shoup(x, K.v[i], K.vs[i], q);
        else r = comp == 0 ? addmod(x, K.v[i], q) : x;
        out[idx] = r;
    }
}
hipError_t launch_scalar(const DevTables& T, int op, const u64* a, u64* out, int ncomp, int l, const ScalarConsts& K,
                         hipStream_t st) {
    if (l > kMaxScalarLimbs) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_scalar, dim3(eltwise_grid((size_t)ncomp * l * T.N)), dim3(256), 0, st, T, op, a, out, ncomp, l,
                       K);
    return hipGetLastError();
}

// ModRaise: the q0 limb of each component (coefficient form after k_ntt_inv) lifted to its
// centred representative in (-q0/2, q0/2] and reduced into all L0 data limbs, then NTT.
__global__ void k_mod_raise_lift(DevTables T, const u64* __restrict__ coef, u64* __restrict__ out, int ncomp) {
    const int N = T.N, L = T.L0;
    const u64 q0 = PK(T, 0).q, half = q0 >> 1;
    const size_t total = (size_t)ncomp * L * N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        const int n = (int)(idx % N);
        const size_t li = idx / N;
        const int i = (int)(li % L), comp = (int)(li / L);
        const u64 x = coef[(size_t)comp * N + n], qi = PK(T, i).q;
        u64 r;
        if (x <= half) r = x % qi;                        // non-negative representative
        else {                                            // x - q0 < 0
            const u64 m = (q0 - x) % qi;
            r = m ? qi - m : 0;
        }
        out[idx] = r;
    }
}
// in: ncomp components of l limbs (NTT form), limb 0 used; out: ncomp x L0 limbs; scratch: ncomp x N
hipError_t launch_mod_raise(const DevTables& T, const u64* in, int l, u64* out, u64* scratch, int ncomp,
                            hipStream_t st) {
    const size_t N = T.N;
    hipError_t e = hipMemcpy2DAsync(scratch, 8 * N, in, 8 * N * l, 8 * N, ncomp, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
    e = launch_ntt_inv(T, scratch, 1, 1, ncomp, N, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_mod_raise_lift, dim3(eltwise_grid((size_t)ncomp * T.L0 * N)), dim3(256), 0, st, T, scratch, out,
                       ncomp);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_ntt_fwd(T, out, T.L0, T.L0, ncomp, (size_t)T.L0 * N, st);
}

// Exact 128-bit integer coefficients (hi signed, lo unsigned: x = hi 2^64 + lo) -> every limb, NTT
// (fhs_encode_precise: bootstrapping transform plaintexts).
__global__ void k_reduce_i128(DevTables T, const int64_t* hi, const u64* lo, int count, u64* const* outs, int l) {
    const int N = T.N;
    const size_t total = (size_t)count * l * N;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        const int n = (int)(idx % N);
        const size_t rest = idx / N;
        const int i = (int)(rest % l);
        const size_t v = rest / l;
        const PrimeK& P = PK(T, i);
        const u64 q = P.q;
        const int64_t h = hi[v * N + n];
        u64 hm = (u64)(h < 0 ? -(h + 1) : h) % q;                 // |h| - [h < 0], no overflow
        if (h < 0) hm = submod(0, (hm + 1) % q, q);
        const u64 t64 = (0 - q) % q;                              // 2^64 mod q
        const u64 r = addmod(mulmod(hm, t64, P), lo[v * N + n] % q, q);
        outs[v][(size_t)i * N + n] = r;
    }
}
hipError_t launch_encode_int128(const DevTables& T, const int64_t* hi, const u64* lo, int count, u64* const* outs_dev,
                                int l, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_reduce_i128, dim3(eltwise_grid((size_t)count * l * T.N)), dim3(256), 0, st, T, hi, lo, count,
                       outs_dev, l);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    FHS_DISPATCH_LOGN(T.logN, {
        hipLaunchKernelGGL((k_ntt_fwd_ptrs<LOGN>), dim3(l, count), dim3(ntt_threads<LOGN>()), 0, st, T, outs_dev, l);
    });
    return hipGetLastError();
}

}  // namespace fhs
