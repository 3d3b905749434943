// fhs_ntt.h -- negacyclic NTT cores for one RNS limb per workgroup (gfx950).
//
// Layout: a limb of N = 2^LOGN uint64 lives in LDS (N + N/16 words, one pad word per 16 to break
// the power-of-two strides; 136 KiB at N = 16384 -> one workgroup per CU, 16 waves of 64).  The
// T = N/EPT threads (EPT = 16 elements per thread by default) sweep the stages in passes of up to RL = 3 or 4 stages (radix-8 / radix-16):
// per pass each thread loads a group of 2^R elements from LDS into registers, runs the R butterfly
// stages there, and stores the group back.  RL = 4 gives LOGN = 14 as 4+4+4+2 (four LDS sweeps);
// RL = 3 (3+3+3+3+2) halves the live registers for kernels that keep other state in registers
// (k_modup_ip holds 32 accumulator words per thread).
//
// Transform convention (same as the oracle, oracle/ckks_oracle.c ock_ntt_fwd/inv):
//   forward  Cooley-Tukey, natural -> bit-reversed:   out[i] = a(psi^(2 rev(i) + 1))
//   inverse  Gentleman-Sande, bit-reversed -> natural, scaled by N^-1 (folded into stage 0)
// Twiddles tw[2k] = psi^rev(k) (inverse table: psi^-rev(k)), tw[2k+1] = Shoup companion.
// Values are Harvey-lazy: forward keeps [0, 4q) (input must be < 4q), inverse keeps [0, 2q).
#pragma once
#include "fhs_modarith.h"

namespace fhs {

__device__ __forceinline__ int lds_pad(int e) { return e + (e >> 4); }
// lds_pad(j0 + k TL) for the k-th element of a butterfly group, base = lds_pad(j0), as base plus a
// compile-time offset wherever that is exact, so the LDS accesses take immediate offsets instead of
// three address instructions each: TL % 16 == 0 (the stride adds whole pad blocks), or a group
// that lies inside one aligned 16-word block (its span TL GS divides 16 and j0 % (TL GS) < TL).
// lds_pad(tid + c TH) for the c-th row of a thread's strided sweep: lds_pad(tid) + a compile-time
// offset when TH % 16 == 0 (c is unrolled, so the LDS access takes it as an immediate offset)
template <int TH>
__device__ __forceinline__ int row_pad(int tid, int c) {
    if constexpr (TH % 16 == 0)
        return lds_pad(tid) + c * (TH + TH / 16);
    else
        return lds_pad(tid + c * TH);
}
// When TL divides 16 and a group's span TL GS is a multiple of 16, the group's start j0 = blk TL GS + off
// has j0 % 16 = off < TL, so (j0 + k TL) >> 4 = (j0 >> 4) + (k TL) / 16: again base plus a compile-time
// offset (the radix-8 pass with TL = 8 of the half-limb transforms that start at stage 1).
template <int TL, int GS>
__device__ __forceinline__ int grp_pad(int j0, int base, int k) {
    if constexpr (TL % 16 == 0)
        return base + k * (TL + TL / 16);
    else if constexpr (16 % (TL * GS) == 0)
        return base + k * TL;
    else if constexpr (16 % TL == 0 && (TL * GS) % 16 == 0)
        return base + k * TL + (k * TL) / 16;
    else
        return lds_pad(j0 + k * TL);
}

__device__ __forceinline__ void ld_tw(const u64* __restrict__ tw, int idx, u64& w, u64& wp) {
    const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(tw + 2 * idx);
    w = v.x;
    wp = v.y;
}

// One pass over stages [S, S+R) (forward numbering: stage s has m = 2^s blocks, stride N>>(s+1)).
// Groups: {j0 + k*TL : k < 2^R}, j0 = blk*2*TF + off, off < TL; thread tid owns groups
// gid = tid + c*T for c < (N/2^R)/T.
// LAZY (forward only): no conditional subtraction at all; a value that entered below B leaves
// stage s below B + 2 s q (the Shoup product is < 2q for any 64-bit input), so 14 stages from
// B = 4q stay below 32q < 2^64 for q < 2^59 (host flag PrimeK.pm bit 7).
// When a group's block index is wave-uniform (TL >= 64) it is read through readfirstlane so the
// twiddle loads become scalar loads.
// hoff != 0 runs the pass on one half of a twice-larger transform whose first stage was done
// elsewhere: half h uses the global twiddles of its blocks, index ((2 + h) << s) + block = local
// index + ((1 + h) << s), so hoff = 1 + h (forward only).
// NOFOLD (inverse only): the transform is one half of a twice-larger inverse, so its last stage is
// an ordinary stage (twiddle through hoff) and the N^-1 fold happens in the caller's final stage.
template <int LOGN, int S, int R, bool FWD, int EPT, bool LAZY = false, bool NOFOLD = false>
__device__ __forceinline__ void ntt_pass(u64* lds, int tid, const u64* __restrict__ tw, u64 q, u64 s0, u64 s0s,
                                         u64 s1, u64 s1s, int hoff = 0) {
    constexpr int N = 1 << LOGN, T = N / EPT;
    constexpr int TF = N >> (S + 1);
    constexpr int TL = TF >> (R - 1);
    constexpr int GS = 1 << R;
    constexpr int NG = EPT / GS;
    const u64 q2 = 2 * q;
#pragma unroll 1
    for (int c = 0; c < NG; ++c) {
        const int gid = tid + c * T;
        const int blk = TL >= 64 ? __builtin_amdgcn_readfirstlane(gid) / TL : gid / TL, off = gid % TL;
        const int j0 = blk * 2 * TF + off;
        const int base = lds_pad(j0);
#define FHS_GRP_ADDR(k) grp_pad<TL, GS>(j0, base, (k))
        u64 x[GS];
#pragma unroll
        for (int k = 0; k < GS; ++k) x[k] = lds[FHS_GRP_ADDR(k)];
        if constexpr (FWD) {
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int half = GS >> (u + 1);
#pragma unroll
                for (int k = 0; k < GS; ++k) {
                    if (k & half) continue;
                    u64 w, wp;
                    ld_tw(tw, ((1 + hoff) << (S + u)) + blk * (1 << u) + (k >> (R - u)), w, wp);
                    u64 X = x[k];
                    if constexpr (!LAZY) X = X >= q2 ? X - q2 : X;
                    const u64 t = shoup_lazy(x[k + half], w, wp, q);
                    x[k] = X + t;
                    x[k + half] = X + (q2 - t);
                }
            }
        } else {
#pragma unroll
            for (int u = R - 1; u >= 0; --u) {
                const int half = GS >> (u + 1);
#pragma unroll
                for (int k = 0; k < GS; ++k) {
                    if (k & half) continue;
                    const u64 X = x[k], Y = x[k + half];
                    if (!NOFOLD && S == 0 && u == 0) {   // last GS stage: fold N^-1 (and any caller scale)
                        x[k] = shoup_lazy(X + Y, s0, s0s, q);
                        x[k + half] = shoup_lazy(X - Y + q2, s1, s1s, q);
                    } else {
                        u64 w, wp;
                        ld_tw(tw, ((1 + hoff) << (S + u)) + blk * (1 << u) + (k >> (R - u)), w, wp);
                        const u64 s = X + Y;
                        x[k] = s >= q2 ? s - q2 : s;
                        x[k + half] = shoup_lazy(X - Y + q2, w, wp, q);
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < GS; ++k) lds[FHS_GRP_ADDR(k)] = x[k];
#undef FHS_GRP_ADDR
    }
}

// Wave-local passes (round 5).  A pass whose butterfly groups have TL <= W (W = 64 lanes, or all T threads
// when there are fewer) hands wave w exactly the blocks [GS (W w + c T), + W GS) for c < EPT / GS (lanes take
// consecutive gids, TL divides W, a group spans GS TL elements): the same elements in every such pass of the
// same radix.  Between two of them no
// workgroup barrier is needed -- the LDS operations of one wave execute in issue order, and
// wave_barrier() keeps the compiler from moving LDS accesses across the pass boundary -- and after the last
// one the caller may read its own wave's blocks (wl_elem) without a barrier either.  PMC (profiles/r05,
// k_modup_h): 35 % of wave cycles parked on s_waitcnt / barriers, 25 % of SIMD cycles without VALU issue.
#ifndef FHS_NTT_WAVELOCAL
#define FHS_NTT_WAVELOCAL 1
#endif
// The hand-off between two wave-local passes (and at a wave-local head or tail): wave_barrier alone is IntrNoMem
// in LLVM, so it does not stop the compiler from moving one lane's LDS read above another lane's LDS write; the
// wavefront-scope release / acquire fences around it make that ordering a compiler constraint.  At wavefront
// scope they emit no instruction (the wave's LDS operations already execute in issue order).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int LOGN, int S, int R>
constexpr int pass_tl() { return R > 0 ? ((1 << LOGN) >> (S + 1)) >> (R - 1) : 0; }
// lanes of a wave that take part: 64, or all T = N / EPT threads when the transform has fewer (one wave)
template <int LOGN, int EPT>
constexpr int wl_width() { return (1 << LOGN) / EPT < 64 ? (1 << LOGN) / EPT : 64; }
template <int LOGN, int RL, int S>
constexpr int pass_r() { return (LOGN - S) < RL ? (LOGN - S) : RL; }
// element index of output q (q < EPT, compile-time) of thread tid after a wave-local transform (WL) whose
// passes have radix 2^R: block c = q / GS of the wave, row r = q % GS, lane-consecutive
template <int LOGN, int EPT, int GS>
__device__ __forceinline__ int wl_base(int tid) {
    constexpr int W = wl_width<LOGN, EPT>();
    return GS * W * (tid / W) + (tid % W);
}
template <int LOGN, int EPT, int GS>
constexpr int wl_off(int q) { return GS * ((1 << LOGN) / EPT) * (q / GS) + wl_width<LOGN, EPT>() * (q % GS); }

template <int LOGN, int RL, int S, int EPT, bool LAZY, bool WL = false>
__device__ __forceinline__ void fwd_from(u64* lds, int tid, const u64* __restrict__ tw, u64 q, int hoff) {
    if constexpr (S < LOGN) {
        constexpr int R = pass_r<LOGN, RL, S>();
        ntt_pass<LOGN, S, R, true, EPT, LAZY>(lds, tid, tw, q, 0, 0, 0, 0, hoff);
        constexpr int S2 = S + R;
        constexpr int W = wl_width<LOGN, EPT>();
        constexpr bool here = WL && pass_tl<LOGN, S, R>() <= W;
        constexpr bool next = S2 >= LOGN || (pass_r<LOGN, RL, S2>() == R && pass_tl<LOGN, S2, pass_r<LOGN, RL, S2>()>() <= W);
        if constexpr (here && next)
            wave_lds_sync();
        else
            __syncthreads();
        fwd_from<LOGN, RL, S2, EPT, LAZY, WL>(lds, tid, tw, q, hoff);
    }
}
// inverse: chunks [0,RL), [RL,2RL), ... processed last-to-first.  WL (every pass radix RL from S0): the
// barrier after pass S is skipped when the pass executed next (S - RL) is wave-local too (TL <= 64 for both;
// see fwd_from) -- the deep passes, which run first; a caller that wrote its input wave-locally (wl_base +
// wl_off) needs no barrier before the transform either.
template <int LOGN, int RL, int S, int EPT, bool NOFOLD = false, bool WL = false, int S0 = 0>
__device__ __forceinline__ void inv_from(u64* lds, int tid, const u64* __restrict__ tw, u64 q, u64 s0, u64 s0s,
                                         u64 s1, u64 s1s, int hoff = 0) {
    if constexpr (S < LOGN) {
        constexpr int R = pass_r<LOGN, RL, S>();
        inv_from<LOGN, RL, S + R, EPT, NOFOLD, WL, S0>(lds, tid, tw, q, s0, s0s, s1, s1s, hoff);
        ntt_pass<LOGN, S, R, false, EPT, false, NOFOLD>(lds, tid, tw, q, s0, s0s, s1, s1s, hoff);
        if constexpr (WL && R == RL && S - RL >= S0 && pass_tl<LOGN, S, R>() <= wl_width<LOGN, EPT>() &&
                      pass_tl<LOGN, S - RL, RL>() <= wl_width<LOGN, EPT>())
            wave_lds_sync();
        else
            __syncthreads();
    }
}

// Forward transform in LDS.  Entry: input (< 4q) at padded natural positions, after a barrier.
// Exit: bit-reversed-order output, after a barrier: < 4q (Harvey) or < (4 + 2 LOGN) q when
// `lazy` (wave-uniform; RedU::lazy); fwd_canon() maps either to [0, q).
// S0 > 0: stages [0, S0) were done by the caller (in registers), the passes start at stage S0.
// WL: wave-local tail (above): the exit barrier is dropped when the last pass is wave-local, so the caller
// must read only its wave's outputs (wl_base + wl_off) until its next barrier.
template <int LOGN, int RL = 3, int EPT = 16, int S0 = 0, bool WL = false>
__device__ __forceinline__ void ntt_fwd_lds(u64* lds, int tid, const u64* __restrict__ tw, u64 q, bool lazy,
                                            int hoff = 0) {
    static_assert(LOGN >= 7 && LOGN <= 14, "LDS-resident NTT supports 128 <= N <= 16384");
    static_assert(EPT >= 16 && (EPT & (EPT - 1)) == 0, "EPT must be a power of two >= 16");
    if (lazy)
        fwd_from<LOGN, RL, S0, EPT, true, WL>(lds, tid, tw, q, hoff);
    else
        fwd_from<LOGN, RL, S0, EPT, false, WL>(lds, tid, tw, q, hoff);
}
// true when ntt_fwd_lds<LOGN, RL, EPT, S0, true> leaves its outputs wave-local (every pass radix 2^RL, the
// last wave-local): the caller reads wl_base + wl_off with GS = 2^RL
template <int LOGN, int RL, int S0, int EPT = 16>
constexpr bool fwd_exit_wave_local() {
    return (LOGN - S0) % RL == 0 && pass_tl<LOGN, LOGN - RL, RL>() <= wl_width<LOGN, EPT>();
}
// Inverse transform in LDS; the final stage multiplies by (s0, s1) = (N^-1 c, psi^-1 N^-1 c) for a
// per-limb constant c.  Exit: natural-order output in [0, 2q), after a barrier.
// Inverse on one half (h = hoff - 1) of a 2^(LOGN+1)-point inverse: all of its stages except the
// global last one, which the caller applies to the (e, e + 2^LOGN) pairs.  Output in [0, 2q).
// S0 > 0: stages [0, S0) are left to the caller (done in registers afterwards).
template <int LOGN, int RL = 3, int EPT = 16, int S0 = 0, bool WL = false>
__device__ __forceinline__ void ntt_inv_half_lds(u64* lds, int tid, const u64* __restrict__ tw, u64 q, int hoff) {
    static_assert(!WL || (LOGN - S0) % RL == 0, "wave-local inverse passes need one radix throughout");
    if constexpr (WL) wave_lds_sync();   // the caller's wave-local head writes (no workgroup barrier before)
    inv_from<LOGN, RL, S0, EPT, true, WL, S0>(lds, tid, tw, q, 0, 0, 0, 0, hoff);
}
template <int LOGN, int RL = 3, int EPT = 16>
__device__ __forceinline__ void ntt_inv_lds(u64* lds, int tid, const u64* __restrict__ tw, u64 q, u64 s0, u64 s0s,
                                            u64 s1, u64 s1s) {
    static_assert(LOGN >= 8 && LOGN <= 14, "LDS-resident NTT supports 256 <= N <= 16384");
    inv_from<LOGN, RL, 0, EPT>(lds, tid, tw, q, s0, s0s, s1, s1s);
}

}  // namespace fhs
