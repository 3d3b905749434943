// CPU emulation of the device forward/inverse NTT passes (fhs_ntt.h) against a direct evaluation.
// Build: g++ -O2 -std=c++17 -Itools/debug/shim -Ifhe-spear_amd/csrc tools/debug/ntt_emu.cpp
// Each pass is run for every "thread" in turn, which is exactly the barrier-separated semantics.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include "fhs_ntt.h"
using namespace fhs;
typedef unsigned __int128 u128h;
static u64 mm(u64 a, u64 b, u64 q) { return (u64)((u128h)a * b % q); }
static u64 pw(u64 b, u64 e, u64 q) { u64 r = 1; while (e) { if (e & 1) r = mm(r, b, q); b = mm(b, b, q); e >>= 1; } return r; }
static unsigned rev(unsigned x, int bits) { unsigned r = 0; for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1) << (bits - 1 - i); return r; }
static bool isprime(u64 n) { if (n < 2) return false; for (u64 d : {2ull,3ull,5ull,7ull,11ull,13ull,17ull,19ull,23ull,29ull,31ull,37ull}) { if (n % d == 0) return n == d; }
  u64 d = n - 1; int s = 0; while (!(d & 1)) { d >>= 1; ++s; }
  for (u64 a : {2ull,3ull,5ull,7ull,11ull,13ull,17ull,19ull,23ull,29ull,31ull,37ull}) { u64 x = pw(a, d, n); if (x == 1 || x == n - 1) continue; bool ok = false;
    for (int r = 1; r < s; ++r) { x = mm(x, x, n); if (x == n - 1) { ok = true; break; } } if (!ok) return false; } return true; }

template <int LOGN, int RL, int S, bool LAZY>
static void fwd_emu(u64* lds, const u64* tw, u64 q) {
    if constexpr (S < LOGN) {
        constexpr int R = (LOGN - S) < RL ? (LOGN - S) : RL;
        for (int tid = 0; tid < (1 << LOGN) / 16; ++tid) ntt_pass<LOGN, S, R, true, 16, LAZY>(lds, tid, tw, q, 0, 0, 0, 0);
        fwd_emu<LOGN, RL, S + R, LAZY>(lds, tw, q);
    }
}
template <int LOGN, int RL, int S>
static void inv_emu(u64* lds, const u64* tw, u64 q, u64 s0, u64 s0s, u64 s1, u64 s1s) {
    if constexpr (S < LOGN) {
        constexpr int R = (LOGN - S) < RL ? (LOGN - S) : RL;
        inv_emu<LOGN, RL, S + R>(lds, tw, q, s0, s0s, s1, s1s);
        for (int tid = 0; tid < (1 << LOGN) / 16; ++tid) ntt_pass<LOGN, S, R, false, 16>(lds, tid, tw, q, s0, s0s, s1, s1s);
    }
}

template <int LOGN, bool LAZY>
static int run(int bits, int RLsel) {
    const int N = 1 << LOGN;
    u64 q = ((1ull << bits) - 1) / (2 * N) * (2 * N) + 1;
    while (!isprime(q)) q -= 2 * N;
    // minimal primitive 2N-th root not needed: any primitive 2N-th root gives a valid check
    u64 g = 2, psi = 0;
    for (;; ++g) { psi = pw(g, (q - 1) / (2 * N), q); if (pw(psi, N, q) == q - 1) break; }
    std::vector<u64> tw(2 * N), twi(2 * N);
    const u64 ipsi = pw(psi, q - 2, q);
    for (int k = 0; k < N; ++k) {
        tw[2 * rev(k, LOGN)] = pw(psi, k, q); twi[2 * rev(k, LOGN)] = pw(ipsi, k, q);
    }
    for (int k = 0; k < N; ++k) { tw[2 * k + 1] = (u64)(((u128h)tw[2 * k] << 64) / q); twi[2 * k + 1] = (u64)(((u128h)twi[2 * k] << 64) / q); }
    std::mt19937_64 rng(bits * 7 + LOGN);
    std::vector<u64> a(N), lds(N + N / 16);
    for (auto& x : a) x = rng() % q;
    for (int e = 0; e < N; ++e) lds[lds_pad(e)] = a[e];
    if (RLsel == 3) fwd_emu<LOGN, 3, 0, LAZY>(lds.data(), tw.data(), q); else fwd_emu<LOGN, 4, 0, LAZY>(lds.data(), tw.data(), q);
    int bad = 0;
    const u64 bound = LAZY ? (u64)(4 + 2 * LOGN) * q : 4 * q;
    for (int i = 0; i < N; ++i) {
        const u64 x = pw(psi, 2 * rev(i, LOGN) + 1, q);
        u64 v = 0, xp = 1;
        for (int k = 0; k < N; ++k) { v = (v + mm(a[k], xp, q)) % q; xp = mm(xp, x, q); }
        const u64 got = lds[lds_pad(i)];
        if (got >= bound || got % q != v) { if (bad < 3) printf("  fwd i=%d got %llu (mod q %llu) want %llu\n", i, (unsigned long long)got, (unsigned long long)(got % q), (unsigned long long)v); ++bad; }
    }
    // inverse back (canonicalise first)
    for (int i = 0; i < N; ++i) lds[lds_pad(i)] %= q;
    const u64 ninv = pw(N, q - 2, q), w1 = mm(twi[2], ninv, q);
    inv_emu<LOGN, 3, 0>(lds.data(), twi.data(), q, ninv, (u64)(((u128h)ninv << 64) / q), w1, (u64)(((u128h)w1 << 64) / q));
    for (int i = 0; i < N; ++i) if (lds[lds_pad(i)] % q != a[i] || lds[lds_pad(i)] >= 2 * q) { if (bad < 6) printf("  inv i=%d\n", i); ++bad; }
    printf("LOGN=%d bits=%d lazy=%d RL=%d bad=%d\n", LOGN, bits, (int)LAZY, RLsel, bad);
    return bad;
}
// Transforms whose first forward stage (last inverse stage) is done outside the LDS passes, as the
// half-limb kernels' register radix-4 does: the harness applies stage 0 with the same butterfly, the
// passes start at stage 1 (ntt_fwd_lds / ntt_inv_half_lds with S0 = 1; at LOGN = 13 this includes the
// radix-8 pass with TL = 8 whose LDS offsets are compile-time, fhs_ntt.h grp_pad).
template <int LOGN, bool LAZY>
static int run_s1(int bits) {
    const int N = 1 << LOGN, NH = N / 2;
    u64 q = ((1ull << bits) - 1) / (2 * N) * (2 * N) + 1;
    while (!isprime(q)) q -= 2 * N;
    u64 g = 2, psi = 0;
    for (;; ++g) { psi = pw(g, (q - 1) / (2 * N), q); if (pw(psi, N, q) == q - 1) break; }
    std::vector<u64> tw(2 * N), twi(2 * N);
    const u64 ipsi = pw(psi, q - 2, q);
    for (int k = 0; k < N; ++k) { tw[2 * rev(k, LOGN)] = pw(psi, k, q); twi[2 * rev(k, LOGN)] = pw(ipsi, k, q); }
    for (int k = 0; k < N; ++k) { tw[2 * k + 1] = (u64)(((u128h)tw[2 * k] << 64) / q); twi[2 * k + 1] = (u64)(((u128h)twi[2 * k] << 64) / q); }
    std::mt19937_64 rng(bits * 13 + LOGN);
    std::vector<u64> a(N), x(N), lds(N + N / 16);
    for (auto& v : a) v = rng() % q;
    for (int e = 0; e < NH; ++e) {   // stage 0: (e, e + N/2), twiddle tw[1]
        const u64 t = shoup_lazy(a[e + NH], tw[2], tw[3], q);
        x[e] = a[e] + t;
        x[e + NH] = a[e] + (2 * q - t);
    }
    for (int e = 0; e < N; ++e) lds[lds_pad(e)] = x[e];
    fwd_emu<LOGN, 3, 1, LAZY>(lds.data(), tw.data(), q);
    int bad = 0;
    const u64 bound = LAZY ? (u64)(4 + 2 * LOGN) * q : 4 * q;
    for (int i = 0; i < N; i += (i % 97 == 0 ? 1 : 13)) {   // a sample of outputs (direct evaluation is O(N^2))
        const u64 xe = pw(psi, 2 * rev(i, LOGN) + 1, q);
        u64 v = 0, xp = 1;
        for (int k = 0; k < N; ++k) { v = (v + mm(a[k], xp, q)) % q; xp = mm(xp, xe, q); }
        const u64 got = lds[lds_pad(i)];
        if (got >= bound || got % q != v) { if (bad < 3) printf("  fwd_s1 i=%d\n", i); ++bad; }
    }
    for (int i = 0; i < N; ++i) lds[lds_pad(i)] %= q;
    inv_emu<LOGN, 3, 1>(lds.data(), twi.data(), q, 0, 0, 0, 0);   // stages >= 1 (no fold there)
    const u64 ninv = pw(N, q - 2, q), w1 = mm(twi[2], ninv, q);
    const u64 ns = (u64)(((u128h)ninv << 64) / q), w1s = (u64)(((u128h)w1 << 64) / q);
    for (int e = 0; e < NH; ++e) {   // stage 0 with N^-1 folded in, as inv_quad_last2 / inv_limb do
        const u64 X = lds[lds_pad(e)], Y = lds[lds_pad(e + NH)];
        const u64 r0 = shoup_lazy(X + Y, ninv, ns, q), r1 = shoup_lazy(X - Y + 2 * q, w1, w1s, q);
        if (r0 % q != a[e] || r1 % q != a[e + NH] || r0 >= 2 * q || r1 >= 2 * q) { if (bad < 6) printf("  inv_s1 e=%d\n", e); ++bad; }
    }
    printf("S0=1 LOGN=%d bits=%d lazy=%d bad=%d\n", LOGN, bits, (int)LAZY, bad);
    return bad;
}
// acc3_reduce_pm (ModUp conversion reduction) at its extreme inputs: ns = 3 source limbs of
// 60-bit residues, v = 3, for 59- and 60-bit pseudo-Mersenne primes
static int test_acc3_reduce() {
    int bad = 0;
    std::mt19937_64 rng(5);
    for (int bits : {59, 60}) {
        const int N = 16384;
        u64 q = ((1ull << bits) - 1) / (2 * N) * (2 * N) + 1;
        while (!isprime(q)) q -= 2 * N;
        const unsigned d = (unsigned)((1ull << bits) - q);
        const u64 p30 = (1ull << 30) - 1;
        for (int it = 0; it < 200000; ++it) {
            u64 L, M, H;
            if (it < 8) {   // corners
                L = (it & 1) ? 3 * p30 * p30 + 3 * (q - 1) : 0;
                M = (it & 2) ? 6 * p30 * p30 : 0;
                H = (it & 4) ? 3 * p30 * p30 : 0;
            } else {
                L = rng() % (3 * p30 * p30 + 3 * (q - 1) + 1);
                M = rng() % (6 * p30 * p30 + 1);
                H = rng() % (3 * p30 * p30 + 1);
            }
            const u64 r = acc3_reduce_pm(L, M, H, bits, d);
            const u128h x = (u128h)L + ((u128h)M << 30) + ((u128h)H << 60);
            if (r >= 2 * q || r % q != (u64)(x % q)) { if (bad < 3) printf("  acc3 bits=%d it=%d\n", bits, it); ++bad; }
        }
    }
    printf("acc3_reduce_pm bad=%d\n", bad);
    return bad;
}

int main() {
    int bad = test_acc3_reduce();
    bad += run<8, false>(59, 3) + run<8, true>(59, 3) + run<10, false>(59, 3) + run<10, true>(59, 3);
    bad += run<10, true>(59, 4) + run<9, true>(58, 3) + run<10, false>(60, 3) + run<11, true>(59, 3);
    bad += run_s1<13, true>(59) + run_s1<13, false>(60) + run_s1<10, true>(59);
    printf(bad ? "FAIL\n" : "OK\n");
    return bad != 0;
}
