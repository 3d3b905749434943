// CPU check of the wave-local NTT passes (fhs_ntt.h, round 5): wherever fwd_from / inv_from replace the
// workgroup barrier between two passes by a wave barrier, every element a thread touches in the second pass
// must have been written in the first by a thread of its own wave (64 lanes, or wl_width when the transform
// has fewer threads); and where a forward transform exits wave-locally (fwd_exit_wave_local), the elements a
// thread wrote in the last pass must be exactly wl_base(tid) + wl_off(q), q < EPT -- the positions the
// kernels then read without a barrier.  The element sets come from running fhs_ntt.h's own ntt_pass one
// thread at a time on random data and diffing the LDS array (a butterfly group is read and written in place).
// Build: g++ -O2 -std=c++17 -DFHS_ASM_SHOUP=0 -Itools/debug/shim -Ifhe-spear_amd/csrc tools/debug/wl_check.cpp
#include <cstdio>
#include <algorithm>
#include <random>
#include <vector>
#include "fhs_ntt.h"
using namespace fhs;

static const u64 Q = 576460752303439873ull;   // any odd modulus < 2^59 will do: only positions matter

static std::vector<u64> g_tw;

// element sets of one pass, thread by thread; returns the per-thread element lists (natural indices)
template <int LOGN, int S, int R, bool FWD, int EPT>
static std::vector<std::vector<int>> run_pass(std::vector<u64>& lds, const std::vector<int>& pos2e) {
    constexpr int N = 1 << LOGN, T = N / EPT;
    std::vector<std::vector<int>> sets(T);
    std::vector<u64> before;
    for (int t = 0; t < T; ++t) {
        before = lds;
        ntt_pass<LOGN, S, R, FWD, EPT, true>(lds.data(), t, g_tw.data(), Q, 1, 0, 1, 0, 1);
        for (size_t p = 0; p < lds.size(); ++p)
            if (lds[p] != before[p]) sets[t].push_back(pos2e[p]);
    }
    return sets;
}

static int check_local(const char* what, int W, const std::vector<std::vector<int>>& prev,
                       const std::vector<std::vector<int>>& next, int N) {
    std::vector<int> owner(N, -1);
    for (size_t t = 0; t < prev.size(); ++t)
        for (int e : prev[t]) owner[e] = (int)t;
    int bad = 0;
    for (size_t t = 0; t < next.size(); ++t)
        for (int e : next[t])
            if (owner[e] < 0 || owner[e] / W != (int)t / W) {
                if (bad < 3) printf("  %s: thread %zu touches element %d written by thread %d\n", what, t, e, owner[e]);
                ++bad;
            }
    return bad;
}

// forward passes from S0 with radix RL, as fwd_from<..., WL = true>
template <int LOGN, int RL, int S, int EPT, int S0>
static int fwd_chain(std::vector<u64>& lds, const std::vector<int>& pos2e, std::vector<std::vector<int>>& prev,
                     bool prev_skip) {
    if constexpr (S < LOGN) {
        constexpr int R = pass_r<LOGN, RL, S>();
        constexpr int W = wl_width<LOGN, EPT>();
        auto sets = run_pass<LOGN, S, R, true, EPT>(lds, pos2e);
        int bad = 0;
        if (prev_skip) bad += check_local("fwd", W, prev, sets, 1 << LOGN);
        constexpr int S2 = S + R;
        constexpr bool here = pass_tl<LOGN, S, R>() <= W;
        constexpr bool next = S2 >= LOGN || (pass_r<LOGN, RL, S2>() == R && pass_tl<LOGN, S2, pass_r<LOGN, RL, S2>()>() <= W);
        prev = sets;
        return bad + fwd_chain<LOGN, RL, S2, EPT, S0>(lds, pos2e, prev, here && next);
    }
    return 0;
}

template <int LOGN, int RL, int EPT, int S0>
static int check_fwd() {
    constexpr int N = 1 << LOGN, T = N / EPT;
    std::vector<u64> lds(N + N / 16);
    std::vector<int> pos2e(lds.size(), -1);
    for (int e = 0; e < N; ++e) pos2e[lds_pad(e)] = e;
    std::mt19937_64 rng(LOGN * 131 + RL * 7 + S0);
    for (int e = 0; e < N; ++e) lds[lds_pad(e)] = rng() % Q;
    std::vector<std::vector<int>> last;
    int bad = fwd_chain<LOGN, RL, S0, EPT, S0>(lds, pos2e, last, false);
    int nskip = 0;
    if constexpr (fwd_exit_wave_local<LOGN, RL, S0, EPT>()) {   // the callers' wl_base + wl_off reads
        constexpr int GS = 1 << RL;
        std::vector<std::vector<int>> reads(T);
        std::vector<int> hit(N, 0);
        for (int t = 0; t < T; ++t)
            for (int q = 0; q < EPT; ++q) {
                const int e = wl_base<LOGN, EPT, GS>(t) + wl_off<LOGN, EPT, GS>(q);
                reads[t].push_back(e);
                ++hit[e];
            }
        nskip = check_local("exit", wl_width<LOGN, EPT>(), last, reads, N);
        for (int e = 0; e < N; ++e)   // and the reads cover every output once
            if (hit[e] != 1) {
                if (nskip < 3) printf("  exit: element %d read %d times\n", e, hit[e]);
                ++nskip;
            }
    }
    printf("fwd LOGN=%d RL=%d EPT=%d S0=%d exit_wave_local=%d bad=%d\n", LOGN, RL, EPT, S0,
           (int)fwd_exit_wave_local<LOGN, RL, S0, EPT>(), bad + nskip);
    return bad + nskip;
}

// inverse passes from the deepest chunk down to S0, as inv_from<..., WL = true, S0>
template <int LOGN, int RL, int EPT, int S0>
static int check_inv() {
    constexpr int N = 1 << LOGN;
    constexpr int W = wl_width<LOGN, EPT>();
    std::vector<u64> lds(N + N / 16);
    std::vector<int> pos2e(lds.size(), -1);
    for (int e = 0; e < N; ++e) pos2e[lds_pad(e)] = e;
    std::mt19937_64 rng(LOGN * 17 + RL + S0);
    for (int e = 0; e < N; ++e) lds[lds_pad(e)] = rng() % Q;
    // chunk starts S0, S0 + RL, ... executed last-to-first
    std::vector<int> starts;
    for (int s = S0; s < LOGN; s += RL) starts.push_back(s);
    int bad = 0;
    std::vector<std::vector<int>> prev;
    bool skip = false;
    if constexpr ((LOGN - S0) % RL == 0) {
        // wave-local head (k_ks_intt_h, inv_limb): each thread stores its input at wl_base + wl_off with no
        // barrier before the deepest pass
        constexpr int T = N / EPT, GS = 1 << RL;
        prev.assign(T, {});
        for (int t = 0; t < T; ++t)
            for (int q = 0; q < EPT; ++q) prev[t].push_back(wl_base<LOGN, EPT, GS>(t) + wl_off<LOGN, EPT, GS>(q));
        skip = true;
    }
    for (int i = (int)starts.size() - 1; i >= 0; --i) {
        std::vector<std::vector<int>> sets;
        bool local_after = false;
        auto run = [&](auto sc) {
            constexpr int S = decltype(sc)::value;
            constexpr int R = pass_r<LOGN, RL, S>();
            sets = run_pass<LOGN, S, R, false, EPT>(lds, pos2e);
            if constexpr (S - RL >= S0)
                local_after = R == RL && pass_tl<LOGN, S, R>() <= W && pass_tl<LOGN, S - RL, RL>() <= W;
        };
        switch (starts[i]) {   // S is a template argument: the chunk starts a transform of <= 14 stages can have
#define FHS_CASE(k) case k: if constexpr (k < LOGN && (k - S0) % RL == 0 && k >= S0) run(std::integral_constant<int, k>{}); break;
            FHS_CASE(0) FHS_CASE(1) FHS_CASE(2) FHS_CASE(3) FHS_CASE(4) FHS_CASE(5) FHS_CASE(6) FHS_CASE(7)
            FHS_CASE(8) FHS_CASE(9) FHS_CASE(10) FHS_CASE(11) FHS_CASE(12) FHS_CASE(13)
#undef FHS_CASE
        }
        if (skip) bad += check_local("inv", W, prev, sets, N);
        prev = sets;
        skip = local_after;
    }
    printf("inv LOGN=%d RL=%d EPT=%d S0=%d bad=%d\n", LOGN, RL, EPT, S0, bad);
    return bad;
}

int main() {
    g_tw.resize(2 * 2 * 16384);
    std::mt19937_64 rng(5);
    for (size_t i = 0; i < g_tw.size(); i += 2) { g_tw[i] = rng() % Q; g_tw[i + 1] = rng(); }
    int bad = 0;
    // the kernels' shapes: half limbs of N = 16384 (LOGN 13) and 32768 (14) after a register radix-4 (S0 = 1),
    // whole limbs with S0 = 0, one-wave transforms (N = 1024: 64 threads -> wl_width 64; N = 512: 32)
    bad += check_fwd<13, 3, 16, 1>();
    bad += check_fwd<14, 3, 16, 1>();
    bad += check_fwd<14, 3, 16, 2>();   // N = 32768 half limbs after the radix-8 first stages (fwd_oct_first3)
    bad += check_fwd<13, 3, 16, 0>();
    bad += check_fwd<12, 3, 16, 0>();
    bad += check_fwd<10, 3, 16, 1>();
    bad += check_fwd<9, 3, 16, 0>();
    bad += check_fwd<13, 4, 16, 1>();
    bad += check_inv<13, 3, 16, 1>();
    bad += check_inv<14, 3, 16, 1>();
    bad += check_inv<13, 3, 16, 0>();
    bad += check_inv<10, 3, 16, 1>();
    bad += check_inv<9, 3, 16, 0>();
    bad += check_inv<13, 4, 16, 1>();
    bad += check_inv<14, 4, 16, 1>();
    bad += check_fwd<14, 4, 16, 1>();
    printf(bad ? "FAIL\n" : "OK\n");
    return bad ? 1 : 0;
}
