// fhs_host.hip -- host side of libfhespear_hip.so: parameter tables, object lifetime, key
// generation, CKKS encode/decode, and every extern "C" entry point of include/fhespear.h.
//
// Runtime model (MI355X-first):
//  - one context = one device + one HIP stream; device blocks come from hipMalloc behind a bounded
//    per-size caching free list reused in stream order, so a free never synchronises the host;
//  - calls on a context are serialised by a mutex (ctypes drops the GIL; bg:223-249 may call
//    from a thread pool);
//  - rotations are DEFERRED and batched: fhs_rotate allocates the output and queues the
//    key-switch; the queue is flushed as one batched key-switch by the next operation that is
//    not a rotation at the same level.  The reference's baby-step loop (bg:215-220) issues G-1
//    independent rotations back to back; batching turns 39 workgroups per rotation into
//    39 (G-1) workgroups per launch.  Each rotation is computed exactly as it would be alone.
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <csignal>
#include <atomic>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstring>
#include <map>
#include <unordered_map>
#include <chrono>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fhespear.h"
#include "fhs_kernels.h"
#include "fhs_modarith.h"

using fhs::DevTables;
using fhs::KsItem;
typedef unsigned __int128 hu128;

// ============================================================================ errors
static thread_local std::string g_err;
static fhs_status fail(fhs_status code, const std::string& msg) {
    g_err = msg;
    return code;
}
// FHESPEAR_SEGV_TRACE=1: print a native backtrace on SIGSEGV (diagnostics for faults outside
// Python frames, e.g. during process teardown, where faulthandler is no longer installed)
static void segv_trace(int sig) {
    void* fr[64];
    const int n = backtrace(fr, 64);
    static const char hdr[] = "[fhespear] native backtrace:\n";
    (void)!write(2, hdr, sizeof(hdr) - 1);
    backtrace_symbols_fd(fr, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
__attribute__((constructor)) static void segv_trace_install() {
    if (getenv("FHESPEAR_SEGV_TRACE")) signal(SIGSEGV, segv_trace);
}
static fhs_status hip_fail(hipError_t e, const char* where) {
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation)
        return fail(FHS_ERR_OOM, std::string("HIP out of memory in ") + where);
    return fail(FHS_ERR_HIP, std::string("HIP error in ") + where + ": " + hipGetErrorString(e));
}
#define HIPCHK(expr, where)                                  \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return hip_fail(_e, where);    \
    } while (0)

extern "C" const char* fhs_last_error(void) { return g_err.c_str(); }
extern "C" const char* fhs_version(void) { return "fhespear-mi355x 0.1 (gfx950)"; }
extern "C" int fhs_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
extern "C" fhs_status fhs_device_pci_bus_id(int device, char* buf, int len) {
    if (!buf || len < 13) return fail(FHS_ERR_INVALID, "device_pci_bus_id: buffer of at least 13 bytes");
    hipError_t e = hipDeviceGetPCIBusId(buf, len, device);
    if (e != hipSuccess) return hip_fail(e, "device_pci_bus_id");
    return FHS_OK;
}

// ============================================================================ host number theory
static inline uint64_t h_mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)(((hu128)a * b) % q); }
static uint64_t h_pow(uint64_t b, uint64_t e, uint64_t q) {
    uint64_t r = 1 % q;
    b %= q;
    while (e) {
        if (e & 1) r = h_mulmod(r, b, q);
        b = h_mulmod(b, b, q);
        e >>= 1;
    }
    return r;
}
static uint64_t h_inv(uint64_t a, uint64_t q) { return h_pow(a % q, q - 2, q); }
static uint64_t h_shoup(uint64_t w, uint64_t q) { return (uint64_t)(((hu128)w << 64) / q); }

// q = 2^b - d qualifies for pm_reduce128 (fhs_modarith.h) when its three folds provably take
// every 128-bit input below 2q: B_{k+1} = (B_k >> b) d + 2^b - 1 from B_0 = 2^128 - 1, with the
// fold-2 quotient < 2^64 and the fold-3 quotient < 2^32.  Returns the PrimeK.pm word or 0.
static uint64_t pm_word(uint64_t q, int logN) {
    int b = 64 - __builtin_clzll(q);
    if (b < 40 || b > 62) return 0;
    const uint64_t d = (1ull << b) - q;
    if (d >= (1ull << 32)) return 0;
    const hu128 lim = ((hu128)1 << b) - 1;
    const hu128 B0 = ~(hu128)0;
    const hu128 h1 = B0 >> b;                       // < 2^88: product with d may overflow -> check
    if ((h1 >> 96) != 0) return 0;
    const hu128 B1 = h1 * d + lim;                  // h1 < 2^96, d < 2^32 -> < 2^128
    if (B1 < h1 * d) return 0;
    const hu128 h2 = B1 >> b;
    if ((h2 >> 64) != 0) return 0;
    const hu128 B2 = h2 * d + lim;
    const hu128 h3 = B2 >> b;
    if ((h3 >> 32) != 0) return 0;
    const hu128 B3 = h3 * d + lim;
    if (B3 >= 2 * (hu128)q) return 0;
    const bool lazy = (hu128)q * (uint64_t)(4 + 2 * logN) < ((hu128)1 << 64);   // fhs_ntt.h LAZY bound
    return (d << 8) | (lazy ? 128u : 0u) | (uint64_t)b;
}

// A 59-bit prime q = 2^59 - d with d < 2^27: the precondition of convert3x_b59's bounds.
static bool b59_prime(uint64_t q) { return q < (1ull << 59) && (1ull << 59) - q < (1ull << 27); }
// Bit 40 of PrimeK.pm: the ModUp conversion may reduce its split-30 sums directly
// (fhs_modarith.h acc3_reduce_pm): with ns <= P source limbs (< 2^60 each) and the v (Q mod m)
// correction folded into L, every intermediate of that routine stays in its word and the result is
// below 2q.  Checked here with exact bounds for this prime.
static bool conv_pm_ok(uint64_t q, int ns) {
    const int b = 64 - __builtin_clzll(q);
    if (b < 40 || b > 60 || ns < 1 || ns > 7) return false;
    const hu128 d = ((hu128)1 << b) - q;
    const hu128 p30 = ((hu128)1 << 30) - 1, M64 = ~(hu128)0 >> 64;   // 2^64 - 1
    const hu128 Lmax = (hu128)ns * p30 * p30 + (hu128)ns * (q - 1);
    const hu128 Mmax = (hu128)2 * ns * p30 * p30, Hmax = (hu128)ns * p30 * p30;
    const int sh = b - 30;
    const hu128 Amax = Lmax + ((((hu128)1 << sh) - 1) << 30);
    const hu128 Bmax = (Mmax >> sh) + (Hmax << (60 - b));
    if (Lmax > M64 || Mmax > M64 || Amax > M64 || Bmax > M64) return false;
    if ((Bmax >> 64) != 0 || d >= ((hu128)1 << 32)) return false;
    const hu128 Smax = Amax + Bmax * d;   // < 2^96
    const hu128 Sh = Smax >> b;
    if (Sh >= ((hu128)1 << 32)) return false;
    const hu128 rmax = (((hu128)1 << b) - 1) + Sh * d;
    return rmax < 2 * (hu128)q;
}
// X form of the centred extension for full 3-limb digits (fhs_modarith.h centered_x_pack /
// convert3x_value, fhs_kernels.hip k_centered_x): per digit j (primes 3j..3j+2, j < dnum with 3j + 3 <=
// L0) the exact Q_S / q_u, the rounding thresholds ((2k - 1) Q_S + 1) / 2 and 2^179 - v Q_S (192-bit
// words, little-endian) into xd[j][32]; per prime m the base-2^60 weights 2^60, 2^120 mod m (split-30
// packed) and -2^179 mod m into xt[i][4].  |X| < Q_S / 2 < 2^179 (three primes below 2^60; < 2^176 for the
// 59-bit chain), so U = X + 2^179 lies in (0, 2^180): exactly three 60-bit words.
static void modup_xform_tables(const uint64_t* primes, int K, int L0, int dnum, uint64_t* xd, uint64_t* xt) {
    auto mul192 = [](const uint64_t a[3], uint64_t m, uint64_t r[3]) {   // r = a m mod 2^192
        hu128 cy = 0;
        for (int w = 0; w < 3; ++w) {
            const hu128 t = (hu128)a[w] * m + cy;
            r[w] = (uint64_t)t;
            cy = t >> 64;
        }
    };
    for (int j = 0; j < dnum && 3 * j + 3 <= L0; ++j) {
        const uint64_t* q3 = &primes[3 * j];
        uint64_t* d = &xd[(size_t)j * 32];
        for (int u = 0; u < 3; ++u) {
            const hu128 h = (hu128)q3[(u + 1) % 3] * q3[(u + 2) % 3];
            d[2 * u] = (uint64_t)h;
            d[2 * u + 1] = (uint64_t)(h >> 64);
        }
        const uint64_t one[3] = {1, 0, 0};
        uint64_t Q[3], t[3];
        mul192(one, q3[0], t);
        mul192(t, q3[1], Q);
        mul192(Q, q3[2], t);
        std::copy(t, t + 3, Q);
        for (int k = 1; k <= 3; ++k) {   // ((2k - 1) Q + 1) / 2: (2k - 1) Q is odd, so + 1 is carry-free
            uint64_t m[3];
            mul192(Q, (uint64_t)(2 * k - 1), m);
            m[0] += 1;
            uint64_t* th = d + 6 + 3 * (k - 1);
            th[0] = (m[0] >> 1) | (m[1] << 63);
            th[1] = (m[1] >> 1) | (m[2] << 63);
            th[2] = m[2] >> 1;
        }
        for (int v = 0; v <= 3; ++v) {   // 2^179 - v Q
            uint64_t m[3];
            mul192(Q, (uint64_t)v, m);
            uint64_t* c = d + 15 + 3 * v;
            const uint64_t top[3] = {0, 0, 1ull << (179 - 128)};
            uint64_t br = 0;
            for (int w = 0; w < 3; ++w) {
                const hu128 s = (hu128)top[w] - m[w] - br;
                c[w] = (uint64_t)s;
                br = (uint64_t)(s >> 64) ? 1 : 0;
            }
        }
    }
    for (int i = 0; i < K; ++i) {
        const uint64_t m = primes[i];
        uint64_t p60 = 1 % m;
        for (int e = 0; e < 60; ++e) p60 = h_mulmod(p60, 2, m);
        const uint64_t p120 = h_mulmod(p60, p60, m);
        uint64_t p179 = 1 % m;
        for (int e = 0; e < 179; ++e) p179 = h_mulmod(p179, 2, m);
        xt[(size_t)i * 4 + 0] = p60;   // convert3x_value takes it as one 32-bit word (< 2^30 checked by the caller)
        xt[(size_t)i * 4 + 1] = pack30(p120);
        xt[(size_t)i * 4 + 2] = p179 ? m - p179 : 0;
    }
}
static bool h_is_prime(uint64_t n) {
    if (n < 2) return false;
    const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (uint64_t p : bases) {
        if (n == p) return true;
        if (n % p == 0) return false;
    }
    uint64_t d = n - 1;
    int s = 0;
    while (!(d & 1)) { d >>= 1; ++s; }
    for (uint64_t a : bases) {
        uint64_t x = h_pow(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int r = 1; r < s && comp; ++r) {
            x = h_mulmod(x, x, n);
            if (x == n - 1) comp = false;
        }
        if (comp) return false;
    }
    return true;
}
static uint32_t h_bitrev(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}
// minimal primitive 2N-th root of unity mod q (SEAL / Phantom convention)
static uint64_t h_min_root(uint64_t q, uint64_t N) {
    const uint64_t cof = (q - 1) / (2 * N);
    uint64_t g = 0;
    for (uint64_t c = 2;; ++c) {
        g = h_pow(c, cof, q);
        if (h_pow(g, N, q) == q - 1) break;
    }
    const uint64_t g2 = h_mulmod(g, g, q);
    uint64_t best = g, cur = g;
    for (uint64_t k = 1; k < N; ++k) {
        cur = h_mulmod(cur, g2, q);
        if (cur < best) best = cur;
    }
    return best;
}

extern "C" fhs_status fhs_create_coeff_modulus(uint64_t N, const int* bits, int n, uint64_t* out) {
    if (!bits || !out || n <= 0 || N < 2 || (N & (N - 1))) return fail(FHS_ERR_INVALID, "create_coeff_modulus: bad args");
    const uint64_t fac = 2 * N;
    std::map<int, std::vector<uint64_t>> pool;
    std::map<int, int> need, used;
    for (int i = 0; i < n; ++i) {
        if (bits[i] < 2 || bits[i] > 61) return fail(FHS_ERR_INVALID, "create_coeff_modulus: bit size must be in [2, 61]");
        need[bits[i]]++;
    }
    for (auto& kv : need) {
        const int b = kv.first;
        uint64_t v = ((uint64_t)1 << b) - fac + 1;
        const uint64_t lo = (uint64_t)1 << (b - 1);
        while ((int)pool[b].size() < kv.second && v > lo) {
            if (h_is_prime(v)) pool[b].push_back(v);
            v -= fac;
        }
        if ((int)pool[b].size() < kv.second) return fail(FHS_ERR_INVALID, "create_coeff_modulus: not enough primes");
    }
    for (int i = 0; i < n; ++i) out[i] = pool[bits[i]][used[bits[i]]++];
    return FHS_OK;
}

extern "C" uint64_t fhs_galois_elt_from_step(int step, uint64_t N) {
    const uint64_t m = 2 * N;
    if (step == 0) return m - 1;
    const uint64_t slots = N / 2;
    uint64_t s = step > 0 ? (uint64_t)step : slots - (uint64_t)(-(int64_t)step);
    s %= slots;
    uint64_t e = 1;
    for (uint64_t i = 0; i < s; ++i) e = (e * 5) & (m - 1);
    return e;
}

// ============================================================================ objects
struct PendingRot {
    KsItem item;
    fhs_ciphertext* out;
    const fhs_ciphertext* in;
};

struct fhs_context {
    int device = 0;
    hipStream_t st = nullptr;
    std::recursive_mutex mu;
    uint64_t N = 0;
    int logN = 0, L0 = 0, P = 0, K = 0, dnum = 0;
    std::vector<uint64_t> q;
    std::vector<uint64_t> elts;
    DevTables T{};
    std::vector<void*> tables;     // device allocations owned by the context
    void* items_dev = nullptr;     // KsItem[kMaxItems]
    void* ptrs_dev = nullptr;      // pointer arrays for BSGS (2 x kMaxPtrs)
    std::vector<PendingRot> pending;
    int pending_l = -1;
    std::set<const void*> pending_refs;   // inputs and outputs of queued rotations (destroy must flush)
    std::set<const void*> pending_outs;   // outputs of queued rotations (a consumer must flush)
    int debug_fail_flushes = 0;           // fhs_debug_fail_next_flushes (testing hook)
    std::vector<std::complex<double>> fft_w;   // exp(2 pi i k / N), k < N
    std::vector<std::complex<double>> dec_twist;   // (cos, sin)(pi k / N), k < N
    std::vector<uint64_t> slot_index;          // (5^j mod 2N - 1)/2, j < N/2
    std::atomic<uint64_t> bytes_live{0};
    // lifetime: the caller's reference + one per live object (ciphertext, plaintext, key), so objects
    // may be destroyed after fhs_context_destroy (Python finalisation order is arbitrary)
    std::atomic<int> refs{1};
    // caching allocator: freed device blocks are kept per exact size and reused in stream order
    // (every use of a block is ordered on `st`, aux-stream work is joined back into `st`).  A large
    // device allocation costs host time per GB and a free synchronises (tools/microbench/
    // alloc.hip); ciphertexts and plaintexts come in a handful of sizes, so almost every allocation
    // after warm-up is a free-list pop.  Trimmed on out-of-memory, at context destruction and exit.
    std::unordered_map<size_t, std::vector<void*>> free_blocks;
    // imported switching keys (fhs_*_keys_import): key -> its explicit a_j [dnum][K][N]
    std::unordered_map<const void*, uint64_t*> key_a;
    size_t cached_bytes = 0;
    // bounded: a chain walks down the levels, so every level brings new sizes and the sizes of the
    // levels behind it go cold.  Over the cap, whole sizes are evicted least-recently-used first
    // (a 13-block d=2048 chain otherwise parked 135 GB here).  FHESPEAR_CACHE_BYTES overrides.
    size_t cache_cap = 0;
    uint64_t cache_tick = 0;
    std::unordered_map<size_t, uint64_t> size_tick;   // last dalloc/dfree of each size
    // kernel timer (bench): events around the timed kernel launches
    // per-kernel event timer (fhs_kernel_timer): bitmask of fhs::KernelId, completed pairs per id
    uint32_t timer_mask = 0;
    std::vector<hipEvent_t> timer_open;                              // begin event per id
    std::vector<std::vector<std::pair<hipEvent_t, hipEvent_t>>> timer_pairs;
    fhs::KTimer ktimer{};
    // pinned staging ring for launch descriptors (stage_h2d): kRingSegs segments; leaving a segment
    // records an event, re-entering it waits for that event (recorded a whole ring earlier)
    unsigned char* ring = nullptr;
    size_t ring_head = 0;          // next free byte; always inside segment ring_seg (or at its end)
    int ring_seg = 0;
    static constexpr size_t kRingBytes = 16u << 20;
    static constexpr int kRingSegs = 8;
    static constexpr size_t kSegBytes = kRingBytes / kRingSegs;
    hipEvent_t ring_ev[kRingSegs] = {};
    uint64_t ring_waits = 0, ring_blocked = 0;   // segment re-entries; of those, the ones that had to wait
    fhs::Stager stager{};
    std::map<std::pair<int, int>, std::vector<uint64_t>> crt_cache;   // decoder tables per (kk, l) (crt_tables)
    // pinned, grow-only: the decoder's slots (and flags) come back through it
    double* readback = nullptr;
    size_t readback_bytes = 0;
    // grow-only scratch buffers reused across calls (stream order makes reuse safe): a large
    // allocation costs host time per GB
    // SEAL-convention hoisting (fhs_kernels.h SealHoist): the per-(key, level) corrections [2][l+P][N],
    // the zero flag (device word + pinned host word) and the counts of hoisted / fallback flushes
    std::map<std::pair<const uint64_t*, int>, uint64_t*> seal_corr;
    size_t seal_corr_bytes = 0;
    size_t seal_corr_cap = 0;     // bound on seal_corr_bytes (1/16 of the context's device; FHESPEAR_SEAL_CORR_BYTES)
    fhs::SealHoist seal_hoist{};
    enum { SCR_KS, SCR_BSGS_INNER, SCR_BSGS_WS, SCR_BSGS_SUM, SCR_RESCALE, SCR_ENC_PTRS, SCR_COUNT };
    uint64_t* scr[SCR_COUNT] = {};
    size_t scr_bytes[SCR_COUNT] = {};
    static constexpr int kMaxItems = 512;
    static constexpr int kMaxPtrs = 1 << 16;
};

struct fhs_ciphertext {
    fhs_context* ctx;
    uint64_t* d;
    int ncomp, ci, l;
    double scale;
    // the queued rotation that was to produce it could not run (flush failed, e.g. out of memory): its limbs are
    // undefined and every later use fails (drop_pending)
    bool lost = false;
};
// One device block shared by the plaintexts of a batch (new_pts): a block per plaintext cost a hipMalloc per
// diagonal and, once a chain walking down the levels pushed the cache over its cap, thousands of hipFree's
// (round-5 cfg5 leg: 0.5-4.7 s per FFN block instead of ~0.2).  Freed when its last plaintext is destroyed.
struct PtSlab {
    uint64_t* base;
    size_t bytes;
    int refs;
};
struct fhs_plaintext {
    fhs_context* ctx;
    uint64_t* d;
    int ci, l;
    double scale;
    PtSlab* slab = nullptr;   // non-null: d points into a batch's shared block
    // compact shadow of a periodic plaintext (encode_rows_dev): word e >> tlog of each limb (N >> tlog words)
    // equals dense word e; read by the fused BSGS's Hadamard only (2^-tlog of the diagonal bytes).  Plaintexts
    // are immutable, so the two never diverge; every other op reads d.
    uint64_t* dc = nullptr;
    int tlog = 0;
    PtSlab* cslab = nullptr;
};
struct fhs_secret_key {
    fhs_context* ctx;
    uint64_t* s;   // K limbs, NTT
    PrfKey key;    // 256-bit PRF key all secret randomness is drawn from
    uint64_t ctr;  // symmetric-encryption counter
    uint64_t pk_gen = 0;   // public keys generated so far (each gets its own mask stream)
};
struct fhs_public_key {
    fhs_context* ctx;
    uint64_t* pk;  // 2 x L0
    PrfKey rng;    // encryption-mask key: a PRF output of the secret key (reveals nothing about it)
    uint64_t ctr;
};
struct fhs_relin_key {
    fhs_context* ctx;
    uint64_t* key;
};
struct fhs_galois_keys {
    fhs_context* ctx;
    std::map<uint64_t, uint64_t*> keys;
};

static void ctx_retain(fhs_context* c) { c->refs.fetch_add(1); }

// Live contexts, for the out-of-memory path (every context's cached blocks on the device are
// released before the retry) and for the process-exit release.  Device blocks come from plain
// hipMalloc behind the per-size cache: round 1 used stream-ordered pools with an infinite release
// threshold, and a process exiting with a multi-GB pool still mapped crashed inside libamdhip64's
// exit handler (a 13-block d=2048 FFN chain with 135 GB cached), and a pool that had been driven to
// out-of-memory left the next process exit crashing too.  release_at_exit is registered with atexit()
// after the first context's stream exists (i.e. after HIP registered its own handlers), so it runs
// first and returns every cached block.
static std::mutex g_live_mu;
static std::set<fhs_context*> g_live;
static void trim_cache(fhs_context* c);
static void release_at_exit() {
    // try_lock, as trim_other_caches: a thread still inside a context (holding c->mu, possibly about
    // to take g_live_mu on its out-of-memory path) keeps that context's cache rather than deadlock exit
    std::lock_guard<std::mutex> lk(g_live_mu);
    for (fhs_context* c : g_live) {
        std::unique_lock<std::recursive_mutex> cl(c->mu, std::try_to_lock);
        if (cl.owns_lock()) trim_cache(c);
    }
}
static void ctx_release(fhs_context* c);

// switching key in HBM: b_j [dnum][K][N] then the dnum seeds of the uniform a_j, which the key
// inner product regenerates on the fly (SAMPLE_SEEDED): half the bytes of storing (b_j, a_j)
static size_t key_words(const fhs_context* c) { return (size_t)c->dnum * c->K * c->N + (size_t)c->dnum; }
// exported / oracle layout: [dnum][2][K][N]
static size_t key_words_full(const fhs_context* c) { return (size_t)c->dnum * 2 * c->K * c->N; }
static void dfree(fhs_context* c, void* p, size_t bytes);
// an imported key's explicit a_j (null for generated keys, whose a_j are regenerated from seeds)
static const uint64_t* key_akey(const fhs_context* c, const uint64_t* key) {
    auto it = c->key_a.find(key);
    return it == c->key_a.end() ? nullptr : it->second;
}
static void drop_seal_corr(fhs_context* c, const uint64_t* key);
static void free_key(fhs_context* c, uint64_t* key) {
    drop_seal_corr(c, key);
    auto it = c->key_a.find(key);
    if (it != c->key_a.end()) {
        dfree(c, it->second, 8ull * c->dnum * c->K * c->N);
        c->key_a.erase(it);
    }
    dfree(c, key, 8 * key_words(c));
}

static void ctx_sync(fhs_context* c) {
    hipStreamSynchronize(c->st);
}
// every cached block back to the device (the caller holds c->mu)
static void trim_cache(fhs_context* c) {
    if (c->free_blocks.empty()) return;
    if (getenv("FHESPEAR_TRACE_LIFETIME"))
        fprintf(stderr, "[fhespear] trim: %zu cached bytes in %zu sizes, %llu live\n", c->cached_bytes,
                c->free_blocks.size(), (unsigned long long)c->bytes_live.load());
    ctx_sync(c);   // a cached block may still be read by queued work
    for (auto& kv : c->free_blocks)
        for (void* p : kv.second) (void)hipFree(p);
    c->free_blocks.clear();
    c->cached_bytes = 0;
}
// out-of-memory retry: the other contexts on the device give their caches back too (try_lock: a
// context busy on another thread keeps its cache rather than risk a lock-order inversion)
static void trim_other_caches(fhs_context* self) {
    std::lock_guard<std::mutex> lk(g_live_mu);
    for (fhs_context* c : g_live) {
        if (c == self || c->device != self->device) continue;
        std::unique_lock<std::recursive_mutex> cl(c->mu, std::try_to_lock);
        if (cl.owns_lock()) trim_cache(c);
    }
}
static void evict_cold(fhs_context* c, size_t keep) {
    std::vector<void*> victims;
    while (c->cached_bytes > c->cache_cap) {
        size_t victim = 0;
        uint64_t oldest = ~0ull;
        for (auto& kv : c->free_blocks)
            if (kv.first != keep && !kv.second.empty() && c->size_tick[kv.first] < oldest) {
                oldest = c->size_tick[kv.first];
                victim = kv.first;
            }
        if (!victim) victim = keep;   // only the size in hand is cached: shed its blocks
        auto& v = c->free_blocks[victim];
        while (!v.empty() && c->cached_bytes > c->cache_cap) {
            victims.push_back(v.back());
            v.pop_back();
            c->cached_bytes -= victim;
        }
        if (v.empty()) c->free_blocks.erase(victim);
    }
    if (victims.empty()) return;
    ctx_sync(c);
    for (void* p : victims) (void)hipFree(p);
}
// FHESPEAR_CONTIG_BYTES=n (default 0 = never): allocations of at least n bytes ask for physically contiguous memory
// (hipDeviceMallocContiguous), falling back to plain hipMalloc when refused.  Round 6 (tools/debug/alloc_spread.py,
// profiles/r06/alloc_spread/): the Hadamard's time follows where its 9.66 GB diagonal slab lands in HBM -- the same
// process, clocks and data re-allocated ten times ran 1.79-2.02 ms (hipMalloc) and 1.75-2.01 ms (contiguous), the
// contiguous placements mostly at the fast end (mean -2 % and -6 % on two boxes); but on the bench's own
// allocation sequence both landed at 2.00-2.05 ms (4 + 4 interleaved runs, profiles/r06/alloc_spread/ab_bench.txt),
// so it stays off.
static hipError_t dev_malloc(void** v, size_t bytes) {
    static const size_t contig = [] {
        const char* e = getenv("FHESPEAR_CONTIG_BYTES");
        return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)0;
    }();
    if (contig && bytes >= contig) {
        if (hipExtMallocWithFlags(v, bytes, hipDeviceMallocContiguous) == hipSuccess) return hipSuccess;
        (void)hipGetLastError();
    }
    return hipMalloc(v, bytes);
}
static hipError_t dalloc(fhs_context* c, uint64_t** p, size_t bytes) {
    bytes = bytes ? bytes : 8;
    c->size_tick[bytes] = ++c->cache_tick;
    auto it = c->free_blocks.find(bytes);
    if (it != c->free_blocks.end() && !it->second.empty()) {
        *p = static_cast<uint64_t*>(it->second.back());
        it->second.pop_back();
        c->cached_bytes -= bytes;
        c->bytes_live += bytes;
        return hipSuccess;
    }
    void* v = nullptr;
    hipError_t e = dev_malloc(&v, bytes);
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {   // give every cache back, retry once
        (void)hipGetLastError();
        trim_cache(c);
        trim_other_caches(c);
        e = dev_malloc(&v, bytes);
    }
    if (e == hipSuccess) {
        *p = (uint64_t*)v;
        c->bytes_live += bytes;
    } else {
        (void)hipGetLastError();   // not sticky: the next launch's hipGetLastError must not see it
    }
    return e;
}
static void dfree(fhs_context* c, void* p, size_t bytes) {
    if (!p) return;
    bytes = bytes ? bytes : 8;
    c->free_blocks[bytes].push_back(p);
    c->cached_bytes += bytes;
    c->bytes_live -= bytes;
    c->size_tick[bytes] = ++c->cache_tick;
    if (c->cached_bytes > c->cache_cap) evict_cold(c, bytes);
}

static hipError_t scratch(fhs_context* c, int slot, size_t bytes, uint64_t** p) {
    if (bytes > c->scr_bytes[slot]) {
        if (c->scr[slot]) dfree(c, c->scr[slot], c->scr_bytes[slot]);
        c->scr[slot] = nullptr;
        c->scr_bytes[slot] = 0;
        hipError_t e = dalloc(c, &c->scr[slot], bytes);
        if (e != hipSuccess) return e;
        c->scr_bytes[slot] = bytes;
    }
    *p = c->scr[slot];
    return hipSuccess;
}

static fhs_status new_ct(fhs_context* c, int ncomp, int ci, double scale, fhs_ciphertext** out) {
    const int l = c->L0 + 1 - ci;
    if (l < 1) return fail(FHS_ERR_LEVEL, "chain index out of range");
    auto* ct = new fhs_ciphertext{c, nullptr, ncomp, ci, l, scale};
    hipError_t e = dalloc(c, &ct->d, 8ull * ncomp * l * c->N);
    if (e != hipSuccess) {
        delete ct;
        return hip_fail(e, "ciphertext allocation");
    }
    ctx_retain(c);
    *out = ct;
    return FHS_OK;
}
static fhs_status new_pt(fhs_context* c, int ci, double scale, fhs_plaintext** out) {
    const int l = c->L0 + 1 - ci;
    if (l < 1) return fail(FHS_ERR_LEVEL, "chain index out of range");
    auto* pt = new fhs_plaintext{c, nullptr, ci, l, scale};
    hipError_t e = dalloc(c, &pt->d, 8ull * l * c->N);
    if (e != hipSuccess) {
        delete pt;
        return hip_fail(e, "plaintext allocation");
    }
    ctx_retain(c);
    *out = pt;
    return FHS_OK;
}
// A block of at least *bytes: a cached block up to 1.5x the request is taken whole (*bytes becomes its size),
// so the batches of a chain walking down the levels reuse the larger blocks the levels above left in the
// cache instead of allocating (and, over the cap, freeing) one per level.
static hipError_t dalloc_fit(fhs_context* c, uint64_t** p, size_t* bytes) {
    size_t best = 0;
    for (auto& kv : c->free_blocks)
        if (!kv.second.empty() && kv.first >= *bytes && kv.first <= *bytes + *bytes / 2 && (!best || kv.first < best))
            best = kv.first;
    if (best) *bytes = best;
    return dalloc(c, p, *bytes);
}
// `count` new plaintexts at chain index ci in one device block (PtSlab, dalloc_fit).  On failure nothing is
// left allocated and outs[0..count) are null.
static fhs_status new_pts(fhs_context* c, size_t count, int ci, double scale, fhs_plaintext** outs) {
    const int l = c->L0 + 1 - ci;
    if (l < 1) return fail(FHS_ERR_LEVEL, "chain index out of range");
    for (size_t k = 0; k < count; ++k) outs[k] = nullptr;
    if (count == 0) return FHS_OK;
    if (count == 1) return new_pt(c, ci, scale, outs);
    // FHESPEAR_PT_PAD_WORDS (experiment, default 0): words of padding between a slab's plaintexts (read per call)
    const char* padv = getenv("FHESPEAR_PT_PAD_WORDS");
    const size_t pad = padv ? (strtoull(padv, nullptr, 10) + 1) & ~(size_t)1 : 0;
    const size_t per = (size_t)l * c->N + pad;
    auto* slab = new PtSlab{nullptr, 8 * count * per, 0};
    hipError_t e = dalloc_fit(c, &slab->base, &slab->bytes);
    if (e != hipSuccess) {
        delete slab;
        return hip_fail(e, "plaintext allocation");
    }
    if (getenv("FHESPEAR_TRACE_SLABS"))
        fprintf(stderr, "[fhespear] slab %p: %zu plaintexts, %zu bytes (block %zu)\n", (void*)slab->base, count,
                8 * count * per, slab->bytes);
    for (size_t k = 0; k < count; ++k) {
        outs[k] = new fhs_plaintext{c, slab->base + k * per, ci, l, scale, slab};
        ++slab->refs;
        ctx_retain(c);
    }
    return FHS_OK;
}
static size_t ct_bytes(const fhs_ciphertext* ct) { return 8ull * ct->ncomp * ct->l * ct->ctx->N; }
static size_t pt_bytes(const fhs_plaintext* pt) { return 8ull * pt->l * pt->ctx->N; }
// The dense limbs of a plaintext.  A compact-only one (a periodic diagonal batch, encode_rows_dev) gets them on first
// use -- expanded from its shadow on the stream (k_expand_compact) and kept for the rest of its life, so the fused
// BSGS, which reads the shadow, never pays for them.  Plaintexts are immutable: the two copies never diverge.
static hipError_t pt_dense(fhs_context* c, const fhs_plaintext* cpt, const uint64_t** out) {
    auto* pt = const_cast<fhs_plaintext*>(cpt);
    if (!pt->d) {
        if (!pt->dc) return hipErrorInvalidValue;
        uint64_t* d = nullptr;
        hipError_t e = dalloc(c, &d, pt_bytes(pt));
        if (e != hipSuccess) return e;
        e = fhs::launch_expand_compact(pt->dc, d, pt->l, c->N, pt->tlog, c->st);
        if (e != hipSuccess) {
            dfree(c, d, pt_bytes(pt));
            return e;
        }
        pt->d = d;
    }
    *out = pt->d;
    return hipSuccess;
}
#define PT_DENSE(var, pt, where)        \
    const uint64_t* var = nullptr;      \
    HIPCHK(pt_dense(c, (pt), &var), where)

// ---------------------------------------------------------------- timing events
// A pool of timing events per device: hipEventCreate can take milliseconds now and then (it may
// allocate a signal through the driver), so the timing hooks -- the bench's per-step events
// (fhs_event_record) and the per-kernel brackets (timer_rec) -- take pre-created events instead of
// creating them between enqueued launches, where a slow creation leaves the GPU idle inside an open
// bracket.  fhs_kernel_timer_arm tops the pool up before a timed region.
static std::mutex g_ev_mu;
static std::map<int, std::vector<hipEvent_t>> g_ev_free;
static std::unordered_map<hipEvent_t, int> g_ev_dev;
// events belong to the device current at creation: create on `dev`, whatever the calling thread has
// current (one thread may drive contexts on two GPUs), and leave the caller's current device as it was
static hipError_t ev_create_on(int dev, hipEvent_t* e) {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) cur = -1;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return hipErrorInvalidDevice;
    hipError_t r = hipEventCreate(e);
    if (cur >= 0 && cur != dev) (void)hipSetDevice(cur);
    return r;
}
static hipEvent_t ev_get(int dev) {
    {
        std::lock_guard<std::mutex> lk(g_ev_mu);
        auto& v = g_ev_free[dev];
        if (!v.empty()) {
            hipEvent_t e = v.back();
            v.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    if (ev_create_on(dev, &e) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_ev_mu);
    g_ev_dev[e] = dev;
    return e;
}
static void ev_put(hipEvent_t e) {
    if (!e) return;
    std::lock_guard<std::mutex> lk(g_ev_mu);
    auto it = g_ev_dev.find(e);
    if (it == g_ev_dev.end()) {
        hipEventDestroy(e);
        return;
    }
    g_ev_free[it->second].push_back(e);
}
static void ev_reserve(int dev, size_t n) {
    std::vector<hipEvent_t> made;
    {
        std::lock_guard<std::mutex> lk(g_ev_mu);
        if (g_ev_free[dev].size() >= n) return;
        n -= g_ev_free[dev].size();
    }
    for (size_t k = 0; k < n; ++k) {
        hipEvent_t e = nullptr;
        if (ev_create_on(dev, &e) != hipSuccess) break;
        made.push_back(e);
    }
    std::lock_guard<std::mutex> lk(g_ev_mu);
    for (hipEvent_t e : made) {
        g_ev_dev[e] = dev;
        g_ev_free[dev].push_back(e);
    }
}

// ---------------------------------------------------------------- host-side latency trace
// FHESPEAR_HOST_TRACE=1 prints the host time of each section of the BSGS entry point (stderr); used
// to check that no call blocks on the GPU queue (tools/debug/host_timing.py).
struct HostTrace {
    bool on;
    std::chrono::steady_clock::time_point t0;
    HostTrace() : on(getenv("FHESPEAR_HOST_TRACE") != nullptr), t0(std::chrono::steady_clock::now()) {}
    void mark(const char* what) {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[fhs host] %-28s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    }
};

// ---------------------------------------------------------------- staging
// Small host->device copies on the context stream.  A pageable-source hipMemcpyAsync returns only
// once the copy has run, i.e. once the stream has drained up to it, which would serialise the host
// with the GPU on every launch; staging through a pinned ring keeps the host ahead of the queue.
// The ring is cut into kRingSegs segments and a copy never straddles two.  Leaving segment k records
// an event on the stream after k's last copy; before k is written again -- a whole ring (16 MB of
// descriptors, hundreds of BSGS steps) later -- the host waits for that event, which has long
// completed.  Round 1-3 synchronised the whole stream on every wrap instead: the queue drained to
// empty, and any host delay right after it (e.g. an event creation, see timer_rec) left the GPU idle
// inside whatever kernel bracket was open.
static hipError_t stage_h2d(void* user, void* dst, const void* src, size_t bytes) {
    fhs_context* c = static_cast<fhs_context*>(user);
    constexpr size_t SEG = fhs_context::kSegBytes;
    if (!c->ring || bytes > SEG) {
        hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->st);
        return e == hipSuccess ? hipStreamSynchronize(c->st) : e;
    }
    const int seg = c->ring_seg;
    if (c->ring_head + bytes > (size_t)(seg + 1) * SEG) {   // leave segment `seg` for the next one
        hipEvent_t& out = c->ring_ev[seg];
        if (!out && hipEventCreateWithFlags(&out, hipEventDisableTiming) != hipSuccess) out = nullptr;
        hipError_t e = out ? hipEventRecord(out, c->st) : hipStreamSynchronize(c->st);
        if (e != hipSuccess) return e;
        const int next = (seg + 1) % fhs_context::kRingSegs;
        if (hipEvent_t in = c->ring_ev[next]) {
            ++c->ring_waits;
            if (hipEventQuery(in) == hipErrorNotReady) {
                ++c->ring_blocked;
                e = hipEventSynchronize(in);
                if (e != hipSuccess) return e;
            }
        }
        c->ring_seg = next;
        c->ring_head = (size_t)next * SEG;
    }
    unsigned char* p = c->ring + c->ring_head;
    memcpy(p, src, bytes);
    c->ring_head += (bytes + 255) & ~(size_t)255;
    return hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, c->st);
}

// ---------------------------------------------------------------- SEAL-convention hoisting
// FHESPEAR_SEAL_HOIST=0 keeps SEAL's per-rotation decomposition for every flush (A/B and test knob)
static bool seal_hoist_enabled() {
    const char* v = getenv("FHESPEAR_SEAL_HOIST");
    return !v || strcmp(v, "0") != 0;
}
static size_t seal_corr_bytes(const fhs_context* c, int l) { return 8ull * 2 * (l + c->P) * c->N; }
// the corrections of `key` (null: of every key), returned to the block cache in stream order
static void drop_seal_corr(fhs_context* c, const uint64_t* key) {
    for (auto it = c->seal_corr.begin(); it != c->seal_corr.end();) {
        if (key && it->first.first != key) { ++it; continue; }
        dfree(c, it->second, seal_corr_bytes(c, it->first.second));
        c->seal_corr_bytes -= seal_corr_bytes(c, it->first.second);
        it = c->seal_corr.erase(it);
    }
}
// The correction of every rotated item of a flush (computed once per (key, level) and kept with the key),
// and the zero-flag buffers.  Bounded: past FHESPEAR_SEAL_CORR_BYTES (default 1/16 of HBM) the cache is
// emptied before this flush's corrections are made (a chain walks down the levels; the corrections of the
// levels behind it go cold).
static hipError_t seal_prepare(fhs_context* c, std::vector<KsItem>& items, int l) {
    fhs::SealHoist& sh = c->seal_hoist;
    hipError_t e = hipSuccess;
    if (!sh.zflag_dev) {
        uint64_t* z = nullptr;
        e = dalloc(c, &z, 8);
        if (e != hipSuccess) return e;
        sh.zflag_dev = reinterpret_cast<unsigned*>(z);
    }
    if (!sh.zflag_host) {
        void* h = nullptr;
        e = hipHostMalloc(&h, 64, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        sh.zflag_host = static_cast<unsigned*>(h);
    }
    const size_t cap = c->seal_corr_cap;   // per context, from its own device (context_create)
    size_t need = 0;
    for (const KsItem& it : items)
        if (it.elt != 1 && !c->seal_corr.count({it.key, l})) need += seal_corr_bytes(c, l);
    if (need && c->seal_corr_bytes + need > cap) drop_seal_corr(c, nullptr);
    uint64_t* mask = nullptr;
    for (KsItem& it : items) {
        if (it.elt == 1) continue;
        auto f = c->seal_corr.find({it.key, l});
        if (f == c->seal_corr.end()) {
            if (!mask && (e = dalloc(c, &mask, 8ull * c->K * c->N)) != hipSuccess) break;
            uint64_t* corr = nullptr;
            if ((e = dalloc(c, &corr, seal_corr_bytes(c, l))) != hipSuccess) break;
            e = fhs::launch_seal_corr(c->T, it.key, it.akey, it.elt, l, mask, corr, c->st);
            if (e != hipSuccess) {
                dfree(c, corr, seal_corr_bytes(c, l));
                break;
            }
            f = c->seal_corr.emplace(std::make_pair(it.key, l), corr).first;
            c->seal_corr_bytes += seal_corr_bytes(c, l);
        }
        it.corr = f->second;
    }
    if (mask) dfree(c, mask, 8ull * c->K * c->N);
    return e;
}

// ---------------------------------------------------------------- deferred rotations
// Every flush empties the queue.  One that cannot launch marks its outputs lost (every later use of them fails
// loudly, live_ct) and no later flush may launch a key switch on inputs or outputs the caller has destroyed
// meanwhile -- the round-5 world-8 rehearsal's rank-0 abort: a flush failed out of memory, the queue kept its
// pointers, the objects were freed (and their blocks returned to the device when the cache was trimmed), and the
// next flush's key switch read and wrote freed memory.
static fhs_status drop_pending(fhs_context* c, fhs_status st) {
    if (st != FHS_OK)
        for (PendingRot& p : c->pending) p.out->lost = true;
    c->pending.clear();
    c->pending_refs.clear();
    c->pending_outs.clear();
    c->pending_l = -1;
    return st;
}
static fhs_status flush(fhs_context* c) {
    if (c->pending.empty()) return FHS_OK;
    const int R = (int)c->pending.size(), l = c->pending_l;
    // distinct inputs: rotations of the same ciphertext share one (hoisted) ModUp
    std::vector<KsItem> items(R);
    std::vector<const uint64_t*> uniq;
    std::map<const uint64_t*, int> idx;
    for (int r = 0; r < R; ++r) {
        items[r] = c->pending[r].item;
        auto ins = idx.emplace(items[r].a, (int)uniq.size());
        if (ins.second) uniq.push_back(items[r].a);
        items[r].src = (uint64_t)ins.first->second;
    }
    const int U = (int)uniq.size();
    const size_t wsb = fhs::keyswitch_workspace_bytes(c->T, R, U, l);
    uint64_t* ws = nullptr;
    HostTrace ht;
    hipError_t e = c->debug_fail_flushes > 0 ? (--c->debug_fail_flushes, hipErrorOutOfMemory)
                                             : scratch(c, fhs_context::SCR_KS, wsb, &ws);
    ht.mark("flush: workspace");
    if (e != hipSuccess) return drop_pending(c, hip_fail(e, "key-switch workspace"));
    fhs::SealHoist* sh = nullptr;
    if (c->T.ks_seal && U < R && seal_hoist_enabled()) {   // SEAL convention: one ModUp per shared input
        e = seal_prepare(c, items, l);
        if (e == hipSuccess) sh = &c->seal_hoist;
        else if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
            for (auto& it : items) it.corr = nullptr;   // no room for the corrections: per-rotation path
            e = hipSuccess;
        }
        ht.mark("flush: seal corrections");
        if (e != hipSuccess) return drop_pending(c, hip_fail(e, "seal corrections"));
    }
    e = fhs::launch_keyswitch(c->T, items.data(), R, reinterpret_cast<const fhs::u64* const*>(uniq.data()), U, l, ws,
                              wsb, c->items_dev, c->stager, c->st, c->timer_mask ? &c->ktimer : nullptr, sh);
    ht.mark("flush: launch keyswitch");
    if (e != hipSuccess) return drop_pending(c, hip_fail(e, "key-switch launch"));
    return drop_pending(c, FHS_OK);
}

struct Guard {
    fhs_context* c;
    std::lock_guard<std::recursive_mutex> lk;
    explicit Guard(fhs_context* c_) : c(c_), lk(c_->mu) {}
};
// a ciphertext whose producing rotation was dropped (drop_pending) is not an operand
static fhs_status live_ct(const fhs_ciphertext* a) {
    if (a && a->lost) return fail(FHS_ERR_INVALID, "ciphertext lost: the queued rotation producing it could not run "
                                                   "(an earlier call reported why)");
    return FHS_OK;
}
#define LIVE(ct)                                   \
    do {                                           \
        fhs_status _ls = live_ct(ct);              \
        if (_ls != FHS_OK) return _ls;             \
    } while (0)
#define ENTER(ctx)                                                           \
    if (!(ctx)) return fail(FHS_ERR_INVALID, "null context");               \
    Guard _g(ctx);                                                           \
    (void)hipGetLastError(); /* a failed HIP call of an earlier entry is not this one's */ \
    do {                                                                     \
        fhs_status _s = flush(ctx);                                          \
        if (_s != FHS_OK) return _s;                                         \
    } while (0)

// ============================================================================ context
extern "C" fhs_status fhs_context_create(uint64_t N, const uint64_t* primes, int nprimes, int special,
                                         const uint64_t* galois_elts, int n_elts, int device, fhs_context** out) {
    if (!primes || !out) return fail(FHS_ERR_INVALID, "context_create: null argument");
    segv_trace_install();
    if (N < 256 || N > 32768 || (N & (N - 1)))
        return fail(FHS_ERR_INVALID, "context_create: poly_modulus_degree must be a power of two in [256, 32768]");
    if (special < 1 || special >= nprimes) return fail(FHS_ERR_INVALID, "context_create: bad special modulus size");
    const int L0 = nprimes - special;
    if (L0 % special != 0)
        return fail(FHS_ERR_INVALID,
                    "context_create: data primes (L0) must be a multiple of special_modulus_size (README.md:59)");
    if (special > 8) return fail(FHS_ERR_INVALID, "context_create: special_modulus_size > 8 unsupported");
    for (int i = 0; i < nprimes; ++i) {
        if (primes[i] >= (1ull << 60) || (primes[i] - 1) % (2 * N) != 0 || !h_is_prime(primes[i]))
            return fail(FHS_ERR_INVALID, "context_create: every modulus must be a prime < 2^60 (SEAL's 60-bit "
                                         "limit; Acc3 in fhs_modarith.h relies on it), = 1 mod 2N");
        for (int j = 0; j < i; ++j)
            if (primes[j] == primes[i]) return fail(FHS_ERR_INVALID, "context_create: duplicate modulus");
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(FHS_ERR_NODEVICE, "no HIP device: libfhespear_hip needs an MI355X (gfx950)");
    if (device < 0 || device >= ndev) return fail(FHS_ERR_INVALID, "context_create: bad device index");
    HIPCHK(hipSetDevice(device), "hipSetDevice");

    auto c = std::make_unique<fhs_context>();
    c->device = device;
    c->N = N;
    while ((1ull << c->logN) < N) c->logN++;
    c->K = nprimes;
    c->P = special;
    c->L0 = L0;
    c->dnum = (L0 + special - 1) / special;
    c->q.assign(primes, primes + nprimes);
    HIPCHK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking), "hipStreamCreate");
    {
        static std::once_flag exit_once;
        std::call_once(exit_once, [] { atexit(release_at_exit); });
        size_t free_b = 0, total_b = 0;
        (void)hipMemGetInfo(&free_b, &total_b);
        c->cache_cap = total_b / 4;
        if (const char* e = getenv("FHESPEAR_CACHE_BYTES")) c->cache_cap = strtoull(e, nullptr, 10);
        // SEAL-hoisting corrections: 1/16 of this context's device (seal_prepare)
        c->seal_corr_cap = total_b ? total_b / 16 : (size_t)16 << 30;
        if (const char* e = getenv("FHESPEAR_SEAL_CORR_BYTES")) c->seal_corr_cap = strtoull(e, nullptr, 10);
    }
    if (galois_elts && n_elts > 0) {
        c->elts.assign(galois_elts, galois_elts + n_elts);
    } else {   // default: +-2^k steps and conjugation (SEAL/Phantom create_galois_keys default)
        std::set<uint64_t> s;
        for (uint64_t k = 1; k < N / 2; k <<= 1) {
            s.insert(fhs_galois_elt_from_step((int)k, N));
            s.insert(fhs_galois_elt_from_step(-(int)k, N));
        }
        s.insert(2 * N - 1);
        c->elts.assign(s.begin(), s.end());
    }
    for (uint64_t e : c->elts)
        if ((e & 1) == 0 || e >= 2 * N) return fail(FHS_ERR_INVALID, "context_create: invalid galois element");

    const int K = nprimes, P = special, dnum = c->dnum;
    // ---- per-prime constants and twiddles
    std::vector<PrimeK> pk(K);
    std::vector<uint64_t> twf((size_t)K * N * 2), twi((size_t)K * N * 2);
    for (int i = 0; i < K; ++i) {
        const uint64_t q = primes[i];
        const hu128 r = (~(hu128)0) / q;
        const uint64_t psi = h_min_root(q, N), ipsi = h_inv(psi, q);
        uint64_t pw = 1, ipw = 1;
        for (uint64_t k = 0; k < N; ++k) {
            const uint32_t rv = h_bitrev((uint32_t)k, c->logN);
            twf[((size_t)i * N + rv) * 2] = pw;
            twi[((size_t)i * N + rv) * 2] = ipw;
            pw = h_mulmod(pw, psi, q);
            ipw = h_mulmod(ipw, ipsi, q);
        }
        for (uint64_t k = 0; k < N; ++k) {
            twf[((size_t)i * N + k) * 2 + 1] = h_shoup(twf[((size_t)i * N + k) * 2], q);
            twi[((size_t)i * N + k) * 2 + 1] = h_shoup(twi[((size_t)i * N + k) * 2], q);
        }
        const uint64_t ninv = h_inv(N % q, q);
        const uint64_t w1n = h_mulmod(twi[((size_t)i * N + 1) * 2], ninv, q);
        pk[i] = PrimeK{q, (uint64_t)r, (uint64_t)(r >> 64), ninv, h_shoup(ninv, q), w1n, h_shoup(w1n, q), pm_word(q, c->logN) | (pm_word(q, c->logN) && conv_pm_ok(q, special) ? (1ull << 40) : 0ull)};
    }
    // ---- ModUp tables per level l: digit j covers [jP, min(jP+P, l))
    std::vector<uint64_t> mu_intt((size_t)(L0 + 1) * L0 * 4, 0), mu_hat((size_t)(L0 + 1) * dnum * P * K, 0);
    for (int l = 1; l <= L0; ++l) {
        const int dn = (l + P - 1) / P;
        for (int j = 0; j < dn; ++j) {
            const int s0 = j * P, s1 = std::min(s0 + P, l), ns = s1 - s0;
            for (int u = 0; u < ns; ++u) {
                const int i = s0 + u;
                const uint64_t q = primes[i];
                uint64_t hat = 1;
                for (int v = 0; v < ns; ++v)
                    if (v != u) hat = h_mulmod(hat, primes[s0 + v] % q, q);
                const uint64_t ih = h_inv(hat, q);
                const uint64_t a = h_mulmod(pk[i].ninv, ih, q), b = h_mulmod(pk[i].w1ninv, ih, q);
                uint64_t* d = &mu_intt[((size_t)l * L0 + i) * 4];
                d[0] = a; d[1] = h_shoup(a, q); d[2] = b; d[3] = h_shoup(b, q);
                for (int t = 0; t < K; ++t) {
                    const uint64_t m = primes[t];
                    uint64_t h = 1;
                    for (int v = 0; v < ns; ++v)
                        if (v != u) h = h_mulmod(h, primes[s0 + v] % m, m);
                    mu_hat[(((size_t)l * dnum + j) * P + u) * K + t] = h;
                }
            }
        }
    }
    // ---- centred-extension tables: floor(2^128/q_u) per digit source, Q_S and ns Q_S mod every prime
    std::vector<uint64_t> mu_R((size_t)(L0 + 1) * dnum * P * 2, 0), mu_Q((size_t)(L0 + 1) * dnum * K * 2, 0);
    for (int l = 1; l <= L0; ++l) {
        const int dn = (l + P - 1) / P;
        for (int j = 0; j < dn; ++j) {
            const int s0 = j * P, s1 = std::min(s0 + P, l), ns = s1 - s0;
            for (int u = 0; u < ns; ++u) {
                const hu128 R = (~(hu128)0) / primes[s0 + u];
                mu_R[(((size_t)l * dnum + j) * P + u) * 2 + 0] = (uint64_t)R;
                mu_R[(((size_t)l * dnum + j) * P + u) * 2 + 1] = (uint64_t)(R >> 64);
            }
            for (int t = 0; t < K; ++t) {
                const uint64_t m = primes[t];
                uint64_t Qm = 1;
                for (int u = 0; u < ns; ++u) Qm = h_mulmod(Qm, primes[s0 + u] % m, m);
                mu_Q[(((size_t)l * dnum + j) * K + t) * 2 + 0] = Qm;
                mu_Q[(((size_t)l * dnum + j) * K + t) * 2 + 1] = h_mulmod(Qm, (uint64_t)ns, m);
            }
        }
    }
    std::vector<uint64_t> mu_xd((size_t)dnum * 32, 0), mu_xt((size_t)K * 4, 0);
    if (P == 3) modup_xform_tables(primes, K, L0, dnum, mu_xd.data(), mu_xt.data());
    // ---- ModDown tables
    // X form of the special digit (fhs_kernels.hip k_special_x): Y = sum_k y_k (P/p_k) < 3P stored as
    // base-2^60 words -- no centring (thresholds all ones), no offset (C_0 = 0); needs 3P < 2^180, so
    // special primes below 2^59
    std::vector<uint64_t> md_xd(32, 0);
    bool md_x_ok = P == 3;
    for (int k = 0; k < P && md_x_ok; ++k) md_x_ok = primes[L0 + k] < (1ull << 59);
    if (md_x_ok) {
        for (int u = 0; u < 3; ++u) {
            const hu128 h = (hu128)primes[L0 + (u + 1) % 3] * primes[L0 + (u + 2) % 3];
            md_xd[2 * u] = (uint64_t)h;
            md_xd[2 * u + 1] = (uint64_t)(h >> 64);
        }
        for (int w = 6; w < 15; ++w) md_xd[w] = ~0ull;
    }
    std::vector<uint64_t> md_intt((size_t)P * 4), md_hat((size_t)P * L0), md_pinv((size_t)4 * L0);
    for (int k = 0; k < P; ++k) {
        const int pi = L0 + k;
        const uint64_t p = primes[pi];
        uint64_t hat = 1;
        for (int v = 0; v < P; ++v)
            if (v != k) hat = h_mulmod(hat, primes[L0 + v] % p, p);
        const uint64_t ih = h_inv(hat, p);
        const uint64_t a = h_mulmod(pk[pi].ninv, ih, p), b = h_mulmod(pk[pi].w1ninv, ih, p);
        md_intt[k * 4 + 0] = a; md_intt[k * 4 + 1] = h_shoup(a, p);
        md_intt[k * 4 + 2] = b; md_intt[k * 4 + 3] = h_shoup(b, p);
        for (int i = 0; i < L0; ++i) {
            const uint64_t q = primes[i];
            uint64_t h = 1;
            for (int v = 0; v < P; ++v)
                if (v != k) h = h_mulmod(h, primes[L0 + v] % q, q);
            md_hat[(size_t)k * L0 + i] = h;
        }
    }
    for (int i = 0; i < L0; ++i) {
        const uint64_t q = primes[i];
        uint64_t pm = 1;
        for (int k = 0; k < P; ++k) pm = h_mulmod(pm, primes[L0 + k] % q, q);
        const uint64_t pinv = h_inv(pm, q);
        md_pinv[2 * i] = pinv;
        md_pinv[2 * i + 1] = h_shoup(pinv, q);
        md_pinv[2 * L0 + i] = pm;
        md_pinv[3 * L0 + i] = P == 1 ? (primes[L0] >> 1) % q : 0;   // SEAL ModDown rounding (P = 1)
    }
    // ---- rescale tables: level l (limbs) drops q_{l-1}
    std::vector<uint64_t> rs((size_t)(L0 + 1) * L0 * 4, 0);
    for (int l = 2; l <= L0; ++l) {
        const uint64_t ql = primes[l - 1], half = ql >> 1;
        for (int i = 0; i < l - 1; ++i) {
            const uint64_t q = primes[i];
            const uint64_t inv = h_inv(ql % q, q);
            uint64_t* d = &rs[((size_t)l * L0 + i) * 4];
            d[0] = inv; d[1] = h_shoup(inv, q); d[2] = half % q; d[3] = half;
        }
    }
    // ---- 2^e mod q for exact double reduction
    std::vector<uint64_t> pow2((size_t)K * 1088);
    for (int i = 0; i < K; ++i) {
        uint64_t v = 1 % primes[i];
        for (int e = 0; e < 1088; ++e) {
            pow2[(size_t)i * 1088 + e] = v;
            v = h_mulmod(v, 2, primes[i]);
        }
    }
    auto up = [&](const void* src, size_t bytes, const void** dst) -> hipError_t {
        void* d = nullptr;
        hipError_t e = hipMalloc(&d, bytes);
        if (e != hipSuccess) return e;
        c->tables.push_back(d);
        e = hipMemcpy(d, src, bytes, hipMemcpyHostToDevice);
        *dst = d;
        return e;
    };
    DevTables& T = c->T;
    T.N = (int)N; T.logN = c->logN; T.L0 = L0; T.P = P; T.K = K; T.dnum = dnum;
    T.max_qbits = 0;
    for (int i = 0; i < K; ++i) T.max_qbits = std::max(T.max_qbits, 64 - __builtin_clzll(c->q[i]));
    // ModUp's specialised conversion: 3-limb digits with every target on the pseudo-Mersenne fold (the
    // generic loop is then not compiled into the kernel), one-limb digits, or the generic loop
    bool all_cpm = true;
    for (int i = 0; i < K; ++i) all_cpm = all_cpm && ((pk[i].pm >> 40) & 1);
    bool small_e1 = true;   // the X form's weight 2^60 mod m below 2^30 for every prime (modup_xform_tables)
    for (int i = 0; i < K && P == 3; ++i) small_e1 = small_e1 && mu_xt[(size_t)i * 4] < (1ull << 30);
    T.modup_dp = (P == 3 && L0 % 3 == 0 && all_cpm && small_e1) ? 3 : (P == 1 ? 1 : 0);
    T.md_xform = T.modup_dp == 3 && md_x_ok;
    // every prime 2^59 - d with d < 2^27 (SEAL's 59-bit Create() primes at N <= 65536): the X-form
    // conversions reduce with compile-time folds (convert3x_b59)
    bool b59 = T.modup_dp == 3;
    for (int i = 0; i < K && b59; ++i) b59 = b59_prime(c->q[i]);
    T.conv_b59 = b59;
    bool all59 = true;
    for (int i = 0; i < K && all59; ++i) all59 = b59_prime(c->q[i]);
    T.all_b59 = all59;
    // the B59 kernels compile the forward NTT's lazy mode in for N <= 16384 (fhs_kernels.hip lazy_of): every
    // prime must carry the lazy bit there, which q < 2^59 implies -- checked, not assumed
    for (int i = 0; i < K && (b59 || all59) && c->logN <= 14; ++i)
        if (!((pk[i].pm >> 7) & 1))
            return fail(FHS_ERR_INVALID, "context: a 59-bit prime without the lazy NTT bound (internal)");
    HIPCHK(up(pk.data(), sizeof(PrimeK) * K, &T.primes), "tables");
    HIPCHK(up(twf.data(), 8 * twf.size(), (const void**)&T.tw_fwd), "tables");
    HIPCHK(up(twi.data(), 8 * twi.size(), (const void**)&T.tw_inv), "tables");
    HIPCHK(up(mu_intt.data(), 8 * mu_intt.size(), (const void**)&T.modup_intt), "tables");
    HIPCHK(up(mu_hat.data(), 8 * mu_hat.size(), (const void**)&T.modup_hat), "tables");
    HIPCHK(up(mu_R.data(), 8 * mu_R.size(), (const void**)&T.modup_R), "tables");
    HIPCHK(up(mu_Q.data(), 8 * mu_Q.size(), (const void**)&T.modup_Q), "tables");
    HIPCHK(up(mu_xd.data(), 8 * mu_xd.size(), (const void**)&T.modup_xd), "tables");
    HIPCHK(up(mu_xt.data(), 8 * mu_xt.size(), (const void**)&T.modup_xt), "tables");
    HIPCHK(up(md_xd.data(), 8 * md_xd.size(), (const void**)&T.md_xd), "tables");
    HIPCHK(up(md_intt.data(), 8 * md_intt.size(), (const void**)&T.md_intt), "tables");
    HIPCHK(up(md_hat.data(), 8 * md_hat.size(), (const void**)&T.md_hat), "tables");
    HIPCHK(up(md_pinv.data(), 8 * md_pinv.size(), (const void**)&T.md_pinv), "tables");
    HIPCHK(up(rs.data(), 8 * rs.size(), (const void**)&T.rescale), "tables");
    HIPCHK(up(pow2.data(), 8 * pow2.size(), (const void**)&T.pow2), "tables");
    // host encoder / decoder tables
    c->fft_w.resize(N);
    for (uint64_t k = 0; k < N; ++k) c->fft_w[k] = std::polar(1.0, 2.0 * M_PI * (double)k / (double)N);
    c->dec_twist.resize(N);
    for (uint64_t k = 0; k < N; ++k)
        c->dec_twist[k] = {std::cos(M_PI * (double)k / (double)N), std::sin(M_PI * (double)k / (double)N)};
    c->slot_index.resize(N / 2);
    uint64_t e5 = 1;
    for (uint64_t j = 0; j < N / 2; ++j) {
        c->slot_index[j] = (e5 - 1) / 2;
        e5 = (e5 * 5) & (2 * N - 1);
    }
    {   // GPU decoder tables (fhs_kernels.hip k_decode_fft): the host decoder's own values
        const size_t H = N / 2;
        std::vector<double> dw(2 * H), dt(2 * H);
        std::vector<unsigned> dp(H);
        for (size_t k = 0; k < H; ++k) {
            dw[2 * k] = c->fft_w[2 * k].real();
            dw[2 * k + 1] = c->fft_w[2 * k].imag();
            dt[2 * k] = c->dec_twist[k].real();
            dt[2 * k + 1] = c->dec_twist[k].imag();
            dp[k] = (unsigned)(c->slot_index[k] >> 1);
        }
        HIPCHK(up(dw.data(), 8 * dw.size(), (const void**)&T.dec_w), "tables");
        HIPCHK(up(dt.data(), 8 * dt.size(), (const void**)&T.dec_twist), "tables");
        HIPCHK(up(dp.data(), 4 * dp.size(), (const void**)&T.dec_pos), "tables");
    }
    {   // GPU encoder tables (fhs_kernels.hip k_encode)
        const size_t H = N / 2;
        const int logH = c->logN - 1;
        std::vector<double> ew(2 * H), et(2 * H);
        std::vector<unsigned> ep(H);
        for (size_t k = 0; k < H; ++k) {
            const double th = -2.0 * M_PI * (double)k / (double)H;
            ew[2 * k] = std::cos(th);
            ew[2 * k + 1] = std::sin(th);
            const double tz = -M_PI * (double)k / (double)N;
            et[2 * k] = 2.0 / (double)N * std::cos(tz);
            et[2 * k + 1] = 2.0 / (double)N * std::sin(tz);
        }
        uint64_t e5 = 1;
        for (size_t j = 0; j < H; ++j) {
            ep[j] = h_bitrev((uint32_t)((e5 - 1) / 4), logH);
            e5 = (e5 * 5) & (2 * N - 1);
        }
        HIPCHK(up(ew.data(), 8 * ew.size(), (const void**)&T.enc_w), "tables");
        HIPCHK(up(et.data(), 8 * et.size(), (const void**)&T.enc_twist), "tables");
        HIPCHK(up(ep.data(), 4 * ep.size(), (const void**)&T.enc_pos), "tables");
    }
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->ring), fhs_context::kRingBytes, hipHostMallocDefault),
           "staging ring");
    c->stager = fhs::Stager{c.get(), stage_h2d};
    HIPCHK(hipMalloc(&c->items_dev, (sizeof(KsItem) + sizeof(void*)) * fhs_context::kMaxItems), "items buffer");
    c->tables.push_back(c->items_dev);
    HIPCHK(hipMalloc(&c->ptrs_dev, sizeof(void*) * 2 * fhs_context::kMaxPtrs), "pointer buffer");
    c->tables.push_back(c->ptrs_dev);
    {
        std::lock_guard<std::mutex> lk(g_live_mu);
        g_live.insert(c.get());
    }
    *out = c.release();
    return FHS_OK;
}

static void ctx_free(fhs_context* c) {
    const bool trace = getenv("FHESPEAR_TRACE_LIFETIME") != nullptr;
    if (trace)
        fprintf(stderr, "[fhespear] context %p: freeing (%zu cached bytes, %llu live)\n", (void*)c, c->cached_bytes,
                (unsigned long long)c->bytes_live.load());
    {
        Guard g(c);
        flush(c);
        hipStreamSynchronize(c->st);
        ctx_sync(c);
        for (void* p : c->tables) hipFree(p);
        for (auto& kv : c->seal_corr) hipFree(kv.second);
        c->seal_corr.clear();
        if (c->seal_hoist.zflag_dev) hipFree(c->seal_hoist.zflag_dev);
        if (c->seal_hoist.zflag_host) hipHostFree(c->seal_hoist.zflag_host);
        for (int k = 0; k < fhs_context::SCR_COUNT; ++k)
            if (c->scr[k]) hipFree(c->scr[k]);
        {
            std::lock_guard<std::mutex> lk(g_live_mu);
            g_live.erase(c);
        }
        for (auto& kv : c->free_blocks)
            for (void* p : kv.second) hipFree(p);
        c->free_blocks.clear();
        if (c->ring) hipHostFree(c->ring);
        if (c->readback) hipHostFree(c->readback);
        for (hipEvent_t e : c->ring_ev)
            if (e) hipEventDestroy(e);
        for (auto& v : c->timer_pairs)
            for (auto& pr : v) { ev_put(pr.first); ev_put(pr.second); }
        for (hipEvent_t e : c->timer_open)
            if (e) ev_put(e);
        hipStreamDestroy(c->st);
    }
    delete c;
    if (trace) fprintf(stderr, "[fhespear] context %p: freed\n", (void*)c);
}
static void ctx_release(fhs_context* c) {
    if (c->refs.fetch_sub(1) == 1) ctx_free(c);
}
extern "C" fhs_status fhs_context_destroy(fhs_context* c) {
    if (!c) return FHS_OK;
    ctx_release(c);
    return FHS_OK;
}
extern "C" fhs_status fhs_context_info(const fhs_context* c, uint64_t* N, int* L0, int* P, int* n_elts) {
    if (!c) return fail(FHS_ERR_INVALID, "null context");
    if (N) *N = c->N;
    if (L0) *L0 = c->L0;
    if (P) *P = c->P;
    if (n_elts) *n_elts = (int)c->elts.size();
    return FHS_OK;
}
extern "C" fhs_status fhs_context_galois_elts(const fhs_context* c, uint64_t* out) {
    if (!c || !out) return fail(FHS_ERR_INVALID, "null argument");
    std::copy(c->elts.begin(), c->elts.end(), out);
    return FHS_OK;
}
extern "C" fhs_status fhs_synchronize(fhs_context* c) {
    ENTER(c);
    HIPCHK(hipStreamSynchronize(c->st), "hipStreamSynchronize");
    return FHS_OK;
}
extern "C" fhs_status fhs_memory_in_use(fhs_context* c, uint64_t* bytes) {
    if (!c || !bytes) return fail(FHS_ERR_INVALID, "null argument");
    *bytes = c->bytes_live.load();
    return FHS_OK;
}

// ============================================================================ sampling helpers
// sm64: fhs_modarith.h (host + device)
// 256 bits from the OS entropy pool (a secret key created without a caller-supplied key)
static bool os_random(void* buf, size_t n) {
    FILE* f = fopen("/dev/urandom", "rb");
    if (!f) return false;
    const size_t got = fread(buf, 1, n, f);
    fclose(f);
    return got == n;
}
static uint64_t prf_u64(const PrfKey& K, uint64_t sid) {
    uint64_t w0, w1;
    prf128(K, sid, 0, w0, w1);
    return w0;
}
static uint64_t stream_id(uint64_t kind, uint64_t a, uint64_t b) { return (kind << 56) | (a << 16) | b; }
// Reproducible randomness for parity checks (FHESPEAR_PARITY_RNG set: tests/conftest.py, bench.py, smoke):
// encryption counters start at 0 and a public key's mask key is PRF(secret key, generation) alone, so a
// seeded key reproduces the oracle's ciphertexts.  Otherwise each secret key's symmetric-encryption
// counter starts at a fresh random offset and each public key's mask key has 256 fresh random bits
// mixed in: a secret key recreated from the same 32 key bytes (another process, another context) never
// repeats an encryption mask, which would reveal the difference of the two messages.
// Only the exact value "1" enables it (0, empty or anything else leaves the secure default), and the
// first use in a process says so on stderr: ciphertexts made in this mode reuse mask streams across
// processes and must never leave a test.
static bool parity_rng() {
    const char* v = getenv("FHESPEAR_PARITY_RNG");
    if (!v || strcmp(v, "1") != 0) return false;
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true))
        fprintf(stderr, "[fhespear] FHESPEAR_PARITY_RNG=1: deterministic encryption randomness (parity tests "
                        "only; never for real data)\n");
    return true;
}
enum { ST_SECRET = 1, ST_PUBKEY = 2, ST_RELIN = 3, ST_GALOIS = 4, ST_ENC_SYM = 5, ST_ENC_ASYM = 6, ST_PK_RNG = 7 };

// sample a small polynomial (ternary/CBD) over `limbs` primes and NTT it
static hipError_t sample_small_ntt(fhs_context* c, int mode, const PrfKey& K, uint64_t sid, uint64_t* out, int limbs) {
    hipError_t e = fhs::launch_sample(c->T, mode, K, sid, out, limbs, c->st);
    if (e != hipSuccess) return e;
    return fhs::launch_ntt_fwd(c->T, out, limbs, limbs, 1, 0, c->st);
}

// ============================================================================ keys
extern "C" fhs_status fhs_secret_key_create(fhs_context* c, const uint8_t* key32, fhs_secret_key** out) {
    ENTER(c);
    if (!out) return fail(FHS_ERR_INVALID, "null out");
    PrfKey K{};
    if (key32) {
        for (int w = 0; w < 8; ++w)
            K.k[w] = (uint32_t)key32[4 * w] | ((uint32_t)key32[4 * w + 1] << 8) | ((uint32_t)key32[4 * w + 2] << 16) |
                     ((uint32_t)key32[4 * w + 3] << 24);
    } else if (!os_random(K.k, sizeof(K.k))) {
        return fail(FHS_ERR_INVALID, "secret_key: /dev/urandom unavailable");
    }
    uint64_t ctr0 = 0;   // stream ids carry 40 counter bits: a random start below 2^39 leaves 2^39 encryptions
    if (!parity_rng() && !os_random(&ctr0, sizeof ctr0)) return fail(FHS_ERR_INVALID, "secret_key: /dev/urandom unavailable");
    auto* sk = new fhs_secret_key{c, nullptr, K, ctr0 & ((1ull << 39) - 1)};
    hipError_t e = dalloc(c, &sk->s, 8ull * c->K * c->N);
    if (e != hipSuccess) { delete sk; return hip_fail(e, "secret key"); }
    e = sample_small_ntt(c, fhs::SAMPLE_TERNARY, sk->key, stream_id(ST_SECRET, 0, 0), sk->s, c->K);
    if (e != hipSuccess) { delete sk; return hip_fail(e, "secret key sampling"); }
    ctx_retain(c);
    *out = sk;
    return FHS_OK;
}
extern "C" fhs_status fhs_secret_key_destroy(fhs_secret_key* sk) {
    if (!sk) return FHS_OK;
    fhs_context* c = sk->ctx;
    { Guard g(c); flush(c); dfree(c, sk->s, 8ull * c->K * c->N); }
    delete sk;
    ctx_release(c);
    return FHS_OK;
}

static fhs_status gen_switch_key(fhs_context* c, const PrfKey& K, uint64_t base, const uint64_t* s, const uint64_t* snew,
                                 uint64_t** key_out) {
    uint64_t* key = nullptr;
    hipError_t e = dalloc(c, &key, 8 * key_words(c));
    if (e != hipSuccess) return hip_fail(e, "switching key");
    const size_t S = (size_t)c->K * c->N;
    uint64_t* tmp = nullptr;   // e | a
    e = dalloc(c, &tmp, 16 * S);
    if (e != hipSuccess) { dfree(c, key, 8 * key_words(c)); return hip_fail(e, "switching key"); }
    uint64_t* ebuf = tmp;
    uint64_t* abuf = tmp + S;
    std::vector<uint64_t> seeds(c->dnum);
    for (int j = 0; j < c->dnum && e == hipSuccess; ++j) {
        seeds[j] = prf_u64(K, base | (uint64_t)(2 * j));   // public seed of a_j: a PRF output
        e = fhs::launch_sample(c->T, fhs::SAMPLE_SEEDED, K, seeds[j], abuf, c->K, c->st);
        if (e == hipSuccess) e = sample_small_ntt(c, fhs::SAMPLE_CBD, K, base | (uint64_t)(2 * j + 1), ebuf, c->K);
        if (e == hipSuccess) e = fhs::launch_switch_key_assemble(c->T, key + (size_t)j * S, abuf, ebuf, s, snew, j, c->st);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(key + (size_t)c->dnum * S, seeds.data(), 8 * seeds.size(),
                                            hipMemcpyHostToDevice, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);   // `seeds` is a host temporary
    dfree(c, tmp, 16 * S);
    if (e != hipSuccess) { dfree(c, key, 8 * key_words(c)); return hip_fail(e, "switching key generation"); }
    *key_out = key;
    return FHS_OK;
}
// [dnum][2][K][N] with the a_j regenerated from their seeds (the oracle's layout)
static fhs_status export_switch_key(fhs_context* c, const uint64_t* key, uint64_t* host) {
    const size_t S = (size_t)c->K * c->N;
    if (const uint64_t* akey = key_akey(c, key)) {   // imported: (b_j, a_j) as given
        for (int j = 0; j < c->dnum; ++j) {
            HIPCHK(hipMemcpyAsync(host + (size_t)j * 2 * S, key + (size_t)j * S, 8 * S, hipMemcpyDeviceToHost, c->st),
                   "key export");
            HIPCHK(hipMemcpyAsync(host + ((size_t)j * 2 + 1) * S, akey + (size_t)j * S, 8 * S, hipMemcpyDeviceToHost,
                                  c->st), "key export");
        }
        HIPCHK(hipStreamSynchronize(c->st), "key export");
        return FHS_OK;
    }
    std::vector<uint64_t> seeds(c->dnum);
    HIPCHK(hipMemcpyAsync(seeds.data(), key + (size_t)c->dnum * S, 8 * seeds.size(), hipMemcpyDeviceToHost, c->st),
           "key export");
    HIPCHK(hipStreamSynchronize(c->st), "key export");
    uint64_t* full = nullptr;
    HIPCHK(dalloc(c, &full, 8 * key_words_full(c)), "key export");
    hipError_t e = hipSuccess;
    for (int j = 0; j < c->dnum && e == hipSuccess; ++j) {
        e = hipMemcpyAsync(full + (size_t)j * 2 * S, key + (size_t)j * S, 8 * S, hipMemcpyDeviceToDevice, c->st);
        if (e == hipSuccess) e = fhs::launch_sample(c->T, fhs::SAMPLE_SEEDED, PrfKey{}, seeds[j], full + ((size_t)j * 2 + 1) * S, c->K, c->st);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(host, full, 8 * key_words_full(c), hipMemcpyDeviceToHost, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);
    dfree(c, full, 8 * key_words_full(c));
    if (e != hipSuccess) return hip_fail(e, "key export");
    return FHS_OK;
}

extern "C" fhs_status fhs_gen_relin_key(fhs_context* c, fhs_secret_key* sk, fhs_relin_key** out) {
    ENTER(c);
    if (!sk || !out) return fail(FHS_ERR_INVALID, "null argument");
    uint64_t* s2 = nullptr;
    HIPCHK(dalloc(c, &s2, 8ull * c->K * c->N), "relin key");
    HIPCHK(fhs::launch_key_prod(c->T, sk->s, sk->s, s2, c->K, c->st), "relin key");
    auto* rk = new fhs_relin_key{c, nullptr};
    fhs_status s = gen_switch_key(c, sk->key, stream_id(ST_RELIN, 0, 0), sk->s, s2, &rk->key);
    dfree(c, s2, 8ull * c->K * c->N);
    if (s != FHS_OK) { delete rk; return s; }
    ctx_retain(c);
    *out = rk;
    return FHS_OK;
}
extern "C" fhs_status fhs_relin_key_destroy(fhs_relin_key* rk) {
    if (!rk) return FHS_OK;
    fhs_context* c = rk->ctx;
    { Guard g(c); flush(c); free_key(c, rk->key); }
    delete rk;
    ctx_release(c);
    return FHS_OK;
}

extern "C" fhs_status fhs_create_galois_keys(fhs_context* c, fhs_secret_key* sk, const uint64_t* elts, int n,
                                             fhs_galois_keys** out) {
    ENTER(c);
    if (!sk || !out) return fail(FHS_ERR_INVALID, "null argument");
    std::vector<uint64_t> list = (elts && n > 0) ? std::vector<uint64_t>(elts, elts + n) : c->elts;
    auto* gk = new fhs_galois_keys{c, {}};
    uint64_t* sn = nullptr;
    hipError_t e = dalloc(c, &sn, 8ull * c->K * c->N);
    if (e != hipSuccess) { delete gk; return hip_fail(e, "galois keys"); }
    for (uint64_t elt : list) {
        if (gk->keys.count(elt)) continue;
        if ((elt & 1) == 0 || elt >= 2 * c->N) { e = hipErrorInvalidValue; break; }
        e = fhs::launch_galois_perm(c->T, sk->s, sn, c->K, elt, c->st);
        if (e != hipSuccess) break;
        uint64_t* key = nullptr;
        fhs_status s = gen_switch_key(c, sk->key, stream_id(ST_GALOIS, elt, 0), sk->s, sn, &key);
        if (s != FHS_OK) {
            dfree(c, sn, 8ull * c->K * c->N);
            for (auto& kv : gk->keys) free_key(c, kv.second);
            delete gk;
            return s;
        }
        gk->keys[elt] = key;
    }
    dfree(c, sn, 8ull * c->K * c->N);
    if (e != hipSuccess) {
        for (auto& kv : gk->keys) free_key(c, kv.second);
        delete gk;
        return hip_fail(e, "galois key generation");
    }
    ctx_retain(c);
    *out = gk;
    return FHS_OK;
}
extern "C" fhs_status fhs_galois_keys_destroy(fhs_galois_keys* gk) {
    if (!gk) return FHS_OK;
    fhs_context* c = gk->ctx;
    {
        Guard g(c);
        flush(c);
        for (auto& kv : gk->keys) free_key(c, kv.second);
    }
    delete gk;
    ctx_release(c);
    return FHS_OK;
}
extern "C" fhs_status fhs_galois_keys_has(const fhs_galois_keys* gk, uint64_t elt, int* has) {
    if (!gk || !has) return fail(FHS_ERR_INVALID, "null argument");
    *has = gk->keys.count(elt) ? 1 : 0;
    return FHS_OK;
}
extern "C" fhs_status fhs_galois_keys_bytes(const fhs_galois_keys* gk, uint64_t* bytes) {
    if (!gk || !bytes) return fail(FHS_ERR_INVALID, "null argument");
    *bytes = (uint64_t)gk->keys.size() * 8 * key_words(gk->ctx);
    return FHS_OK;
}

static fhs_status export_dev(fhs_context* c, const void* d, size_t bytes, void* host) {
    HIPCHK(hipMemcpyAsync(host, d, bytes, hipMemcpyDeviceToHost, c->st), "export");
    HIPCHK(hipStreamSynchronize(c->st), "export sync");
    return FHS_OK;
}
extern "C" fhs_status fhs_galois_key_export(fhs_context* c, const fhs_galois_keys* gk, uint64_t elt, uint64_t* host) {
    ENTER(c);
    if (!gk || !host) return fail(FHS_ERR_INVALID, "null argument");
    auto it = gk->keys.find(elt);
    if (it == gk->keys.end()) return fail(FHS_ERR_KEY, "galois key not present");
    return export_switch_key(c, it->second, host);
}
extern "C" fhs_status fhs_relin_key_export(fhs_context* c, const fhs_relin_key* rk, uint64_t* host) {
    ENTER(c);
    if (!rk || !host) return fail(FHS_ERR_INVALID, "null argument");
    return export_switch_key(c, rk->key, host);
}
// ---- key import ("identical keys": a key set produced elsewhere, e.g. by SEAL, in the export layout)
static bool canonical_limbs(const fhs_context* c, const uint64_t* host, int nlimbs, int limb0) {
    for (int i = 0; i < nlimbs; ++i) {
        const uint64_t q = c->q[(limb0 + i) % c->K];
        const uint64_t* v = host + (size_t)i * c->N;
        for (uint64_t n = 0; n < c->N; ++n)
            if (v[n] >= q) return false;
    }
    return true;
}
// host [dnum][2][K][N] -> b_j in the key, a_j in a companion allocation (key_a)
static fhs_status import_switch_key(fhs_context* c, const uint64_t* host, uint64_t** key_out) {
    const size_t S = (size_t)c->K * c->N;
    for (int j = 0; j < 2 * c->dnum; ++j)
        if (!canonical_limbs(c, host + (size_t)j * S, c->K, 0))
            return fail(FHS_ERR_INVALID, "key import: residues must be canonical (< q_i) in [dnum][2][K][N] order");
    uint64_t *key = nullptr, *a = nullptr;
    HIPCHK(dalloc(c, &key, 8 * key_words(c)), "key import");
    hipError_t e = dalloc(c, &a, 8ull * c->dnum * S);
    if (e != hipSuccess) { dfree(c, key, 8 * key_words(c)); return hip_fail(e, "key import"); }
    for (int j = 0; j < c->dnum && e == hipSuccess; ++j) {
        e = hipMemcpyAsync(key + (size_t)j * S, host + (size_t)j * 2 * S, 8 * S, hipMemcpyHostToDevice, c->st);
        if (e == hipSuccess)
            e = hipMemcpyAsync(a + (size_t)j * S, host + ((size_t)j * 2 + 1) * S, 8 * S, hipMemcpyHostToDevice, c->st);
    }
    if (e == hipSuccess) e = hipMemsetAsync(key + (size_t)c->dnum * S, 0, 8 * c->dnum, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);   // pageable host source
    if (e != hipSuccess) {
        dfree(c, a, 8ull * c->dnum * S);
        dfree(c, key, 8 * key_words(c));
        return hip_fail(e, "key import");
    }
    c->key_a[key] = a;
    *key_out = key;
    return FHS_OK;
}
extern "C" fhs_status fhs_galois_keys_import(fhs_context* c, const uint64_t* elts, int n, const uint64_t* host,
                                             fhs_galois_keys** out) {
    ENTER(c);
    if (!elts || n < 1 || !host || !out) return fail(FHS_ERR_INVALID, "galois_keys_import: bad args");
    auto* gk = new fhs_galois_keys{c, {}};
    for (int k = 0; k < n; ++k) {
        if ((elts[k] & 1) == 0 || elts[k] >= 2 * c->N || gk->keys.count(elts[k])) {
            for (auto& kv : gk->keys) free_key(c, kv.second);
            delete gk;
            return fail(FHS_ERR_INVALID, "galois_keys_import: invalid or repeated galois element");
        }
        uint64_t* key = nullptr;
        fhs_status s = import_switch_key(c, host + (size_t)k * key_words_full(c), &key);
        if (s != FHS_OK) {
            for (auto& kv : gk->keys) free_key(c, kv.second);
            delete gk;
            return s;
        }
        gk->keys[elts[k]] = key;
    }
    ctx_retain(c);
    *out = gk;
    return FHS_OK;
}
extern "C" fhs_status fhs_relin_key_import(fhs_context* c, const uint64_t* host, fhs_relin_key** out) {
    ENTER(c);
    if (!host || !out) return fail(FHS_ERR_INVALID, "null argument");
    auto* rk = new fhs_relin_key{c, nullptr};
    fhs_status s = import_switch_key(c, host, &rk->key);
    if (s != FHS_OK) { delete rk; return s; }
    ctx_retain(c);
    *out = rk;
    return FHS_OK;
}
extern "C" fhs_status fhs_secret_key_import(fhs_context* c, const uint64_t* host, fhs_secret_key** out) {
    ENTER(c);
    if (!host || !out) return fail(FHS_ERR_INVALID, "null argument");
    if (!canonical_limbs(c, host, c->K, 0)) return fail(FHS_ERR_INVALID, "secret_key_import: residues must be < q_i");
    PrfKey K{};
    if (!os_random(K.k, sizeof(K.k))) return fail(FHS_ERR_INVALID, "secret_key_import: /dev/urandom unavailable");
    auto* sk = new fhs_secret_key{c, nullptr, K, 0};   // fresh encryption randomness
    hipError_t e = dalloc(c, &sk->s, 8ull * c->K * c->N);
    if (e == hipSuccess) e = hipMemcpyAsync(sk->s, host, 8ull * c->K * c->N, hipMemcpyHostToDevice, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);
    if (e != hipSuccess) {
        if (sk->s) dfree(c, sk->s, 8ull * c->K * c->N);
        delete sk;
        return hip_fail(e, "secret_key_import");
    }
    ctx_retain(c);
    *out = sk;
    return FHS_OK;
}
// key-switch convention of the context (fhs_kernels.h DevTables::ks_seal)
extern "C" fhs_status fhs_context_set_key_switch_mode(fhs_context* c, int mode) {
    ENTER(c);
    if (mode != FHS_KS_EXACT && mode != FHS_KS_SEAL) return fail(FHS_ERR_INVALID, "key switch mode: 0 exact, 1 seal");
    if (mode == FHS_KS_SEAL && c->P != 1)
        return fail(FHS_ERR_INVALID, "key switch mode seal: SEAL's switch_key_inplace has one special prime (P = 1)");
    c->T.ks_seal = mode == FHS_KS_SEAL;
    drop_seal_corr(c, nullptr);
    return FHS_OK;
}
extern "C" fhs_status fhs_seal_hoist_stats(fhs_context* c, uint64_t* hoisted, uint64_t* fallback) {
    ENTER(c);
    if (!hoisted || !fallback) return fail(FHS_ERR_INVALID, "null argument");
    *hoisted = c->seal_hoist.hoisted;
    *fallback = c->seal_hoist.fallback;
    return FHS_OK;
}
extern "C" fhs_status fhs_context_key_switch_mode(const fhs_context* c, int* mode) {
    if (!c || !mode) return fail(FHS_ERR_INVALID, "null argument");
    *mode = c->T.ks_seal ? FHS_KS_SEAL : FHS_KS_EXACT;
    return FHS_OK;
}
extern "C" fhs_status fhs_secret_key_export(fhs_context* c, const fhs_secret_key* sk, uint64_t* host) {
    ENTER(c);
    if (!sk || !host) return fail(FHS_ERR_INVALID, "null argument");
    return export_dev(c, sk->s, 8ull * c->K * c->N, host);
}

extern "C" fhs_status fhs_gen_public_key(fhs_context* c, fhs_secret_key* sk, fhs_public_key** out) {
    ENTER(c);
    if (!sk || !out) return fail(FHS_ERR_INVALID, "null argument");
    auto* pk = new fhs_public_key{c, nullptr, PrfKey{}, 1ull << 20};
    // rng = 256 PRF bits of stream (ST_PK_RNG, generation): two public keys of one secret key never
    // share encryption masks (their key material is the same, so shared masks would reveal m1 - m2)
    const uint64_t gen = sk->pk_gen++;
    for (int w = 0; w < 4; ++w) {
        uint64_t w0, w1;
        prf128(sk->key, stream_id(ST_PK_RNG, gen, 0), (uint32_t)w, w0, w1);
        pk->rng.k[2 * w] = (uint32_t)w0;
        pk->rng.k[2 * w + 1] = (uint32_t)(w0 >> 32);
    }
    if (!parity_rng()) {   // fresh bits: the same secret key recreated elsewhere never repeats a mask stream
        PrfKey nonce{};
        if (!os_random(nonce.k, sizeof nonce.k)) { delete pk; return fail(FHS_ERR_INVALID, "public key: /dev/urandom unavailable"); }
        for (int w = 0; w < 8; ++w) pk->rng.k[w] ^= nonce.k[w];
    }
    const size_t S = (size_t)c->L0 * c->N;
    hipError_t e = dalloc(c, &pk->pk, 16 * S);
    if (e != hipSuccess) { delete pk; return hip_fail(e, "public key"); }
    uint64_t* eb = nullptr;
    e = dalloc(c, &eb, 8 * S);
    if (e == hipSuccess)
        e = fhs::launch_sample(c->T, fhs::SAMPLE_UNIFORM, sk->key, stream_id(ST_PUBKEY, 0, 0), pk->pk + S, c->L0, c->st);
    if (e == hipSuccess)
        e = sample_small_ntt(c, fhs::SAMPLE_CBD, sk->key, stream_id(ST_PUBKEY, 0, 1), eb, c->L0);
    if (e == hipSuccess)
        e = fhs::launch_encrypt_combine(c->T, 0, pk->pk, pk->pk + S, sk->s, nullptr, nullptr, eb, nullptr, nullptr,
                                        c->L0, c->st);
    dfree(c, eb, 8 * S);
    if (e != hipSuccess) { dfree(c, pk->pk, 16 * S); delete pk; return hip_fail(e, "public key generation"); }
    ctx_retain(c);
    *out = pk;
    return FHS_OK;
}
extern "C" fhs_status fhs_public_key_destroy(fhs_public_key* pk) {
    if (!pk) return FHS_OK;
    fhs_context* c = pk->ctx;
    { Guard g(c); flush(c); dfree(c, pk->pk, 16ull * c->L0 * c->N); }
    delete pk;
    ctx_release(c);
    return FHS_OK;
}
extern "C" fhs_status fhs_public_key_export(fhs_context* c, const fhs_public_key* pk, uint64_t* host) {
    ENTER(c);
    if (!pk || !host) return fail(FHS_ERR_INVALID, "null argument");
    return export_dev(c, pk->pk, 16ull * c->L0 * c->N, host);
}

// ============================================================================ object API
static bool pending_uses(fhs_context* c, const void* p) { return c->pending_refs.count(p) != 0; }

extern "C" fhs_status fhs_ciphertext_destroy(fhs_ciphertext* ct) {
    if (!ct) return FHS_OK;
    fhs_context* c = ct->ctx;
    {
        Guard g(c);
        if (pending_uses(c, ct)) flush(c);
        dfree(c, ct->d, ct_bytes(ct));
    }
    delete ct;
    ctx_release(c);
    return FHS_OK;
}
extern "C" fhs_status fhs_plaintext_destroy(fhs_plaintext* pt) {
    if (!pt) return FHS_OK;
    fhs_context* c = pt->ctx;
    {
        Guard g(c);
        if (pt->slab) {
            if (--pt->slab->refs == 0) {
                dfree(c, pt->slab->base, pt->slab->bytes);
                delete pt->slab;
            }
        } else {
            dfree(c, pt->d, pt_bytes(pt));
        }
        if (pt->cslab && --pt->cslab->refs == 0) {
            dfree(c, pt->cslab->base, pt->cslab->bytes);
            delete pt->cslab;
        }
    }
    delete pt;
    ctx_release(c);
    return FHS_OK;
}
// Output array of a batch creator: cleared on entry; if the call fails part-way (e.g. device OOM,
// which bg:1164-1170 catches to fall back to on-the-fly encoding) the plaintexts already created
// are destroyed and their slots reset to null, so a failed batch leaves no HBM behind.
static void destroy_obj(fhs_plaintext* p) { fhs_plaintext_destroy(p); }
static void destroy_obj(fhs_ciphertext* p) { fhs_ciphertext_destroy(p); }
template <class Obj>
struct BatchOutT {
    Obj** outs;
    size_t n;
    bool kept = false;
    BatchOutT(Obj** o, size_t count) : outs(o), n(o ? count : 0) {
        for (size_t i = 0; i < n; ++i) outs[i] = nullptr;
    }
    fhs_status keep(fhs_status st) {
        kept = st == FHS_OK;
        return st;
    }
    ~BatchOutT() {
        if (kept) return;
        for (size_t i = 0; i < n; ++i)
            if (outs[i]) {
                destroy_obj(outs[i]);
                outs[i] = nullptr;
            }
    }
};
using BatchOut = BatchOutT<fhs_plaintext>;
// Largest batch one launch takes (its item count is a grid dimension of the sampler, NTT, combine, decrypt
// and CRT kernels, and its scratch is count x l x N words); bigger batches are processed in chunks of this
// many items, with the same results as one call per item
static constexpr int kMaxBatch = 4096;
extern "C" fhs_status fhs_ciphertext_info(const fhs_ciphertext* ct, int* ncomp, int* ci, int* l, double* scale) {
    if (!ct) return fail(FHS_ERR_INVALID, "null ciphertext");
    if (ncomp) *ncomp = ct->ncomp;
    if (ci) *ci = ct->ci;
    if (l) *l = ct->l;
    if (scale) *scale = ct->scale;
    return FHS_OK;
}
extern "C" fhs_status fhs_ciphertext_set_scale(fhs_ciphertext* ct, double scale) {
    if (!ct) return fail(FHS_ERR_INVALID, "null ciphertext");
    ct->scale = scale;
    return FHS_OK;
}
extern "C" fhs_status fhs_plaintext_info(const fhs_plaintext* pt, int* ci, int* l, double* scale) {
    if (!pt) return fail(FHS_ERR_INVALID, "null plaintext");
    if (ci) *ci = pt->ci;
    if (l) *l = pt->l;
    if (scale) *scale = pt->scale;
    return FHS_OK;
}
extern "C" fhs_status fhs_ciphertext_export(fhs_context* c, const fhs_ciphertext* ct, uint64_t* host) {
    ENTER(c);
    if (!ct || !host) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(ct);
    return export_dev(c, ct->d, ct_bytes(ct), host);
}
extern "C" fhs_status fhs_plaintext_export(fhs_context* c, const fhs_plaintext* pt, uint64_t* host) {
    ENTER(c);
    if (!pt || !host) return fail(FHS_ERR_INVALID, "null argument");
    PT_DENSE(pd, pt, "plaintext_export");
    return export_dev(c, pd, pt_bytes(pt), host);
}
extern "C" fhs_status fhs_ciphertext_import(fhs_context* c, const uint64_t* host, int ncomp, int ci, double scale,
                                            fhs_ciphertext** out) {
    ENTER(c);
    if (!host || !out || ncomp < 2 || ncomp > 3) return fail(FHS_ERR_INVALID, "ciphertext_import: bad args");
    fhs_ciphertext* ct;
    fhs_status s = new_ct(c, ncomp, ci, scale, &ct);
    if (s != FHS_OK) return s;
    HIPCHK(hipMemcpyAsync(ct->d, host, ct_bytes(ct), hipMemcpyHostToDevice, c->st), "ciphertext_import");
    HIPCHK(hipStreamSynchronize(c->st), "ciphertext_import");
    *out = ct;
    return FHS_OK;
}
extern "C" fhs_status fhs_plaintext_import(fhs_context* c, const uint64_t* host, int ci, double scale,
                                           fhs_plaintext** out) {
    ENTER(c);
    if (!host || !out) return fail(FHS_ERR_INVALID, "plaintext_import: bad args");
    fhs_plaintext* pt;
    fhs_status s = new_pt(c, ci, scale, &pt);
    if (s != FHS_OK) return s;
    HIPCHK(hipMemcpyAsync(pt->d, host, pt_bytes(pt), hipMemcpyHostToDevice, c->st), "plaintext_import");
    HIPCHK(hipStreamSynchronize(c->st), "plaintext_import");
    *out = pt;
    return FHS_OK;
}
extern "C" fhs_status fhs_debug_fail_next_flushes(fhs_context* c, int count) {
    if (!c || count < 0) return fail(FHS_ERR_INVALID, "debug_fail_next_flushes: bad args");
    Guard g(c);
    c->debug_fail_flushes = count;
    return FHS_OK;
}
extern "C" fhs_status fhs_ciphertext_device_ptr(const fhs_ciphertext* ct, void** dptr, uint64_t* bytes) {
    if (!ct || !dptr) return fail(FHS_ERR_INVALID, "null argument");
    fhs_context* c = ct->ctx;
    Guard g(c);
    fhs_status s = flush(c);
    if (s != FHS_OK) return s;
    LIVE(ct);
    *dptr = ct->d;
    if (bytes) *bytes = ct_bytes(ct);
    return FHS_OK;
}

// ============================================================================ encoder
// slots z_j sit at the evaluation point zeta^(5^j); encode solves m(zeta^(5^j)) = scale z_j with
// a length-N complex DFT over the odd exponents (pb:141-149).
// Forward N-point complex FFT for decode (the only user): iterative radix-2, products written out
// as (ac - bd, ad + bc) so no __muldc3 call (std::complex's NaN-recovering multiply) is made.
static void fft_inplace(std::vector<std::complex<double>>& a, const std::vector<std::complex<double>>& w, int logN,
                        size_t wstride = 1) {
    const size_t n = a.size();
    for (size_t i = 0; i < n; ++i) {
        const size_t r = h_bitrev((uint32_t)i, logN);
        if (r > i) std::swap(a[i], a[r]);
    }
    double* x = reinterpret_cast<double*>(a.data());
    const double* wt = reinterpret_cast<const double*>(w.data());
    for (size_t len = 2; len <= n; len <<= 1) {
        const size_t step = n / len * wstride, h = len / 2;
        for (size_t i = 0; i < n; i += len) {
            for (size_t k = 0; k < h; ++k) {
                const double wr = wt[2 * k * step], wi = wt[2 * k * step + 1];
                double* u = x + 2 * (i + k);
                double* v = x + 2 * (i + k + h);
                const double vr = v[0] * wr - v[1] * wi, vi = v[0] * wi + v[1] * wr;
                v[0] = u[0] - vr;
                v[1] = u[1] - vi;
                u[0] += vr;
                u[1] += vi;
            }
        }
    }
}

// values: count vectors of n complex (re,im) (or real when is_real); produces rounded coefficients

// The encoder's periodic-row detection (fhs_kernels.hip k_enc_period): *tl = a scratch of one byte per row, or null
// when no row can take the sparse form (fewer values than slots, a ring below 512, FHESPEAR_ENCODE_DENSE=1)
static hipError_t enc_periods(fhs_context* c, const double* dvals, size_t cnt, size_t n, size_t stride, bool is_real,
                              uint64_t** tl, size_t* tbytes) {
    *tl = nullptr;
    *tbytes = 0;
    static const bool dense = getenv("FHESPEAR_ENCODE_DENSE") != nullptr;
    const int smax = fhs::encode_sparse_max_log(c->logN);
    if (dense || smax < 1 || n != c->N / 2 || cnt == 0) return hipSuccess;
    const size_t tb = (cnt + 7) & ~(size_t)7;
    hipError_t e = dalloc(c, tl, tb);
    if (e != hipSuccess) {
        *tl = nullptr;
        return e;
    }
    *tbytes = tb;
    return fhs::launch_enc_period(dvals, (int)cnt, n, stride, is_real, smax, reinterpret_cast<unsigned char*>(*tl),
                                  c->st);
}
// Encode `cnt` value rows already in HBM (row v at dvals + v * stride doubles) into new plaintexts.
// A batch of >= 32 rows (diagonal batches, not a client's few vectors) whose every row is periodic (tlog >= 1, read
// back after k_enc_period: one wait per batch) is stored compact only, at the batch's smallest tlog
// (fhs_plaintext::dc): the fused BSGS's Hadamard reads it as it is, every other op through pt_dense.  Otherwise (or
// without room for the compact block, or FHESPEAR_ENCODE_NO_SHADOW=1) the batch is dense.
static fhs_status new_pts_compact(fhs_context* c, size_t count, int ci, double scale, int tlog, fhs_plaintext** outs) {
    const int l = c->L0 + 1 - ci;
    const size_t per = (size_t)l * (c->N >> tlog);
    auto* cs = new PtSlab{nullptr, 8 * count * per, 0};
    hipError_t e = dalloc_fit(c, &cs->base, &cs->bytes);
    if (e != hipSuccess) {
        delete cs;
        return hip_fail(e, "plaintext allocation");
    }
    for (size_t k = 0; k < count; ++k) {
        outs[k] = new fhs_plaintext{c, nullptr, ci, l, scale};
        outs[k]->dc = cs->base + k * per;
        outs[k]->tlog = tlog;
        outs[k]->cslab = cs;
        ++cs->refs;
        ctx_retain(c);
    }
    return FHS_OK;
}
// ss_hint >= 0: the caller knows every row is periodic at tlog >= ss_hint (encode_diag_rows' tiled rows), so the
// compact factor needs no read-back of the periods (no host wait); -1: read them back.  rows_known: every row's
// tlog IS ss_hint >= 1 and only its first (N/2) >> ss_hint values are in HBM (stride apart): no detection either.
static fhs_status encode_rows_dev(fhs_context* c, const double* dvals, size_t cnt, size_t n, size_t stride,
                                  bool is_real, double scale, int ci, fhs_plaintext** outs, int ss_hint = -1,
                                  bool rows_known = false) {
    const int l = c->L0 + 1 - ci;
    if (l < 1) return fail(FHS_ERR_LEVEL, "chain index out of range");
    // fused reduction + NTT through a scratch of rounded coefficients (FHESPEAR_ENCODE_UNFUSED=1: the
    // encoder reduces into every limb and the NTT runs in place -- same limbs, A/B and test knob)
    static const bool unfused = getenv("FHESPEAR_ENCODE_UNFUSED") != nullptr;
    static const bool no_shadow = getenv("FHESPEAR_ENCODE_NO_SHADOW") != nullptr;
    uint64_t *coef = nullptr, *tl = nullptr, *dptrs = nullptr;
    const size_t cbytes = 8 * cnt * c->N;
    size_t tbytes = 0;
    hipError_t e = hipSuccess;
    if (!unfused) e = dalloc(c, &coef, cbytes);
    if (e == hipSuccess && rows_known) {
        tbytes = (cnt + 7) & ~(size_t)7;
        e = dalloc(c, &tl, tbytes);
        if (e == hipSuccess) e = hipMemsetAsync(tl, ss_hint, cnt, c->st);
    } else if (e == hipSuccess) {
        e = enc_periods(c, dvals, cnt, n, stride, is_real, &tl, &tbytes);
    }
    int ss = 0;
    if (e == hipSuccess && tl && coef && !no_shadow && c->T.max_qbits <= 59 && cnt >= 32 && ss_hint >= 0) {
        ss = ss_hint;
    } else if (e == hipSuccess && tl && coef && !no_shadow && c->T.max_qbits <= 59 && cnt >= 32) {
        std::vector<unsigned char> th(cnt);
        e = hipMemcpyAsync(th.data(), tl, cnt, hipMemcpyDeviceToHost, c->st);
        if (e == hipSuccess) e = hipStreamSynchronize(c->st);
        if (e == hipSuccess) ss = *std::min_element(th.begin(), th.end());
    }
    fhs_status s0 = FHS_OK;
    if (e == hipSuccess && ss > 0 && new_pts_compact(c, cnt, ci, scale, ss, outs) != FHS_OK) {
        (void)hipGetLastError();   // no room for the compact block: a dense batch
        ss = 0;
    }
    if (e == hipSuccess && ss == 0) s0 = new_pts(c, cnt, ci, scale, outs);
    std::vector<uint64_t*> ptrs(2 * cnt, nullptr);
    if (e == hipSuccess && s0 == FHS_OK) {
        for (size_t v = 0; v < cnt; ++v) {
            ptrs[v] = outs[v]->d;   // null for a compact batch
            ptrs[cnt + v] = outs[v]->dc;
        }
        e = scratch(c, fhs_context::SCR_ENC_PTRS, 16 * cnt, &dptrs);
    }
    if (e == hipSuccess && s0 == FHS_OK) e = stage_h2d(c, dptrs, ptrs.data(), 16 * cnt);
    if (e == hipSuccess && s0 == FHS_OK)
        e = fhs::launch_encode(c->T, dvals, (int)cnt, n, stride, is_real, scale, reinterpret_cast<fhs::u64* const*>(dptrs),
                               l, c->st, reinterpret_cast<double*>(coef), reinterpret_cast<const unsigned char*>(tl),
                               ss ? reinterpret_cast<fhs::u64* const*>(dptrs + cnt) : nullptr, ss);
    if (tl) dfree(c, tl, tbytes);
    if (coef) dfree(c, coef, cbytes);
    if (s0 != FHS_OK) return s0;
    return e == hipSuccess ? FHS_OK : hip_fail(e, "encode");
}
static fhs_status encode_checks(fhs_context* c, size_t n, double scale, int ci) {
    if (n > c->N / 2) return fail(FHS_ERR_INVALID, "encode: more values than slots");
    if (!(scale > 0) || !std::isfinite(scale)) return fail(FHS_ERR_INVALID, "encode: bad scale");
    const int l = c->L0 + 1 - ci;
    if (ci < 1 || l < 1) return fail(FHS_ERR_LEVEL, "encode: chain index out of range");
    return FHS_OK;
}
static fhs_status encode_many(fhs_context* c, const double* vals, size_t count, size_t n, bool is_real, double scale,
                              int ci, fhs_plaintext** outs) {
    fhs_status st = encode_checks(c, n, scale, ci);
    if (st != FHS_OK) return st;
    if (count == 0) return FHS_OK;
    BatchOut bo(outs, count);
    const size_t stride = is_real ? n : 2 * n;
    // values -> HBM (the copy completes before returning: the caller's buffer may be reused), then
    // FFT + exact reduction + NTT on the GPU (k_encode, k_ntt_fwd_ptrs), stream-ordered
    const size_t chunk = 4096;
    HostTrace ht;
    for (size_t base = 0; base < count; base += chunk) {
        const size_t cnt = std::min(chunk, count - base);
        uint64_t* dvals = nullptr;
        HIPCHK(dalloc(c, &dvals, std::max<size_t>(8, 8 * cnt * stride)), "encode staging");
        if (stride) {   // stage_h2d: through the pinned ring, no host wait, when it fits a segment (a client
                        // batch of a few vectors), else a copy + synchronisation
            hipError_t e = stage_h2d(c, dvals, vals + base * stride, 8 * cnt * stride);
            if (e != hipSuccess) { dfree(c, dvals, 8 * cnt * stride); return hip_fail(e, "encode upload"); }
        }
        ht.mark("encode: upload");
        fhs_status s = encode_rows_dev(c, reinterpret_cast<const double*>(dvals), cnt, n, stride, is_real, scale, ci,
                                       outs + base);
        dfree(c, dvals, std::max<size_t>(8, 8 * cnt * stride));
        ht.mark("encode: objects+launch");
        if (ht.on) { hipStreamSynchronize(c->st); ht.mark("encode: gpu"); }
        if (s != FHS_OK) return s;
    }
    return bo.keep(FHS_OK);
}

// Extension (no reference symbol): the whole caller-side diagonal pipeline of bg:198-203 +
// bg:361-432 on the device -- upload the D x D matrix once (D^2 doubles instead of D x slots),
// gather the rolled, tiled diagonal rows in HBM, encode them.  Values identical to
// encode_*_vector_batch on the host-prepared rows, hence identical limbs.
// The encoder behind encode_matrix_diagonals: diagonal rows `rows[0..nrows)` (indices into 0..D-1, any
// order) of the D x D view, giant group g rolled by g G, tiled, encoded -- out[k] is row rows[k].  Runs
// of consecutive indices are gathered by one launch each (a sharded matvec's rank needs a contiguous
// range of giant groups, or on a grid the same baby share of every group of its column).
static fhs_status encode_diag_rows(fhs_context* c, const double* M1, const double* M2, int64_t ld, int trans, int D,
                                   int G, double scale, int ci, const int* rows, int nrows, fhs_plaintext** out) {
    if (!M1 || !out || (nrows > 0 && !rows)) return fail(FHS_ERR_INVALID, "encode_diagonals: null argument");
    if (D < 1 || G < 1 || G > D) return fail(FHS_ERR_INVALID, "encode_diagonals: need 1 <= G <= D");
    if (ld < D) return fail(FHS_ERR_INVALID, "encode_diagonals: leading dimension below D");
    for (int k = 0; k < nrows; ++k)
        if (rows[k] < 0 || rows[k] >= D) return fail(FHS_ERR_INVALID, "encode_diagonals: row index out of range");
    const size_t n = c->N / 2;
    if ((size_t)D > n) return fail(FHS_ERR_INVALID, "encode_diagonals: dimension larger than the slot count");
    fhs_status st = encode_checks(c, n, scale, ci);
    if (st != FHS_OK) return st;
    const bool is_real = M2 == nullptr;
    BatchOut bo(out, (size_t)nrows);
    const size_t mb = 8ull * D * D;
    uint64_t *dm = nullptr, *dvals = nullptr;
    HIPCHK(dalloc(c, &dm, mb * (is_real ? 1 : 2)), "encode_diagonals matrix");
    // D rows of D doubles, `ld` apart on the host, packed on the device (no host-side copy of a view)
    hipError_t e = hipMemcpy2DAsync(dm, 8ull * D, M1, 8ull * ld, 8ull * D, D, hipMemcpyHostToDevice, c->st);
    if (e == hipSuccess && !is_real)
        e = hipMemcpy2DAsync((char*)dm + mb, 8ull * D, M2, 8ull * ld, 8ull * D, D, hipMemcpyHostToDevice, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);   // caller's buffers may be reused on return
    const double* m1 = reinterpret_cast<const double*>(dm);
    const double* m2 = is_real ? nullptr : reinterpret_cast<const double*>((char*)dm + mb);
    // the gathered rows repeat with period D (slot j reads column j mod D): periodic at t = n / D when that is a power
    // of two, so the compact factor is known without reading the detected periods back
    int ss_hint = 0;
    if (n % (size_t)D == 0 && ((n / D) & (n / D - 1)) == 0)
        ss_hint = std::min(__builtin_ctzll((unsigned long long)(n / D)), fhs::encode_sparse_max_log(c->logN));
    // The sparse encoder reads only each row's first (N/2) >> ss_hint values, so with ss_hint >= 1 only those are
    // gathered (a whole number of periods) and the periods are not detected: every row takes tlog = ss_hint -- the
    // largest power-of-two period the detector would find in a row of period D (one with a smaller period, e.g. a
    // constant diagonal, keeps the same factor; its encoding is the same polynomial up to the FFT's rounding).
    // FHESPEAR_ENCODE_DENSE=1 / FHESPEAR_ENCODE_UNFUSED=1 keep the full rows and the detector.
    static const bool full_rows = getenv("FHESPEAR_ENCODE_DENSE") || getenv("FHESPEAR_ENCODE_UNFUSED");
    const bool known = ss_hint >= 1 && !full_rows;
    const size_t ng = known ? n >> ss_hint : n, gstride = is_real ? ng : 2 * ng;
    const size_t chunk = 2048;
    for (size_t base = 0; e == hipSuccess && st == FHS_OK && base < (size_t)nrows; base += chunk) {
        const size_t cnt = std::min(chunk, (size_t)nrows - base);
        e = dalloc(c, &dvals, 8 * cnt * gstride);
        if (e != hipSuccess) break;
        for (size_t k = 0; e == hipSuccess && k < cnt;) {   // one gather per run of consecutive rows
            size_t r = 1;
            while (k + r < cnt && rows[base + k + r] == rows[base + k] + (int)r) ++r;
            e = fhs::launch_diag_gather(m1, m2, D, G, (int)ng, rows[base + k], (int)r, trans ? 1 : 0,
                                        reinterpret_cast<double*>(dvals) + k * gstride, c->st);
            k += r;
        }
        if (e == hipSuccess)
            st = encode_rows_dev(c, reinterpret_cast<const double*>(dvals), cnt, n, gstride, is_real, scale, ci,
                                 out + base, ss_hint, known);
        dfree(c, dvals, 8 * cnt * gstride);
    }
    dfree(c, dm, mb * (is_real ? 1 : 2));
    if (e != hipSuccess) return hip_fail(e, "encode_diagonals");
    return bo.keep(st);
}
extern "C" fhs_status fhs_encode_diagonals_ex(fhs_context* c, const double* M1, const double* M2, int64_t ld, int trans,
                                              int D, int G, double scale, int ci, fhs_plaintext** out) {
    ENTER(c);
    std::vector<int> rows(D > 0 ? D : 0);
    for (int k = 0; k < (int)rows.size(); ++k) rows[k] = k;
    return encode_diag_rows(c, M1, M2, ld, trans, D, G, scale, ci, rows.data(), (int)rows.size(), out);
}
extern "C" fhs_status fhs_encode_diagonals_rows(fhs_context* c, const double* M1, const double* M2, int64_t ld,
                                                int trans, int D, int G, double scale, int ci, const int* rows,
                                                int nrows, fhs_plaintext** out) {
    ENTER(c);
    return encode_diag_rows(c, M1, M2, ld, trans, D, G, scale, ci, rows, nrows, out);
}
extern "C" fhs_status fhs_encode_diagonals(fhs_context* c, const double* M1, const double* M2, int D, int G,
                                           double scale, int ci, fhs_plaintext** out) {
    return fhs_encode_diagonals_ex(c, M1, M2, D, 0, D, G, scale, ci, out);
}

// Extended-precision encoder for constant plaintexts (bootstrapping transforms): the f64 FFT of
// the GPU encoder has relative error ~2^-52 log n, i.e. hundreds of integer units at scale 2^59,
// which CoeffToSlot multiplies by |I| ~ K (DESIGN.md §3 bootstrapping).  Here the N/2-point DFT
// runs on the host in x87 long double (64-bit mantissa), each coefficient is rounded exactly to a
// 128-bit integer (hi, lo), and the device reduces it mod every limb and runs the NTT.
static void encode_precise_rows(const fhs_context* c, const double* vals, size_t n_in, size_t r0, size_t r1,
                                long double scale, int64_t* hi, uint64_t* lo, std::atomic<int>* overflow) {
    typedef std::complex<long double> cl;
    const size_t N = c->N, n = N / 2;
    int logn = 0;
    while (((size_t)1 << logn) < n) ++logn;
    const long double pi = acosl(-1.0L);
    std::vector<cl> w(n / 2), tw(n), a(n);
    for (size_t t = 0; t < n / 2; ++t) w[t] = cl(cosl(2 * pi * t / n), -sinl(2 * pi * t / n));   // omega^-t
    for (size_t k = 0; k < n; ++k)                                                              // (2/N) zeta^-k
        tw[k] = cl(cosl(pi * k / N), -sinl(pi * k / N)) * (2.0L / (long double)N);
    const long double two64 = 18446744073709551616.0L;
    for (size_t r = r0; r < r1; ++r) {
        std::fill(a.begin(), a.end(), cl(0, 0));
        for (size_t j = 0; j < n_in; ++j) {                       // Z[s_j] = z_j, 5^j = 4 s_j + 1
            const size_t s = (size_t)(c->slot_index[j] >> 1);
            a[h_bitrev((uint32_t)s, logn)] = cl(vals[(r * n_in + j) * 2], vals[(r * n_in + j) * 2 + 1]);
        }
        for (size_t len = 2; len <= n; len <<= 1) {               // DIT, natural-order output
            const size_t step = n / len;
            for (size_t i = 0; i < n; i += len)
                for (size_t k = 0; k < len / 2; ++k) {
                    const cl u = a[i + k], v = a[i + k + len / 2] * w[k * step];
                    a[i + k] = u + v;
                    a[i + k + len / 2] = u - v;
                }
        }
        for (size_t k = 0; k < n; ++k) {
            const cl ck = a[k] * tw[k];
            const long double part[2] = {ck.real() * scale, ck.imag() * scale};
            for (int h = 0; h < 2; ++h) {
                const long double x = roundl(part[h]);
                if (!(fabsl(x) < 0x1p126L)) { overflow->store(1); continue; }
                const long double xh = floorl(x / two64);
                const size_t idx = r * N + k + (size_t)h * n;
                hi[idx] = (int64_t)xh;
                lo[idx] = (uint64_t)(x - xh * two64);
            }
        }
    }
}
extern "C" fhs_status fhs_encode_precise(fhs_context* c, const double* re_im, size_t count, size_t n, double scale,
                                         int ci, fhs_plaintext** outs) {
    ENTER(c);
    if ((!re_im && n) || !outs) return fail(FHS_ERR_INVALID, "encode_precise: null argument");
    if (n > c->N / 2) return fail(FHS_ERR_INVALID, "encode_precise: more values than slots");
    if (!(scale > 0) || !std::isfinite(scale) || scale > 0x1p126) return fail(FHS_ERR_INVALID, "encode_precise: bad scale");
    const int l = c->L0 + 1 - ci;
    if (ci < 1 || l < 1) return fail(FHS_ERR_LEVEL, "encode: chain index out of range");
    if (count == 0) return FHS_OK;
    BatchOut bo(outs, count);
    const size_t N = c->N;
    std::vector<int64_t> hi(count * N);
    std::vector<uint64_t> lo(count * N);
    const size_t nth = std::max<size_t>(1, std::min<size_t>({count, 16, (size_t)std::thread::hardware_concurrency()}));
    std::vector<std::thread> th;
    std::atomic<int> overflow{0};
    for (size_t t = 0; t < nth; ++t)
        th.emplace_back(encode_precise_rows, c, re_im, n, count * t / nth, count * (t + 1) / nth, (long double)scale,
                        hi.data(), lo.data(), &overflow);
    for (auto& x : th) x.join();
    if (overflow.load()) return fail(FHS_ERR_INVALID, "encode_precise: |value x scale| >= 2^126 (or not finite)");
    uint64_t* dbuf = nullptr;
    HIPCHK(dalloc(c, &dbuf, 16 * count * N), "encode_precise staging");
    hipError_t e = hipMemcpyAsync(dbuf, hi.data(), 8 * count * N, hipMemcpyHostToDevice, c->st);
    if (e == hipSuccess) e = hipMemcpyAsync(dbuf + count * N, lo.data(), 8 * count * N, hipMemcpyHostToDevice, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);
    std::vector<uint64_t*> ptrs(count);
    if (e == hipSuccess) {
        fhs_status s = new_pts(c, count, ci, scale, outs);
        if (s != FHS_OK) { dfree(c, dbuf, 16 * count * N); return s; }
        for (size_t v = 0; v < count; ++v) ptrs[v] = outs[v]->d;
    }
    uint64_t* dptrs = nullptr;
    if (e == hipSuccess) e = scratch(c, fhs_context::SCR_ENC_PTRS, 8 * count, &dptrs);
    if (e == hipSuccess) e = stage_h2d(c, dptrs, ptrs.data(), 8 * count);
    if (e == hipSuccess)
        e = fhs::launch_encode_int128(c->T, reinterpret_cast<const int64_t*>(dbuf), dbuf + count * N, (int)count,
                                      reinterpret_cast<fhs::u64* const*>(dptrs), l, c->st);
    dfree(c, dbuf, 16 * count * N);
    if (e != hipSuccess) return hip_fail(e, "encode_precise");
    return bo.keep(FHS_OK);
}

extern "C" fhs_status fhs_encode(fhs_context* c, const double* re_im, size_t n, double scale, int ci,
                                 fhs_plaintext** out) {
    ENTER(c);
    if ((!re_im && n) || !out) return fail(FHS_ERR_INVALID, "encode: null argument");
    return encode_many(c, re_im, 1, n, false, scale, ci, out);
}
extern "C" fhs_status fhs_encode_real(fhs_context* c, const double* v, size_t n, double scale, int ci,
                                      fhs_plaintext** out) {
    ENTER(c);
    if ((!v && n) || !out) return fail(FHS_ERR_INVALID, "encode: null argument");
    return encode_many(c, v, 1, n, true, scale, ci, out);
}
extern "C" fhs_status fhs_encode_batch(fhs_context* c, const double* re_im, size_t count, size_t n, double scale,
                                       int ci, fhs_plaintext** out) {
    ENTER(c);
    if (!re_im || !out) return fail(FHS_ERR_INVALID, "encode_batch: null argument");
    return encode_many(c, re_im, count, n, false, scale, ci, out);
}
extern "C" fhs_status fhs_encode_real_batch(fhs_context* c, const double* v, size_t count, size_t n, double scale,
                                            int ci, fhs_plaintext** out) {
    ENTER(c);
    if (!v || !out) return fail(FHS_ERR_INVALID, "encode_batch: null argument");
    return encode_many(c, v, count, n, true, scale, ci, out);
}

// CRT-compose l residues of each coefficient to a centred double (multi-precision, host)
static void crt_compose(const fhs_context* c, const std::vector<uint64_t>& limbs, int l, std::vector<double>& out) {
    const size_t N = c->N;
    const int W = l + 1;
    std::vector<uint64_t> Q(W, 0);
    Q[0] = 1;
    for (int i = 0; i < l; ++i) {
        hu128 carry = 0;
        for (int w = 0; w < W; ++w) {
            const hu128 t = (hu128)Q[w] * c->q[i] + carry;
            Q[w] = (uint64_t)t;
            carry = t >> 64;
        }
    }
    std::vector<uint64_t> hat((size_t)l * W, 0), ihat(l);
    for (int i = 0; i < l; ++i) {
        uint64_t* h = &hat[(size_t)i * W];
        h[0] = 1;
        uint64_t hm = 1;
        for (int k = 0; k < l; ++k) {
            if (k == i) continue;
            hu128 carry = 0;
            for (int w = 0; w < W; ++w) {
                const hu128 t = (hu128)h[w] * c->q[k] + carry;
                h[w] = (uint64_t)t;
                carry = t >> 64;
            }
            hm = h_mulmod(hm, c->q[k] % c->q[i], c->q[i]);
        }
        ihat[i] = h_inv(hm, c->q[i]);
    }
    std::vector<uint64_t> ihat_s(l);
    for (int i = 0; i < l; ++i) ihat_s[i] = (uint64_t)(((hu128)ihat[i] << 64) / c->q[i]);
    std::vector<uint64_t> halfQ(W);
    for (int w = 0; w < W; ++w) halfQ[w] = (Q[w] >> 1) | (w + 1 < W ? Q[w + 1] << 63 : 0);
    out.assign(N, 0.0);
    const unsigned nth = std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), l <= 6 ? 8 : 32));
    std::vector<std::thread> th;
    for (unsigned tix = 0; tix < nth; ++tix)
        th.emplace_back([&, tix]() {
            std::vector<uint64_t> x(W + 1);
            for (size_t n = tix; n < N; n += nth) {
                std::fill(x.begin(), x.end(), 0);
                for (int i = 0; i < l; ++i) {
                    // y = limb * ihat mod q by Shoup (ihat_s = floor(ihat 2^64 / q)); limbs are < q
                    const uint64_t a = limbs[(size_t)i * N + n], qi = c->q[i];
                    const uint64_t qh = (uint64_t)(((hu128)a * ihat_s[i]) >> 64);
                    uint64_t y = a * ihat[i] - qh * qi;
                    if (y >= qi) y -= qi;
                    hu128 carry = 0;
                    const uint64_t* h = &hat[(size_t)i * W];
                    for (int w = 0; w < W; ++w) {
                        const hu128 t = (hu128)h[w] * y + x[w] + carry;
                        x[w] = (uint64_t)t;
                        carry = t >> 64;
                    }
                    x[W] += (uint64_t)carry;
                    for (;;) {   // x < 2Q: at most one subtraction
                        bool ge = x[W] != 0;
                        if (!ge) {
                            ge = true;
                            for (int w = W - 1; w >= 0; --w)
                                if (x[w] != Q[w]) { ge = x[w] > Q[w]; break; }
                        }
                        if (!ge) break;
                        uint64_t br = 0;
                        for (int w = 0; w < W; ++w) {
                            const uint64_t qa = Q[w] + br;
                            const uint64_t nb = (qa < br) || (x[w] < qa);
                            x[w] -= qa;
                            br = nb;
                        }
                        x[W] -= br;
                    }
                }
                bool neg = false;
                for (int w = W - 1; w >= 0; --w)
                    if (x[w] != halfQ[w]) { neg = x[w] > halfQ[w]; break; }
                if (neg) {
                    uint64_t br = 0;
                    for (int w = 0; w < W; ++w) {
                        const uint64_t xa = x[w] + br;
                        const uint64_t nb = (xa < br) || (Q[w] < xa);
                        x[w] = Q[w] - xa;
                        br = nb;
                    }
                }
                double v = 0;
                for (int w = W - 1; w >= 0; --w) v = v * 18446744073709551616.0 + (double)x[w];
                out[n] = neg ? -v : v;
            }
        });
    for (auto& t : th) t.join();
}

// Coefficients of a decrypted plaintext are |x| = |m| scale + noise: the centred CRT over the first
// k limbs (prod q_i >= scale 2^72) is the same integer as over all l, hence the same double, whenever
// |x| < Q_k / 2 -- every plaintext whose coefficients are below 2^71 scale, the range CKKS decoding is
// meant for.  The GPU composes k+1 limbs and checks the result against every other limb (it must equal
// the coefficient's residue mod each q_e): all agree exactly when the composition IS the coefficient
// (both lie in (-Q_l/2, Q_l/2) and agree mod Q_l), so any larger coefficient -- which would otherwise
// decode to an aliased value -- is detected and the decoder composes all l limbs instead.
// FHESPEAR_DECODE_FULL=1 always composes all l limbs.
static int decode_limbs(const fhs_context* c, double scale, int l) {
    double bits = 0, need = std::log2(std::max(scale, 1.0)) + 72.0;
    for (int i = 0; i < l; ++i) {
        bits += std::log2((double)c->q[i]);
        if (bits >= need) return i + 1;
    }
    return l;
}
// constants of the centred CRT over the first l limbs for the GPU composition (l <= kCrtMaxL): the
// same Q, hat, inv-hat (+ Shoup companion) and Q/2 words crt_compose derives on the host
static void crt_consts(const fhs_context* c, int l, fhs::CrtConsts& K) {
    K = fhs::CrtConsts{};
    K.l = l;
    K.W = l + 1;
    const int W = K.W;
    K.Q[0] = 1;
    for (int i = 0; i < l; ++i) {
        hu128 carry = 0;
        for (int w = 0; w < W; ++w) {
            const hu128 t = (hu128)K.Q[w] * c->q[i] + carry;
            K.Q[w] = (uint64_t)t;
            carry = t >> 64;
        }
    }
    for (int i = 0; i < l; ++i) {
        uint64_t* h = K.hat[i];
        h[0] = 1;
        uint64_t hm = 1;
        for (int k = 0; k < l; ++k) {
            if (k == i) continue;
            hu128 carry = 0;
            for (int w = 0; w < W; ++w) {
                const hu128 t = (hu128)h[w] * c->q[k] + carry;
                h[w] = (uint64_t)t;
                carry = t >> 64;
            }
            hm = h_mulmod(hm, c->q[k] % c->q[i], c->q[i]);
        }
        K.q[i] = c->q[i];
        K.ihat[i] = h_inv(hm, c->q[i]);
        K.ihat_s[i] = (uint64_t)(((hu128)K.ihat[i] << 64) / c->q[i]);
    }
    for (int w = 0; w < W; ++w) K.halfQ[w] = (K.Q[w] >> 1) | (w + 1 < W ? K.Q[w + 1] << 63 : 0);
}
// INTT of the first lv limbs and the centred CRT composition of the first k on the GPU, checked against
// limbs k..lv-1 (*exact = every coefficient matched them); N doubles to the host
// The composition constants of the first kk limbs and the check tables of limbs kk..l-1 ([CrtConsts as
// words][l - kk vtabs of kCrtVtabWords]), built once per (kk, l) and kept in the context: a client decodes
// the same few levels over and over
static const std::vector<uint64_t>& crt_tables(fhs_context* c, int kk, int l) {
    std::vector<uint64_t>& tab = c->crt_cache[std::make_pair(kk, l)];
    if (!tab.empty()) return tab;
    constexpr size_t KW = sizeof(fhs::CrtConsts) / 8;
    static_assert(sizeof(fhs::CrtConsts) % 8 == 0, "CrtConsts packs into words");
    fhs::CrtConsts K;
    crt_consts(c, kk, K);
    tab.assign(KW + (size_t)(l - kk) * fhs::kCrtVtabWords, 0);
    std::memcpy(tab.data(), &K, sizeof(K));
    for (int x = 0; x < l - kk; ++x) {
        uint64_t* v = tab.data() + KW + (size_t)x * fhs::kCrtVtabWords;
        const uint64_t q = c->q[kk + x];
        const hu128 R = (~(hu128)0) / q;
        v[0] = q;
        v[1] = (uint64_t)R;
        v[2] = (uint64_t)(R >> 64);
        const uint64_t t64 = (uint64_t)((((hu128)1) << 64) % q);
        uint64_t pw = 1 % q;
        for (int w = 0; w < K.W; ++w) {
            v[3 + w] = pw;
            pw = h_mulmod(pw, t64, q);
        }
    }
    return tab;
}
static fhs_status decode_coeffs_dev(fhs_context* c, const fhs_plaintext* pt, int k, int lv, std::vector<double>& m,
                                    bool* exact) {
    const size_t N = c->N, bytes = 8ull * lv * N;
    const int nx = lv - k;
    fhs::CrtConsts K;
    crt_consts(c, k, K);
    std::vector<uint64_t> vt((size_t)nx * fhs::kCrtVtabWords, 0);
    for (int e = 0; e < nx; ++e) {
        uint64_t* v = vt.data() + (size_t)e * fhs::kCrtVtabWords;
        const uint64_t q = c->q[k + e];
        const hu128 R = (~(hu128)0) / q;   // floor(2^128 / q) for odd q
        v[0] = q;
        v[1] = (uint64_t)R;
        v[2] = (uint64_t)(R >> 64);
        const uint64_t t64 = (uint64_t)((((hu128)1) << 64) % q);
        uint64_t pw = 1 % q;
        for (int w = 0; w < K.W; ++w) {
            v[3 + w] = pw;
            pw = h_mulmod(pw, t64, q);
        }
    }
    const size_t extra_b = 8 * vt.size() + 8;   // vtab, then the mismatch flag
    uint64_t *tmp = nullptr, *dbl = nullptr, *aux = nullptr;
    HIPCHK(dalloc(c, &tmp, bytes), "decode");
    hipError_t e = dalloc(c, &dbl, 8 * N);
    if (e != hipSuccess) { dfree(c, tmp, bytes); return hip_fail(e, "decode"); }
    e = dalloc(c, &aux, extra_b);
    if (e != hipSuccess) { dfree(c, dbl, 8 * N); dfree(c, tmp, bytes); return hip_fail(e, "decode"); }
    unsigned* flag = reinterpret_cast<unsigned*>(aux + vt.size());
    unsigned hflag = 0;
    const uint64_t* pd = nullptr;
    e = pt_dense(c, pt, &pd);
    if (e == hipSuccess) e = hipMemcpyAsync(tmp, pd, bytes, hipMemcpyDeviceToDevice, c->st);
    if (e == hipSuccess && nx > 0) e = stage_h2d(c, aux, vt.data(), 8 * vt.size());
    if (e == hipSuccess) e = hipMemsetAsync(flag, 0, 4, c->st);
    if (e == hipSuccess) e = fhs::launch_ntt_inv(c->T, tmp, lv, lv, 1, 0, c->st);
    if (e == hipSuccess)
        e = fhs::launch_crt_compose(K, tmp, reinterpret_cast<double*>(dbl), (int)N, c->st, tmp + (size_t)k * N, nx, aux,
                                    flag);
    m.resize(N);
    if (e == hipSuccess) e = hipMemcpyAsync(m.data(), dbl, 8 * N, hipMemcpyDeviceToHost, c->st);
    if (e == hipSuccess) e = hipMemcpyAsync(&hflag, flag, 4, hipMemcpyDeviceToHost, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);
    dfree(c, aux, extra_b);
    dfree(c, dbl, 8 * N);
    dfree(c, tmp, bytes);
    if (e != hipSuccess) return hip_fail(e, "decode");
    *exact = hflag == 0;
    return FHS_OK;
}
static fhs_status decode_coeffs(fhs_context* c, const fhs_plaintext* pt, int k, std::vector<uint64_t>& host) {
    const size_t N = c->N, bytes = 8ull * k * N;
    uint64_t* tmp = nullptr;
    PT_DENSE(pd, pt, "decode");
    HIPCHK(dalloc(c, &tmp, bytes), "decode");
    HIPCHK(hipMemcpyAsync(tmp, pd, bytes, hipMemcpyDeviceToDevice, c->st), "decode");
    HIPCHK(fhs::launch_ntt_inv(c->T, tmp, k, k, 1, 0, c->st), "decode");
    host.resize((size_t)k * N);
    HIPCHK(hipMemcpyAsync(host.data(), tmp, bytes, hipMemcpyDeviceToHost, c->st), "decode");
    HIPCHK(hipStreamSynchronize(c->st), "decode");
    dfree(c, tmp, bytes);
    return FHS_OK;
}
// centred coefficients of the first k limbs as doubles: composed on the GPU up to kCrtMaxL limbs (same
// arithmetic, same doubles as the host composition, which FHESPEAR_DECODE_HOST_CRT=1 forces)
static fhs_status decode_compose(fhs_context* c, const fhs_plaintext* pt, int k, std::vector<double>& m) {
    static const bool host_crt = getenv("FHESPEAR_DECODE_HOST_CRT") != nullptr;   // A/B and test knob
    bool unused;
    if (k <= fhs::kCrtMaxL && !host_crt) return decode_coeffs_dev(c, pt, k, k, m, &unused);
    std::vector<uint64_t> host;
    const fhs_status s = decode_coeffs(c, pt, k, host);
    if (s != FHS_OK) return s;
    crt_compose(c, host, k, m);
    return FHS_OK;
}
// slots z_j = m(zeta^(5^j)) = sum_{k < N/2} (m_k + i m_{k+N/2}) zeta^k omega^(s_j k), omega = zeta^4,
// 5^j = 4 s_j + 1: an N/2-point FFT of the twisted half-pairs, read at s_j = slot_index[j] / 2; the first
// `nslots` slots to re_im
static void decode_slots(const fhs_context* c, const double* m, double scale, size_t nslots, double* re_im) {
    const size_t n = c->N / 2;
    std::vector<std::complex<double>> v(n);
    for (size_t k2 = 0; k2 < n; ++k2) {
        const double a = m[k2] / scale, b = m[k2 + n] / scale;
        const double cr = c->dec_twist[k2].real(), ci = c->dec_twist[k2].imag();
        v[k2] = {a * cr - b * ci, a * ci + b * cr};
    }
    fft_inplace(v, c->fft_w, c->logN - 1, 2);
    for (size_t j = 0; j < nslots; ++j) {
        const std::complex<double> z = v[c->slot_index[j] >> 1];
        re_im[2 * j] = z.real();
        re_im[2 * j + 1] = z.imag();
    }
}
static hipError_t readback_buf(fhs_context* c, size_t bytes, double** out) {
    if (bytes > c->readback_bytes) {   // every earlier use ended with a stream synchronisation
        if (c->readback) hipHostFree(c->readback);
        c->readback = nullptr;
        c->readback_bytes = 0;
        const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&c->readback), bytes, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        c->readback_bytes = bytes;
    }
    *out = c->readback;
    return hipSuccess;
}

// Decode `count` plaintexts to their first `nslots` slots (out: count x nslots x (re, im)), all on the GPU:
// per plaintext the INTT, centred CRT composition of the limbs the scale needs (+1) and the check against
// the rest (decode_coeffs_dev's arithmetic); then one k_decode_fft + gather over all of them; only the
// slots come back, through the pinned readback buffer, after ONE synchronisation.  A plaintext whose
// check fails (an aliased coefficient) or that needs more limbs than the GPU composition takes is
// composed exactly from all its limbs (decode_compose) and decoded on its own.  FHESPEAR_DECODE_HOST_FFT=1
// runs the slot FFT on the host instead (decode_slots: the same operations, so the same doubles; A/B and
// test knob).
// cts non-null (with sk): the items are ciphertexts, decrypted straight into the INTT's buffer
// (fhs_decrypt_decode_batch) instead of plaintexts copied there
static fhs_status decode_many(fhs_context* c, const fhs_plaintext* const* pts, int count, int nslots, double* re_im,
                              const fhs_ciphertext* const* cts = nullptr, fhs_secret_key* sk = nullptr) {
    const size_t N = c->N, n = N / 2;
    if ((!pts && !cts) || (cts && !sk) || !re_im || count < 0 || nslots < 1 || (size_t)nslots > n)
        return fail(FHS_ERR_INVALID, "decode: bad arguments");
    if (cts)
        for (int i = 0; i < count; ++i) LIVE(cts[i]);
    auto lv = [&](int i) { return cts ? cts[i]->l : pts[i]->l; };
    auto scl = [&](int i) { return cts ? cts[i]->scale : pts[i]->scale; };
    if (count == 0) return FHS_OK;
    static const bool full = getenv("FHESPEAR_DECODE_FULL") != nullptr;       // A/B and test knobs
    static const bool host_crt = getenv("FHESPEAR_DECODE_HOST_CRT") != nullptr;
    static const bool host_fft = getenv("FHESPEAR_DECODE_HOST_FFT") != nullptr;
    std::vector<int> fast(count, 0), kks(count, 0);
    size_t tmp_words = 0, vt_words = 0;
    for (int i = 0; i < count; ++i) {
        if (cts ? !cts[i] : !pts[i]) return fail(FHS_ERR_INVALID, "decode: null plaintext or ciphertext");
        const int l = lv(i), k = full ? l : decode_limbs(c, scl(i), l);
        kks[i] = std::min(l, k + 1);
        fast[i] = kks[i] < l && kks[i] <= fhs::kCrtMaxL && !host_crt;
        if (fast[i]) {
            tmp_words += (size_t)l * N;
            vt_words += (size_t)(l - kks[i]) * fhs::kCrtVtabWords;
        }
    }
    // aux (one staged copy up to the flags): the scales, every fast item's check table (vtab), its
    // composition job (fhs::CrtJob), the ciphertext pointers (cts), the zeroed check flags, then the slots;
    // flags and slots come back in one copy
    constexpr size_t JW = sizeof(fhs::CrtJob) / 8;
    static_assert(sizeof(fhs::CrtJob) % 8 == 0, "CrtJob packs into words");
    int nf = 0, lf = -1, max_nx = 0;
    bool one_l = true, one_nc = true;
    for (int i = 0; i < count; ++i) {
        if (!fast[i]) continue;
        one_l &= lf < 0 || lv(i) == lf;
        one_nc &= !cts || cts[i]->ncomp == cts[0]->ncomp;
        lf = lv(i);
        max_nx = std::max(max_nx, lv(i) - kks[i]);
        ++nf;
    }
    const size_t FW = ((size_t)count + 1) / 2, J0 = (size_t)count + vt_words, P0 = J0 + (size_t)nf * JW,
                 A0 = P0 + (cts ? (size_t)count : 0);
    const size_t slot_words = host_fft ? 0 : 2 * (size_t)nslots * count;
    const size_t aux_words = A0 + FW + slot_words;
    HostTrace ht;
    const size_t per_out = host_fft ? N : 2 * (size_t)nslots;   // doubles back per item
    const size_t dbl_b = 8 * N * count, spec_b = 16 * n * count;
    uint64_t *tmp = nullptr, *dbl = nullptr, *aux = nullptr, *spec = nullptr;
    double* rb = nullptr;
    hipError_t e = readback_buf(c, 8 * (FW + per_out * count), &rb);
    if (e == hipSuccess && tmp_words) e = dalloc(c, &tmp, 8 * tmp_words);
    if (e == hipSuccess) e = dalloc(c, &dbl, dbl_b);
    if (e == hipSuccess) e = dalloc(c, &aux, 8 * aux_words);
    if (e == hipSuccess && !host_fft) e = dalloc(c, &spec, spec_b);
    const unsigned* hflag = reinterpret_cast<const unsigned*>(rb);
    double* rslots = rb + FW;
    const double* dscales = reinterpret_cast<const double*>(aux);
    unsigned* dflag = reinterpret_cast<unsigned*>(aux + A0);
    uint64_t* dout = aux + A0 + FW;
    std::vector<uint64_t> head(A0 + FW, 0);
    for (int i = 0; i < count; ++i) {
        const double sc = scl(i);
        std::memcpy(&head[i], &sc, 8);
    }
    size_t vo = (size_t)count, jo = J0, to = 0;
    for (int i = 0; i < count; ++i) {
        if (!fast[i]) continue;
        const int l = lv(i), kk = kks[i], nx = l - kk;
        const std::vector<uint64_t>& tab = crt_tables(c, kk, l);   // [CrtConsts][nx vtabs], cached per (kk, l)
        fhs::CrtJob J{};
        std::memcpy(&J.K, tab.data(), sizeof(fhs::CrtConsts));
        std::memcpy(head.data() + vo, tab.data() + sizeof(fhs::CrtConsts) / 8, 8 * (size_t)nx * fhs::kCrtVtabWords);
        J.limbs = tmp + to;
        J.out = reinterpret_cast<double*>(dbl) + (size_t)i * N;
        J.extra = tmp + to + (size_t)kk * N;
        J.vtab = aux + vo;
        J.flag = dflag + i;
        J.nx = nx;
        std::memcpy(head.data() + jo, &J, sizeof(J));
        vo += (size_t)nx * fhs::kCrtVtabWords;
        jo += JW;
        to += (size_t)l * N;
    }
    if (cts)
        for (int i = 0; i < count; ++i) head[P0 + i] = reinterpret_cast<uint64_t>(cts[i]->d);
    if (e == hipSuccess) e = stage_h2d(c, aux, head.data(), 8 * head.size());
    // coefficient form: the fast items side by side (decrypted there, or copied), one INTT launch over all
    // of them when they share a level (the usual client batch), else one per item
    if (cts && nf == count && one_l && one_nc) {
        if (e == hipSuccess)
            e = fhs::launch_decrypt_many(c->T, reinterpret_cast<const fhs::u64* const*>(aux + P0), count, cts[0]->ncomp,
                                         sk->s, tmp, (size_t)lf * N, lf, c->st);
    } else {
        to = 0;
        for (int i = 0; e == hipSuccess && i < count; ++i) {
            if (!fast[i]) continue;
            const int l = lv(i);
            const uint64_t* pd = nullptr;
            if (!cts) e = pt_dense(c, pts[i], &pd);
            if (e == hipSuccess)
                e = cts ? fhs::launch_decrypt(c->T, cts[i]->d, cts[i]->ncomp, sk->s, tmp + to, l, c->st)
                        : hipMemcpyAsync(tmp + to, pd, 8ull * l * N, hipMemcpyDeviceToDevice, c->st);
            if (e == hipSuccess && !one_l) e = fhs::launch_ntt_inv(c->T, tmp + to, l, l, 1, 0, c->st);
            to += (size_t)l * N;
        }
    }
    if (e == hipSuccess && nf > 0 && one_l) e = fhs::launch_ntt_inv(c->T, tmp, lf, lf, nf, (size_t)lf * N, c->st);
    if (e == hipSuccess && nf > 0)
        e = fhs::launch_crt_compose_jobs(reinterpret_cast<const fhs::CrtJob*>(aux + J0), nf, max_nx, (int)N, c->st);
    // the slots of every item (a slow one's are recomputed below), then flags + slots in one copy back
    if (e == hipSuccess && !host_fft)
        e = fhs::launch_decode_slots(c->T, reinterpret_cast<const double*>(dbl), dscales, count,
                                     reinterpret_cast<double*>(spec), nslots, reinterpret_cast<double*>(dout), c->st);
    if (e == hipSuccess) e = hipMemcpyAsync(rb, dflag, 8 * (FW + slot_words), hipMemcpyDeviceToHost, c->st);
    if (e == hipSuccess && host_fft) e = hipMemcpyAsync(rslots, dbl, 8 * per_out * count, hipMemcpyDeviceToHost, c->st);
    ht.mark("decode: enqueue");
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);
    ht.mark("decode: gpu");
    fhs_status st = e == hipSuccess ? FHS_OK : hip_fail(e, "decode");
    std::vector<double> m;
    for (int i = 0; st == FHS_OK && i < count; ++i) {
        if (fast[i] && hflag[i] == 0) continue;
        if (cts) {   // exact: all limbs, from the decrypted plaintext
            fhs_plaintext* pt = nullptr;
            st = fhs_decrypt(c, sk, cts[i], &pt);
            if (st == FHS_OK) st = decode_compose(c, pt, pt->l, m);
            if (pt) fhs_plaintext_destroy(pt);
        } else {
            st = decode_compose(c, pts[i], pts[i]->l, m);   // exact: all limbs
        }
        if (st != FHS_OK) break;
        double* slot = rslots + (size_t)i * per_out;
        if (host_fft) {
            std::copy(m.begin(), m.end(), slot);
            continue;
        }
        double* di = reinterpret_cast<double*>(dbl) + (size_t)i * N;
        e = hipMemcpyAsync(di, m.data(), 8 * N, hipMemcpyHostToDevice, c->st);
        if (e == hipSuccess)
            e = fhs::launch_decode_slots(c->T, di, dscales + i, 1, reinterpret_cast<double*>(spec), nslots,
                                         reinterpret_cast<double*>(dout), c->st);
        if (e == hipSuccess) e = hipMemcpyAsync(slot, dout, 8 * per_out, hipMemcpyDeviceToHost, c->st);
        if (e == hipSuccess) e = hipStreamSynchronize(c->st);
        if (e != hipSuccess) st = hip_fail(e, "decode");
    }
    for (int i = 0; st == FHS_OK && i < count; ++i) {
        double* out = re_im + (size_t)i * 2 * nslots;
        if (host_fft)
            decode_slots(c, rslots + (size_t)i * N, scl(i), (size_t)nslots, out);
        else
            std::memcpy(out, rslots + (size_t)i * per_out, 8 * per_out);
    }
    ht.mark("decode: slots");
    if (spec) dfree(c, spec, spec_b);
    if (aux) dfree(c, aux, 8 * aux_words);
    if (dbl) dfree(c, dbl, dbl_b);
    if (tmp) dfree(c, tmp, 8 * tmp_words);
    return st;
}
extern "C" fhs_status fhs_decode(fhs_context* c, const fhs_plaintext* pt, double* re_im) {
    ENTER(c);
    if (!pt || !re_im) return fail(FHS_ERR_INVALID, "decode: null argument");
    return decode_many(c, &pt, 1, (int)(c->N / 2), re_im);
}
extern "C" fhs_status fhs_decrypt_decode_batch(fhs_context* c, fhs_secret_key* sk, const fhs_ciphertext* const* cts,
                                               int count, int nslots, double* re_im) {
    ENTER(c);
    if (!sk || !cts || !re_im || count < 0 || nslots < 1 || (size_t)nslots > c->N / 2)
        return fail(FHS_ERR_INVALID, "decrypt_decode_batch: bad arguments");
    for (int i0 = 0; i0 < count; i0 += kMaxBatch) {   // grid rows and scratch bound one launch
        const fhs_status s = decode_many(c, nullptr, std::min(kMaxBatch, count - i0), nslots,
                                         re_im + (size_t)i0 * 2 * nslots, cts + i0, sk);
        if (s != FHS_OK) return s;
    }
    return FHS_OK;
}
// Client-side batch (the client-aided block decrypts 2-3 outputs per stage): decode_many over all of
// them, one synchronisation, only the first `nslots` slots of each back to the host.
extern "C" fhs_status fhs_decode_batch(fhs_context* c, const fhs_plaintext* const* pts, int count, int nslots,
                                       double* re_im) {
    ENTER(c);
    if (!pts || !re_im || count < 0 || nslots < 1 || (size_t)nslots > c->N / 2)
        return fail(FHS_ERR_INVALID, "decode_batch: bad arguments");
    for (int i0 = 0; i0 < count; i0 += kMaxBatch) {
        const fhs_status s = decode_many(c, pts + i0, std::min(kMaxBatch, count - i0), nslots,
                                         re_im + (size_t)i0 * 2 * nslots);
        if (s != FHS_OK) return s;
    }
    return FHS_OK;
}

// ============================================================================ encryption
extern "C" fhs_status fhs_encrypt_symmetric(fhs_context* c, fhs_secret_key* sk, const fhs_plaintext* pt,
                                            fhs_ciphertext** out) {
    ENTER(c);
    if (!sk || !pt || !out) return fail(FHS_ERR_INVALID, "encrypt: null argument");
    const uint64_t ctr = sk->ctr++;
    fhs_ciphertext* ct;
    fhs_status s = new_ct(c, 2, pt->ci, pt->scale, &ct);
    if (s != FHS_OK) return s;
    const int l = pt->l;
    const size_t S = (size_t)l * c->N;
    uint64_t* eb = nullptr;
    HIPCHK(dalloc(c, &eb, 8 * S), "encrypt");
    HIPCHK(fhs::launch_sample(c->T, fhs::SAMPLE_UNIFORM, sk->key, stream_id(ST_ENC_SYM, ctr, 0), ct->d + S, l, c->st), "encrypt");
    HIPCHK(sample_small_ntt(c, fhs::SAMPLE_CBD, sk->key, stream_id(ST_ENC_SYM, ctr, 1), eb, l), "encrypt");
    PT_DENSE(pd, pt, "encrypt");
    HIPCHK(fhs::launch_encrypt_combine(c->T, 0, ct->d, ct->d + S, sk->s, nullptr, nullptr, eb, nullptr, pd, l, c->st),
           "encrypt");
    dfree(c, eb, 8 * S);
    *out = ct;
    return FHS_OK;
}
// `count` symmetric encryptions at l limbs into new ciphertexts outs[i] (chain index ci, scale scales[i]):
// of the plaintexts pts[i], or (pts null) of the rounded message coefficients `coef` already in HBM
// (count x N doubles, launch_encode_coef) -- encode and encrypt fused.  Counters as `count` calls.
static fhs_status encrypt_sym_core(fhs_context* c, fhs_secret_key* sk, int count, int l, int ci, const double* scales,
                                   const fhs_plaintext* const* pts, const double* coef, fhs_ciphertext** outs) {
    BatchOutT<fhs_ciphertext> bo(outs, count);
    const size_t S = (size_t)l * c->N;
    for (int i = 0; i < count; ++i) {
        fhs_ciphertext* ct;
        fhs_status s = new_ct(c, 2, ci, scales[i], &ct);
        if (s != FHS_OK) return s;
        outs[i] = ct;
    }
    const uint64_t ctr0 = sk->ctr;
    sk->ctr += (uint64_t)count;
    const uint64_t step = stream_id(0, 1, 0);   // consecutive counters: stream ids 2^16 apart
    std::vector<uint64_t*> ptrs(2 * (size_t)count, nullptr);
    for (int i = 0; i < count; ++i) {
        ptrs[i] = outs[i]->d;
        if (pts) {
            const uint64_t* pd = nullptr;
            HIPCHK(pt_dense(c, pts[i], &pd), "encrypt");
            ptrs[count + i] = const_cast<uint64_t*>(pd);
        }
    }
    uint64_t *eb = nullptr, *dptrs = nullptr, *small = nullptr;
    const size_t small_b = ((size_t)c->N * count + 7) & ~(size_t)7;
    HIPCHK(dalloc(c, &eb, 8 * S * count), "encrypt");
    hipError_t e = dalloc(c, &dptrs, 16 * (size_t)count);
    if (e == hipSuccess) e = dalloc(c, &small, small_b);
    if (e == hipSuccess) e = stage_h2d(c, dptrs, ptrs.data(), 16 * (size_t)count);
    if (e == hipSuccess)
        e = fhs::launch_encrypt_sym_batch(c->T, sk->key, stream_id(ST_ENC_SYM, ctr0, 0), stream_id(ST_ENC_SYM, ctr0, 1),
                                          step, reinterpret_cast<fhs::u64* const*>(dptrs), sk->s,
                                          pts ? reinterpret_cast<const fhs::u64* const*>(dptrs + count) : nullptr,
                                          count, l, reinterpret_cast<signed char*>(small), eb, c->st, coef);
    if (small) dfree(c, small, small_b);
    if (dptrs) dfree(c, dptrs, 16 * (size_t)count);
    dfree(c, eb, 8 * S * count);
    return bo.keep(e == hipSuccess ? FHS_OK : hip_fail(e, "encrypt"));
}
extern "C" fhs_status fhs_encrypt_symmetric_batch(fhs_context* c, fhs_secret_key* sk, const fhs_plaintext* const* pts,
                                                  int count, fhs_ciphertext** outs) {
    ENTER(c);
    if (!sk || !pts || !outs || count < 0) return fail(FHS_ERR_INVALID, "encrypt_batch: bad arguments");
    for (int i = 0; i < count; ++i)
        if (!pts[i]) return fail(FHS_ERR_INVALID, "encrypt_batch: null plaintext");
    bool same = count > 0;
    for (int i = 1; i < count; ++i) same &= pts[i]->l == pts[0]->l && pts[i]->ci == pts[0]->ci;
    if (!same) {   // mixed levels: one at a time (the same counters in the same order); a failure destroys
                   // the ciphertexts already made, as the batched path does
        BatchOutT<fhs_ciphertext> bo(outs, count);
        for (int i = 0; i < count; ++i) {
            const fhs_status s = fhs_encrypt_symmetric(c, sk, pts[i], &outs[i]);
            if (s != FHS_OK) return s;
        }
        return bo.keep(FHS_OK);
    }
    // chunks of kMaxBatch (grid rows and scratch bound the launch); counters stay consecutive, so the
    // ciphertexts are those of one call per plaintext
    BatchOutT<fhs_ciphertext> bo(outs, count);
    std::vector<double> scales(count);
    for (int i = 0; i < count; ++i) scales[i] = pts[i]->scale;
    for (int i0 = 0; i0 < count; i0 += kMaxBatch) {
        const int n = std::min(kMaxBatch, count - i0);
        const fhs_status s = encrypt_sym_core(c, sk, n, pts[0]->l, pts[0]->ci, scales.data() + i0, pts + i0, nullptr,
                                              outs + i0);
        if (s != FHS_OK) return s;
    }
    return bo.keep(FHS_OK);
}
// Extension (the client's encrypt_replicated of a stage's inputs, bg:53-58 / 124-127, in one pass):
// encode `count` vectors of n values (real, or interleaved re/im) at `scale` and chain index ci and encrypt
// them with sk -- limb for limb fhs_encode[_real]_batch followed by fhs_encrypt_symmetric_batch, without
// the plaintexts: the message's rounded coefficients go into the error's NTT.
extern "C" fhs_status fhs_encode_encrypt_symmetric_batch(fhs_context* c, fhs_secret_key* sk, const double* values,
                                                         size_t count, size_t n, int is_real, double scale, int ci,
                                                         fhs_ciphertext** outs) {
    ENTER(c);
    if (!sk || !outs || (!values && count && n)) return fail(FHS_ERR_INVALID, "encode_encrypt: null argument");
    fhs_status st = encode_checks(c, n, scale, ci);
    if (st != FHS_OK) return st;
    if (count == 0) return FHS_OK;
    if (count > (size_t)kMaxBatch) return fail(FHS_ERR_INVALID, "encode_encrypt: at most 4096 vectors per call");
    const size_t stride = is_real ? n : 2 * n, N = c->N;
    const int l = c->L0 + 1 - ci;
    uint64_t *dvals = nullptr, *coef = nullptr;
    const size_t vb = std::max<size_t>(8, 8 * count * stride), cb = 8 * count * N;
    HIPCHK(dalloc(c, &dvals, vb), "encode_encrypt");
    hipError_t e = dalloc(c, &coef, cb);
    if (e == hipSuccess && stride) e = stage_h2d(c, dvals, values, 8 * count * stride);
    uint64_t* tl = nullptr;   // periodic rows: the sparse encoding, as encode_*_batch gives them
    size_t tbytes = 0;
    if (e == hipSuccess)
        e = enc_periods(c, reinterpret_cast<const double*>(dvals), count, n, stride, is_real != 0, &tl, &tbytes);
    if (e == hipSuccess)
        e = fhs::launch_encode_coef(c->T, reinterpret_cast<const double*>(dvals), (int)count, n, stride, is_real != 0,
                                    scale, reinterpret_cast<double*>(coef), c->st, reinterpret_cast<const unsigned char*>(tl));
    if (tl) dfree(c, tl, tbytes);
    if (e == hipSuccess) {
        std::vector<double> scales(count, scale);
        st = encrypt_sym_core(c, sk, (int)count, l, ci, scales.data(), nullptr, reinterpret_cast<const double*>(coef),
                              outs);
    } else {
        st = hip_fail(e, "encode_encrypt");
    }
    if (coef) dfree(c, coef, cb);
    dfree(c, dvals, vb);
    return st;
}
extern "C" fhs_status fhs_encrypt_asymmetric(fhs_context* c, fhs_public_key* pk, const fhs_plaintext* pt,
                                             fhs_ciphertext** out) {
    ENTER(c);
    if (!pk || !pt || !out) return fail(FHS_ERR_INVALID, "encrypt: null argument");
    const uint64_t ctr = pk->ctr++;
    fhs_ciphertext* ct;
    fhs_status s = new_ct(c, 2, pt->ci, pt->scale, &ct);
    if (s != FHS_OK) return s;
    const int l = pt->l;
    const size_t S = (size_t)l * c->N, SL = (size_t)c->L0 * c->N;
    uint64_t* tmp = nullptr;
    HIPCHK(dalloc(c, &tmp, 24 * S), "encrypt");
    uint64_t *u = tmp, *e0 = tmp + S, *e1 = tmp + 2 * S;
    HIPCHK(sample_small_ntt(c, fhs::SAMPLE_TERNARY, pk->rng, stream_id(ST_ENC_ASYM, ctr, 0), u, l), "encrypt");
    HIPCHK(sample_small_ntt(c, fhs::SAMPLE_CBD, pk->rng, stream_id(ST_ENC_ASYM, ctr, 1), e0, l), "encrypt");
    HIPCHK(sample_small_ntt(c, fhs::SAMPLE_CBD, pk->rng, stream_id(ST_ENC_ASYM, ctr, 2), e1, l), "encrypt");
    PT_DENSE(pd, pt, "encrypt");
    HIPCHK(fhs::launch_encrypt_combine(c->T, 1, ct->d, ct->d + S, pk->pk, pk->pk + SL, u, e0, e1, pd, l, c->st),
           "encrypt");
    dfree(c, tmp, 24 * S);
    *out = ct;
    return FHS_OK;
}
extern "C" fhs_status fhs_decrypt(fhs_context* c, fhs_secret_key* sk, const fhs_ciphertext* ct, fhs_plaintext** out) {
    ENTER(c);
    if (!sk || !ct || !out) return fail(FHS_ERR_INVALID, "decrypt: null argument");
    LIVE(ct);
    fhs_plaintext* pt;
    fhs_status s = new_pt(c, ct->ci, ct->scale, &pt);
    if (s != FHS_OK) return s;
    HIPCHK(fhs::launch_decrypt(c->T, ct->d, ct->ncomp, sk->s, pt->d, ct->l, c->st), "decrypt");
    *out = pt;
    return FHS_OK;
}

// ============================================================================ evaluator
static fhs_status same_level(const fhs_ciphertext* a, const fhs_ciphertext* b) {
    if (a->ci != b->ci) return fail(FHS_ERR_LEVEL, "operands are at different chain indices");
    return FHS_OK;
}
static bool scales_close(double a, double b) { return std::fabs(a - b) <= 1e-9 * std::max(std::fabs(a), std::fabs(b)); }

static fhs_status binop(fhs_context* c, int op, const fhs_ciphertext* a, const fhs_ciphertext* b, fhs_ciphertext** out) {
    if (!a || !b || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    LIVE(b);
    fhs_status s = same_level(a, b);
    if (s != FHS_OK) return s;
    if (a->ncomp != b->ncomp) return fail(FHS_ERR_INVALID, "ciphertext sizes differ");
    if (!scales_close(a->scale, b->scale)) return fail(FHS_ERR_SCALE, "scale mismatch");
    fhs_ciphertext* r;
    s = new_ct(c, a->ncomp, a->ci, a->scale, &r);
    if (s != FHS_OK) return s;
    const size_t cs = (size_t)a->l * c->N;
    HIPCHK(fhs::launch_eltwise(c->T, op, a->d, b->d, r->d, a->ncomp, a->l, cs, cs, c->st), "eltwise");
    *out = r;
    return FHS_OK;
}
extern "C" fhs_status fhs_add(fhs_context* c, const fhs_ciphertext* a, const fhs_ciphertext* b, fhs_ciphertext** out) {
    ENTER(c);
    return binop(c, fhs::OP_ADD, a, b, out);
}
extern "C" fhs_status fhs_sub(fhs_context* c, const fhs_ciphertext* a, const fhs_ciphertext* b, int negate,
                              fhs_ciphertext** out) {
    ENTER(c);
    return binop(c, negate ? fhs::OP_SUBNEG : fhs::OP_SUB, a, b, out);
}
extern "C" fhs_status fhs_negate(fhs_context* c, const fhs_ciphertext* a, fhs_ciphertext** out) {
    ENTER(c);
    if (!a || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    fhs_ciphertext* r;
    fhs_status s = new_ct(c, a->ncomp, a->ci, a->scale, &r);
    if (s != FHS_OK) return s;
    const size_t cs = (size_t)a->l * c->N;
    HIPCHK(fhs::launch_eltwise(c->T, fhs::OP_NEG, a->d, nullptr, r->d, a->ncomp, a->l, cs, 0, c->st), "negate");
    *out = r;
    return FHS_OK;
}
static fhs_status plainop(fhs_context* c, int op, const fhs_ciphertext* a, const fhs_plaintext* p, fhs_ciphertext** out) {
    if (!a || !p || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    if (a->ci != p->ci) return fail(FHS_ERR_LEVEL, "ciphertext and plaintext are at different chain indices");
    const double sc = op == fhs::OP_MULP ? a->scale * p->scale : a->scale;
    if (op != fhs::OP_MULP && !scales_close(a->scale, p->scale)) return fail(FHS_ERR_SCALE, "scale mismatch");
    fhs_ciphertext* r;
    fhs_status s = new_ct(c, a->ncomp, a->ci, sc, &r);
    if (s != FHS_OK) return s;
    const size_t cs = (size_t)a->l * c->N;
    PT_DENSE(pd, p, "plain op");
    HIPCHK(fhs::launch_eltwise(c->T, op, a->d, pd, r->d, a->ncomp, a->l, cs, 0, c->st), "plain op");
    *out = r;
    return FHS_OK;
}
extern "C" fhs_status fhs_add_plain(fhs_context* c, const fhs_ciphertext* a, const fhs_plaintext* p, fhs_ciphertext** out) {
    ENTER(c);
    return plainop(c, fhs::OP_ADDP, a, p, out);
}
extern "C" fhs_status fhs_sub_plain(fhs_context* c, const fhs_ciphertext* a, const fhs_plaintext* p, fhs_ciphertext** out) {
    ENTER(c);
    return plainop(c, fhs::OP_SUBP, a, p, out);
}
extern "C" fhs_status fhs_multiply_plain(fhs_context* c, const fhs_ciphertext* a, const fhs_plaintext* p,
                                         fhs_ciphertext** out) {
    ENTER(c);
    return plainop(c, fhs::OP_MULP, a, p, out);
}
extern "C" fhs_status fhs_multiply(fhs_context* c, const fhs_ciphertext* a, const fhs_ciphertext* b, fhs_ciphertext** out) {
    ENTER(c);
    if (!a || !b || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    LIVE(b);
    fhs_status s = same_level(a, b);
    if (s != FHS_OK) return s;
    if (a->ncomp != 2 || b->ncomp != 2) return fail(FHS_ERR_INVALID, "multiply expects 2-component ciphertexts");
    fhs_ciphertext* r;
    s = new_ct(c, 3, a->ci, a->scale * b->scale, &r);
    if (s != FHS_OK) return s;
    HIPCHK(fhs::launch_tensor(c->T, a->d, b->d, r->d, a->l, c->st), "multiply");
    *out = r;
    return FHS_OK;
}

static fhs_status run_keyswitch(fhs_context* c, std::vector<KsItem>& items, int l) {
    const int R = (int)items.size();
    std::vector<const uint64_t*> uniq;
    for (int r = 0; r < R; ++r) {
        items[r].src = (uint64_t)uniq.size();
        uniq.push_back(items[r].a);
    }
    const size_t wsb = fhs::keyswitch_workspace_bytes(c->T, R, R, l);
    uint64_t* ws = nullptr;
    HIPCHK(scratch(c, fhs_context::SCR_KS, wsb, &ws), "key-switch workspace");
    hipError_t e = fhs::launch_keyswitch(c->T, items.data(), R, reinterpret_cast<const fhs::u64* const*>(uniq.data()), R,
                                         l, ws, wsb, c->items_dev, c->stager, c->st, nullptr);
    if (e != hipSuccess) return hip_fail(e, "key-switch");
    return FHS_OK;
}

extern "C" fhs_status fhs_relinearize(fhs_context* c, const fhs_ciphertext* a, const fhs_relin_key* rk,
                                      fhs_ciphertext** out) {
    ENTER(c);
    if (!a || !rk || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    if (a->ncomp != 3) return fail(FHS_ERR_INVALID, "relinearize expects a 3-component ciphertext");
    fhs_ciphertext* r;
    fhs_status s = new_ct(c, 2, a->ci, a->scale, &r);
    if (s != FHS_OK) return s;
    const size_t S = (size_t)a->l * c->N;
    std::vector<KsItem> it{KsItem{a->d + 2 * S, a->d, a->d + S, rk->key, r->d, r->d + S, 1, 0, key_akey(c, rk->key)}};
    s = run_keyswitch(c, it, a->l);
    if (s != FHS_OK) return s;
    *out = r;
    return FHS_OK;
}

extern "C" fhs_status fhs_rescale_to_next(fhs_context* c, const fhs_ciphertext* a, fhs_ciphertext** out) {
    ENTER(c);
    if (!a || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    if (a->l < 2) return fail(FHS_ERR_LEVEL, "rescale_to_next: no level left (end of modulus switching chain)");
    fhs_ciphertext* r;
    fhs_status s = new_ct(c, a->ncomp, a->ci + 1, a->scale / (double)c->q[a->l - 1], &r);
    if (s != FHS_OK) return s;
    uint64_t* scr = nullptr;
    HIPCHK(scratch(c, fhs_context::SCR_RESCALE, 8ull * a->ncomp * c->N, &scr), "rescale");
    HIPCHK(fhs::launch_rescale(c->T, a->d, r->d, scr, a->ncomp, a->l, c->st), "rescale");
    *out = r;
    return FHS_OK;
}

static fhs_status drop_ct(fhs_context* c, const fhs_ciphertext* a, int ci, fhs_ciphertext** out) {
    LIVE(a);
    if (ci < a->ci) return fail(FHS_ERR_LEVEL, "mod_switch_to: cannot switch to a higher level");
    fhs_ciphertext* r;
    fhs_status s = new_ct(c, a->ncomp, ci, a->scale, &r);
    if (s != FHS_OK) return s;
    const size_t row = 8ull * r->l * c->N, pitch = 8ull * a->l * c->N;
    HIPCHK(hipMemcpy2DAsync(r->d, row, a->d, pitch, row, a->ncomp, hipMemcpyDeviceToDevice, c->st), "mod_switch");
    *out = r;
    return FHS_OK;
}
extern "C" fhs_status fhs_mod_switch_to_next(fhs_context* c, const fhs_ciphertext* a, fhs_ciphertext** out) {
    ENTER(c);
    if (!a || !out) return fail(FHS_ERR_INVALID, "null argument");
    if (a->l < 2) return fail(FHS_ERR_LEVEL, "mod_switch_to_next: end of modulus switching chain");
    return drop_ct(c, a, a->ci + 1, out);
}
extern "C" fhs_status fhs_mod_switch_to(fhs_context* c, const fhs_ciphertext* a, int ci, fhs_ciphertext** out) {
    ENTER(c);
    if (!a || !out) return fail(FHS_ERR_INVALID, "null argument");
    if (ci > c->L0) return fail(FHS_ERR_LEVEL, "mod_switch_to: chain index out of range");
    return drop_ct(c, a, ci, out);
}
static fhs_status drop_pt(fhs_context* c, const fhs_plaintext* a, int ci, fhs_plaintext** out) {
    if (ci < a->ci || ci > c->L0) return fail(FHS_ERR_LEVEL, "mod_switch_to: bad target chain index");
    fhs_plaintext* r;
    fhs_status s = new_pt(c, ci, a->scale, &r);
    if (s != FHS_OK) return s;
    PT_DENSE(pd, a, "mod_switch");
    HIPCHK(hipMemcpyAsync(r->d, pd, pt_bytes(r), hipMemcpyDeviceToDevice, c->st), "mod_switch");
    *out = r;
    return FHS_OK;
}
extern "C" fhs_status fhs_plain_mod_switch_to_next(fhs_context* c, const fhs_plaintext* a, fhs_plaintext** out) {
    ENTER(c);
    if (!a || !out) return fail(FHS_ERR_INVALID, "null argument");
    return drop_pt(c, a, a->ci + 1, out);
}
extern "C" fhs_status fhs_plain_mod_switch_to(fhs_context* c, const fhs_plaintext* a, int ci, fhs_plaintext** out) {
    ENTER(c);
    if (!a || !out) return fail(FHS_ERR_INVALID, "null argument");
    return drop_pt(c, a, ci, out);
}

// rotation: queued, flushed as one batched key-switch (see file header)
static fhs_status queue_rotation(fhs_context* c, const fhs_ciphertext* a, uint64_t elt, const fhs_galois_keys* gk,
                                 fhs_ciphertext** out) {
    if (!a || !gk || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    if (a->ncomp != 2) return fail(FHS_ERR_INVALID, "rotate expects a 2-component ciphertext");
    auto it = gk->keys.find(elt);
    if (it == gk->keys.end()) return fail(FHS_ERR_KEY, "galois key for this rotation step is not present");
    if (!c->pending.empty() && (c->pending_l != a->l || (int)c->pending.size() >= fhs_context::kMaxItems ||
                                c->pending_outs.count(a))) {
        fhs_status s = flush(c);
        if (s != FHS_OK) return s;
    }
    fhs_ciphertext* r;
    fhs_status s = new_ct(c, 2, a->ci, a->scale, &r);
    if (s != FHS_OK) return s;
    const size_t S = (size_t)a->l * c->N;
    c->pending.push_back(PendingRot{KsItem{a->d + S, a->d, nullptr, it->second, r->d, r->d + S, elt, 0,
                                           key_akey(c, it->second)}, r, a});
    c->pending_l = a->l;
    c->pending_refs.insert(r);
    c->pending_refs.insert(a);
    c->pending_outs.insert(r);
    *out = r;
    return FHS_OK;
}
extern "C" fhs_status fhs_rotate(fhs_context* c, const fhs_ciphertext* a, int step, const fhs_galois_keys* gk,
                                 fhs_ciphertext** out) {
    if (!c) return fail(FHS_ERR_INVALID, "null context");
    Guard g(c);
    if (step == 0 || std::abs(step) >= (int)(c->N / 2)) {
        if (step == 0) return fail(FHS_ERR_INVALID, "rotate: step 0 (use apply_galois for conjugation)");
        return fail(FHS_ERR_INVALID, "rotate: |step| must be < slot count");
    }
    return queue_rotation(c, a, fhs_galois_elt_from_step(step, c->N), gk, out);
}
extern "C" fhs_status fhs_apply_galois(fhs_context* c, const fhs_ciphertext* a, uint64_t elt, const fhs_galois_keys* gk,
                                       fhs_ciphertext** out) {
    if (!c) return fail(FHS_ERR_INVALID, "null context");
    Guard g(c);
    return queue_rotation(c, a, elt, gk, out);
}
extern "C" fhs_status fhs_rotate_many(fhs_context* c, const fhs_ciphertext* const* in, const int* steps, int n,
                                      const fhs_galois_keys* gk, fhs_ciphertext** out) {
    if (!c) return fail(FHS_ERR_INVALID, "null context");
    Guard g(c);
    for (int i = 0; i < n; ++i) {
        fhs_status s = queue_rotation(c, in[i], fhs_galois_elt_from_step(steps[i], c->N), gk, &out[i]);
        if (s != FHS_OK) return s;
    }
    return flush(c);
}

// ============================================================================ fused BSGS
// giant_elts: null = 5^(g G) (the matvec, bg:478-483); else B Galois elements, giant_elts[0] = 1.
// rescale = false leaves the sum at the product scale (last SlotToCoeff group of the bootstrap).
// ptl > 0: pt_ptrs are the diagonals' compact shadows (pts_ptl)
static fhs_status bsgs_core(fhs_context* c, const fhs_ciphertext* const* baby, int G, const uint64_t* const* pt_ptrs,
                            int D, int B, int ci, double pt_scale, const fhs_galois_keys* gk, fhs_ciphertext** out,
                            const uint64_t* giant_elts = nullptr, bool rescale = true, int ptl = 0) {
    if (G < 1 || D < 1 || !baby) return fail(FHS_ERR_INVALID, "bsgs: bad G/D");
    const int Beff = std::min(B, (D + G - 1) / G);
    if (Beff < 1) return fail(FHS_ERR_INVALID, "bsgs: no giant groups");
    if (G > 2048 || (size_t)D + G > (size_t)fhs_context::kMaxPtrs) return fail(FHS_ERR_INVALID, "bsgs: too many diagonals");
    const int l = baby[0]->l;
    for (int b = 0; b < G; ++b) {
        if (!baby[b] || baby[b]->l != l || baby[b]->ncomp != 2 || baby[b]->ci != ci)
            return fail(FHS_ERR_LEVEL, "bsgs: baby steps and diagonals must share one chain index");
        LIVE(baby[b]);
    }
    if (rescale && l < 2) return fail(FHS_ERR_LEVEL, "bsgs: no level left for the final rescale");
    if (giant_elts && giant_elts[0] != 1) return fail(FHS_ERR_INVALID, "linear_transform: giant group 0 must be the identity");
    HostTrace ht;
    std::vector<const uint64_t*> keys(Beff, nullptr), akeys(Beff, nullptr);
    for (int g = 1; g < Beff; ++g) {
        const uint64_t elt = giant_elts ? giant_elts[g] : fhs_galois_elt_from_step(g * G, c->N);
        auto it = gk->keys.find(elt);
        if (it == gk->keys.end()) return fail(FHS_ERR_KEY, "bsgs: galois key for a giant step is missing");
        keys[g] = it->second;
        akeys[g] = key_akey(c, it->second);
    }
    const size_t S = (size_t)l * c->N;
    // pointer arrays -> device
    std::vector<const uint64_t*> ptrs(G + D);
    for (int b = 0; b < G; ++b) ptrs[b] = baby[b]->d;
    for (int k = 0; k < D; ++k) ptrs[G + k] = pt_ptrs[k];
    ht.mark("keys+ptrs");
    HIPCHK(stage_h2d(c, c->ptrs_dev, ptrs.data(), sizeof(void*) * (G + D)), "bsgs");
    ht.mark("stage ptrs");
    const uint64_t* const* dbaby = reinterpret_cast<const uint64_t* const*>(c->ptrs_dev);
    const uint64_t* const* dpts = dbaby + G;
    uint64_t* inner = nullptr;
    HIPCHK(scratch(c, fhs_context::SCR_BSGS_INNER, 8ull * Beff * 2 * S, &inner), "bsgs inner products");
    const fhs::KTimer* tm = c->timer_mask ? &c->ktimer : nullptr;
    const size_t wsb = std::max<size_t>(8, fhs::bsgs_workspace_bytes(c->T, Beff - 1, l));
    uint64_t* ws = nullptr;
    HIPCHK(scratch(c, fhs_context::SCR_BSGS_WS, wsb, &ws), "bsgs workspace");
    uint64_t* sum = nullptr;
    HIPCHK(scratch(c, fhs_context::SCR_BSGS_SUM, 16 * S, &sum), "bsgs sum");
    ht.mark("workspaces");
    HIPCHK(fhs::launch_bsgs(c->T, dbaby, dpts, G, Beff, D, l, keys.data(), akeys.data(), giant_elts, inner, sum, ws, wsb,
                            c->items_dev, c->stager, c->st, tm, ptl),
           "bsgs");
    ht.mark("launch bsgs");
    fhs_ciphertext* r;
    if (!rescale) {
        fhs_status s = new_ct(c, 2, ci, baby[0]->scale * pt_scale, &r);
        if (s != FHS_OK) return s;
        HIPCHK(hipMemcpyAsync(r->d, sum, 8 * 2 * S, hipMemcpyDeviceToDevice, c->st), "linear_transform");
        *out = r;
        return FHS_OK;
    }
    fhs_status s = new_ct(c, 2, ci + 1, baby[0]->scale * pt_scale / (double)c->q[l - 1], &r);
    if (s != FHS_OK) return s;
    uint64_t* scr = nullptr;
    HIPCHK(scratch(c, fhs_context::SCR_RESCALE, 16ull * c->N, &scr), "bsgs rescale");
    HIPCHK(fhs::launch_rescale(c->T, sum, r->d, scr, 2, l, c->st, tm), "bsgs rescale");
    ht.mark("rescale+frees");
    *out = r;
    return FHS_OK;
}

// The Hadamard reads the diagonals' compact shadows when every one has one at the same tlog (encode_rows_dev; the
// same products, 2^-tlog of the bytes), else the dense limbs.  FHESPEAR_BSGS_DENSE=1 always reads the dense limbs.
static int pts_ptl(const fhs_context* c, const fhs_plaintext* const* pts, int D) {
    static const bool dense = getenv("FHESPEAR_BSGS_DENSE") != nullptr;
    if (dense || D < 1 || c->T.max_qbits > 59 || !pts[0]->dc) return 0;
    for (int k = 1; k < D; ++k)
        if (!pts[k]->dc || pts[k]->tlog != pts[0]->tlog) return 0;
    return pts[0]->tlog;
}
extern "C" fhs_status fhs_bsgs_multiply_accumulate(fhs_context* c, const fhs_ciphertext* const* baby, int G,
                                                   const fhs_plaintext* const* pts, int D, int B,
                                                   const fhs_galois_keys* gk, fhs_ciphertext** out) {
    ENTER(c);
    if (!pts || !gk || !out || !baby) return fail(FHS_ERR_INVALID, "null argument");
    std::vector<const uint64_t*> p(D);
    for (int k = 0; k < D; ++k) {
        if (!pts[k] || pts[k]->ci != baby[0]->ci) return fail(FHS_ERR_LEVEL, "bsgs: diagonal at a different chain index");
        if (!scales_close(pts[k]->scale, pts[0]->scale)) return fail(FHS_ERR_SCALE, "bsgs: diagonal scales differ");
    }
    const int ptl = pts_ptl(c, pts, D);
    for (int k = 0; k < D; ++k) {
        p[k] = pts[k]->dc;
        if (!ptl) HIPCHK(pt_dense(c, pts[k], &p[k]), "bsgs");
    }
    return bsgs_core(c, baby, G, p.data(), D, B, baby[0]->ci, pts[0]->scale, gk, out, nullptr, true, ptl);
}

// The Hadamard half of the fused BSGS alone: outs[g] = sum_{b < G} baby[b] (.) pts[g G + b], g < B, not
// rescaled (scale baby * pt).  Used by the baby-step-sharded latency mode (fhespear_dist.bsgs_baby_sharded):
// a rank holding baby steps b in its share forms every giant group's partial inner product.
// inner products of the B groups into dst ([g][2][l][N] words, device memory), stream-ordered
static fhs_status inner_products_core(fhs_context* c, const fhs_ciphertext* const* baby, int G,
                                      const fhs_plaintext* const* pts, int B, uint64_t* dst) {
    if (G < 1 || G > 2048 || B < 1) return fail(FHS_ERR_INVALID, "bsgs_inner_products: 1 <= G <= 2048, B >= 1");
    const int D = B * G, ci = baby[0]->ci, l = baby[0]->l;
    if ((size_t)D + G > (size_t)fhs_context::kMaxPtrs) return fail(FHS_ERR_INVALID, "bsgs_inner_products: too many plaintexts");
    std::vector<const uint64_t*> ptrs(G + D);
    for (int b = 0; b < G; ++b) {
        if (!baby[b] || baby[b]->l != l || baby[b]->ncomp != 2 || baby[b]->ci != ci)
            return fail(FHS_ERR_LEVEL, "bsgs_inner_products: baby steps must share one chain index");
        LIVE(baby[b]);
        ptrs[b] = baby[b]->d;
    }
    for (int k = 0; k < D; ++k) {
        if (!pts[k] || pts[k]->ci != ci) return fail(FHS_ERR_LEVEL, "bsgs_inner_products: plaintext at a different chain index");
        if (!scales_close(pts[k]->scale, pts[0]->scale)) return fail(FHS_ERR_SCALE, "bsgs_inner_products: plaintext scales differ");
    }
    const int ptl = pts_ptl(c, pts, D);
    for (int k = 0; k < D; ++k) {
        ptrs[G + k] = pts[k]->dc;
        if (!ptl) HIPCHK(pt_dense(c, pts[k], &ptrs[G + k]), "bsgs_inner_products");
    }
    HIPCHK(stage_h2d(c, c->ptrs_dev, ptrs.data(), sizeof(void*) * (G + D)), "bsgs_inner_products");
    const uint64_t* const* dbaby = reinterpret_cast<const uint64_t* const*>(c->ptrs_dev);
    HIPCHK(fhs::launch_bsgs_inner(c->T, dbaby, dbaby + G, G, 0, B, D, l, dst, c->st, ptl), "bsgs_inner_products");
    return FHS_OK;
}
extern "C" fhs_status fhs_bsgs_inner_products(fhs_context* c, const fhs_ciphertext* const* baby, int G,
                                              const fhs_plaintext* const* pts, int B, fhs_ciphertext** outs) {
    ENTER(c);
    if (!pts || !outs || !baby || !baby[0]) return fail(FHS_ERR_INVALID, "null argument");
    const int ci = baby[0]->ci;
    const size_t S = (size_t)baby[0]->l * c->N;
    uint64_t* inner = nullptr;
    HIPCHK(scratch(c, fhs_context::SCR_BSGS_INNER, 8ull * std::max(B, 1) * 2 * S, &inner), "bsgs_inner_products");
    fhs_status cs = inner_products_core(c, baby, G, pts, B, inner);
    if (cs != FHS_OK) return cs;
    std::vector<fhs_ciphertext*> made;
    for (int g = 0; g < B; ++g) {
        fhs_ciphertext* r;
        fhs_status st = new_ct(c, 2, ci, baby[0]->scale * pts[0]->scale, &r);
        if (st == FHS_OK && hipMemcpyAsync(r->d, inner + (size_t)g * 2 * S, 16 * S, hipMemcpyDeviceToDevice, c->st) != hipSuccess)
            st = fail(FHS_ERR_HIP, "bsgs_inner_products: copy");
        if (st != FHS_OK) {
            for (fhs_ciphertext* m : made) fhs_ciphertext_destroy(m);
            return st;
        }
        made.push_back(r);
        outs[g] = r;
    }
    return FHS_OK;
}

// fhs_bsgs_inner_products into caller device memory (e.g. a torch buffer that a reduce-scatter then
// sums): group g at dst + g 2 l N words, ordered on the context stream (fhs_context_stream).
extern "C" fhs_status fhs_bsgs_inner_products_device(fhs_context* c, const fhs_ciphertext* const* baby, int G,
                                                     const fhs_plaintext* const* pts, int B, uint64_t* dst) {
    ENTER(c);
    if (!pts || !dst || !baby || !baby[0]) return fail(FHS_ERR_INVALID, "null argument");
    return inner_products_core(c, baby, G, pts, B, dst);
}

// The giant-step half of the fused BSGS alone: out = sum_j rot_{elts[j]}(inners[j]), every rotation's
// key switch summed before one ModDown (k_giant_sum / k_giant_final), not rescaled.  elts[0] may be 1
// (an unrotated term); otherwise a zero term takes group 0's place.  The baby-step-sharded latency mode
// (fhespear_dist.bsgs_baby_sharded) finishes a rank's giant groups with it.
// src(j): device address of term j's 2 l N words
template <class Src>
static fhs_status giant_steps_core(fhs_context* c, Src src, int k, int ci, double scale, const uint64_t* elts,
                                   const fhs_galois_keys* gk, fhs_ciphertext** out) {
    const int l = c->L0 + 1 - ci;
    for (int j = 0; j < k; ++j) {
        if ((elts[j] & 1) == 0 || elts[j] >= 2 * c->N) return fail(FHS_ERR_INVALID, "bsgs_giant_steps: bad Galois element");
        if (j > 0 && elts[j] == 1) return fail(FHS_ERR_INVALID, "bsgs_giant_steps: only the first term may be unrotated");
    }
    const int pad = elts[0] == 1 ? 0 : 1, B = k + pad;   // group 0 = the unrotated term (or zero)
    std::vector<uint64_t> ge(B, 1);
    std::vector<const uint64_t*> keys(B, nullptr), akeys(B, nullptr);
    for (int g = 1; g < B; ++g) {
        ge[g] = elts[g - pad];
        auto it = gk->keys.find(ge[g]);
        if (it == gk->keys.end()) return fail(FHS_ERR_KEY, "bsgs_giant_steps: galois key missing");
        keys[g] = it->second;
        akeys[g] = key_akey(c, it->second);
    }
    const size_t S = (size_t)l * c->N;
    uint64_t *inner = nullptr, *ws = nullptr, *sum = nullptr;
    HIPCHK(scratch(c, fhs_context::SCR_BSGS_INNER, 8ull * B * 2 * S, &inner), "bsgs_giant_steps");
    if (pad) HIPCHK(hipMemsetAsync(inner, 0, 16 * S, c->st), "bsgs_giant_steps");
    for (int j = 0; j < k; ++j)
        HIPCHK(hipMemcpyAsync(inner + (size_t)(j + pad) * 2 * S, src(j), 16 * S, hipMemcpyDeviceToDevice, c->st),
               "bsgs_giant_steps");
    const size_t wsb = std::max<size_t>(8, fhs::bsgs_workspace_bytes(c->T, B - 1, l));
    HIPCHK(scratch(c, fhs_context::SCR_BSGS_WS, wsb, &ws), "bsgs_giant_steps");
    HIPCHK(scratch(c, fhs_context::SCR_BSGS_SUM, 16 * S, &sum), "bsgs_giant_steps");
    const fhs::KTimer* tm = c->timer_mask ? &c->ktimer : nullptr;
    HIPCHK(fhs::launch_bsgs(c->T, nullptr, nullptr, 1, B, B, l, keys.data(), akeys.data(), ge.data(), inner, sum, ws, wsb,
                            c->items_dev, c->stager, c->st, tm),
           "bsgs_giant_steps");
    fhs_ciphertext* r;
    fhs_status s = new_ct(c, 2, ci, scale, &r);
    if (s != FHS_OK) return s;
    HIPCHK(hipMemcpyAsync(r->d, sum, 16 * S, hipMemcpyDeviceToDevice, c->st), "bsgs_giant_steps");
    *out = r;
    return FHS_OK;
}
extern "C" fhs_status fhs_bsgs_giant_steps(fhs_context* c, const fhs_ciphertext* const* inners, int k,
                                           const uint64_t* elts, const fhs_galois_keys* gk, fhs_ciphertext** out) {
    ENTER(c);
    if (!inners || !elts || !gk || !out || k < 1 || !inners[0]) return fail(FHS_ERR_INVALID, "null argument");
    if (k > 511) return fail(FHS_ERR_INVALID, "bsgs_giant_steps: 1 <= k <= 511");
    const int l = inners[0]->l, ci = inners[0]->ci;
    for (int j = 0; j < k; ++j) {
        if (!inners[j] || inners[j]->ncomp != 2 || inners[j]->l != l || inners[j]->ci != ci)
            return fail(FHS_ERR_LEVEL, "bsgs_giant_steps: inner products must be 2-component at one chain index");
        LIVE(inners[j]);
        if (!scales_close(inners[j]->scale, inners[0]->scale)) return fail(FHS_ERR_SCALE, "bsgs_giant_steps: scales differ");
    }
    return giant_steps_core(c, [&](int j) { return inners[j]->d; }, k, ci, inners[0]->scale, elts, gk, out);
}
// the same over k terms laid out contiguously in caller device memory (term j at src + j 2 l N words,
// l = L0 + 1 - chain_index), e.g. the slice a reduce-scatter handed this rank
extern "C" fhs_status fhs_bsgs_giant_steps_device(fhs_context* c, const uint64_t* src, int k, int chain_index,
                                                  double scale, const uint64_t* elts, const fhs_galois_keys* gk,
                                                  fhs_ciphertext** out) {
    ENTER(c);
    if (!src || !elts || !gk || !out) return fail(FHS_ERR_INVALID, "null argument");
    if (k < 1 || k > 511) return fail(FHS_ERR_INVALID, "bsgs_giant_steps: 1 <= k <= 511");
    if (chain_index < 1 || chain_index > c->L0) return fail(FHS_ERR_LEVEL, "bsgs_giant_steps: bad chain index");
    const size_t W = 2 * (size_t)(c->L0 + 1 - chain_index) * c->N;
    return giant_steps_core(c, [&](int j) { return src + (size_t)j * W; }, k, chain_index, scale, elts, gk, out);
}

extern "C" fhs_status fhs_linear_transform(fhs_context* c, const fhs_ciphertext* const* baby, int G,
                                           const fhs_plaintext* const* pts, int D, int B, const uint64_t* giant_elts,
                                           const fhs_galois_keys* gk, int rescale, fhs_ciphertext** out) {
    ENTER(c);
    if (!pts || !gk || !out || !baby || !giant_elts) return fail(FHS_ERR_INVALID, "null argument");
    if (B < 1 || D != B * G) return fail(FHS_ERR_INVALID, "linear_transform: expects D = B * G plaintexts");
    std::vector<const uint64_t*> p(D);
    for (int k = 0; k < D; ++k) {
        if (!pts[k] || pts[k]->ci != baby[0]->ci) return fail(FHS_ERR_LEVEL, "linear_transform: plaintext at a different chain index");
        if (!scales_close(pts[k]->scale, pts[0]->scale)) return fail(FHS_ERR_SCALE, "linear_transform: plaintext scales differ");
    }
    const int ptl = pts_ptl(c, pts, D);
    for (int k = 0; k < D; ++k) {
        p[k] = pts[k]->dc;
        if (!ptl) HIPCHK(pt_dense(c, pts[k], &p[k]), "linear_transform");
    }
    for (int g = 0; g < B; ++g)
        if ((giant_elts[g] & 1) == 0 || giant_elts[g] >= 2 * c->N) return fail(FHS_ERR_INVALID, "linear_transform: bad Galois element");
    return bsgs_core(c, baby, G, p.data(), D, B, baby[0]->ci, pts[0]->scale, gk, out, giant_elts, rescale != 0, ptl);
}

// ============================================================================ bootstrapping primitives
// exact residue of the integer-valued double p modulo q
static uint64_t dbl_int_mod(double p, uint64_t q) {
    const bool neg = p < 0;
    const double a = std::fabs(p);
    uint64_t r;
    if (a < 18446744073709551616.0) {
        r = (uint64_t)a % q;
    } else {
        int e;
        const double f = std::frexp(a, &e);              // a = f 2^e, f in [0.5, 1)
        const uint64_t m = (uint64_t)std::ldexp(f, 53);  // exact 53-bit mantissa
        r = h_mulmod(m % q, h_pow(2, (uint64_t)(e - 53), q), q);
    }
    return neg && r ? q - r : r;
}
static fhs_status scalar_consts(fhs_context* c, double v, int l, fhs::ScalarConsts& K) {
    if (!std::isfinite(v)) return fail(FHS_ERR_INVALID, "constant is not finite");
    if (l > fhs::kMaxScalarLimbs) return fail(FHS_ERR_INVALID, "too many limbs for a constant op");
    const double p = std::round(v);                      // half away from zero
    for (int i = 0; i < l; ++i) {
        K.v[i] = dbl_int_mod(p, c->q[i]);
        K.vs[i] = h_shoup(K.v[i], c->q[i]);
    }
    return FHS_OK;
}
extern "C" fhs_status fhs_multiply_const(fhs_context* c, const fhs_ciphertext* a, double value, double const_scale,
                                         fhs_ciphertext** out) {
    ENTER(c);
    if (!a || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    if (!(const_scale > 0) || !std::isfinite(const_scale)) return fail(FHS_ERR_INVALID, "multiply_const: bad scale");
    fhs::ScalarConsts K;
    fhs_status s = scalar_consts(c, value * const_scale, a->l, K);
    if (s != FHS_OK) return s;
    fhs_ciphertext* r;
    s = new_ct(c, a->ncomp, a->ci, a->scale * const_scale, &r);
    if (s != FHS_OK) return s;
    HIPCHK(fhs::launch_scalar(c->T, fhs::SCALAR_MUL, a->d, r->d, a->ncomp, a->l, K, c->st), "multiply_const");
    *out = r;
    return FHS_OK;
}
extern "C" fhs_status fhs_add_const(fhs_context* c, const fhs_ciphertext* a, double value, fhs_ciphertext** out) {
    ENTER(c);
    if (!a || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    fhs::ScalarConsts K;
    fhs_status s = scalar_consts(c, value * a->scale, a->l, K);
    if (s != FHS_OK) return s;
    fhs_ciphertext* r;
    s = new_ct(c, a->ncomp, a->ci, a->scale, &r);
    if (s != FHS_OK) return s;
    HIPCHK(fhs::launch_scalar(c->T, fhs::SCALAR_ADD, a->d, r->d, a->ncomp, a->l, K, c->st), "add_const");
    *out = r;
    return FHS_OK;
}
extern "C" fhs_status fhs_mod_raise(fhs_context* c, const fhs_ciphertext* a, fhs_ciphertext** out) {
    ENTER(c);
    if (!a || !out) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(a);
    if (a->ncomp != 2) return fail(FHS_ERR_INVALID, "mod_raise expects a 2-component ciphertext");
    fhs_ciphertext* r;
    fhs_status s = new_ct(c, 2, 1, a->scale, &r);
    if (s != FHS_OK) return s;
    uint64_t* scr = nullptr;
    HIPCHK(scratch(c, fhs_context::SCR_RESCALE, 16ull * c->N, &scr), "mod_raise");
    HIPCHK(fhs::launch_mod_raise(c->T, a->d, a->l, r->d, scr, 2, c->st), "mod_raise");
    *out = r;
    return FHS_OK;
}

// ---- EvalMod orchestration in C++ (ckks_bootstrapper._evalmod, pyPhantom/bootstrap.py).  The same
// op sequence as the Python restatement (which the oracle runs): ~300 small ops per EvalMod, whose
// per-call Python overhead dominated the bootstrap.  Every double expression mirrors the Python one
// (same IEEE operations in the same order), so the limbs are identical.
namespace {
struct Ct {   // owning ciphertext handle
    fhs_ciphertext* p = nullptr;
    Ct() = default;
    explicit Ct(fhs_ciphertext* x) : p(x) {}
    Ct(const Ct&) = delete;
    Ct& operator=(const Ct&) = delete;
    Ct(Ct&& o) noexcept : p(o.p) { o.p = nullptr; }
    Ct& operator=(Ct&& o) noexcept {
        if (this != &o) {
            reset();
            p = o.p;
            o.p = nullptr;
        }
        return *this;
    }
    ~Ct() { reset(); }
    void reset() {
        if (p) fhs_ciphertext_destroy(p);
        p = nullptr;
    }
    fhs_ciphertext* release() {
        fhs_ciphertext* x = p;
        p = nullptr;
        return x;
    }
};
struct EmErr {
    fhs_status s;
};
inline void em_try(fhs_status s) {
    if (s != FHS_OK) throw EmErr{s};
}

struct EvalMod {
    fhs_context* c;
    const fhs_relin_key* rk;
    std::map<int, Ct> own;   // T_k computed here (T_1 is borrowed)
    std::map<int, const fhs_ciphertext*> T;

    double q_drop(int ci) const { return (double)c->q[c->L0 - ci]; }   // Bootstrapper._q_drop
    Ct mod_switch(const fhs_ciphertext* a, int ci) {
        fhs_ciphertext* r;
        em_try(fhs_mod_switch_to(c, a, ci, &r));
        return Ct(r);
    }
    Ct mul(const fhs_ciphertext* a, const fhs_ciphertext* b) {   // Bootstrapper._mul
        const int ci = std::max(a->ci, b->ci);
        Ct ta, tb;
        if (a->ci < ci) {
            ta = mod_switch(a, ci);
            a = ta.p;
        }
        if (b->ci < ci) {
            tb = mod_switch(b, ci);
            b = tb.p;
        }
        fhs_ciphertext *m, *r, *s;
        em_try(fhs_multiply(c, a, b, &m));
        Ct M(m);
        em_try(fhs_relinearize(c, M.p, rk, &r));
        Ct R(r);
        em_try(fhs_rescale_to_next(c, R.p, &s));
        return Ct(s);
    }
    Ct add(const fhs_ciphertext* a, const fhs_ciphertext* b) {
        fhs_ciphertext* r;
        em_try(fhs_add(c, a, b, &r));
        return Ct(r);
    }
    Ct sub(const fhs_ciphertext* a, const fhs_ciphertext* b) {
        fhs_ciphertext* r;
        em_try(fhs_sub(c, a, b, 0, &r));
        return Ct(r);
    }
    Ct add_const(const fhs_ciphertext* a, double v) {
        fhs_ciphertext* r;
        em_try(fhs_add_const(c, a, v, &r));
        return Ct(r);
    }
    // value * a landing exactly at (ci, scale): Bootstrapper._scalar
    Ct scalar(const fhs_ciphertext* a, double value, int ci, double scale) {
        if (a->ci > ci - 1) throw EmErr{fail(FHS_ERR_LEVEL, "evalmod: scalar product target level too low")};
        Ct t;
        if (a->ci < ci - 1) {
            t = mod_switch(a, ci - 1);
            a = t.p;
        }
        fhs_ciphertext *m, *r;
        em_try(fhs_multiply_const(c, a, value, scale * q_drop(ci - 1) / a->scale, &m));
        Ct M(m);
        em_try(fhs_rescale_to_next(c, M.p, &r));
        r->scale = scale;
        return Ct(r);
    }
    // Bootstrapper._align: borrowed when already there, else a scalar product by 1.0
    const fhs_ciphertext* align(const fhs_ciphertext* a, int ci, double scale, Ct& hold) {
        if (a->ci == ci && std::fabs(a->scale - scale) <= 1e-9 * scale) return a;
        hold = scalar(a, 1.0, ci, scale);
        return hold.p;
    }
    static int bitlen(int k) {
        int b = 0;
        while (k >> b) ++b;
        return b;
    }
    const fhs_ciphertext* get(int k) {   // Bootstrapper._cheb_basis.get
        auto it = T.find(k);
        if (it != T.end()) return it->second;
        const int a = (k & (k - 1)) ? 1 << (bitlen(k) - 1) : k / 2, b = k - a;
        Ct out;
        if (a == b) {
            const fhs_ciphertext* ta = get(a);
            Ct P = mul(ta, ta);
            Ct P2 = add(P.p, P.p);
            out = add_const(P2.p, -1.0);
        } else {
            const fhs_ciphertext* ta = get(a);
            const fhs_ciphertext* tb = get(b);
            Ct P = mul(ta, tb);
            Ct P2 = add(P.p, P.p);
            Ct hold;
            const fhs_ciphertext* d = align(get(a - b), P2.p->ci, P2.p->scale, hold);
            out = sub(P2.p, d);
        }
        const fhs_ciphertext* r = out.p;
        own[k] = std::move(out);
        T[k] = r;
        return r;
    }
    // Bootstrapper._cheb_eval: sum_k c_k T_k landing exactly at (ci, scale)
    Ct cheb(std::vector<double> cf, int ci, double scale) {
        int deg = (int)cf.size() - 1;
        while (deg > 0 && cf[deg] == 0.0) --deg;
        if (deg < 8) {
            std::vector<int> ks;
            for (int k = 1; k <= deg; ++k)
                if (cf[k] != 0.0) ks.push_back(k);
            if (ks.empty()) ks.push_back(1);
            Ct acc;
            for (int k : ks) {
                Ct t = scalar(get(k), k <= deg ? cf[k] : 0.0, ci, scale);
                acc = acc.p ? add(acc.p, t.p) : std::move(t);
            }
            return cf[0] != 0.0 ? add_const(acc.p, cf[0]) : std::move(acc);
        }
        const int m = 1 << (bitlen(deg) - 1);
        // cheb_split: T_{m+j} = 2 T_m T_j - T_{m-j} (j >= 1), T_m = T_m T_0
        std::vector<double> c2(cf.begin(), cf.begin() + deg + 1);
        c2.resize(2 * m, 0.0);
        std::vector<double> H(m), L(c2.begin(), c2.begin() + m);
        H[0] = c2[m];
        for (int j = 1; j < m; ++j) H[j] = 2.0 * c2[m + j];
        for (int j = 1; j < m; ++j) L[m - j] -= c2[m + j];
        const fhs_ciphertext* Tm = get(m);
        Ct h = cheb(H, ci - 1, scale * q_drop(ci - 1) / Tm->scale);
        Ct P = mul(h.p, Tm);
        P.p->scale = scale;
        Ct Lc = cheb(L, ci, scale);
        return add(P.p, Lc.p);
    }
};
}  // namespace

extern "C" fhs_status fhs_bootstrap_evalmod(fhs_context* c, const fhs_ciphertext* y, const fhs_relin_key* rk,
                                            const double* cc, const double* cs, int ncoef, int r, int cheb_depth,
                                            fhs_ciphertext** out) {
    ENTER(c);
    if (!y || !rk || !cc || !cs || !out || ncoef < 1 || r < 1) return fail(FHS_ERR_INVALID, "evalmod: bad argument");
    LIVE(y);
    try {
        EvalMod e{c, rk, {}, {}};
        e.T[1] = y;
        for (int k : {2, 3, 4, 5, 6, 7, 8, 16, 32}) e.get(k);
        const int ci = y->ci + cheb_depth;
        Ct cv = e.cheb(std::vector<double>(cc, cc + ncoef), ci, y->scale);
        Ct sv = e.cheb(std::vector<double>(cs, cs + ncoef), ci, y->scale);
        for (int step = 0; step < r; ++step) {   // (c, s) -> ((c + s)(c - s), 2 c s)
            Ct P = e.mul(cv.p, sv.p);
            if (step < r - 1) {
                Ct a = e.add(cv.p, sv.p), b = e.sub(cv.p, sv.p);
                cv = e.mul(a.p, b.p);
            }
            sv = e.add(P.p, P.p);
        }
        *out = sv.release();
        return FHS_OK;
    } catch (const EmErr& err) {
        return err.s;
    }
}

extern "C" fhs_status fhs_host_alloc(uint64_t bytes, void** ptr) {
    if (!ptr) return fail(FHS_ERR_INVALID, "null argument");
    HIPCHK(hipHostMalloc(ptr, bytes ? bytes : 8, hipHostMallocDefault), "pinned host allocation");
    return FHS_OK;
}
extern "C" fhs_status fhs_host_free(void* ptr) {
    if (ptr) HIPCHK(hipHostFree(ptr), "pinned host free");
    return FHS_OK;
}
extern "C" fhs_status fhs_offload_plaintexts(fhs_context* c, const fhs_plaintext* const* pts, int count, uint64_t* host) {
    ENTER(c);
    if (!pts || !host || count < 1) return fail(FHS_ERR_INVALID, "offload: bad args");
    const size_t b = pt_bytes(pts[0]);
    for (int k = 0; k < count; ++k) {
        if (pts[k]->l != pts[0]->l) return fail(FHS_ERR_LEVEL, "offload: plaintexts at different levels");
        PT_DENSE(pd, pts[k], "offload");
        HIPCHK(hipMemcpyAsync((char*)host + (size_t)k * b, pd, b, hipMemcpyDeviceToHost, c->st), "offload");
    }
    HIPCHK(hipStreamSynchronize(c->st), "offload");
    return FHS_OK;
}
extern "C" fhs_status fhs_upload_plaintexts(fhs_context* c, const uint64_t* host, int count, int ci, double scale,
                                            fhs_plaintext** outs) {
    ENTER(c);
    if (!host || !outs || count < 1) return fail(FHS_ERR_INVALID, "upload: bad args");
    BatchOut bo(outs, (size_t)count);
    fhs_status s0 = new_pts(c, (size_t)count, ci, scale, outs);
    if (s0 != FHS_OK) return s0;
    for (int k = 0; k < count; ++k) {
        fhs_plaintext* pt = outs[k];
        HIPCHK(hipMemcpyAsync(pt->d, host + (size_t)k * pt->l * c->N, pt_bytes(pt), hipMemcpyHostToDevice, c->st), "upload");
    }
    HIPCHK(hipStreamSynchronize(c->st), "upload");
    return bo.keep(FHS_OK);
}
extern "C" fhs_status fhs_bsgs_from_cpu(fhs_context* c, const fhs_ciphertext* const* baby, int G, const uint64_t* host,
                                        int D, int B, int ci, double scale, const fhs_galois_keys* gk,
                                        fhs_ciphertext** out) {
    ENTER(c);
    if (!baby || !host || !gk || !out) return fail(FHS_ERR_INVALID, "null argument");
    if (ci != baby[0]->ci) return fail(FHS_ERR_LEVEL, "bsgs_from_cpu: diagonals at a different chain index");
    for (int b = 0; b < G; ++b) LIVE(baby[b]);
    const int l = c->L0 + 1 - ci;
    const size_t bytes = 8ull * D * l * c->N;
    uint64_t* dev = nullptr;
    HIPCHK(dalloc(c, &dev, bytes), "bsgs_from_cpu staging");
    HIPCHK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, c->st), "bsgs_from_cpu upload");
    std::vector<const uint64_t*> p(D);
    for (int k = 0; k < D; ++k) p[k] = dev + (size_t)k * l * c->N;
    fhs_status s = bsgs_core(c, baby, G, p.data(), D, B, ci, scale, gk, out);
    dfree(c, dev, bytes);
    return s;
}

// ============================================================================ measurement hooks
extern "C" fhs_status fhs_random_plaintexts(fhs_context* c, uint64_t seed, int count, int ci, double scale,
                                            fhs_plaintext** outs) {
    ENTER(c);
    if (!outs || count < 1) return fail(FHS_ERR_INVALID, "random_plaintexts: bad args");
    BatchOut bo(outs, (size_t)count);
    fhs_status s0 = new_pts(c, (size_t)count, ci, scale, outs);
    if (s0 != FHS_OK) return s0;
    for (int k = 0; k < count; ++k) {
        fhs_plaintext* pt = outs[k];
        HIPCHK(fhs::launch_sample(c->T, fhs::SAMPLE_TESTDATA, PrfKey{}, sm64(seed ^ sm64((7ull << 56) | (uint64_t)k)), pt->d, pt->l, c->st), "random_plaintexts");
    }
    return bo.keep(FHS_OK);
}
extern "C" fhs_status fhs_event_record(fhs_context* c, void** ev) {
    ENTER(c);
    hipEvent_t e = ev_get(c->device);
    if (!e) return fail(FHS_ERR_HIP, "event: hipEventCreate failed");
    HIPCHK(hipEventRecord(e, c->st), "event");
    *ev = (void*)e;
    return FHS_OK;
}
extern "C" fhs_status fhs_event_elapsed(void* a, void* b, float* ms) {
    HIPCHK(hipEventSynchronize((hipEvent_t)b), "event sync");
    HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b), "event elapsed");
    return FHS_OK;
}
extern "C" fhs_status fhs_event_destroy(void* e) {
    ev_put((hipEvent_t)e);   // back to the pool (events are reused, not destroyed)
    return FHS_OK;
}
static void timer_rec(void* vc, int id, int begin, hipStream_t st) {
    auto* c = static_cast<fhs_context*>(vc);
    if (!(c->timer_mask & (1u << id))) return;
    hipEvent_t e = ev_get(c->device);
    if (!e) return;
    hipEventRecord(e, st);
    if (begin) {
        if (c->timer_open[id]) ev_put(c->timer_open[id]);
        c->timer_open[id] = e;
    } else if (c->timer_open[id]) {
        c->timer_pairs[id].push_back({c->timer_open[id], e});
        c->timer_open[id] = nullptr;
    } else {
        ev_put(e);
    }
}
// Arms the timer for the kernels in `mask` (bit i = fhs::KernelId i) after reporting, for kernel
// `kernel_id`, the time and launch count accumulated since the last reset.
extern "C" fhs_status fhs_kernel_timer(fhs_context* c, int kernel_id, float* ms, int* launches, int reset) {
    ENTER(c);
    HIPCHK(hipStreamSynchronize(c->st), "timer sync");
    if ((int)c->timer_pairs.size() < fhs::KID_COUNT) {
        c->timer_pairs.resize(fhs::KID_COUNT);
        c->timer_open.assign(fhs::KID_COUNT, nullptr);
        c->ktimer = fhs::KTimer{c, timer_rec};
    }
    float tot = 0.f;
    int n = 0;
    if (kernel_id >= 0 && kernel_id < fhs::KID_COUNT)
        for (auto& pr : c->timer_pairs[kernel_id]) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, pr.first, pr.second) == hipSuccess) { tot += t; ++n; }
        }
    if (ms) *ms = tot;
    if (launches) *launches = n;
    if (reset) {
        for (auto& v : c->timer_pairs) {
            for (auto& pr : v) { ev_put(pr.first); ev_put(pr.second); }
            v.clear();
        }
    }
    return FHS_OK;
}
extern "C" fhs_status fhs_kernel_timer_arm(fhs_context* c, uint32_t mask) {
    ENTER(c);
    if (c->timer_pairs.size() < (size_t)fhs::KID_COUNT) {
        c->timer_pairs.resize(fhs::KID_COUNT);
        c->timer_open.assign(fhs::KID_COUNT, nullptr);
        c->ktimer = fhs::KTimer{c, timer_rec};
    }
    c->timer_mask = mask;
    if (mask) ev_reserve(c->device, 2048);   // created here, not between the timed launches
    return FHS_OK;
}
// staging-ring statistics (tests / diagnostics): segment re-entries, and how many had to wait
extern "C" fhs_status fhs_staging_stats(fhs_context* c, uint64_t* reentries, uint64_t* blocked) {
    ENTER(c);
    if (reentries) *reentries = c->ring_waits;
    if (blocked) *blocked = c->ring_blocked;
    return FHS_OK;
}
// device-to-device copy of a ciphertext's limbs into caller memory (RCCL interop); synchronises
static fhs_status copy_to_device(fhs_context* c, const fhs_ciphertext* ct, void* dst, bool sync) {
    if (!ct || !dst) return fail(FHS_ERR_INVALID, "null argument");
    LIVE(ct);
    HIPCHK(hipMemcpyAsync(dst, ct->d, ct_bytes(ct), hipMemcpyDeviceToDevice, c->st), "copy_to_device");
    if (sync) HIPCHK(hipStreamSynchronize(c->st), "copy_to_device");
    return FHS_OK;
}
static fhs_status from_device(fhs_context* c, const void* src, int ncomp, int ci, double scale, fhs_ciphertext** out,
                              bool sync) {
    if (!src || !out) return fail(FHS_ERR_INVALID, "null argument");
    fhs_ciphertext* ct;
    fhs_status s = new_ct(c, ncomp, ci, scale, &ct);
    if (s != FHS_OK) return s;
    hipError_t e = hipMemcpyAsync(ct->d, src, ct_bytes(ct), hipMemcpyDeviceToDevice, c->st);
    if (e == hipSuccess && sync) e = hipStreamSynchronize(c->st);
    if (e != hipSuccess) {
        fhs_ciphertext_destroy(ct);
        return hip_fail(e, "from_device");
    }
    *out = ct;
    return FHS_OK;
}
extern "C" fhs_status fhs_ciphertext_copy_to_device(fhs_context* c, const fhs_ciphertext* ct, void* dst) {
    ENTER(c);
    return copy_to_device(c, ct, dst, true);
}
extern "C" fhs_status fhs_ciphertext_from_device(fhs_context* c, const void* src, int ncomp, int ci, double scale,
                                                 fhs_ciphertext** out) {
    ENTER(c);
    return from_device(c, src, ncomp, ci, scale, out, true);
}
extern "C" fhs_status fhs_ciphertext_copy_to_device_async(fhs_context* c, const fhs_ciphertext* ct, void* dst) {
    ENTER(c);
    return copy_to_device(c, ct, dst, false);
}
extern "C" fhs_status fhs_ciphertext_from_device_async(fhs_context* c, const void* src, int ncomp, int ci, double scale,
                                                       fhs_ciphertext** out) {
    ENTER(c);
    return from_device(c, src, ncomp, ci, scale, out, false);
}
extern "C" fhs_status fhs_context_stream(fhs_context* c, void** stream) {
    ENTER(c);
    if (!stream) return fail(FHS_ERR_INVALID, "null argument");
    *stream = (void*)c->st;
    return FHS_OK;
}

// x (any 64-bit value, or a value < 2m when canonical is asked) congruent to want (< m)?
static bool x_ok(uint64_t x, uint64_t want, uint64_t m, bool lt2m) {
    return (!lt2m || x < 2 * m) && x % m == want;
}
// The ModUp X form's arithmetic on the host (the same __host__ __device__ routines the kernels run):
// y3 (residues of a 3-prime digit q3, after the inverse-hat scaling) -> the centred digit value mod m.
// For a 59-bit target the kernels' convert3x_b59 (folded and unfolded) must give congruent values.
extern "C" fhs_status fhs_debug_modup_xform(const uint64_t* q3, const uint64_t* y3, uint64_t m, uint64_t* out) {
    if (!q3 || !y3 || !out) return FHS_ERR_INVALID;
    const uint64_t w = pm_word(m, 14);
    if (!w || !conv_pm_ok(m, 3)) return fail(FHS_ERR_INVALID, "debug_modup_xform: target not on the pseudo-Mersenne fold");
    for (int u = 0; u < 3; ++u)   // centered_x_pack has three rounding thresholds: S < 3 Q_S needs y < q
        if (y3[u] >= q3[u]) return fail(FHS_ERR_INVALID, "debug_modup_xform: residues must be < q");
    const uint64_t pr[4] = {q3[0], q3[1], q3[2], m};
    uint64_t xd[32] = {0}, xt[16] = {0};
    modup_xform_tables(pr, 4, 3, 1, xd, xt);
    uint64_t words[3];
    centered_x_pack(y3, xd, words);
    const uint64_t* t = xt + 12;
    if (t[0] >= (1ull << 30)) return fail(FHS_ERR_INVALID, "debug_modup_xform: 2^60 mod m >= 2^30 (no X form)");
    const uint64_t x = convert3x_value(words[0], words[1], words[2], (uint32_t)t[0], unpack30(t[1]), t[2],
                                       (unsigned)(w & 127), (unsigned)(w >> 8));
    if (x >= 2 * m) return fail(FHS_ERR_INVALID, "debug_modup_xform: result above 2m");
    *out = x >= m ? x - m : x;
    if (b59_prime(m)) {
        const uint32_t d = (uint32_t)((1ull << 59) - m);
        for (int canon = 0; canon < 2; ++canon)
            if (!x_ok(convert3x_b59(words[0], words[1], words[2], (uint32_t)t[0], unpack30(t[1]), t[2], d, canon), *out,
                      m, canon))
                return fail(FHS_ERR_INVALID, "debug_modup_xform: convert3x_b59 disagrees");
    }
    return FHS_OK;
}
// ModDown's X form on the host (k_special_x + moddown_convert3x arithmetic): y3 (special residues < p_k,
// already scaled by inv(P/p_k)) -> (sum_k y_k P/p_k) mod q, the fast base conversion's value.
extern "C" fhs_status fhs_debug_moddown_xform(const uint64_t* p3, const uint64_t* y3, uint64_t q, uint64_t* out) {
    if (!p3 || !y3 || !out) return FHS_ERR_INVALID;
    const uint64_t w = pm_word(q, 14);
    if (!w || !conv_pm_ok(q, 3)) return fail(FHS_ERR_INVALID, "debug_moddown_xform: target not on the pseudo-Mersenne fold");
    for (int k = 0; k < 3; ++k)
        if (p3[k] >= (1ull << 59)) return fail(FHS_ERR_INVALID, "debug_moddown_xform: special primes must be < 2^59");
    for (int k = 0; k < 3; ++k)
        if (y3[k] >= p3[k]) return fail(FHS_ERR_INVALID, "debug_moddown_xform: residues must be < p");
    uint64_t xd[32] = {0}, xt[4] = {0};
    for (int u = 0; u < 3; ++u) {   // as fhs_context_create's md_xd
        const hu128 h = (hu128)p3[(u + 1) % 3] * p3[(u + 2) % 3];
        xd[2 * u] = (uint64_t)h;
        xd[2 * u + 1] = (uint64_t)(h >> 64);
    }
    for (int i = 6; i < 15; ++i) xd[i] = ~0ull;
    modup_xform_tables(&q, 1, 0, 0, xd, xt);   // the target's weights only (no digit rows: L0 = 0)
    if (xt[0] >= (1ull << 30)) return fail(FHS_ERR_INVALID, "debug_moddown_xform: 2^60 mod q >= 2^30");
    uint64_t words[3];
    centered_x_pack(y3, xd, words);
    const uint64_t x = convert3x_value(words[0], words[1], words[2], (uint32_t)xt[0], unpack30(xt[1]), 0,
                                       (unsigned)(w & 127), (unsigned)(w >> 8));
    if (x >= 2 * q) return fail(FHS_ERR_INVALID, "debug_moddown_xform: result above 2q");
    *out = x >= q ? x - q : x;
    if (b59_prime(q)) {
        const uint32_t d = (uint32_t)((1ull << 59) - q);
        for (int canon = 0; canon < 2; ++canon)
            if (!x_ok(convert3x_b59(words[0], words[1], words[2], (uint32_t)xt[0], unpack30(xt[1]), 0, d, canon), *out,
                      q, canon))
                return fail(FHS_ERR_INVALID, "debug_moddown_xform: convert3x_b59 disagrees");
    }
    return FHS_OK;
}
extern "C" fhs_status fhs_debug_reduce128(uint64_t q, uint64_t lo, uint64_t hi, uint64_t* out, int* pm_used) {
    if (!out || q < 3) return FHS_ERR_INVALID;
    const uint64_t w = pm_word(q, 14);
    if (pm_used) *pm_used = w != 0;
    *out = w ? pm_reduce128(lo, hi, q, (unsigned)(w & 127), (unsigned)(w >> 8))
             : (uint64_t)((((hu128)hi << 64) | lo) % q);
    return FHS_OK;
}
