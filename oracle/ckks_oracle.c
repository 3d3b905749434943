/*
 * ckks_oracle.c -- CPU restatement of the CKKS arithmetic on FHE-SPEAR's BSGS hot path.
 * TEST INFRASTRUCTURE ONLY (see ckks_oracle.h).  Plain C99 + unsigned __int128, no dependencies.
 *
 * Reference anchors (all paths under /root/reference):
 *   create_coeff_modulus  gpu/phantom_binding.cu:81        (SEAL CoeffModulus::Create algorithm)
 *   get_elts_from_steps   gpu/phantom_binding.cu:124-126   (5^step mod 2N; bg:18-26 uses pow(5,step,2N))
 *   rotate                gpu/phantom_binding.cu:203       (automorphism + hybrid key-switch)
 *   multiply_plain / add  gpu/phantom_binding.cu:181, 167  (bg:471, 475, 483)
 *   rescale_to_next       gpu/phantom_binding.cu:185       (bg:484)
 *   multiply/relinearize  gpu/phantom_binding.cu:177, 183  (tf:58-60)
 *   BSGS loop             scripts/bootstrap_generation.py:464-485
 *   encoder               gpu/phantom_binding.cu:138-156   (slot j <-> root zeta^(5^j), slots = N/2)
 */
#include "ckks_oracle.h"
#include <stdlib.h>
#include <string.h>
#include <math.h>

typedef unsigned __int128 u128;

struct ock_ctx {
    uint64_t N;
    int logN;
    int L0, P, K;           /* data primes, special primes, total */
    uint64_t* q;            /* K primes, key-level order */
    uint64_t* psi_rev;      /* K x N  psi^{rev(k)} */
    uint64_t* psi_rev_s;    /* Shoup companions */
    uint64_t* ipsi_rev;     /* K x N  psi^{-rev(k)} */
    uint64_t* ipsi_rev_s;
    uint64_t* n_inv;        /* K */
    int ks_seal;            /* key-switch convention: 0 exact centred (default), 1 SEAL (P = 1) */
};

/* SEAL's switch_key_inplace (P = 1; SEAL evaluator.cpp, published): each data limb of the
 * (already automorphed) target is lifted to the other primes as its residue in [0, q) -- no
 * centring -- and the ModDown adds floor(p/2) to the special limb before converting it and
 * subtracts floor(p/2) mod q_i after, i.e. rounds instead of flooring.  The non-centred lift does not
 * commute with automorphisms, so there is no hoisting in this mode: ock_rotate_hoisted refuses it. */
int ock_ctx_set_ks_mode(ock_ctx* c, int mode) {
    if (mode != 0 && mode != 1) return -1;
    if (mode == 1 && c->P != 1) return -1;
    c->ks_seal = mode;
    return 0;
}

/* ------------------------------------------------------------------ sampling spec */
uint64_t ock_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
uint64_t ock_rnd(uint64_t key, uint64_t ctr) { return ock_splitmix64(key ^ ock_splitmix64(ctr ^ 0xD1B54A32D192ED03ULL)); }

/* ChaCha20 block function, RFC 8439 §2.3 (state: constants, 8 key words, counter, 3 nonce words;
 * 20 rounds as 10 column + diagonal double rounds; output = rounds(state) + state) */
#define ROTL32(v, n) (((v) << (n)) | ((v) >> (32 - (n))))
#define QROUND(a, b, c, d) do { \
    a += b; d ^= a; d = ROTL32(d, 16); c += d; b ^= c; b = ROTL32(b, 12); \
    a += b; d ^= a; d = ROTL32(d, 8);  c += d; b ^= c; b = ROTL32(b, 7); } while (0)
void ock_chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], uint32_t out[16]) {
    uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    for (int i = 0; i < 8; i++) st[4 + i] = key[i];
    st[12] = counter; st[13] = nonce[0]; st[14] = nonce[1]; st[15] = nonce[2];
    uint32_t x[16];
    memcpy(x, st, sizeof x);
    for (int r = 0; r < 10; r++) {
        QROUND(x[0], x[4], x[8], x[12]); QROUND(x[1], x[5], x[9], x[13]);
        QROUND(x[2], x[6], x[10], x[14]); QROUND(x[3], x[7], x[11], x[15]);
        QROUND(x[0], x[5], x[10], x[15]); QROUND(x[1], x[6], x[11], x[12]);
        QROUND(x[2], x[7], x[8], x[13]); QROUND(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) out[i] = x[i] + st[i];
}
/* The secret-randomness PRF: block `ctr` of stream `sid` under the 32-byte key
 * (little-endian words), nonce (lo32 sid, hi32 sid, "FHS1"); w0/w1 = its first two 64-bit words. */
typedef struct { uint32_t k[8]; } prf_key;
static prf_key prf_key_from_bytes(const uint8_t* b) {
    prf_key K;
    for (int w = 0; w < 8; w++)
        K.k[w] = (uint32_t)b[4 * w] | ((uint32_t)b[4 * w + 1] << 8) | ((uint32_t)b[4 * w + 2] << 16) | ((uint32_t)b[4 * w + 3] << 24);
    return K;
}
static void prf128(const prf_key* K, uint64_t sid, uint32_t ctr, uint64_t* w0, uint64_t* w1) {
    uint32_t nonce[3] = {(uint32_t)sid, (uint32_t)(sid >> 32), 0x31534846u}, o[16];
    ock_chacha20_block(K->k, ctr, nonce, o);
    *w0 = (uint64_t)o[0] | ((uint64_t)o[1] << 32);
    *w1 = (uint64_t)o[2] | ((uint64_t)o[3] << 32);
}

enum { ST_SECRET = 1, ST_PUBKEY = 2, ST_RELIN = 3, ST_GALOIS = 4, ST_ENC_SYM = 5, ST_ENC_ASYM = 6, ST_PK_RNG = 7 };
static uint64_t stream_id(uint64_t kind, uint64_t a, uint64_t b) { return (kind << 56) | (a << 16) | b; }

/* ------------------------------------------------------------------ modular helpers */
static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)(((u128)a * b) % q); }
static inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t q) { uint64_t s = a + b; return s >= q ? s - q : s; }
static inline uint64_t submod(uint64_t a, uint64_t b, uint64_t q) { return a >= b ? a - b : a + q - b; }
static uint64_t powmod(uint64_t b, uint64_t e, uint64_t q) {
    uint64_t r = 1 % q; b %= q;
    while (e) { if (e & 1) r = mulmod(r, b, q); b = mulmod(b, b, q); e >>= 1; }
    return r;
}
static uint64_t invmod(uint64_t a, uint64_t q) { return powmod(a, q - 2, q); } /* q prime */
static inline uint64_t shoup_pre(uint64_t w, uint64_t q) { return (uint64_t)(((u128)w << 64) / q); }
static inline uint64_t shoup_mul(uint64_t a, uint64_t w, uint64_t wp, uint64_t q) {
    uint64_t qh = (uint64_t)(((u128)a * wp) >> 64);
    uint64_t r = a * w - qh * q;
    return r >= q ? r - q : r;
}

static int is_prime_u64(uint64_t n) {
    if (n < 2) return 0;
    static const uint64_t small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (int i = 0; i < 12; i++) { if (n == small[i]) return 1; if (n % small[i] == 0) return 0; }
    uint64_t d = n - 1; int s = 0;
    while (!(d & 1)) { d >>= 1; s++; }
    for (int i = 0; i < 12; i++) {
        uint64_t x = powmod(small[i], d, n);
        if (x == 1 || x == n - 1) continue;
        int comp = 1;
        for (int r = 1; r < s; r++) { x = mulmod(x, x, n); if (x == n - 1) { comp = 0; break; } }
        if (comp) return 0;
    }
    return 1;
}

static inline uint32_t bitrev(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

/* ------------------------------------------------------------------ parameters */
/* SEAL CoeffModulus::Create restated: for each bit size, the largest primes p < 2^b with
 * p = 1 (mod 2N), descending; request order decides which prime lands where (pb:81). */
int ock_create_coeff_modulus(uint64_t N, const int* bits, int n, uint64_t* out) {
    uint64_t fac = 2 * N;
    for (int i = 0; i < n; i++) {
        int b = bits[i];
        if (b < 2 || b > 61) return -1;
        int rank = 0;                          /* how many earlier requests share this size */
        for (int k = 0; k < i; k++) if (bits[k] == b) rank++;
        uint64_t v = ((uint64_t)1 << b) - fac + 1, lo = (uint64_t)1 << (b - 1);
        int found = -1;
        while (v > lo) {
            if (is_prime_u64(v)) { found++; if (found == rank) break; }
            v -= fac;
        }
        if (v <= lo) return -2;
        out[i] = v;
    }
    return 0;
}

/* pb:124-126 get_elt_from_step: step>0 rotates left: 5^step mod 2N; step<0: 5^(N/2-|step|);
 * step 0 = conjugation 2N-1.  bg:18-26 builds the same elements with pow(5, step, 2N). */
uint64_t ock_galois_elt_from_step(int step, uint64_t N) {
    uint64_t m = 2 * N;
    if (step == 0) return m - 1;
    uint64_t slots = N / 2;
    uint64_t s = step > 0 ? (uint64_t)step : slots - (uint64_t)(-step);
    s %= slots;
    uint64_t e = 1;
    for (uint64_t i = 0; i < s; i++) e = (e * 5) & (m - 1);
    return e;
}

static uint64_t minimal_2n_root(uint64_t q, uint64_t N) {
    uint64_t m = 2 * N, cof = (q - 1) / m, g = 0;
    for (uint64_t c = 2;; c++) {
        g = powmod(c, cof, q);
        if (powmod(g, N, q) == q - 1) break;   /* order exactly 2N */
    }
    uint64_t g2 = mulmod(g, g, q), best = g, cur = g;
    for (uint64_t k = 1; k < N; k++) { cur = mulmod(cur, g2, q); if (cur < best) best = cur; }
    return best;
}

ock_ctx* ock_ctx_create(uint64_t N, const uint64_t* primes, int nprimes, int special) {
    if (N < 8 || (N & (N - 1)) || special < 1 || special >= nprimes) return NULL;
    ock_ctx* c = (ock_ctx*)calloc(1, sizeof(ock_ctx));
    c->N = N; c->logN = 0; while (((uint64_t)1 << c->logN) < N) c->logN++;
    c->K = nprimes; c->P = special; c->L0 = nprimes - special;
    c->q = (uint64_t*)malloc(sizeof(uint64_t) * nprimes);
    memcpy(c->q, primes, sizeof(uint64_t) * nprimes);
    size_t tab = (size_t)nprimes * N;
    c->psi_rev = (uint64_t*)malloc(8 * tab); c->psi_rev_s = (uint64_t*)malloc(8 * tab);
    c->ipsi_rev = (uint64_t*)malloc(8 * tab); c->ipsi_rev_s = (uint64_t*)malloc(8 * tab);
    c->n_inv = (uint64_t*)malloc(8 * nprimes);
    for (int i = 0; i < nprimes; i++) {
        uint64_t q = primes[i];
        uint64_t psi = minimal_2n_root(q, N), ipsi = invmod(psi, q);
        uint64_t* pr = c->psi_rev + (size_t)i * N; uint64_t* ipr = c->ipsi_rev + (size_t)i * N;
        uint64_t pw = 1, ipw = 1;
        for (uint64_t k = 0; k < N; k++) {
            uint32_t r = bitrev((uint32_t)k, c->logN);
            pr[r] = pw; ipr[r] = ipw;
            pw = mulmod(pw, psi, q); ipw = mulmod(ipw, ipsi, q);
        }
        for (uint64_t k = 0; k < N; k++) {
            c->psi_rev_s[(size_t)i * N + k] = shoup_pre(pr[k], q);
            c->ipsi_rev_s[(size_t)i * N + k] = shoup_pre(ipr[k], q);
        }
        c->n_inv[i] = invmod(N % q, q);
    }
    return c;
}
void ock_ctx_destroy(ock_ctx* c) {
    if (!c) return;
    free(c->q); free(c->psi_rev); free(c->psi_rev_s); free(c->ipsi_rev); free(c->ipsi_rev_s); free(c->n_inv);
    free(c);
}
int ock_ctx_L0(const ock_ctx* c) { return c->L0; }
int ock_ctx_P(const ock_ctx* c) { return c->P; }
uint64_t ock_ctx_N(const ock_ctx* c) { return c->N; }
uint64_t ock_ctx_prime(const ock_ctx* c, int i) { return c->q[i]; }

/* key-level prime index of the i-th limb of an extended (Q_l u P) polynomial */
static inline int ext_prime(const ock_ctx* c, int l, int i) { return i < l ? i : c->L0 + (i - l); }

/* ------------------------------------------------------------------ NTT */
/* forward negacyclic NTT, Cooley-Tukey, natural in -> bit-reversed out:
 * out[i] = a(psi^(2*rev(i)+1)) mod q. */
void ock_ntt_fwd(const ock_ctx* c, uint64_t* a, int pi) {
    uint64_t N = c->N, q = c->q[pi];
    const uint64_t* W = c->psi_rev + (size_t)pi * N; const uint64_t* Ws = c->psi_rev_s + (size_t)pi * N;
    uint64_t t = N;
    for (uint64_t m = 1; m < N; m <<= 1) {
        t >>= 1;
        for (uint64_t i = 0; i < m; i++) {
            uint64_t w = W[m + i], ws = Ws[m + i], j1 = 2 * i * t;
            for (uint64_t j = j1; j < j1 + t; j++) {
                uint64_t x = a[j], y = shoup_mul(a[j + t], w, ws, q);
                a[j] = addmod(x, y, q); a[j + t] = submod(x, y, q);
            }
        }
    }
}
/* inverse, Gentleman-Sande, bit-reversed in -> natural out, includes N^-1 */
void ock_ntt_inv(const ock_ctx* c, uint64_t* a, int pi) {
    uint64_t N = c->N, q = c->q[pi];
    const uint64_t* W = c->ipsi_rev + (size_t)pi * N; const uint64_t* Ws = c->ipsi_rev_s + (size_t)pi * N;
    uint64_t t = 1;
    for (uint64_t m = N >> 1; m >= 1; m >>= 1) {
        for (uint64_t i = 0; i < m; i++) {
            uint64_t w = W[m + i], ws = Ws[m + i], j1 = 2 * i * t;
            for (uint64_t j = j1; j < j1 + t; j++) {
                uint64_t x = a[j], y = a[j + t];
                a[j] = addmod(x, y, q); a[j + t] = shoup_mul(submod(x, y, q), w, ws, q);
            }
        }
        t <<= 1;
    }
    uint64_t ni = c->n_inv[pi], nis = shoup_pre(ni, q);
    for (uint64_t j = 0; j < N; j++) a[j] = shoup_mul(a[j], ni, nis, q);
}

/* X -> X^elt in the NTT domain: out[i] = in[idx((2 rev(i)+1) * elt mod 2N)], idx(e)=rev((e-1)/2) */
void ock_apply_galois_ntt(const ock_ctx* c, const uint64_t* in, uint64_t* out, uint64_t elt) {
    uint64_t N = c->N, m = 2 * N;
    for (uint64_t i = 0; i < N; i++) {
        uint64_t e = 2 * (uint64_t)bitrev((uint32_t)i, c->logN) + 1;
        uint64_t e2 = (e * elt) & (m - 1);
        out[i] = in[bitrev((uint32_t)((e2 - 1) >> 1), c->logN)];
    }
}

/* ------------------------------------------------------------------ element-wise */
void ock_add(const ock_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* out, int ncomp, int l) {
    uint64_t N = c->N;
    for (int k = 0; k < ncomp; k++) for (int i = 0; i < l; i++) {
        size_t o = ((size_t)k * l + i) * N;
        for (uint64_t j = 0; j < N; j++) out[o + j] = addmod(a[o + j], b[o + j], c->q[i]);
    }
}
void ock_sub(const ock_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* out, int ncomp, int l) {
    uint64_t N = c->N;
    for (int k = 0; k < ncomp; k++) for (int i = 0; i < l; i++) {
        size_t o = ((size_t)k * l + i) * N;
        for (uint64_t j = 0; j < N; j++) out[o + j] = submod(a[o + j], b[o + j], c->q[i]);
    }
}
void ock_negate(const ock_ctx* c, const uint64_t* a, uint64_t* out, int ncomp, int l) {
    uint64_t N = c->N;
    for (int k = 0; k < ncomp; k++) for (int i = 0; i < l; i++) {
        size_t o = ((size_t)k * l + i) * N;
        for (uint64_t j = 0; j < N; j++) out[o + j] = a[o + j] ? c->q[i] - a[o + j] : 0;
    }
}
/* pb:181 multiply_plain: c_k <- c_k (.) p  (bg:471) */
void ock_multiply_plain(const ock_ctx* c, const uint64_t* ct, const uint64_t* pt, uint64_t* out, int ncomp, int l) {
    uint64_t N = c->N;
    for (int k = 0; k < ncomp; k++) for (int i = 0; i < l; i++) {
        size_t o = ((size_t)k * l + i) * N, po = (size_t)i * N;
        for (uint64_t j = 0; j < N; j++) out[o + j] = mulmod(ct[o + j], pt[po + j], c->q[i]);
    }
}
void ock_add_plain(const ock_ctx* c, const uint64_t* ct, const uint64_t* pt, uint64_t* out, int ncomp, int l) {
    uint64_t N = c->N;
    memcpy(out, ct, sizeof(uint64_t) * ncomp * l * N);
    for (int i = 0; i < l; i++)
        for (uint64_t j = 0; j < N; j++) out[(size_t)i * N + j] = addmod(ct[(size_t)i * N + j], pt[(size_t)i * N + j], c->q[i]);
}
/* pb:177 multiply (tf:58): (a0 b0, a0 b1 + a1 b0, a1 b1) */
void ock_multiply(const ock_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* out3, int l) {
    uint64_t N = c->N; size_t S = (size_t)l * N;
    for (int i = 0; i < l; i++) {
        uint64_t q = c->q[i];
        for (uint64_t j = 0; j < N; j++) {
            size_t o = (size_t)i * N + j;
            out3[o] = mulmod(a[o], b[o], q);
            out3[S + o] = addmod(mulmod(a[o], b[S + o], q), mulmod(a[S + o], b[o], q), q);
            out3[2 * S + o] = mulmod(a[S + o], b[S + o], q);
        }
    }
}

/* pb:185 rescale_to_next (bg:484): divide by q_{l-1} with rounding, per component */
void ock_rescale_to_next(const ock_ctx* c, const uint64_t* in, uint64_t* out, int ncomp, int l) {
    uint64_t N = c->N; int last = l - 1; uint64_t ql = c->q[last], half = ql >> 1;
    uint64_t* tmp = (uint64_t*)malloc(8 * N); uint64_t* t2 = (uint64_t*)malloc(8 * N);
    for (int k = 0; k < ncomp; k++) {
        memcpy(tmp, in + ((size_t)k * l + last) * N, 8 * N);
        ock_ntt_inv(c, tmp, last);
        for (uint64_t j = 0; j < N; j++) tmp[j] = addmod(tmp[j], half, ql);
        for (int i = 0; i < last; i++) {
            uint64_t q = c->q[i], hq = half % q, inv = invmod(ql % q, q);
            for (uint64_t j = 0; j < N; j++) t2[j] = submod(tmp[j] % q, hq, q);
            ock_ntt_fwd(c, t2, i);
            const uint64_t* a = in + ((size_t)k * l + i) * N;
            uint64_t* o = out + ((size_t)k * last + i) * N;
            for (uint64_t j = 0; j < N; j++) o[j] = mulmod(submod(a[j], t2[j], q), inv, q);
        }
    }
    free(tmp); free(t2);
}

/* ------------------------------------------------------------------ bootstrapping primitives */
/* ModRaise (ckks_bootstrapper.bootstrap, bg:149-154): limb q0 of each component, centred in
 * (-q0/2, q0/2], re-embedded into all L0 data limbs (standard CKKS bootstrapping, Cheon et al. 2018). */
void ock_mod_raise(const ock_ctx* c, const uint64_t* in, int l, int ncomp, uint64_t* out) {
    uint64_t N = c->N; int L = c->L0; uint64_t q0 = c->q[0], half = q0 >> 1;
    uint64_t* x = (uint64_t*)malloc(8 * N);
    for (int k = 0; k < ncomp; k++) {
        memcpy(x, in + (size_t)k * l * N, 8 * N);
        ock_ntt_inv(c, x, 0);
        for (int i = 0; i < L; i++) {
            uint64_t q = c->q[i];
            uint64_t* o = out + ((size_t)k * L + i) * N;
            for (uint64_t j = 0; j < N; j++) {
                if (x[j] <= half) o[j] = x[j] % q;
                else { uint64_t m = (q0 - x[j]) % q; o[j] = m ? q - m : 0; }
            }
            ock_ntt_fwd(c, o, i);
        }
    }
    free(x);
}
/* constant product (op 0: every component times k_i) or sum (op 1: k_i added to component 0);
 * k_i = the integer constant mod q_i (a constant polynomial is constant in the NTT domain) */
void ock_scalar(const ock_ctx* c, int op, const uint64_t* in, const uint64_t* k, uint64_t* out, int ncomp, int l) {
    uint64_t N = c->N;
    for (int comp = 0; comp < ncomp; comp++)
        for (int i = 0; i < l; i++) {
            uint64_t q = c->q[i];
            const uint64_t* a = in + ((size_t)comp * l + i) * N;
            uint64_t* o = out + ((size_t)comp * l + i) * N;
            for (uint64_t j = 0; j < N; j++)
                o[j] = op == 0 ? mulmod(a[j], k[i], q) : (comp == 0 ? addmod(a[j], k[i], q) : a[j]);
        }
}

/* ------------------------------------------------------------------ hybrid key-switch */
/* Exact centred base extension count: v = round(sum_u y_u / q_u) = the number of Q_S to subtract
 * from X = sum_u y_u (Q_S/q_u) so that X - v Q_S lies in (-Q_S/2, Q_S/2).  Fast path: 64-bit
 * fixed-point sum of frac(y_u/q_u) via R_u = floor(2^128/q_u) (error < 2 ns ulp); when the
 * fraction is within 64 ulp of 1/2 the decision is made exactly with multi-word integers.
 * Exactness makes the extension commute with the signed coefficient permutations of Galois
 * automorphisms, so a hoisted ModUp (one per input, rotations applied afterwards) is
 * bit-identical to one ModUp per rotated input.   */
static int ock_centered_count(const uint64_t* y, const uint64_t* qs, int ns) {
    if (ns == 1) return y[0] > (qs[0] >> 1);
    uint64_t lo = 0; int carry = 0;
    for (int u = 0; u < ns; u++) {
        u128 R = (~(u128)0) / qs[u];                       /* floor(2^128 / q) for odd q */
        uint64_t R0 = (uint64_t)R, R1 = (uint64_t)(R >> 64);
        uint64_t F = y[u] * R1 + (uint64_t)(((u128)y[u] * R0) >> 64);
        lo += F; carry += (lo < F);
    }
    uint64_t half = (uint64_t)1 << 63;
    uint64_t d = lo >= half ? lo - half : half - lo;
    if (d > 64) return carry + (lo >= half);
    /* exact: v = carry + [2X >= (2 carry + 1) Q] with X = sum_u y_u prod_{u' != u} q_u' */
    uint64_t X[10] = {0}, Q[10] = {0}, t[10];
    Q[0] = 1;
    for (int u = 0; u < ns; u++) {
        u128 cy = 0;
        for (int w = 0; w < 10; w++) { u128 z = (u128)Q[w] * qs[u] + cy; Q[w] = (uint64_t)z; cy = z >> 64; }
    }
    for (int u = 0; u < ns; u++) {
        memset(t, 0, sizeof t); t[0] = y[u];
        for (int v = 0; v < ns; v++) {
            if (v == u) continue;
            u128 cy = 0;
            for (int w = 0; w < 10; w++) { u128 z = (u128)t[w] * qs[v] + cy; t[w] = (uint64_t)z; cy = z >> 64; }
        }
        u128 cy = 0;
        for (int w = 0; w < 10; w++) { u128 z = (u128)X[w] + t[w] + cy; X[w] = (uint64_t)z; cy = z >> 64; }
    }
    /* lhs = 2X, rhs = (2 carry + 1) Q */
    uint64_t L[10], Rr[10]; u128 cy = 0;
    for (int w = 0; w < 10; w++) { u128 z = ((u128)X[w] << 1) + cy; L[w] = (uint64_t)z; cy = z >> 64; }
    cy = 0;
    for (int w = 0; w < 10; w++) { u128 z = (u128)Q[w] * (uint64_t)(2 * carry + 1) + cy; Rr[w] = (uint64_t)z; cy = z >> 64; }
    int ge = 1;
    for (int w = 9; w >= 0; w--) { if (L[w] != Rr[w]) { ge = L[w] > Rr[w]; break; } }
    return carry + ge;
}
int ock_centered_count_test(const uint64_t* y, const uint64_t* qs, int ns) { return ock_centered_count(y, qs, ns); }

/* Digit j of level l covers data primes [jP, min(jP+P, l)).  ModUp (approximate fast base
 * conversion) -> inner product with key digits over Q_l u P -> ModDown by P (no rounding
 * term).  This is the per-rotation (non-hoisted) key-switch the reference issues at bg:219 and
 * bg:479 through pb:203. */
void ock_keyswitch(const ock_ctx* c, const uint64_t* a, const uint64_t* key, int l,
                   uint64_t* out0, uint64_t* out1) {
    uint64_t N = c->N; int P = c->P, L0 = c->L0, K = c->K, E = l + P;
    int dnum = (l + P - 1) / P;
    uint64_t* acoef = (uint64_t*)malloc(8 * N * l);
    memcpy(acoef, a, 8 * N * l);
    for (int i = 0; i < l; i++) ock_ntt_inv(c, acoef + (size_t)i * N, i);
    uint64_t* acc = (uint64_t*)calloc((size_t)2 * E * N, 8);
    uint64_t* ext = (uint64_t*)malloc(8 * N);
    uint64_t* y = (uint64_t*)malloc(8 * N * P);
    for (int j = 0; j < dnum; j++) {
        int s0 = j * P, s1 = s0 + P < l ? s0 + P : l, ns = s1 - s0;
        for (int u = 0; u < ns; u++) {               /* y_u = a_u * (Q_S/q_u)^{-1} mod q_u */
            int i = s0 + u; uint64_t q = c->q[i], hat = 1;
            for (int v = 0; v < ns; v++) if (v != u) hat = mulmod(hat, c->q[s0 + v] % q, q);
            uint64_t ih = invmod(hat, q);
            for (uint64_t n = 0; n < N; n++) y[(size_t)u * N + n] = mulmod(acoef[(size_t)i * N + n], ih, q);
        }
        for (int t = 0; t < E; t++) {
            int pi = ext_prime(c, l, t); uint64_t m = c->q[pi];
            if (t >= s0 && t < s1) {
                memcpy(ext, a + (size_t)t * N, 8 * N);
            } else {
                uint64_t hm[8], Qm = 1;
                for (int u = 0; u < ns; u++) {
                    uint64_t h = 1;
                    for (int v = 0; v < ns; v++) if (v != u) h = mulmod(h, c->q[s0 + v] % m, m);
                    hm[u] = h;
                    Qm = mulmod(Qm, c->q[s0 + u] % m, m);
                }
                for (uint64_t n = 0; n < N; n++) {
                    uint64_t yy[8];
                    for (int u = 0; u < ns; u++) yy[u] = y[(size_t)u * N + n];
                    int v = c->ks_seal ? 0 : ock_centered_count(yy, c->q + s0, ns);
                    u128 s = 0;
                    for (int u = 0; u < ns; u++) s += (u128)yy[u] * hm[u];
                    uint64_t r = (uint64_t)(s % m);
                    ext[n] = submod(r, mulmod((uint64_t)v, Qm, m), m);   /* X - v Q_S (centred) */
                }
                ock_ntt_fwd(c, ext, pi);
            }
            for (int comp = 0; comp < 2; comp++) {
                const uint64_t* kp = key + (((size_t)j * 2 + comp) * K + pi) * N;
                uint64_t* ap = acc + ((size_t)comp * E + t) * N;
                for (uint64_t n = 0; n < N; n++) ap[n] = addmod(ap[n], mulmod(ext[n], kp[n], m), m);
            }
        }
    }
    /* ModDown */
    uint64_t* yp = (uint64_t*)malloc(8 * N * P);
    for (int comp = 0; comp < 2; comp++) {
        uint64_t* outp = comp ? out1 : out0;
        for (int k = 0; k < P; k++) {
            int pi = L0 + k; uint64_t p = c->q[pi], hat = 1;
            for (int v = 0; v < P; v++) if (v != k) hat = mulmod(hat, c->q[L0 + v] % p, p);
            uint64_t ih = invmod(hat, p);
            uint64_t* dst = yp + (size_t)k * N;
            memcpy(dst, acc + ((size_t)comp * E + l + k) * N, 8 * N);
            ock_ntt_inv(c, dst, pi);
            for (uint64_t n = 0; n < N; n++) dst[n] = mulmod(dst[n], ih, p);
            if (c->ks_seal) for (uint64_t n = 0; n < N; n++) dst[n] = addmod(dst[n], p >> 1, p);
        }
        for (int i = 0; i < l; i++) {
            uint64_t q = c->q[i], hm[8], Pm = 1;
            for (int k = 0; k < P; k++) {
                uint64_t h = 1;
                for (int v = 0; v < P; v++) if (v != k) h = mulmod(h, c->q[L0 + v] % q, q);
                hm[k] = h; Pm = mulmod(Pm, c->q[L0 + k] % q, q);
            }
            uint64_t Pinv = invmod(Pm, q);
            uint64_t halfq = c->ks_seal ? (c->q[L0] >> 1) % q : 0;
            for (uint64_t n = 0; n < N; n++) {
                u128 s = 0;
                for (int k = 0; k < P; k++) s += (u128)yp[(size_t)k * N + n] * hm[k];
                ext[n] = submod((uint64_t)(s % q), halfq, q);
            }
            ock_ntt_fwd(c, ext, i);
            const uint64_t* ap = acc + ((size_t)comp * E + i) * N;
            for (uint64_t n = 0; n < N; n++) outp[(size_t)i * N + n] = mulmod(submod(ap[n], ext[n], q), Pinv, q);
        }
    }
    free(acoef); free(acc); free(ext); free(y); free(yp);
}

void ock_rotate(const ock_ctx* c, const uint64_t* ct, const uint64_t* gkey, uint64_t elt, int l, uint64_t* out) {
    uint64_t N = c->N; size_t S = (size_t)l * N;
    uint64_t* r = (uint64_t*)malloc(8 * 2 * S);
    for (int i = 0; i < l; i++) {
        ock_apply_galois_ntt(c, ct + (size_t)i * N, r + (size_t)i * N, elt);
        ock_apply_galois_ntt(c, ct + S + (size_t)i * N, r + S + (size_t)i * N, elt);
    }
    uint64_t* k0 = (uint64_t*)malloc(8 * S); uint64_t* k1 = (uint64_t*)malloc(8 * S);
    ock_keyswitch(c, r + S, gkey, l, k0, k1);
    for (int i = 0; i < l; i++) for (uint64_t n = 0; n < N; n++) {
        size_t o = (size_t)i * N + n;
        out[o] = addmod(r[o], k0[o], c->q[i]);
        out[S + o] = k1[o];
    }
    free(r); free(k0); free(k1);
}

/* Hoisted rotations of ONE ciphertext: ModUp(c1) once, then per rotation the NTT-domain
 * automorphism of every extended digit, key inner product and ModDown.  With the exact centred
 * extension this equals ock_rotate per element, limb for limb (tests/test_cpu.py). */
void ock_rotate_hoisted(const ock_ctx* c, const uint64_t* ct, const uint64_t* const* gkeys, const uint64_t* elts,
                        int nrot, int l, uint64_t* const* outs) {
    if (c->ks_seal) {   /* no hoisting under SEAL's convention: one rotation at a time */
        for (int r = 0; r < nrot; r++) ock_rotate(c, ct, gkeys[r], elts[r], l, outs[r]);
        return;
    }
    uint64_t N = c->N; int P = c->P, L0 = c->L0, K = c->K, E = l + P;
    int dnum = (l + P - 1) / P;
    size_t S = (size_t)l * N;
    const uint64_t* c1 = ct + S;
    uint64_t* acoef = (uint64_t*)malloc(8 * S);
    memcpy(acoef, c1, 8 * S);
    for (int i = 0; i < l; i++) ock_ntt_inv(c, acoef + (size_t)i * N, i);
    uint64_t* ext = (uint64_t*)malloc(8 * N * (size_t)dnum * E);   /* [j][t][N] */
    for (int j = 0; j < dnum; j++) {
        int s0 = j * P, s1 = s0 + P < l ? s0 + P : l, ns = s1 - s0;
        uint64_t y[8][1];
        (void)y;
        for (int t = 0; t < E; t++) {
            int pi = ext_prime(c, l, t); uint64_t m = c->q[pi];
            uint64_t* dst = ext + ((size_t)j * E + t) * N;
            if (t >= s0 && t < s1) { memcpy(dst, c1 + (size_t)t * N, 8 * N); continue; }
            uint64_t hm[8], ih[8], Qm = 1;
            for (int u = 0; u < ns; u++) {
                uint64_t h = 1, hq = 1, q = c->q[s0 + u];
                for (int v = 0; v < ns; v++) if (v != u) { h = mulmod(h, c->q[s0 + v] % m, m); hq = mulmod(hq, c->q[s0 + v] % q, q); }
                hm[u] = h; ih[u] = invmod(hq, q);
                Qm = mulmod(Qm, c->q[s0 + u] % m, m);
            }
            for (uint64_t n = 0; n < N; n++) {
                uint64_t yy[8];
                for (int u = 0; u < ns; u++) yy[u] = mulmod(acoef[(size_t)(s0 + u) * N + n], ih[u], c->q[s0 + u]);
                int v = ock_centered_count(yy, c->q + s0, ns);
                u128 sum = 0;
                for (int u = 0; u < ns; u++) sum += (u128)yy[u] * hm[u];
                dst[n] = submod((uint64_t)(sum % m), mulmod((uint64_t)v, Qm, m), m);
            }
            ock_ntt_fwd(c, dst, pi);
        }
    }
    uint64_t* perm = (uint64_t*)malloc(8 * N);
    uint64_t* acc = (uint64_t*)malloc(8 * N * 2 * (size_t)E);
    uint64_t* yp = (uint64_t*)malloc(8 * N * P);
    uint64_t* tmp = (uint64_t*)malloc(8 * N);
    for (int r = 0; r < nrot; r++) {
        uint64_t elt = elts[r];
        const uint64_t* key = gkeys[r];
        memset(acc, 0, 8 * N * 2 * (size_t)E);
        for (int j = 0; j < dnum; j++)
            for (int t = 0; t < E; t++) {
                int pi = ext_prime(c, l, t); uint64_t m = c->q[pi];
                ock_apply_galois_ntt(c, ext + ((size_t)j * E + t) * N, perm, elt);
                for (int comp = 0; comp < 2; comp++) {
                    const uint64_t* kp = key + (((size_t)j * 2 + comp) * K + pi) * N;
                    uint64_t* ap = acc + ((size_t)comp * E + t) * N;
                    for (uint64_t n = 0; n < N; n++) ap[n] = addmod(ap[n], mulmod(perm[n], kp[n], m), m);
                }
            }
        uint64_t* out = outs[r];
        for (int comp = 0; comp < 2; comp++) {
            for (int k = 0; k < P; k++) {
                int pi = L0 + k; uint64_t p = c->q[pi], hat = 1;
                for (int v = 0; v < P; v++) if (v != k) hat = mulmod(hat, c->q[L0 + v] % p, p);
                uint64_t ihp = invmod(hat, p);
                uint64_t* dst = yp + (size_t)k * N;
                memcpy(dst, acc + ((size_t)comp * E + l + k) * N, 8 * N);
                ock_ntt_inv(c, dst, pi);
                for (uint64_t n = 0; n < N; n++) dst[n] = mulmod(dst[n], ihp, p);
            }
            for (int i = 0; i < l; i++) {
                uint64_t q = c->q[i], hmk[8], Pm = 1;
                for (int k = 0; k < P; k++) {
                    uint64_t h = 1;
                    for (int v = 0; v < P; v++) if (v != k) h = mulmod(h, c->q[L0 + v] % q, q);
                    hmk[k] = h; Pm = mulmod(Pm, c->q[L0 + k] % q, q);
                }
                uint64_t Pinv = invmod(Pm, q);
                for (uint64_t n = 0; n < N; n++) {
                    u128 sum = 0;
                    for (int k = 0; k < P; k++) sum += (u128)yp[(size_t)k * N + n] * hmk[k];
                    tmp[n] = (uint64_t)(sum % q);
                }
                ock_ntt_fwd(c, tmp, i);
                const uint64_t* ap = acc + ((size_t)comp * E + i) * N;
                uint64_t* o = out + (size_t)comp * S + (size_t)i * N;
                for (uint64_t n = 0; n < N; n++) o[n] = mulmod(submod(ap[n], tmp[n], q), Pinv, q);
            }
        }
        /* + galois(c0) */
        for (int i = 0; i < l; i++) {
            ock_apply_galois_ntt(c, ct + (size_t)i * N, perm, elt);
            for (uint64_t n = 0; n < N; n++) out[(size_t)i * N + n] = addmod(out[(size_t)i * N + n], perm[n], c->q[i]);
        }
    }
    free(acoef); free(ext); free(perm); free(acc); free(yp); free(tmp);
}

void ock_relinearize(const ock_ctx* c, const uint64_t* ct3, const uint64_t* rlk, int l, uint64_t* out) {
    uint64_t N = c->N; size_t S = (size_t)l * N;
    uint64_t* k0 = (uint64_t*)malloc(8 * S); uint64_t* k1 = (uint64_t*)malloc(8 * S);
    ock_keyswitch(c, ct3 + 2 * S, rlk, l, k0, k1);
    for (int i = 0; i < l; i++) for (uint64_t n = 0; n < N; n++) {
        size_t o = (size_t)i * N + n;
        out[o] = addmod(ct3[o], k0[o], c->q[i]);
        out[S + o] = addmod(ct3[S + o], k1[o], c->q[i]);
    }
    free(k0); free(k1);
}

/* bg:464-485 restated: for g < B: inner = sum_b baby[b] (.) pt[gG+b]; rotate by gG (g>0);
 * accumulate; final rescale. */
void ock_bsgs_loop(const ock_ctx* c, const uint64_t* const* baby, const uint64_t* const* pts,
                   const uint64_t* const* gkeys, int G, int B, int D, int l, uint64_t* out) {
    uint64_t N = c->N; size_t S = (size_t)2 * l * N;
    uint64_t* res = (uint64_t*)malloc(8 * S); int have_res = 0;
    uint64_t* inner = (uint64_t*)malloc(8 * S); uint64_t* term = (uint64_t*)malloc(8 * S);
    uint64_t* rot = (uint64_t*)malloc(8 * S);
    for (int g = 0; g < B; g++) {
        int have = 0;
        for (int b = 0; b < G; b++) {
            int k = g * G + b;
            if (k >= D) continue;
            ock_multiply_plain(c, baby[b], pts[k], term, 2, l);
            if (!have) { memcpy(inner, term, 8 * S); have = 1; }
            else ock_add(c, inner, term, inner, 2, l);
        }
        if (!have) continue;
        uint64_t* cur = inner;
        if (g > 0) {
            ock_rotate(c, inner, gkeys[g], ock_galois_elt_from_step(g * G, N), l, rot);
            cur = rot;
        }
        if (!have_res) { memcpy(res, cur, 8 * S); have_res = 1; }
        else ock_add(c, res, cur, res, 2, l);
    }
    ock_rescale_to_next(c, res, out, 2, l);
    free(res); free(inner); free(term); free(rot);
}

/* ------------------------------------------------------------------ sampling */
static uint64_t reduce128(uint64_t hi, uint64_t lo, uint64_t q) { return (uint64_t)((((u128)hi << 64) | lo) % q); }

/* uniform mod q_i in the NTT domain: (w0 2^64 + w1) mod q from block pi N + n (bias < 2^-67) */
static void sample_uniform_ntt(const ock_ctx* c, const prf_key* K, uint64_t sid, int pi, uint64_t* dst) {
    uint64_t N = c->N, q = c->q[pi];
    for (uint64_t n = 0; n < N; n++) {
        uint64_t w0, w1;
        prf128(K, sid, (uint32_t)((uint64_t)pi * N + n), &w0, &w1);
        dst[n] = reduce128(w0, w1, q);
    }
}
/* switching-key `a` components: exactly uniform by rejection from the top bits of one SplitMix64
 * output per try (spec shared with fhs_modarith.h seeded_uniform_x, regenerated on the GPU inside
 * the key inner product instead of being stored) */
uint64_t ock_seeded_uniform(uint64_t key, int pi, uint64_t n, uint64_t q) {
    const uint64_t G = 0x9E3779B97F4A7C15ULL;
    const int bits = 64 - __builtin_clzll(q);
    const uint64_t kx = key + ((((uint64_t)pi) << 20) | n) * G;
    for (uint64_t m = 0;; m++) {
        uint64_t v = ock_splitmix64(kx + (m << 40) * G) >> (64 - bits);
        if (v < q) return v;
    }
}
static void sample_uniform_seeded(const ock_ctx* c, uint64_t key, int pi, uint64_t* dst) {
    for (uint64_t n = 0; n < c->N; n++) dst[n] = ock_seeded_uniform(key, pi, n, c->q[pi]);
}
/* small samplers: 64 PRF bits (w0 of block n) per coefficient */
static uint64_t prf_small(const prf_key* K, uint64_t sid, uint64_t n) {
    uint64_t w0, w1;
    prf128(K, sid, (uint32_t)n, &w0, &w1);
    return w0;
}
static void sample_ternary(const ock_ctx* c, const prf_key* K, uint64_t sid, int64_t* dst) {
    for (uint64_t n = 0; n < c->N; n++) { uint64_t t = prf_small(K, sid, n) % 3; dst[n] = t == 2 ? -1 : (int64_t)t; }
}
static void sample_cbd(const ock_ctx* c, const prf_key* K, uint64_t sid, int64_t* dst) {
    for (uint64_t n = 0; n < c->N; n++) {
        uint64_t v = prf_small(K, sid, n);
        dst[n] = (int64_t)__builtin_popcountll(v & 0x1FFFFFULL) - (int64_t)__builtin_popcountll((v >> 21) & 0x1FFFFFULL);
    }
}
static void small_to_ntt(const ock_ctx* c, const int64_t* s, int pi, uint64_t* dst) {
    uint64_t q = c->q[pi];
    for (uint64_t n = 0; n < c->N; n++) dst[n] = s[n] >= 0 ? (uint64_t)s[n] % q : q - ((uint64_t)(-s[n]) % q);
    ock_ntt_fwd(c, dst, pi);
}

void ock_gen_secret(const ock_ctx* c, const uint8_t* key32, uint64_t* s_ntt) {
    prf_key K = prf_key_from_bytes(key32);
    int64_t* s = (int64_t*)malloc(8 * c->N);
    sample_ternary(c, &K, stream_id(ST_SECRET, 0, 0), s);
    for (int i = 0; i < c->K; i++) small_to_ntt(c, s, i, s_ntt + (size_t)i * c->N);
    free(s);
}

/* key_j = (-a_j s + e_j + [i in digit j] (P mod q_i) s_new,  a_j) over all L0+P limbs */
void ock_gen_switch_key(const ock_ctx* c, const uint8_t* key32, uint64_t stream_base,
                        const uint64_t* s_ntt, const uint64_t* snew, uint64_t* key) {
    prf_key PK = prf_key_from_bytes(key32);
    uint64_t N = c->N; int K = c->K, P = c->P, L0 = c->L0;
    int dnum = (L0 + P - 1) / P;
    int64_t* e = (int64_t*)malloc(8 * N); uint64_t* et = (uint64_t*)malloc(8 * N);
    for (int j = 0; j < dnum; j++) {
        uint64_t ka = prf_small(&PK, stream_base | (uint64_t)(2 * j), 0);   /* public seed of a_j */
        sample_cbd(c, &PK, stream_base | (uint64_t)(2 * j + 1), e);
        for (int i = 0; i < K; i++) {
            uint64_t q = c->q[i];
            uint64_t* k0 = key + (((size_t)j * 2 + 0) * K + i) * N;
            uint64_t* k1 = key + (((size_t)j * 2 + 1) * K + i) * N;
            sample_uniform_seeded(c, ka, i, k1);
            small_to_ntt(c, e, i, et);
            uint64_t Pm = 1;
            for (int k = 0; k < P; k++) Pm = mulmod(Pm, c->q[L0 + k] % q, q);
            int in_digit = (i < L0) && (i / P == j);
            const uint64_t* s = s_ntt + (size_t)i * N; const uint64_t* sn = snew + (size_t)i * N;
            for (uint64_t n = 0; n < N; n++) {
                uint64_t v = submod(et[n], mulmod(k1[n], s[n], q), q);
                if (in_digit) v = addmod(v, mulmod(Pm, sn[n], q), q);
                k0[n] = v;
            }
        }
    }
    free(e); free(et);
}

void ock_gen_galois_key(const ock_ctx* c, const uint8_t* key32, const uint64_t* s_ntt, uint64_t elt, uint64_t* key) {
    uint64_t N = c->N;
    uint64_t* sn = (uint64_t*)malloc(8 * N * c->K);
    for (int i = 0; i < c->K; i++) ock_apply_galois_ntt(c, s_ntt + (size_t)i * N, sn + (size_t)i * N, elt);
    ock_gen_switch_key(c, key32, stream_id(ST_GALOIS, elt, 0), s_ntt, sn, key);
    free(sn);
}
void ock_gen_relin_key(const ock_ctx* c, const uint8_t* key32, const uint64_t* s_ntt, uint64_t* key) {
    uint64_t N = c->N;
    uint64_t* s2 = (uint64_t*)malloc(8 * N * c->K);
    for (int i = 0; i < c->K; i++)
        for (uint64_t n = 0; n < N; n++) s2[(size_t)i * N + n] = mulmod(s_ntt[(size_t)i * N + n], s_ntt[(size_t)i * N + n], c->q[i]);
    ock_gen_switch_key(c, key32, stream_id(ST_RELIN, 0, 0), s_ntt, s2, key);
    free(s2);
}
void ock_gen_public_key(const ock_ctx* c, const uint8_t* key32, const uint64_t* s_ntt, uint64_t* pk) {
    uint64_t N = c->N; int L0 = c->L0;
    prf_key K = prf_key_from_bytes(key32);
    int64_t* e = (int64_t*)malloc(8 * N); uint64_t* et = (uint64_t*)malloc(8 * N);
    sample_cbd(c, &K, stream_id(ST_PUBKEY, 0, 1), e);
    for (int i = 0; i < L0; i++) {
        uint64_t q = c->q[i]; uint64_t* p0 = pk + (size_t)i * N; uint64_t* p1 = pk + ((size_t)L0 + i) * N;
        sample_uniform_ntt(c, &K, stream_id(ST_PUBKEY, 0, 0), i, p1);
        small_to_ntt(c, e, i, et);
        for (uint64_t n = 0; n < N; n++) p0[n] = submod(et[n], mulmod(p1[n], s_ntt[(size_t)i * N + n], q), q);
    }
    free(e); free(et);
}
void ock_encrypt_symmetric(const ock_ctx* c, const uint8_t* key32, uint64_t counter, const uint64_t* s_ntt,
                           const uint64_t* pt, int l, uint64_t* ct) {
    uint64_t N = c->N; size_t S = (size_t)l * N;
    prf_key K = prf_key_from_bytes(key32);
    int64_t* e = (int64_t*)malloc(8 * N); uint64_t* et = (uint64_t*)malloc(8 * N);
    sample_cbd(c, &K, stream_id(ST_ENC_SYM, counter, 1), e);
    for (int i = 0; i < l; i++) {
        uint64_t q = c->q[i]; uint64_t* c0 = ct + (size_t)i * N; uint64_t* c1 = ct + S + (size_t)i * N;
        sample_uniform_ntt(c, &K, stream_id(ST_ENC_SYM, counter, 0), i, c1);
        small_to_ntt(c, e, i, et);
        for (uint64_t n = 0; n < N; n++)
            c0[n] = addmod(submod(et[n], mulmod(c1[n], s_ntt[(size_t)i * N + n], q), q), pt[(size_t)i * N + n], q);
    }
    free(e); free(et);
}
/* the encryption-mask key of the gen-th public key made from a secret key: 256 PRF bits (w0 of
   blocks 0..3) of stream ST_PK_RNG with a = gen (each public key object draws its own masks) */
void ock_pk_rng_key_gen(const uint8_t* key32, uint64_t gen, uint8_t* rng32) {
    prf_key K = prf_key_from_bytes(key32);
    for (int w = 0; w < 4; w++) {
        uint64_t v = prf_small(&K, stream_id(ST_PK_RNG, gen, 0), (uint64_t)w);
        for (int b = 0; b < 8; b++) rng32[8 * w + b] = (uint8_t)(v >> (8 * b));
    }
}
void ock_pk_rng_key(const uint8_t* key32, uint8_t* rng32) { ock_pk_rng_key_gen(key32, 0, rng32); }
void ock_encrypt_asymmetric(const ock_ctx* c, const uint8_t* rng32, uint64_t counter, const uint64_t* pk,
                            const uint64_t* pt, int l, uint64_t* ct) {
    uint64_t N = c->N; size_t S = (size_t)l * N; int L0 = c->L0;
    prf_key R = prf_key_from_bytes(rng32);
    int64_t* u = (int64_t*)malloc(8 * N); int64_t* e0 = (int64_t*)malloc(8 * N); int64_t* e1 = (int64_t*)malloc(8 * N);
    sample_ternary(c, &R, stream_id(ST_ENC_ASYM, counter, 0), u);
    sample_cbd(c, &R, stream_id(ST_ENC_ASYM, counter, 1), e0);
    sample_cbd(c, &R, stream_id(ST_ENC_ASYM, counter, 2), e1);
    uint64_t* ut = (uint64_t*)malloc(8 * N); uint64_t* t0 = (uint64_t*)malloc(8 * N); uint64_t* t1 = (uint64_t*)malloc(8 * N);
    for (int i = 0; i < l; i++) {
        uint64_t q = c->q[i];
        small_to_ntt(c, u, i, ut); small_to_ntt(c, e0, i, t0); small_to_ntt(c, e1, i, t1);
        const uint64_t* p0 = pk + (size_t)i * N; const uint64_t* p1 = pk + ((size_t)L0 + i) * N;
        for (uint64_t n = 0; n < N; n++) {
            ct[(size_t)i * N + n] = addmod(addmod(mulmod(ut[n], p0[n], q), t0[n], q), pt[(size_t)i * N + n], q);
            ct[S + (size_t)i * N + n] = addmod(mulmod(ut[n], p1[n], q), t1[n], q);
        }
    }
    free(u); free(e0); free(e1); free(ut); free(t0); free(t1);
}
/* pyPhantom.random_plaintexts(ctx, seed, count, ...) plaintext k (the bench's i.i.d. uniform diagonals,
 * not secret): stream key sm(seed ^ sm(7 << 56 | k)); limb i, coefficient n = (rnd(2m) 2^64 + rnd(2m+1))
 * mod q_i with m = i N + n (fhs_kernels.hip k_sample, SAMPLE_TESTDATA). */
void ock_random_plaintext(const ock_ctx* c, uint64_t seed, uint64_t k, int l, uint64_t* out) {
    uint64_t key = ock_splitmix64(seed ^ ock_splitmix64((7ULL << 56) | k)), N = c->N;
    for (int i = 0; i < l; i++)
        for (uint64_t n = 0; n < N; n++) {
            uint64_t ctr = 2 * ((uint64_t)i * N + n);
            out[(size_t)i * N + n] = reduce128(ock_rnd(key, ctr), ock_rnd(key, ctr + 1), c->q[i]);
        }
}
void ock_decrypt(const ock_ctx* c, const uint64_t* s_ntt, const uint64_t* ct, int ncomp, int l, uint64_t* pt) {
    uint64_t N = c->N; size_t S = (size_t)l * N;
    for (int i = 0; i < l; i++) {
        uint64_t q = c->q[i];
        for (uint64_t n = 0; n < N; n++) {
            size_t o = (size_t)i * N + n; uint64_t s = s_ntt[o], sp = s, v = ct[o];
            for (int k = 1; k < ncomp; k++) { v = addmod(v, mulmod(ct[k * S + o], sp, q), q); sp = mulmod(sp, s, q); }
            pt[o] = v;
        }
    }
}

/* ------------------------------------------------------------------ encoder */
/* in-place radix-2 complex DFT of length n: X_k = sum_t x_t exp(sign * 2 pi i t k / n) */
static void cfft(double* re, double* im, int n, int sign) {
    int lg = 0; while ((1 << lg) < n) lg++;
    for (int i = 0; i < n; i++) {
        int r = (int)bitrev((uint32_t)i, lg);
        if (r > i) { double t = re[i]; re[i] = re[r]; re[r] = t; t = im[i]; im[i] = im[r]; im[r] = t; }
    }
    for (int len = 2; len <= n; len <<= 1) {
        double ang = sign * 2.0 * M_PI / len;
        for (int i = 0; i < n; i += len) {
            for (int k = 0; k < len / 2; k++) {
                double wr = cos(ang * k), wi = sin(ang * k);
                int a = i + k, b = i + k + len / 2;
                double xr = re[b] * wr - im[b] * wi, xi = re[b] * wi + im[b] * wr;
                re[b] = re[a] - xr; im[b] = im[a] - xi; re[a] += xr; im[a] += xi;
            }
        }
    }
}

/* exact residue of an integral double */
static uint64_t double_to_mod(double x, uint64_t q) {
    int neg = x < 0; double ax = fabs(x); uint64_t r;
    if (ax < 9.2e18) r = (uint64_t)ax % q;
    else {
        int e; double m = frexp(ax, &e);                 /* ax = m 2^e, m in [0.5,1) */
        uint64_t mant = (uint64_t)ldexp(m, 53);          /* ax = mant * 2^(e-53), e-53 >= 0 */
        r = mulmod(mant % q, powmod(2, (uint64_t)(e - 53), q), q);
    }
    return (neg && r) ? q - r : r;
}

/* pb:138-149 encode_{double,complex}_vector: m(zeta^(5^j)) = scale * z_j, zeta = exp(i pi/N),
 * rounded half away from zero, reduced per limb, forward NTT.  values: n complex (re,im). */
void ock_encode_complex(const ock_ctx* c, const double* z, size_t n, double scale, int l, uint64_t* pt) {
    uint64_t N = c->N, M = 2 * N, slots = N / 2;
    double* re = (double*)calloc(N, 8); double* im = (double*)calloc(N, 8);
    uint64_t e = 1;
    for (uint64_t j = 0; j < slots; j++) {
        double zr = j < n ? z[2 * j] : 0.0, zi = j < n ? z[2 * j + 1] : 0.0;
        re[(e - 1) / 2] = zr; im[(e - 1) / 2] = zi;
        re[(M - e - 1) / 2] = zr; im[(M - e - 1) / 2] = -zi;
        e = (e * 5) & (M - 1);
    }
    cfft(re, im, (int)N, -1);                      /* sum_t v_t w^{-tk} */
    double* coef = (double*)malloc(8 * N);
    for (uint64_t k = 0; k < N; k++) {
        double ang = -M_PI * (double)k / (double)N;  /* zeta^{-k} */
        double v = (re[k] * cos(ang) - im[k] * sin(ang)) / (double)N;
        coef[k] = round(v * scale);
    }
    for (int i = 0; i < l; i++) {
        uint64_t* d = pt + (size_t)i * N;
        for (uint64_t k = 0; k < N; k++) d[k] = double_to_mod(coef[k], c->q[i]);
        ock_ntt_fwd(c, d, i);
    }
    free(re); free(im); free(coef);
}

/* CRT-compose limbs 0..l-1 of one coefficient set into centered doubles */
static void crt_to_double(const ock_ctx* c, uint64_t* const* coefs, int l, double* out) {
    uint64_t N = c->N;
    /* Q and Q/q_i as little-endian word arrays of length l+1 */
    int W = l + 1;
    uint64_t* Q = (uint64_t*)calloc(W, 8); Q[0] = 1;
    for (int i = 0; i < l; i++) {
        u128 carry = 0;
        for (int w = 0; w < W; w++) { u128 t = (u128)Q[w] * c->q[i] + carry; Q[w] = (uint64_t)t; carry = t >> 64; }
    }
    uint64_t* hat = (uint64_t*)calloc((size_t)l * W, 8); uint64_t* ihat = (uint64_t*)malloc(8 * l);
    for (int i = 0; i < l; i++) {
        uint64_t* h = hat + (size_t)i * W; h[0] = 1; uint64_t hm = 1;
        for (int k = 0; k < l; k++) {
            if (k == i) continue;
            u128 carry = 0;
            for (int w = 0; w < W; w++) { u128 t = (u128)h[w] * c->q[k] + carry; h[w] = (uint64_t)t; carry = t >> 64; }
            hm = mulmod(hm, c->q[k] % c->q[i], c->q[i]);
        }
        ihat[i] = invmod(hm, c->q[i]);
    }
    uint64_t* x = (uint64_t*)malloc(8 * (W + 1));
    uint64_t* halfQ = (uint64_t*)malloc(8 * W);
    for (int w = 0; w < W; w++) halfQ[w] = (Q[w] >> 1) | (w + 1 < W ? Q[w + 1] << 63 : 0);
    for (uint64_t n = 0; n < N; n++) {
        memset(x, 0, 8 * (W + 1));
        for (int i = 0; i < l; i++) {
            uint64_t y = mulmod(coefs[i][n], ihat[i], c->q[i]);
            u128 carry = 0; uint64_t* h = hat + (size_t)i * W;
            for (int w = 0; w < W; w++) { u128 t = (u128)h[w] * y + x[w] + carry; x[w] = (uint64_t)t; carry = t >> 64; }
            x[W] += (uint64_t)carry;
            /* reduce: while x >= Q subtract Q (x < l*Q, so a few subtractions) */
            for (;;) {
                int ge = 1;
                if (x[W]) ge = 1;
                else for (int w = W - 1; w >= 0; w--) { if (x[w] != Q[w]) { ge = x[w] > Q[w]; break; } }
                if (!ge) break;
                uint64_t br = 0;
                for (int w = 0; w < W; w++) {
                    uint64_t qa = Q[w] + br; uint64_t nb = (qa < br) || (x[w] < qa);
                    x[w] -= qa; br = nb;
                }
                x[W] -= br;
            }
        }
        int neg = 0;
        for (int w = W - 1; w >= 0; w--) { if (x[w] != halfQ[w]) { neg = x[w] > halfQ[w]; break; } }
        if (neg) {  /* x = Q - x */
            uint64_t br = 0;
            for (int w = 0; w < W; w++) {
                uint64_t xa = x[w] + br; uint64_t nb = (xa < br) || (Q[w] < xa);
                x[w] = Q[w] - xa; br = nb;
            }
        }
        double v = 0;
        for (int w = W - 1; w >= 0; w--) v = v * 18446744073709551616.0 + (double)x[w];
        out[n] = neg ? -v : v;
    }
    free(Q); free(hat); free(ihat); free(x); free(halfQ);
}

void ock_decode_complex(const ock_ctx* c, const uint64_t* pt, int l, double scale, double* z) {
    uint64_t N = c->N, M = 2 * N, slots = N / 2;
    uint64_t** co = (uint64_t**)malloc(sizeof(uint64_t*) * l);
    for (int i = 0; i < l; i++) {
        co[i] = (uint64_t*)malloc(8 * N);
        memcpy(co[i], pt + (size_t)i * N, 8 * N);
        ock_ntt_inv(c, co[i], i);
    }
    double* m = (double*)malloc(8 * N);
    crt_to_double(c, co, l, m);
    double* re = (double*)malloc(8 * N); double* im = (double*)malloc(8 * N);
    for (uint64_t k = 0; k < N; k++) {
        double ang = M_PI * (double)k / (double)N, v = m[k] / scale;
        re[k] = v * cos(ang); im[k] = v * sin(ang);
    }
    cfft(re, im, (int)N, +1);
    uint64_t e = 1;
    for (uint64_t j = 0; j < slots; j++) {
        z[2 * j] = re[(e - 1) / 2]; z[2 * j + 1] = im[(e - 1) / 2];
        e = (e * 5) & (M - 1);
    }
    for (int i = 0; i < l; i++) free(co[i]);
    free(co); free(m); free(re); free(im);
}
