/*
 * cpu_port.c -- the CPU BASELINE of bench.py (cpu_baseline, kind "port"): the BSGS matvec of
 * scripts/bootstrap_generation.py:464-485 on host cores, written the way SEAL's evaluator does its
 * CPU arithmetic, so the GPU/CPU ratio compares like with like (SURVEY.md §8(d)
 * "the build's own C++ CPU restatement, OpenMP ... labelled as such"):
 *   - Harvey lazy NTT/INTT with Shoup twiddles (forward values in [0, 4q), inverse in [0, 2q));
 *   - Shoup products for every fixed operand (inverse hats, P^-1, q_last^-1), Barrett reduction of
 *     128-bit lazy sums for the Hadamard (46 products per sum) and the key inner product (dnum terms);
 *   - per-rotation (non-hoisted) hybrid key switching, as the reference's CPU path issues rotations:
 *     exact centred ModUp (the same count as oracle/ckks_oracle.c ock_centered_count), key inner
 *     product, ModDown by P;
 *   - OpenMP over the independent rotations / giant groups of the matvec, and over limbs in the
 *     final sum and rescale;
 *   - cpx_set_ks_mode(c, 1): SEAL's switch_key_inplace convention (P = 1, the oracle's
 *     ock_ctx_set_ks_mode(c, 1), ckks_oracle.c:459,486,496): every limb lifted as its residue in
 *     [0, q) (no centring), ModDown rounded by adding floor(p/2) to the special limb and subtracting
 *     floor(p/2) mod q_i after the conversion -- bench.py's seal_mode.cpu_baseline.
 * TEST INFRASTRUCTURE (bench.py's cpu_baseline leg and tests/ only, never the product path).  Its
 * limbs equal the oracle's (tests/test_cpu.py::test_cpu_port_matches_oracle), so the baseline runs
 * the same arithmetic as the GPU path, not an approximation of it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;

typedef struct {
    u64 N;
    int logN, L0, P, K;
    u64* q;                  /* K primes, key-level order */
    u64 *tw, *tws;           /* K x N: psi^rev(k) and Shoup companions (forward) */
    u64 *itw, *itws;         /* K x N: psi^-rev(k) (inverse) */
    u64 *ninv, *ninvs;       /* K */
    u64 *w1ninv, *w1ninvs;   /* K: psi^-rev(1) N^-1 (last inverse stage) */
    u64 *br0, *br1;          /* K: floor(2^128 / q) (Barrett) */
    int ks_seal;             /* 0 exact centred (default), 1 SEAL's switch_key_inplace rounding (P = 1) */
} cpx_ctx;

static inline u64 mulmod(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }
static inline u64 addmod(u64 a, u64 b, u64 q) { u64 s = a + b; return s >= q ? s - q : s; }
static inline u64 submod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }
static u64 powmod(u64 b, u64 e, u64 q) {
    u64 r = 1 % q; b %= q;
    while (e) { if (e & 1) r = mulmod(r, b, q); b = mulmod(b, b, q); e >>= 1; }
    return r;
}
static u64 invmod(u64 a, u64 q) { return powmod(a, q - 2, q); }
static inline u64 shoup_pre(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }
/* w a mod q in [0, 2q) for any 64-bit a */
static inline u64 shoup_lazy(u64 a, u64 w, u64 wp, u64 q) { return a * w - (u64)(((u128)a * wp) >> 64) * q; }
static inline u64 shoup(u64 a, u64 w, u64 wp, u64 q) { u64 r = shoup_lazy(a, w, wp, q); return r >= q ? r - q : r; }
/* Barrett: x mod q for any 128-bit x, r = floor(2^128 / q) = r1 2^64 + r0 */
static inline u64 barrett(u128 x, u64 q, u64 r0, u64 r1) {
    u64 lo = (u64)x, hi = (u64)(x >> 64);
    u128 t = ((u128)lo * r0) >> 64;
    t += (u128)lo * r1;
    u128 t2 = (u128)hi * r0 + (u64)t;
    u64 qest = hi * r1 + (u64)(t >> 64) + (u64)(t2 >> 64);
    u64 r = lo - qest * q;
    while (r >= q) r -= q;
    return r;
}
static inline uint32_t bitrev(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}
static u64 minimal_2n_root(u64 q, u64 N) {   /* the oracle's (and SEAL's) choice of psi */
    u64 m = 2 * N, cof = (q - 1) / m, g = 0;
    for (u64 c = 2;; c++) { g = powmod(c, cof, q); if (powmod(g, N, q) == q - 1) break; }
    u64 g2 = mulmod(g, g, q), best = g, cur = g;
    for (u64 k = 1; k < N; k++) { cur = mulmod(cur, g2, q); if (cur < best) best = cur; }
    return best;
}

cpx_ctx* cpx_create(u64 N, const u64* primes, int nprimes, int special) {
    cpx_ctx* c = (cpx_ctx*)calloc(1, sizeof(cpx_ctx));
    c->N = N; while (((u64)1 << c->logN) < N) c->logN++;
    c->K = nprimes; c->P = special; c->L0 = nprimes - special;
    size_t tab = (size_t)nprimes * N;
    c->q = (u64*)malloc(8 * nprimes);
    memcpy(c->q, primes, 8 * nprimes);
    c->tw = (u64*)malloc(8 * tab); c->tws = (u64*)malloc(8 * tab);
    c->itw = (u64*)malloc(8 * tab); c->itws = (u64*)malloc(8 * tab);
    c->ninv = (u64*)malloc(8 * nprimes); c->ninvs = (u64*)malloc(8 * nprimes);
    c->w1ninv = (u64*)malloc(8 * nprimes); c->w1ninvs = (u64*)malloc(8 * nprimes);
    c->br0 = (u64*)malloc(8 * nprimes); c->br1 = (u64*)malloc(8 * nprimes);
    #pragma omp parallel for schedule(dynamic, 1)
    for (int i = 0; i < nprimes; i++) {
        u64 q = primes[i], psi = minimal_2n_root(q, N), ipsi = invmod(psi, q), pw = 1, ipw = 1;
        u64 *pr = c->tw + (size_t)i * N, *ipr = c->itw + (size_t)i * N;
        for (u64 k = 0; k < N; k++) {
            uint32_t r = bitrev((uint32_t)k, c->logN);
            pr[r] = pw; ipr[r] = ipw;
            pw = mulmod(pw, psi, q); ipw = mulmod(ipw, ipsi, q);
        }
        for (u64 k = 0; k < N; k++) {
            c->tws[(size_t)i * N + k] = shoup_pre(pr[k], q);
            c->itws[(size_t)i * N + k] = shoup_pre(ipr[k], q);
        }
        c->ninv[i] = invmod(N % q, q);
        c->ninvs[i] = shoup_pre(c->ninv[i], q);
        c->w1ninv[i] = mulmod(ipr[1], c->ninv[i], q);
        c->w1ninvs[i] = shoup_pre(c->w1ninv[i], q);
        u128 R = (~(u128)0) / q;   /* floor((2^128 - 1) / q) = floor(2^128 / q) for odd q */
        c->br0[i] = (u64)R; c->br1[i] = (u64)(R >> 64);
    }
    return c;
}
void cpx_destroy(cpx_ctx* c) {
    if (!c) return;
    free(c->q); free(c->tw); free(c->tws); free(c->itw); free(c->itws); free(c->ninv); free(c->ninvs);
    free(c->w1ninv); free(c->w1ninvs);
    free(c->br0); free(c->br1); free(c);
}

/* Harvey forward NTT (Cooley-Tukey, natural -> bit-reversed), input < 4q, output canonical.  The
 * last two stages (butterfly spans 2 and 1) are unrolled per twiddle, and the final reduction to
 * [0, q) is folded into the last stage (SEAL's arrangement). */
static void ntt_fwd(const cpx_ctx* c, u64* a, int pi) {
    const u64 N = c->N, q = c->q[pi], q2 = 2 * q;
    const u64 *W = c->tw + (size_t)pi * N, *Ws = c->tws + (size_t)pi * N;
    u64 t = N, m = 1;
    for (; t > 4; m <<= 1) {
        t >>= 1;
        for (u64 i = 0; i < m; i++) {
            const u64 w = W[m + i], ws = Ws[m + i];
            u64 *x = a + 2 * i * t, *y = x + t;
            for (u64 j = 0; j < t; j++) {
                u64 X = x[j];
                X = X >= q2 ? X - q2 : X;
                const u64 T = shoup_lazy(y[j], w, ws, q);
                x[j] = X + T;
                y[j] = X - T + q2;
            }
        }
    }
    /* t = 2 */
    for (u64 i = 0; i < m; i++) {
        const u64 w = W[m + i], ws = Ws[m + i];
        u64* x = a + 4 * i;
        u64 X0 = x[0], X1 = x[1];
        X0 = X0 >= q2 ? X0 - q2 : X0;
        X1 = X1 >= q2 ? X1 - q2 : X1;
        const u64 T0 = shoup_lazy(x[2], w, ws, q), T1 = shoup_lazy(x[3], w, ws, q);
        x[0] = X0 + T0; x[1] = X1 + T1;
        x[2] = X0 - T0 + q2; x[3] = X1 - T1 + q2;
    }
    m <<= 1;
    /* t = 1, outputs reduced to [0, q) */
    for (u64 i = 0; i < m; i++) {
        const u64 w = W[m + i], ws = Ws[m + i];
        u64* x = a + 2 * i;
        u64 X = x[0];
        X = X >= q2 ? X - q2 : X;
        const u64 T = shoup_lazy(x[1], w, ws, q);
        u64 u = X + T, v = X - T + q2;
        u = u >= q2 ? u - q2 : u;
        v = v >= q2 ? v - q2 : v;
        x[0] = u >= q ? u - q : u;
        x[1] = v >= q ? v - q : v;
    }
}
/* Harvey inverse NTT (Gentleman-Sande, bit-reversed -> natural) with N^-1 folded into the last
 * stage, input < 2q, canonical output */
static void ntt_inv(const cpx_ctx* c, u64* a, int pi) {
    const u64 N = c->N, q = c->q[pi], q2 = 2 * q;
    const u64 *W = c->itw + (size_t)pi * N, *Ws = c->itws + (size_t)pi * N;
    /* t = 1 */
    for (u64 i = 0; i < N / 2; i++) {
        const u64 w = W[N / 2 + i], ws = Ws[N / 2 + i];
        u64* x = a + 2 * i;
        const u64 X = x[0], Y = x[1], s = X + Y;
        x[0] = s >= q2 ? s - q2 : s;
        x[1] = shoup_lazy(X - Y + q2, w, ws, q);
    }
    u64 t = 2;
    for (u64 m = N >> 2; m >= 2; m >>= 1) {
        for (u64 i = 0; i < m; i++) {
            const u64 w = W[m + i], ws = Ws[m + i];
            u64 *x = a + 2 * i * t, *y = x + t;
            for (u64 j = 0; j < t; j++) {
                const u64 X = x[j], Y = y[j];
                const u64 s = X + Y;
                x[j] = s >= q2 ? s - q2 : s;
                y[j] = shoup_lazy(X - Y + q2, w, ws, q);
            }
        }
        t <<= 1;
    }
    /* last stage (m = 1, t = N/2) with N^-1: x = (X + Y) N^-1, y = (X - Y) w N^-1 */
    const u64 ni = c->ninv[pi], nis = c->ninvs[pi], wn = c->w1ninv[pi], wns = c->w1ninvs[pi];
    u64 *x = a, *y = a + N / 2;
    for (u64 j = 0; j < N / 2; j++) {
        const u64 X = x[j], Y = y[j];
        x[j] = shoup(X + Y, ni, nis, q);
        y[j] = shoup(X - Y + q2, wn, wns, q);
    }
}

/* exact centred count v = round(sum_u y_u / q_u) (oracle ock_centered_count, same decisions) */
static int centered_count(const u64* y, const u64* qs, const u64* R0, const u64* R1, int ns) {
    if (ns == 1) return y[0] > (qs[0] >> 1);
    u64 lo = 0; int carry = 0;
    for (int u = 0; u < ns; u++) {
        u64 F = y[u] * R1[u] + (u64)(((u128)y[u] * R0[u]) >> 64);
        lo += F; carry += (lo < F);
    }
    const u64 half = (u64)1 << 63;
    const u64 d = lo >= half ? lo - half : half - lo;
    if (d > 64) return carry + (lo >= half);
    u64 X[10] = {0}, Q[10] = {0}, t[10];
    Q[0] = 1;
    for (int u = 0; u < ns; u++) {
        u128 cy = 0;
        for (int w = 0; w < 10; w++) { u128 z = (u128)Q[w] * qs[u] + cy; Q[w] = (u64)z; cy = z >> 64; }
    }
    for (int u = 0; u < ns; u++) {
        memset(t, 0, sizeof t); t[0] = y[u];
        for (int v = 0; v < ns; v++) {
            if (v == u) continue;
            u128 cy = 0;
            for (int w = 0; w < 10; w++) { u128 z = (u128)t[w] * qs[v] + cy; t[w] = (u64)z; cy = z >> 64; }
        }
        u128 cy = 0;
        for (int w = 0; w < 10; w++) { u128 z = (u128)X[w] + t[w] + cy; X[w] = (u64)z; cy = z >> 64; }
    }
    u64 L[10], Rr[10]; u128 cy = 0;
    for (int w = 0; w < 10; w++) { u128 z = ((u128)X[w] << 1) + cy; L[w] = (u64)z; cy = z >> 64; }
    cy = 0;
    for (int w = 0; w < 10; w++) { u128 z = (u128)Q[w] * (u64)(2 * carry + 1) + cy; Rr[w] = (u64)z; cy = z >> 64; }
    int ge = 1;
    for (int w = 9; w >= 0; w--) { if (L[w] != Rr[w]) { ge = L[w] > Rr[w]; break; } }
    return carry + ge;
}

static inline int ext_prime(const cpx_ctx* c, int l, int i) { return i < l ? i : c->L0 + (i - l); }

/* hybrid key switch of `a` (NTT form, l limbs) with key [dnum][2][K][N] (oracle layout):
 * out0/out1 (l limbs each).  Single-threaded (called from parallel tasks). */
static void keyswitch(const cpx_ctx* c, const u64* a, const u64* key, int l, u64* out0, u64* out1) {
    const u64 N = c->N;
    const int P = c->P, L0 = c->L0, K = c->K, E = l + P, dnum = (l + P - 1) / P;
    u64* ys = (u64*)malloc(8 * N * l);             /* [a_u (Q_S/q_u)^-1]_{q_u}, coefficient form */
    unsigned char* vc = (unsigned char*)malloc((size_t)dnum * N);
    u64* acc = (u64*)malloc(8 * 2 * (size_t)E * N);
    u64* ext = (u64*)malloc(8 * N);
    u128* s0 = (u128*)malloc(16 * N);
    u128* s1 = (u128*)malloc(16 * N);
    u64 R0[64], R1[64];
    for (int i = 0; i < l; i++) { R0[i] = c->br0[i]; R1[i] = c->br1[i]; }
    for (int j = 0; j < dnum; j++) {
        const int b0 = j * P, b1 = b0 + P < l ? b0 + P : l, ns = b1 - b0;
        for (int u = 0; u < ns; u++) {
            const int i = b0 + u;
            const u64 q = c->q[i];
            u64 hat = 1;
            for (int v = 0; v < ns; v++) if (v != u) hat = mulmod(hat, c->q[b0 + v] % q, q);
            const u64 ih = invmod(hat, q), ihs = shoup_pre(ih, q);
            u64* y = ys + (size_t)i * N;
            memcpy(y, a + (size_t)i * N, 8 * N);
            ntt_inv(c, y, i);
            for (u64 n = 0; n < N; n++) y[n] = shoup(y[n], ih, ihs, q);
        }
        for (u64 n = 0; n < N; n++) {
            u64 yy[8];
            for (int u = 0; u < ns; u++) yy[u] = ys[(size_t)(b0 + u) * N + n];
            vc[(size_t)j * N + n] = c->ks_seal ? 0 : (unsigned char)centered_count(yy, c->q + b0, R0 + b0, R1 + b0, ns);
        }
    }
    for (int t = 0; t < E; t++) {
        const int pi = ext_prime(c, l, t);
        const u64 m = c->q[pi], mr0 = c->br0[pi], mr1 = c->br1[pi];
        memset(s0, 0, 16 * N); memset(s1, 0, 16 * N);
        for (int j = 0; j < dnum; j++) {
            const int b0 = j * P, b1 = b0 + P < l ? b0 + P : l, ns = b1 - b0;
            const u64* src;
            if (t >= b0 && t < b1) {
                src = a + (size_t)t * N;   /* own limb of the digit: the input itself */
            } else {
                u64 hm[8], Qm = 1;
                for (int u = 0; u < ns; u++) {
                    u64 h = 1;
                    for (int v = 0; v < ns; v++) if (v != u) h = mulmod(h, c->q[b0 + v] % m, m);
                    hm[u] = h;
                    Qm = mulmod(Qm, c->q[b0 + u] % m, m);
                }
                const u64 nQ[4] = {0, m - Qm, (u64)(((u128)(m - Qm) * 2) % m), (u64)(((u128)(m - Qm) * 3) % m)};
                for (u64 n = 0; n < N; n++) {
                    u128 s = 0;
                    for (int u = 0; u < ns; u++) s += (u128)ys[(size_t)(b0 + u) * N + n] * hm[u];
                    const int v = vc[(size_t)j * N + n];
                    s += v < 4 ? nQ[v] : (u64)(((u128)(m - Qm) * v) % m);   /* X - v Q_S */
                    ext[n] = barrett(s, m, mr0, mr1);
                }
                ntt_fwd(c, ext, pi);
                src = ext;
            }
            const u64* k0 = key + (((size_t)j * 2 + 0) * K + pi) * N;
            const u64* k1 = key + (((size_t)j * 2 + 1) * K + pi) * N;
            for (u64 n = 0; n < N; n++) {
                s0[n] += (u128)src[n] * k0[n];
                s1[n] += (u128)src[n] * k1[n];
            }
        }
        u64* a0 = acc + ((size_t)0 * E + t) * N;
        u64* a1 = acc + ((size_t)1 * E + t) * N;
        for (u64 n = 0; n < N; n++) {
            a0[n] = barrett(s0[n], m, mr0, mr1);
            a1[n] = barrett(s1[n], m, mr0, mr1);
        }
    }
    /* ModDown by P (no rounding term, as ock_keyswitch) */
    u64* yp = (u64*)malloc(8 * N * P);
    for (int comp = 0; comp < 2; comp++) {
        u64* outp = comp ? out1 : out0;
        for (int k = 0; k < P; k++) {
            const int pi = L0 + k;
            const u64 p = c->q[pi];
            u64 hat = 1;
            for (int v = 0; v < P; v++) if (v != k) hat = mulmod(hat, c->q[L0 + v] % p, p);
            const u64 ih = invmod(hat, p), ihs = shoup_pre(ih, p);
            u64* d = yp + (size_t)k * N;
            memcpy(d, acc + ((size_t)comp * E + l + k) * N, 8 * N);
            ntt_inv(c, d, pi);
            for (u64 n = 0; n < N; n++) d[n] = shoup(d[n], ih, ihs, p);
            if (c->ks_seal) for (u64 n = 0; n < N; n++) d[n] = addmod(d[n], p >> 1, p);
        }
        for (int i = 0; i < l; i++) {
            const u64 q = c->q[i];
            u64 hm[8], Pm = 1;
            for (int k = 0; k < P; k++) {
                u64 h = 1;
                for (int v = 0; v < P; v++) if (v != k) h = mulmod(h, c->q[L0 + v] % q, q);
                hm[k] = h; Pm = mulmod(Pm, c->q[L0 + k] % q, q);
            }
            const u64 Pinv = invmod(Pm, q), Pinvs = shoup_pre(Pinv, q);
            const u64 halfq = c->ks_seal ? (c->q[L0] >> 1) % q : 0;
            for (u64 n = 0; n < N; n++) {
                u128 s = 0;
                for (int k = 0; k < P; k++) s += (u128)yp[(size_t)k * N + n] * hm[k];
                ext[n] = submod(barrett(s, q, c->br0[i], c->br1[i]), halfq, q);
            }
            ntt_fwd(c, ext, i);
            const u64* ap = acc + ((size_t)comp * E + i) * N;
            u64* o = outp + (size_t)i * N;
            for (u64 n = 0; n < N; n++) o[n] = shoup(submod(ap[n], ext[n], q), Pinv, Pinvs, q);
        }
    }
    free(ys); free(vc); free(acc); free(ext); free(s0); free(s1); free(yp);
}

/* pb:203 rotate (one rotation, non-hoisted): automorphism, key switch of c1, + sigma(c0) */
void cpx_rotate(const cpx_ctx* c, const u64* ct, const u64* key, u64 elt, int l, u64* out) {
    const u64 N = c->N, m = 2 * N;
    const size_t S = (size_t)l * N;
    u64* r = (u64*)malloc(8 * 2 * S);
    u64* k0 = (u64*)malloc(8 * S);
    for (u64 i = 0; i < N; i++) {
        const u64 e = 2 * (u64)bitrev((uint32_t)i, c->logN) + 1;
        const u64 src = bitrev((uint32_t)((((e * elt) & (m - 1)) - 1) >> 1), c->logN);
        for (int comp = 0; comp < 2; comp++)
            for (int li = 0; li < l; li++) r[(size_t)comp * S + (size_t)li * N + i] = ct[(size_t)comp * S + (size_t)li * N + src];
    }
    keyswitch(c, r + S, key, l, k0, out + S);
    for (int li = 0; li < l; li++)
        for (u64 n = 0; n < N; n++) {
            const size_t o = (size_t)li * N + n;
            out[o] = addmod(r[o], k0[o], c->q[li]);
        }
    free(r); free(k0);
}

/* inner = sum_{b < bmax} baby[b] (.) pts[b]  (bg:465-476), lazy 128-bit sums (< 2^125 for 128 terms) */
static void hadamard(const cpx_ctx* c, const u64* const* baby, const u64* const* pts, int bmax, int l, u64* inner) {
    const u64 N = c->N;
    const size_t S = (size_t)l * N;
    for (int i = 0; i < l; i++) {
        const u64 q = c->q[i], r0 = c->br0[i], r1 = c->br1[i];
        for (u64 n0 = 0; n0 < N; n0 += 256) {
            u128 a0[256], a1[256];
            memset(a0, 0, sizeof a0); memset(a1, 0, sizeof a1);
            for (int b = 0; b < bmax; b++) {
                const u64* p = pts[b] + (size_t)i * N + n0;
                const u64* x0 = baby[b] + (size_t)i * N + n0;
                const u64* x1 = x0 + S;
                for (int n = 0; n < 256; n++) {
                    a0[n] += (u128)x0[n] * p[n];
                    a1[n] += (u128)x1[n] * p[n];
                }
            }
            for (int n = 0; n < 256; n++) {
                inner[(size_t)i * N + n0 + n] = barrett(a0[n], q, r0, r1);
                inner[S + (size_t)i * N + n0 + n] = barrett(a1[n], q, r0, r1);
            }
        }
    }
}

/* pb:185 rescale_to_next (oracle ock_rescale_to_next), parallel over (component, limb) */
static void rescale(const cpx_ctx* c, const u64* in, u64* out, int l) {
    const u64 N = c->N, ql = c->q[l - 1], half = ql >> 1;
    const int last = l - 1;
    u64* tmp = (u64*)malloc(8 * 2 * N);
    for (int k = 0; k < 2; k++) {
        u64* t = tmp + (size_t)k * N;
        memcpy(t, in + ((size_t)k * l + last) * N, 8 * N);
        ntt_inv(c, t, last);
        for (u64 j = 0; j < N; j++) t[j] = addmod(t[j], half, ql);
    }
    #pragma omp parallel for schedule(dynamic, 1) collapse(2)
    for (int k = 0; k < 2; k++)
        for (int i = 0; i < last; i++) {
            const u64 q = c->q[i], hq = half % q, inv = invmod(ql % q, q), invs = shoup_pre(inv, q);
            u64* t2 = (u64*)malloc(8 * N);
            const u64* t = tmp + (size_t)k * N;
            for (u64 j = 0; j < N; j++) t2[j] = submod(t[j] % q, hq, q);
            ntt_fwd(c, t2, i);
            const u64* a = in + ((size_t)k * l + i) * N;
            u64* o = out + ((size_t)k * last + i) * N;
            for (u64 j = 0; j < N; j++) o[j] = shoup(submod(a[j], t2[j], q), inv, invs, q);
            free(t2);
        }
    free(tmp);
}

static u64 elt_of_step(u64 step, u64 N) {
    u64 e = 1;
    for (u64 s = 0; s < step; s++) e = (e * 5) & (2 * N - 1);
    return e;
}

/* The reference loop bg:464-485 with its baby steps bg:215-220: baby_b = rotate(ct, b), b = 1..G-1
 * (baby_keys[b], non-hoisted); y = rescale(sum_g rotate(sum_b baby_b (.) pts[gG+b], gG))
 * (giant_keys[g], g >= 1).  OpenMP: rotations in parallel, then giant groups in parallel.
 * out: 2 x (l-1) x N.  Returns 0. */
int cpx_matvec(const cpx_ctx* c, const u64* ct, int l, const u64* const* baby_keys, const u64* const* giant_keys,
               const u64* const* pts, int G, int B, int D, u64* out) {
    const u64 N = c->N;
    const size_t S = (size_t)l * N;
    u64* baby = (u64*)malloc(8 * 2 * S * G);
    u64* gsum = (u64*)malloc(8 * 2 * S * B);
    memcpy(baby, ct, 8 * 2 * S);
    #pragma omp parallel for schedule(dynamic, 1)
    for (int b = 1; b < G; b++) cpx_rotate(c, ct, baby_keys[b], elt_of_step(b, N), l, baby + (size_t)b * 2 * S);
    #pragma omp parallel for schedule(dynamic, 1)
    for (int g = 0; g < B; g++) {
        int bmax = D - g * G < G ? D - g * G : G;
        const u64* bp[512];
        for (int b = 0; b < bmax; b++) bp[b] = baby + (size_t)b * 2 * S;
        u64* dst = gsum + (size_t)g * 2 * S;
        if (g == 0) {
            hadamard(c, bp, pts, bmax, l, dst);
        } else {
            u64* inner = (u64*)malloc(8 * 2 * S);
            hadamard(c, bp, pts + (size_t)g * G, bmax, l, inner);
            cpx_rotate(c, inner, giant_keys[g], elt_of_step((u64)g * G, N), l, dst);
            free(inner);
        }
    }
    u64* sum = (u64*)malloc(8 * 2 * S);
    #pragma omp parallel for schedule(static)
    for (int li = 0; li < 2 * l; li++) {
        const u64 q = c->q[li % l];
        u64* s = sum + (size_t)li * N;
        memcpy(s, gsum + (size_t)li * N, 8 * N);
        for (int g = 1; g < B; g++) {
            const u64* x = gsum + (size_t)g * 2 * S + (size_t)li * N;
            for (u64 n = 0; n < N; n++) s[n] = addmod(s[n], x[n], q);
        }
    }
    rescale(c, sum, out, l);
    free(baby); free(gsum); free(sum);
    return 0;
}

int cpx_threads(void) { return omp_get_max_threads(); }
int cpx_set_ks_mode(cpx_ctx* c, int mode) {
    if (mode && c->P != 1) return -1;   /* SEAL's convention has one special prime */
    c->ks_seal = mode != 0;
    return 0;
}
void cpx_set_threads(int n) { if (n > 0) omp_set_num_threads(n); }

/* exported single transforms (tests and timing) */
void cpx_ntt_fwd(const cpx_ctx* c, u64* a, int pi) { ntt_fwd(c, a, pi); }
void cpx_ntt_inv(const cpx_ctx* c, u64* a, int pi) { ntt_inv(c, a, pi); }
