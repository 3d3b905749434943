// fhs_kernels.h -- launch wrappers for the gfx950 kernels (fhs_kernels.hip).  Host-side only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct PrfKey;   // fhs_modarith.h (ChaCha20 key of the secret-randomness PRF)

namespace fhs {

typedef uint64_t u64;

// Device-resident parameter tables (built once per context, fhs_host.hip).
struct DevTables {
    const void* primes;       // PrimeK[K]
    const u64* tw_fwd;        // [K][N][2]  psi^rev(k), Shoup
    const u64* tw_inv;        // [K][N][2]  psi^-rev(k), Shoup
    const u64* modup_intt;    // [L0+1][L0][4]  INTT stage-0 constants with inv_hat folded in
    const u64* modup_hat;     // [L0+1][dnum][P][K]  (Q_S / q_u) mod prime(t)
    const u64* modup_R;       // [L0+1][dnum][P][2]  floor(2^128 / q_u) (centred-extension count)
    const u64* modup_Q;       // [L0+1][dnum][K][2]  Q_S mod prime(t), ns*Q_S mod prime(t)
    const u64* modup_xd;      // [dnum][32]  X form of full 3-limb digits (k_centered_x): Q_S/q_u (2 words
                              // each), rounding thresholds ((2k-1) Q_S + 1)/2 for k = 1..3, 2^179 - v Q_S
                              // for v = 0..3 (3 words each); null unless P = 3
    const u64* modup_xt;      // [K][4]  per prime m: 2^60 mod m (< 2^30), pack30(2^120 mod m), -2^179 mod m
    const u64* md_xd;         // [32]  X form of ModDown's special digit (k_special_x): P/p_k (2 words each),
                              // thresholds never reached (no centring), 0 offset; null unless md_xform
    const u64* md_intt;       // [P][4]  INTT constants with inv(P/p_k) folded in
    const u64* md_hat;        // [P][L0]  (P / p_k) mod q_i
    const u64* md_pinv;       // [L0][2]  P^-1 mod q_i, Shoup; then [L0] P mod q_i; then [L0] floor(p/2) mod q_i (P = 1)
    const u64* rescale;       // [L0+1][L0][4]  inv(q_{l-1}) mod q_i (+Shoup), half mod q_i, half
    const u64* pow2;          // [K][1088] 2^e mod q_i (exact double reduction)
    const double* enc_w;      // [N/2][2]  omega^-k, omega = exp(2 pi i / (N/2))   (GPU encoder FFT)
    const double* enc_twist;  // [N/2][2]  (2/N) zeta^-k, zeta = exp(i pi / N)
    const unsigned* enc_pos;  // [N/2]     rev_{log N - 1}((5^j mod 2N - 1) / 4): LDS slot of z_j
    const double* dec_w;      // [N/2][2]  omega^k (the host decoder's fft_w[2k], bit for bit)   (GPU decoder FFT)
    const double* dec_twist;  // [N/2][2]  zeta^k (the host decoder's dec_twist)
    const unsigned* dec_pos;  // [N/2]     (5^j mod 2N - 1) / 4: spectrum bin of slot j
    int N, logN, L0, P, K, dnum;
    // key-switch convention: 0 = exact centred ModUp, ModDown without rounding (hoistable; the
    // default); 1 = SEAL's switch_key_inplace (P = 1): per-limb lift without centring, automorphism
    // before the decomposition, ModDown rounded by adding floor(p/2)
    int ks_seal;
    int max_qbits;            // bits of the largest prime (<= 59: split-30 high halves < 2^29, fewer folds)
    int md_xform;             // ModDown converts from the X form (P = 3 special primes < 2^59, modup_dp == 3)
    int conv_b59;             // every prime is 2^59 - d with d < 2^27: the X-form conversions use convert3x_b59
    int all_b59;              // every prime is 2^59 - d with d < 2^27 (any digit shape): the one-limb-digit ModUp
                              // and its ModDown take their B59 instantiations (compile-time lazy NTT, folded stores)
    int modup_dp;             // ModUp conversion compiled for this shape: 3 (P = 3, all targets pseudo-
                              // Mersenne with 2^60 mod m < 2^30: modup_convert3x only, at levels
                              // l % 3 == 0), 1 (P = 1:
                              // modup_convert1), 0 (generic)
};
// The ModUp launch shape and the input form it reads are decided by these two predicates only
// (launch_centered writes the X form exactly when launch_modup's k_modup_h<.., 3> reads it).
#ifndef FHS_MODUP_HALF
#define FHS_MODUP_HALF 1       // k_modup_h: half-limb LDS, two workgroups per CU
#endif
#ifndef FHS_NTT_HALF_MIN
#define FHS_NTT_HALF_MIN 14    // generic NTT kernels use the half-limb form (two workgroups per CU) from this LOGN
#endif
// ModUp runs the half-limb kernel k_modup_h (else the full-limb k_modup, which reads residues + counts)
constexpr bool modup_uses_half(int logN) { return (FHS_MODUP_HALF && logN >= 9) || logN >= FHS_NTT_HALF_MIN; }
// ModUp of level l reads the X form (k_centered_x + modup_convert3x) instead of residues + counts: full
// 3-limb digits on the half-limb kernel's DP = 3 instantiation
inline bool modup_xform(const DevTables& T, int l) { return T.modup_dp == 3 && l % 3 == 0 && modup_uses_half(T.logN); }

// One key-switch of a batch: out = KS_key( galois_elt(a) ) + (galois_elt(add0), add1).
// Items whose `a` is the same polynomial share ONE ModUp (hoisting): the exact centred base
// extension commutes with the automorphism, so the result is bit-identical to a ModUp of
// galois_elt(a).  `src` indexes the batch's list of distinct inputs.
struct KsItem {
    const u64* a;        // poly to switch (NTT form, l limbs), un-permuted
    const u64* add0;     // added to output comp 0 (through `elt`), may be null
    const u64* add1;     // added to output comp 1 (identity), may be null
    const u64* key;      // switching key: b [dnum][K][N], then the dnum seeds of the a_j (SAMPLE_SEEDED)
    u64* out0;           // l limbs
    u64* out1;           // l limbs
    u64 elt;             // galois element (1 = identity)
    u64 src;             // index of `a` in the distinct-input list
    const u64* akey;     // imported key: its a_j [dnum][K][N] (null: a_j regenerated from the seeds)
    const u64* corr;     // SEAL convention, hoisted: the item's correction [2][l+P][N] (launch_seal_corr),
                         // added to the key inner product before ModDown; null otherwise
};

// SEAL-convention hoisting (round 5).  SEAL lifts each data limb of the *automorphed* ciphertext without
// centring, so its extension of sigma(a) differs from sigma applied to the extension of a exactly at the
// coefficients sigma negates: there the lift of -y is q_j - y instead of -y (mod p_t), a difference of
// q_j whenever y != 0.  Summed through the key product that is one data-independent term per (Galois
// element, level): corr_c[t] = NTT_t(mask_sigma) . sum_{j != t} (q_j mod p_t) key_j[c][t], so one ModUp
// of `a` serves every rotation of it, limb for limb equal to SEAL's per-rotation decomposition -- unless a
// digit coefficient is exactly 0 (SEAL lifts 0, not q_j): k_centered flags any zero coefficient, the
// host reads the flag and falls back to the per-rotation decomposition.
struct SealHoist {
    unsigned* zflag_dev;    // set by k_centered when a digit coefficient of an input is 0
    unsigned* zflag_host;   // pinned host word the flag is copied to
    unsigned long long hoisted = 0, fallback = 0;   // flushes taken each way
};
// corr ([2][l+P][N]) of the switching key `key` (akey: explicit a_j, or null) for Galois element elt at
// level l; mask_scratch holds K x N words
hipError_t launch_seal_corr(const DevTables& T, const u64* key, const u64* akey, u64 elt, int l, u64* mask_scratch,
                            u64* out, hipStream_t st);

// Optional per-kernel event timer (bench.py): rec(ctx, id, begin, stream) is called around launches.
enum KernelId { KID_BSGS_INNER = 0, KID_MODUP = 1, KID_KS_IP = 2, KID_MODDOWN = 3, KID_KS_INTT = 4, KID_SPECIAL_INTT = 5,
                KID_GIANT_SUM = 6, KID_GIANT_FINAL = 7, KID_RESCALE = 8, KID_COUNT = 10 };
struct KTimer {
    void* ctx;
    void (*rec)(void* ctx, int id, int begin, hipStream_t st);
};
#define FHS_TMARK(tm, id, b, st) do { if (tm) (tm)->rec((tm)->ctx, (id), (b), (st)); } while (0)

// all launchers enqueue on `st` and return hipSuccess or the first launch error
hipError_t launch_ntt_fwd(const DevTables& T, u64* data, int limbs, int l_split, int npoly, size_t poly_stride,
                          hipStream_t st);
hipError_t launch_ntt_inv(const DevTables& T, u64* data, int limbs, int l_split, int npoly, size_t poly_stride,
                          hipStream_t st);
hipError_t launch_eltwise(const DevTables& T, int op, const u64* a, const u64* b, u64* out, int ncomp, int l,
                          size_t a_cstride, size_t b_cstride, hipStream_t st);
hipError_t launch_tensor(const DevTables& T, const u64* a, const u64* b, u64* out3, int l, hipStream_t st);
hipError_t launch_rescale(const DevTables& T, const u64* in, u64* out, u64* scratch, int ncomp, int l,
                          hipStream_t st, const KTimer* tm = nullptr);
// Stream-ordered host->device copy of small launch descriptors (item lists, pointer arrays).  The
// host side stages through pinned memory so the copy never blocks the calling thread on the GPU
// queue; `src` may be reused as soon as the call returns.
struct Stager {
    void* user;
    hipError_t (*h2d)(void* user, void* dst, const void* src, size_t bytes);
};
// items_host[r].src must index uniq_host (U distinct inputs); items_dev holds >= R items + U pointers
// SEAL convention (T.ks_seal): with `sh` non-null and every rotated item carrying its `corr`, inputs shared by
// several items are decomposed once (hoisted, one stream synchronisation to read the zero flag); otherwise
// every item's automorphed input is decomposed on its own
hipError_t launch_keyswitch(const DevTables& T, const KsItem* items_host, int R, const u64* const* uniq_host, int U,
                            int l, u64* workspace, size_t ws_bytes, void* items_dev, const Stager& sg, hipStream_t st,
                            const KTimer* tm, SealHoist* sh = nullptr);
size_t keyswitch_workspace_bytes(const DevTables& T, int R, int U, int l);

// Hadamard + giant steps of the fused BSGS (fhs_kernels.hip launch_bsgs), enqueued on `st`.
size_t bsgs_workspace_bytes(const DevTables& T, int R, int l);
// giant_elts (host, B entries, may be null): Galois element of giant group g (g >= 1); null means
// 5^(g G) mod 2N (the BSGS matvec of bg:464-485).  Group 0 is never rotated.  pts_dev null: no Hadamard, `inner`
// already holds the B inner products ([g][2][l][N]; giant steps only).
hipError_t launch_bsgs(const DevTables& T, const u64* const* baby_dev, const u64* const* pts_dev, int G, int B, int D,
                       int l, const u64* const* keys_host, const u64* const* akeys_host, const u64* giant_elts, u64* inner,
                       u64* out, u64* workspace, size_t ws_bytes, void* items_dev, const Stager& sg, hipStream_t st,
                       const KTimer* tm, int ptl = 0);
// inner[g] = sum_{b < G, gG + b < D} baby[b] (.) pts[gG + b] for g in [g0, g1) (k_bsgs_inner), inner laid out
// [g][2][l][N].  ptl > 0: pts_dev are compact diagonals (word e >> ptl of each limb of l N >> ptl words holds dense
// word e: the periodic plaintexts' shadow, fhs_host.hip encode_rows_dev), 59-bit chains only.
hipError_t launch_bsgs_inner(const DevTables& T, const u64* const* baby_dev, const u64* const* pts_dev, int G, int g0,
                             int g1, int D, int l, u64* inner, hipStream_t st, int ptl = 0);
// CKKS encode on the GPU: `count` vectors of n values (real, or interleaved re/im), stride doubles
// apart in device memory, to plaintexts outs[0..count) at l limbs, NTT form.
// tlog (device, count bytes, or null): each row's periodicity from launch_enc_period -- rows with tlog > 0 are
// encoded through the sparse form (fhs_kernels.hip k_enc_period).
hipError_t launch_encode(const DevTables& T, const double* vals, int count, size_t n, size_t stride, bool is_real,
                         double scale, u64* const* outs_dev, int l, hipStream_t st,
                         double* coef_scratch = nullptr, const unsigned char* tlog = nullptr,
                         u64* const* couts_dev = nullptr, int ss = 0);
// couts_dev (with coef_scratch and tlog, every row's tlog >= ss >= 1): each plaintext's compact shadow too, l limbs of
// N >> ss words, word e >> ss = dense word e
// per row (n = N/2 values) the largest s <= smax with the row periodic of period (N/2) >> s, into tlog[row]
hipError_t launch_enc_period(const double* vals, int count, size_t n, size_t stride, bool is_real, int smax,
                             unsigned char* tlog, hipStream_t st);
int encode_sparse_max_log(int logN);   // the smax the encoder supports at this ring (0: none)
// dense limbs (l x N) of a compact plaintext (l x N >> tl, word e >> tl = dense word e)
hipError_t launch_expand_compact(const u64* dc, u64* d, int l, int N, int tl, hipStream_t st);
// SAMPLE_UNIFORM / TERNARY / CBD draw from the ChaCha20 PRF stream (K, sid); SAMPLE_SEEDED expands
// the public seed `sid` (switching-key a_j); SAMPLE_TESTDATA is the non-secret SplitMix64 uniform of
// random_plaintexts (K unused)
// A batch of npoly polynomials: polynomial y draws stream sid + y sid_step into outs_dev[y] (device
// pointer array), or out + y l N when outs_dev is null -- the same values as npoly single calls.
hipError_t launch_sample(const DevTables& T, int mode, const ::PrfKey& K, u64 sid, u64* out, int l, hipStream_t st,
                         int npoly = 1, u64 sid_step = 0, u64* const* outs_dev = nullptr);
// b_j = e - a_j s + [limb in digit j] (P mod q) s_new  (switching-key component 0 of digit j)
hipError_t launch_switch_key_assemble(const DevTables& T, u64* b_out, const u64* a, const u64* e_ntt, const u64* s_ntt,
                                      const u64* snew_ntt, int digit, hipStream_t st);
hipError_t launch_galois_perm(const DevTables& T, const u64* in, u64* out, int limbs, u64 elt, hipStream_t st);
// `count` symmetric encryptions: ciphertext y (cts_dev[y]: c0 then c1, l limbs each) of plaintext pts_dev[y]
// with mask stream sid_mask + y sid_step and CBD error stream sid_err + y sid_step -- the values of
// launch_sample (UNIFORM, CBD) + launch_ntt_fwd + launch_encrypt_combine(mode 0) per ciphertext.
// Scratch: small (count x N bytes), eb (count x l x N words).
hipError_t launch_encrypt_sym_batch(const DevTables& T, const ::PrfKey& K, u64 sid_mask, u64 sid_err, u64 sid_step,
                                    u64* const* cts_dev, const u64* s, const u64* const* pts_dev, int count, int l,
                                    signed char* small, u64* eb, hipStream_t st, const double* coef = nullptr);
// coef (count x N rounded message coefficients, launch_encode_coef) instead of pts_dev (null): encode and
// encrypt fused -- the message enters the error's NTT, the same limbs as encoding then encrypting.
hipError_t launch_encode_coef(const DevTables& T, const double* vals, int count, size_t n, size_t stride, bool is_real,
                              double scale, double* coef, hipStream_t st, const unsigned char* tlog = nullptr);
hipError_t launch_encrypt_combine(const DevTables& T, int mode, u64* c0, u64* c1, const u64* s_or_pk0, const u64* pk1,
                                  const u64* u_ntt, const u64* e0, const u64* e1, const u64* pt, int l, hipStream_t st);
hipError_t launch_decrypt(const DevTables& T, const u64* ct, int ncomp, const u64* s, u64* out, int l, hipStream_t st);
// `count` ciphertexts (device pointer array; each ncomp components at l limbs) decrypted to out + i out_stride
hipError_t launch_decrypt_many(const DevTables& T, const u64* const* cts_dev, int count, int ncomp, const u64* s, u64* out,
                               size_t out_stride, int l, hipStream_t st);
hipError_t launch_diag_gather(const double* M1, const double* M2, int D, int G, int n, int k0, int rows, int trans,
                              double* out, hipStream_t st);
// CKKS decode of `count` centred coefficient vectors (m: count x N doubles in HBM) to their first nslots
// slots (out: count x nslots x (re, im)), slot j of vector i = FFT_{N/2}(twist (m_k + i m_{k+N/2}) / scale_i)
// at bin dec_pos[j]; spec: count x N/2 x 2 doubles of scratch.  The host decoder's operations in its order,
// no contraction, so the same doubles (fhs_host.hip decode_slots).  scales: device, count doubles.
hipError_t launch_decode_slots(const DevTables& T, const double* m, const double* scales, int count, double* spec,
                               int nslots, double* out, hipStream_t st);
hipError_t launch_encode_reduce(const DevTables& T, const double* coef, int count, u64* out, int l, hipStream_t st);
hipError_t launch_key_prod(const DevTables& T, const u64* a, const u64* b, u64* out, int limbs, hipStream_t st);
// Centred CRT composition of the first l <= kCrtMaxL limbs (coefficient form) of one polynomial into
// doubles, the exact integer converted word by word from the top (the host decoder's arithmetic,
// fhs_host.hip crt_compose, so both give the same doubles)
constexpr int kCrtMaxL = 7;
struct CrtConsts {
    int l, W;
    u64 q[kCrtMaxL], ihat[kCrtMaxL], ihat_s[kCrtMaxL];
    u64 hat[kCrtMaxL][kCrtMaxL + 1];
    u64 Q[kCrtMaxL + 1], halfQ[kCrtMaxL + 1];
};
// verify (optional, nx > 0): the composed integer x (|x| < Q_l / 2 of the first l limbs, centred) must
// also agree with every further limb -- extra[e][n] (coefficient form) == x mod q_e for e < nx, vtab[e] =
// {q_e, floor(2^128/q_e) lo, hi, (2^64)^w mod q_e for w < W}; any mismatch (x aliased: the coefficient is
// too large for l limbs) sets *flag
hipError_t launch_crt_compose(const CrtConsts& K, const u64* limbs, double* out, int N, hipStream_t st,
                              const u64* extra = nullptr, int nx = 0, const u64* vtab = nullptr,
                              unsigned* flag = nullptr);
constexpr int kCrtVtabWords = 3 + kCrtMaxL + 1;   // per extra limb in vtab
// one composition of a batch (launch_crt_compose_jobs): the arguments of launch_crt_compose in HBM
struct CrtJob {
    CrtConsts K;
    const u64* limbs;
    double* out;
    const u64* extra;
    const u64* vtab;
    unsigned* flag;
    int nx, pad;
};
hipError_t launch_crt_compose_jobs(const CrtJob* jobs_dev, int count, int max_nx, int N, hipStream_t st);

// per-limb constants for k_scalar (value mod q_i and its Shoup companion)
constexpr int kMaxScalarLimbs = 64;
struct ScalarConsts {
    u64 v[kMaxScalarLimbs];
    u64 vs[kMaxScalarLimbs];
};
enum ScalarOp { SCALAR_MUL = 0, SCALAR_ADD = 1 };
hipError_t launch_scalar(const DevTables& T, int op, const u64* a, u64* out, int ncomp, int l, const ScalarConsts& K,
                         hipStream_t st);
// ModRaise (bootstrapping): limb 0 of each component -> centred lift to all L0 data limbs (NTT form)
hipError_t launch_mod_raise(const DevTables& T, const u64* in, int l, u64* out, u64* scratch, int ncomp,
                            hipStream_t st);

// exact 128-bit integer coefficients (x = hi 2^64 + lo) reduced into every limb, then NTT
hipError_t launch_encode_int128(const DevTables& T, const int64_t* hi, const u64* lo, int count, u64* const* outs_dev,
                                int l, hipStream_t st);

enum EltOp { OP_ADD = 0, OP_SUB = 1, OP_NEG = 2, OP_MULP = 3, OP_ADDP = 4, OP_SUBP = 5, OP_SUBNEG = 6 };
enum SampleMode { SAMPLE_UNIFORM = 0, SAMPLE_TERNARY = 1, SAMPLE_CBD = 2, SAMPLE_SEEDED = 3, SAMPLE_TESTDATA = 4 };

}  // namespace fhs
