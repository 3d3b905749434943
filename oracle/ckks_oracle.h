/*
 * ckks_oracle.h -- CPU restatement of the CKKS arithmetic behind FHE-SPEAR's BSGS hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product (fhe-spear_amd/, libfhespear_hip.so)
 * never links, loads or calls it.
 *
 * The reference's arithmetic lives in the un-vendored PhantomFHE fork;
 * its Python surface is gpu/phantom_binding.cu (pb) and the callers are
 * scripts/bootstrap_generation.py (bg) and test_fully_enc_bsgs.py (tf).  Every function here
 * cites the reference call site whose semantics it restates.  Limb-level parity against
 * PhantomFHE / SEAL is UNPINNED (neither is available offline); the oracle is
 * pinned by (1) published known answers (SEAL CoeffModulus primes), (2) algebraic identities
 * (NTT = polynomial evaluation, automorphism = X -> X^k), and (3) golden vectors produced by
 * running the reference's own BSGS orchestration (bg:435-485) on this oracle
 * (tests/golden/make_golden.py).
 *
 * Layout (shared with the HIP library's import/export): a polynomial is [limb][N] uint64,
 * NTT form in bit-reversed evaluation order (ock_ntt_fwd); a ciphertext is [comp][limb][N];
 * a switching key is [digit][comp][L0+P key-level limbs][N].
 */
#ifndef CKKS_ORACLE_H
#define CKKS_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ock_ctx ock_ctx;

/* --- deterministic sampling spec (shared with libfhespear_hip) --- */
uint64_t ock_splitmix64(uint64_t x);
uint64_t ock_rnd(uint64_t key, uint64_t ctr);   /* test data only (random plaintexts) */
/* ChaCha20 block (RFC 8439 §2.3): the PRF all secret randomness is drawn from */
void ock_chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], uint32_t out[16]);
/* the public key's encryption-mask key, derived from the secret key's 32 bytes */
void ock_pk_rng_key(const uint8_t* key32, uint8_t* rng32);
void ock_pk_rng_key_gen(const uint8_t* key32, uint64_t gen, uint8_t* rng32);
/* uniform residue mod q from (key, prime index, coefficient) by rejection (switching-key a_j) */
uint64_t ock_seeded_uniform(uint64_t key, int pi, uint64_t n, uint64_t q);

/* SEAL/Phantom CoeffModulus::Create (pb:81 create_coeff_modulus). 0 on success. */
int ock_create_coeff_modulus(uint64_t N, const int* bits, int n, uint64_t* out);
uint64_t ock_galois_elt_from_step(int step, uint64_t N);       /* pb:124-126 */

ock_ctx* ock_ctx_create(uint64_t N, const uint64_t* primes, int nprimes, int special);
/* key-switch convention: 0 exact centred (default), 1 SEAL switch_key_inplace (P = 1); 0 on success */
int ock_ctx_set_ks_mode(ock_ctx* c, int mode);
void ock_ctx_destroy(ock_ctx* c);
int ock_ctx_L0(const ock_ctx* c);
int ock_ctx_P(const ock_ctx* c);
uint64_t ock_ctx_N(const ock_ctx* c);
uint64_t ock_ctx_prime(const ock_ctx* c, int i);                /* key-level index */

/* ---- per-limb transforms (prime index = key-level index) ---- */
void ock_ntt_fwd(const ock_ctx* c, uint64_t* a, int prime_idx);
void ock_ntt_inv(const ock_ctx* c, uint64_t* a, int prime_idx);
void ock_apply_galois_ntt(const ock_ctx* c, const uint64_t* in, uint64_t* out, uint64_t elt);

/* ---- element-wise ciphertext ops (l = number of data limbs at the operand level) ---- */
void ock_add(const ock_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* out, int ncomp, int l);
void ock_sub(const ock_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* out, int ncomp, int l);
void ock_negate(const ock_ctx* c, const uint64_t* a, uint64_t* out, int ncomp, int l);
/* bootstrapping primitives (ckks_bootstrapper, bg:149-154): ModRaise of limb q0 to all L0 limbs;
 * constant product (op 0) / sum into component 0 (op 1) with per-limb residues k[i] */
void ock_mod_raise(const ock_ctx* c, const uint64_t* in, int l, int ncomp, uint64_t* out);
void ock_scalar(const ock_ctx* c, int op, const uint64_t* in, const uint64_t* k, uint64_t* out, int ncomp, int l);
void ock_multiply_plain(const ock_ctx* c, const uint64_t* ct, const uint64_t* pt, uint64_t* out, int ncomp, int l);
void ock_add_plain(const ock_ctx* c, const uint64_t* ct, const uint64_t* pt, uint64_t* out, int ncomp, int l);
void ock_multiply(const ock_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* out3, int l);
/* divide-and-round by q_{l-1}; out has ncomp x (l-1) limbs */
void ock_rescale_to_next(const ock_ctx* c, const uint64_t* in, uint64_t* out, int ncomp, int l);

/* hybrid key-switch of poly a (NTT, l limbs) with key [dnum][2][L0+P][N]; out0/out1 l limbs */
void ock_keyswitch(const ock_ctx* c, const uint64_t* a, const uint64_t* key, int l,
                   uint64_t* out0, uint64_t* out1);
/* exact centred base-extension count (exposed for tests) */
int ock_centered_count_test(const uint64_t* y, const uint64_t* qs, int ns);
/* rotate = galois(elt) + key-switch of c1 (pb:203) */
void ock_rotate(const ock_ctx* c, const uint64_t* ct, const uint64_t* gkey, uint64_t elt, int l, uint64_t* out);
/* nrot rotations of one ciphertext with a single (hoisted) ModUp; identical limbs to ock_rotate */
void ock_rotate_hoisted(const ock_ctx* c, const uint64_t* ct, const uint64_t* const* gkeys, const uint64_t* elts,
                        int nrot, int l, uint64_t* const* outs);
/* relinearize 3-component ct with relin key (pb:183) */
void ock_relinearize(const ock_ctx* c, const uint64_t* ct3, const uint64_t* rlk, int l, uint64_t* out);

/* reference BSGS loop bg:464-485 (fallback semantics of bsgs_multiply_accumulate):
 * baby: G cts at l limbs; pts: D plaintexts at l limbs; gkeys[g] = key for step g*G (g>=1).
 * out: 2 x (l-1) limbs (after the final rescale). */
void ock_bsgs_loop(const ock_ctx* c, const uint64_t* const* baby, const uint64_t* const* pts,
                   const uint64_t* const* gkeys_by_giant, int G, int B, int D, int l, uint64_t* out);

/* ---- keys & encryption (ChaCha20 PRF keyed by the secret key's 32 bytes; deterministic) ---- */
void ock_gen_secret(const ock_ctx* c, const uint8_t* key32, uint64_t* s_ntt /* L0+P limbs */);
void ock_gen_switch_key(const ock_ctx* c, const uint8_t* key32, uint64_t stream_base,
                        const uint64_t* s_ntt, const uint64_t* snew_ntt, uint64_t* key);
void ock_gen_galois_key(const ock_ctx* c, const uint8_t* key32, const uint64_t* s_ntt, uint64_t elt, uint64_t* key);
void ock_gen_relin_key(const ock_ctx* c, const uint8_t* key32, const uint64_t* s_ntt, uint64_t* key);
void ock_gen_public_key(const ock_ctx* c, const uint8_t* key32, const uint64_t* s_ntt, uint64_t* pk /* 2 x L0 */);
void ock_encrypt_symmetric(const ock_ctx* c, const uint8_t* key32, uint64_t counter, const uint64_t* s_ntt,
                           const uint64_t* pt, int l, uint64_t* ct);
/* rng32: ock_pk_rng_key of the secret key (the public key's own mask key) */
void ock_encrypt_asymmetric(const ock_ctx* c, const uint8_t* rng32, uint64_t counter, const uint64_t* pk,
                            const uint64_t* pt, int l, uint64_t* ct);
void ock_decrypt(const ock_ctx* c, const uint64_t* s_ntt, const uint64_t* ct, int ncomp, int l, uint64_t* pt);
/* the bench's random plaintext k of seed (pyPhantom.random_plaintexts, not secret) at l limbs */
void ock_random_plaintext(const ock_ctx* c, uint64_t seed, uint64_t k, int l, uint64_t* out);

/* ---- CKKS encoder (pb:138-156); slots = N/2; values interleaved (re, im) ---- */
void ock_encode_complex(const ock_ctx* c, const double* re_im, size_t n, double scale, int l, uint64_t* pt);
void ock_decode_complex(const ock_ctx* c, const uint64_t* pt, int l, double scale, double* re_im);

#ifdef __cplusplus
}
#endif
#endif
