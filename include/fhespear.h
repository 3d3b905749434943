/*
 * fhespear.h -- C ABI of libfhespear_hip.so, the MI355X-native CKKS engine behind FHE-SPEAR's
 * BSGS diagonal matrix-vector path.
 *
 * It replaces gpu/phantom_binding.cu (the pybind11 module `pyPhantom`, pb) and the un-vendored
 * PhantomFHE arithmetic under it.  Each entry point names the reference binding/call site it
 * stands in for.  The Python module fhe-spear_amd/python/pyPhantom binds these with ctypes
 * (INTEGRATION.md shows the binding and the fhe_common.py switch).
 *
 * Conventions
 *  - Plain pointers and sizes only; objects are opaque handles freed with *_destroy.
 *  - Every function returns an fhs_status (0 = OK); fhs_last_error() returns a thread-local
 *    message for the last failure.  FHS_ERR_OOM messages contain "out of memory" (the reference
 *    string-matches that text, scripts/bootstrap_generation.py:1164-1166).
 *  - Ciphertexts/plaintexts are device-resident in HBM: [comp][limb][N] uint64, NTT form,
 *    bit-reversed evaluation order.  chain_index c holds L0 + 1 - c data limbs (pb:144, tf:33).
 *  - All work is ordered on one HIP stream per context; calls are serialised per context and
 *    are safe from several host threads (bg:223-249).  Functions that return host data
 *    synchronise the stream.
 */
#ifndef FHESPEAR_H
#define FHESPEAR_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int fhs_status;
enum {
    FHS_OK = 0,
    FHS_ERR_INVALID = 1,      /* bad argument / unsupported parameter */
    FHS_ERR_OOM = 2,          /* device or host allocation failed ("out of memory") */
    FHS_ERR_HIP = 3,          /* HIP runtime error */
    FHS_ERR_LEVEL = 4,        /* operands at different chain indices / no level left */
    FHS_ERR_SCALE = 5,        /* scale mismatch on add */
    FHS_ERR_KEY = 6,          /* missing Galois key for a rotation step */
    FHS_ERR_NODEVICE = 7      /* no HIP device available */
};

typedef struct fhs_context fhs_context;
typedef struct fhs_ciphertext fhs_ciphertext;
typedef struct fhs_plaintext fhs_plaintext;
typedef struct fhs_secret_key fhs_secret_key;
typedef struct fhs_public_key fhs_public_key;
typedef struct fhs_relin_key fhs_relin_key;
typedef struct fhs_galois_keys fhs_galois_keys;

const char* fhs_last_error(void);
const char* fhs_version(void);
int fhs_device_count(void);
/* PCI bus id of HIP device `device` (e.g. "0000:05:00.0"), for the multi-rank line's device check.  Replaces
 * no pb symbol (extension). */
fhs_status fhs_device_pci_bus_id(int device, char* buf, int len);
/* Testing hook (extension, replaces no pb symbol): the next `count` flushes of queued rotations on `ctx` fail as
 * out of memory before launching, so the drop-the-queue path (queued outputs marked lost, later uses rejected)
 * can be exercised without exhausting HBM. */
fhs_status fhs_debug_fail_next_flushes(fhs_context* ctx, int count);

/* ---- parameters (pb:78-98) ---- */
/* pb:81 create_coeff_modulus: SEAL CoeffModulus::Create (largest primes = 1 mod 2N per size) */
fhs_status fhs_create_coeff_modulus(uint64_t N, const int* bit_sizes, int n, uint64_t* primes_out);
/* pb:124-126 get_elt_from_step(s): 5^s mod 2N (s<0 -> 5^(N/2-|s|), s=0 -> 2N-1) */
uint64_t fhs_galois_elt_from_step(int step, uint64_t N);

/* pb:85-98 params + context(params).  primes: key-level list, the last `special` are the
 * special primes; galois_elts: the set create_galois_keys will generate (NULL/0 = default
 * power-of-two steps + conjugation, as Phantom does when set_galois_elts is not called). */
fhs_status fhs_context_create(uint64_t N, const uint64_t* primes, int nprimes, int special,
                              const uint64_t* galois_elts, int n_elts, int device, fhs_context** out);
fhs_status fhs_context_destroy(fhs_context* ctx);
fhs_status fhs_context_info(const fhs_context* ctx, uint64_t* N, int* L0, int* P, int* n_elts);
fhs_status fhs_context_galois_elts(const fhs_context* ctx, uint64_t* elts_out);
fhs_status fhs_synchronize(fhs_context* ctx);
/* bytes currently held by the context's device pool (diagnostics) */
fhs_status fhs_memory_in_use(fhs_context* ctx, uint64_t* bytes);

/* ---- keys (pb:100-124) ---- */
/* pb:100 secret_key(ctx).  All secret randomness is ChaCha20 keyed by key32:
 * deterministic for a caller-supplied key (tests: the integer seed, 32 bytes little-endian). */
fhs_status fhs_secret_key_create(fhs_context* ctx, const uint8_t* key32 /* 32 bytes, NULL: /dev/urandom */,
                                 fhs_secret_key** out);
fhs_status fhs_secret_key_destroy(fhs_secret_key* sk);
fhs_status fhs_gen_public_key(fhs_context* ctx, fhs_secret_key* sk, fhs_public_key** out);      /* pb:102 */
fhs_status fhs_gen_relin_key(fhs_context* ctx, fhs_secret_key* sk, fhs_relin_key** out);        /* pb:103 */
/* pb:104 create_galois_keys: keys for elts (NULL/0 = the context's set) */
fhs_status fhs_create_galois_keys(fhs_context* ctx, fhs_secret_key* sk, const uint64_t* elts, int n,
                                  fhs_galois_keys** out);
fhs_status fhs_public_key_destroy(fhs_public_key* pk);
fhs_status fhs_relin_key_destroy(fhs_relin_key* rk);
fhs_status fhs_galois_keys_destroy(fhs_galois_keys* gk);
fhs_status fhs_galois_keys_has(const fhs_galois_keys* gk, uint64_t elt, int* has);
/* export one switching key [dnum][2][L0+P][N] (parity tests) */
fhs_status fhs_galois_key_export(fhs_context* ctx, const fhs_galois_keys* gk, uint64_t elt, uint64_t* host);
fhs_status fhs_relin_key_export(fhs_context* ctx, const fhs_relin_key* rk, uint64_t* host);
fhs_status fhs_secret_key_export(fhs_context* ctx, const fhs_secret_key* sk, uint64_t* host /* [L0+P][N] */);
/* Key import in the export layout ("identical Galois keys": a key set made elsewhere, e.g. SEAL's
 * KSwitchKeys with key_vector[j].data(0|1), P = 1).  Residues must be canonical.  Imported keys keep
 * their a_j explicitly (generated keys regenerate them from seeds).  Replaces no pb symbol: the
 * binding had no import; TenSEAL's key loading is the analogue. */
fhs_status fhs_galois_keys_import(fhs_context* ctx, const uint64_t* elts, int n,
                                  const uint64_t* host /* [n][dnum][2][L0+P][N] */, fhs_galois_keys** out);
fhs_status fhs_relin_key_import(fhs_context* ctx, const uint64_t* host /* [dnum][2][L0+P][N] */, fhs_relin_key** out);
fhs_status fhs_secret_key_import(fhs_context* ctx, const uint64_t* host /* [L0+P][N], NTT form */,
                                 fhs_secret_key** out);
/* Key-switch convention: FHS_KS_EXACT (default; exact centred ModUp, ModDown without
 * rounding, hoistable) or FHS_KS_SEAL (P = 1 only: SEAL's switch_key_inplace -- per-limb lift without
 * centring, automorphism before the decomposition, ModDown rounded by adding floor(p/2)). */
#define FHS_KS_EXACT 0
#define FHS_KS_SEAL 1
fhs_status fhs_context_set_key_switch_mode(fhs_context* ctx, int mode);
fhs_status fhs_context_key_switch_mode(const fhs_context* ctx, int* mode);
/* SEAL convention: batched rotations of one ciphertext share one decomposition (the same limbs as SEAL's
 * per-rotation decomposition via a per-(Galois key, level) correction); a digit coefficient
 * equal to 0 falls back to the per-rotation path.  Counts of flushes taken each way. */
fhs_status fhs_seal_hoist_stats(fhs_context* ctx, uint64_t* hoisted, uint64_t* fallback);
fhs_status fhs_public_key_export(fhs_context* ctx, const fhs_public_key* pk, uint64_t* host /* [2][L0][N] */);
fhs_status fhs_galois_keys_bytes(const fhs_galois_keys* gk, uint64_t* bytes);

/* ---- objects (pb:157-163) ---- */
fhs_status fhs_ciphertext_destroy(fhs_ciphertext* ct);
fhs_status fhs_plaintext_destroy(fhs_plaintext* pt);
fhs_status fhs_ciphertext_info(const fhs_ciphertext* ct, int* ncomp, int* chain_index, int* nlimbs, double* scale);
fhs_status fhs_ciphertext_set_scale(fhs_ciphertext* ct, double scale);                              /* pb:163 */
fhs_status fhs_plaintext_info(const fhs_plaintext* pt, int* chain_index, int* nlimbs, double* scale);
fhs_status fhs_ciphertext_export(fhs_context* ctx, const fhs_ciphertext* ct, uint64_t* host);
fhs_status fhs_ciphertext_import(fhs_context* ctx, const uint64_t* host, int ncomp, int chain_index, double scale,
                                 fhs_ciphertext** out);
fhs_status fhs_plaintext_export(fhs_context* ctx, const fhs_plaintext* pt, uint64_t* host);
fhs_status fhs_plaintext_import(fhs_context* ctx, const uint64_t* host, int chain_index, double scale,
                                fhs_plaintext** out);
/* device pointer of the limb data (zero-copy interop with torch / RCCL) */
fhs_status fhs_ciphertext_device_ptr(const fhs_ciphertext* ct, void** dptr, uint64_t* bytes);

/* ---- CKKS encoder (pb:128-156) ---- */
/* values: n complex numbers interleaved (re, im); n <= N/2, zero padded.  pb:141-149 */
fhs_status fhs_encode(fhs_context* ctx, const double* re_im, size_t n, double scale, int chain_index,
                      fhs_plaintext** out);
/* batch: count vectors of n complex values each (bg:382 encode_*_vector_batch).
 * Lifetime (every batch creator: encode batches, random_plaintexts, upload_plaintexts, encode_matrix_diagonals):
 * the plaintexts of one call share one device block (a slab of up to 1.5x the request, reused from the cache),
 * returned to the cache only when the LAST of them is destroyed -- keeping one diagonal of a batch keeps the whole
 * batch's HBM, and fhs_context memory_in_use counts the slab as long as any of them lives.  Destroy batches as
 * a whole, or create plaintexts that must outlive their batch with a single-plaintext call. */
fhs_status fhs_encode_batch(fhs_context* ctx, const double* re_im, size_t count, size_t n, double scale,
                            int chain_index, fhs_plaintext** out_array);
/* real-valued fast paths: values are n doubles */
fhs_status fhs_encode_real(fhs_context* ctx, const double* values, size_t n, double scale, int chain_index,
                           fhs_plaintext** out);
fhs_status fhs_encode_real_batch(fhs_context* ctx, const double* values, size_t count, size_t n, double scale,
                                 int chain_index, fhs_plaintext** out_array);
/* pb:150-156 decode: writes N/2 complex (re, im) */
fhs_status fhs_decode(fhs_context* ctx, const fhs_plaintext* pt, double* re_im_out);
/* decode of `count` plaintexts with one device synchronisation (the client's decrypt_vec of a block
 * stage, bg:784-892): the first `nslots` slots of each, re_im_out = count x nslots x (re, im); the same
 * doubles as fhs_decode */
fhs_status fhs_decode_batch(fhs_context* ctx, const fhs_plaintext* const* pts, int count, int nslots,
                            double* re_im_out);

/* ---- encryption (pb:105-116) ---- */
fhs_status fhs_encrypt_symmetric(fhs_context* ctx, fhs_secret_key* sk, const fhs_plaintext* pt, fhs_ciphertext** out);
/* `count` symmetric encryptions in one pass (the client's inputs of a block stage, bg:784-892): the same
 * ciphertexts as `count` fhs_encrypt_symmetric calls in order (each takes the key's next encryption
 * counter); the samplers and NTTs run once over the whole batch */
fhs_status fhs_encrypt_symmetric_batch(fhs_context* ctx, fhs_secret_key* sk, const fhs_plaintext* const* pts, int count,
                                       fhs_ciphertext** out_array);
/* Extension: encode `count` vectors of n values (is_real: n doubles each; else n interleaved (re, im)) at
 * `scale` / `chain_index` and encrypt them with sk in one pass -- the same ciphertexts as
 * fhs_encode[_real]_batch + fhs_encrypt_symmetric_batch (no plaintext objects; count <= 4096) */
fhs_status fhs_encode_encrypt_symmetric_batch(fhs_context* ctx, fhs_secret_key* sk, const double* values, size_t count,
                                              size_t n, int is_real, double scale, int chain_index,
                                              fhs_ciphertext** out_array);
/* Extension: decrypt `count` ciphertexts with sk and decode the first `nslots` slots of each (re_im_out =
 * count x nslots x (re, im)) -- the doubles of fhs_decrypt + fhs_decode_batch, without the plaintexts */
fhs_status fhs_decrypt_decode_batch(fhs_context* ctx, fhs_secret_key* sk, const fhs_ciphertext* const* cts, int count,
                                    int nslots, double* re_im_out);
fhs_status fhs_encrypt_asymmetric(fhs_context* ctx, fhs_public_key* pk, const fhs_plaintext* pt, fhs_ciphertext** out);
fhs_status fhs_decrypt(fhs_context* ctx, fhs_secret_key* sk, const fhs_ciphertext* ct, fhs_plaintext** out);

/* ---- evaluator (pb:165-205); every op returns a NEW object ---- */
fhs_status fhs_add(fhs_context* ctx, const fhs_ciphertext* a, const fhs_ciphertext* b, fhs_ciphertext** out);       /* pb:167 */
fhs_status fhs_sub(fhs_context* ctx, const fhs_ciphertext* a, const fhs_ciphertext* b, int negate, fhs_ciphertext** out); /* pb:173 */
fhs_status fhs_negate(fhs_context* ctx, const fhs_ciphertext* a, fhs_ciphertext** out);                            /* pb:165 */
fhs_status fhs_add_plain(fhs_context* ctx, const fhs_ciphertext* a, const fhs_plaintext* p, fhs_ciphertext** out);  /* pb:169 */
fhs_status fhs_sub_plain(fhs_context* ctx, const fhs_ciphertext* a, const fhs_plaintext* p, fhs_ciphertext** out);  /* pb:175 */
fhs_status fhs_multiply_plain(fhs_context* ctx, const fhs_ciphertext* a, const fhs_plaintext* p, fhs_ciphertext** out); /* pb:181 */
fhs_status fhs_multiply(fhs_context* ctx, const fhs_ciphertext* a, const fhs_ciphertext* b, fhs_ciphertext** out);  /* pb:177 */
fhs_status fhs_relinearize(fhs_context* ctx, const fhs_ciphertext* a, const fhs_relin_key* rk, fhs_ciphertext** out); /* pb:183 */
fhs_status fhs_rescale_to_next(fhs_context* ctx, const fhs_ciphertext* a, fhs_ciphertext** out);                   /* pb:185 */
fhs_status fhs_mod_switch_to_next(fhs_context* ctx, const fhs_ciphertext* a, fhs_ciphertext** out);                /* pb:191-193 */
fhs_status fhs_mod_switch_to(fhs_context* ctx, const fhs_ciphertext* a, int chain_index, fhs_ciphertext** out);    /* pb:198-199 */
fhs_status fhs_plain_mod_switch_to_next(fhs_context* ctx, const fhs_plaintext* a, fhs_plaintext** out);            /* pb:187-189 */
fhs_status fhs_plain_mod_switch_to(fhs_context* ctx, const fhs_plaintext* a, int chain_index, fhs_plaintext** out);/* pb:195-196 */
/* pb:203 rotate: left rotation of the N/2 slots by `step` (bg:219, bg:479) */
fhs_status fhs_rotate(fhs_context* ctx, const fhs_ciphertext* a, int step, const fhs_galois_keys* gk, fhs_ciphertext** out);
/* pb:201 apply_galois with an explicit element */
fhs_status fhs_apply_galois(fhs_context* ctx, const fhs_ciphertext* a, uint64_t elt, const fhs_galois_keys* gk,
                            fhs_ciphertext** out);
/* batch of rotations of possibly different inputs: out[i] = rotate(in[i], steps[i]) */
fhs_status fhs_rotate_many(fhs_context* ctx, const fhs_ciphertext* const* in, const int* steps, int n,
                           const fhs_galois_keys* gk, fhs_ciphertext** out);

/* ---- fused BSGS (fork-only pyPhantom symbols, bg:459, bg:515) ----
 * Semantics identical, limb for limb, to the loop scripts/bootstrap_generation.py:464-485:
 *   out = rescale( sum_g rot_{gG}( sum_{b: gG+b<D} baby[b] (.) pts[gG+b] ) )
 * baby: G ciphertexts (baby[b] = rot_b(x)); pts: D plaintexts at the baby steps' level. */
fhs_status fhs_bsgs_multiply_accumulate(fhs_context* ctx, const fhs_ciphertext* const* baby, int G,
                                        const fhs_plaintext* const* pts, int D, int B,
                                        const fhs_galois_keys* gk, fhs_ciphertext** out);
/* host staging of pre-encoded diagonals (bg:336-358: offload_plaintexts / upload_plaintexts).
 * host buffer holds count x nlimbs x N uint64 (pinned when allocated by fhs_host_alloc). */
fhs_status fhs_offload_plaintexts(fhs_context* ctx, const fhs_plaintext* const* pts, int count, uint64_t* host);
fhs_status fhs_upload_plaintexts(fhs_context* ctx, const uint64_t* host, int count, int chain_index, double scale,
                                 fhs_plaintext** out_array);
/* bg:449 bsgs_from_cpu: streams diagonals from host memory through the BSGS */
fhs_status fhs_bsgs_from_cpu(fhs_context* ctx, const fhs_ciphertext* const* baby, int G, const uint64_t* host,
                             int D, int B, int chain_index, double scale, const fhs_galois_keys* gk,
                             fhs_ciphertext** out);
fhs_status fhs_host_alloc(uint64_t bytes, void** ptr);   /* pinned host memory */
fhs_status fhs_host_free(void* ptr);

/* ---- CKKS bootstrapping primitives (ckks_bootstrapper, bg:72-74, 110-116, 149-154; tf:243-262;
 * the fork's C++ bootstrapper behind pb is un-vendored) ----
 * Generalised fused BSGS linear transform (CoeffToSlot / SlotToCoeff groups):
 *   out = [rescale]( sum_{g<B} galois_{giant_elts[g]}( sum_{b<G} baby[b] (.) pts[g G + b] ) )
 * D = B * G plaintexts; giant_elts[0] must be 1 (identity group).  rescale = 0 keeps the product
 * scale (baby scale x plaintext scale) and the level. */
fhs_status fhs_linear_transform(fhs_context* ctx, const fhs_ciphertext* const* baby, int G,
                                const fhs_plaintext* const* pts, int D, int B, const uint64_t* giant_elts,
                                const fhs_galois_keys* gk, int rescale, fhs_ciphertext** out);
/* Extension (no reference symbol): the Hadamard half of fhs_bsgs_multiply_accumulate on its own --
 * outs[g] = sum_{b < G} baby[b] (.) pts[g G + b] for g < B (bg:465-476 per giant group), NOT rotated and
 * NOT rescaled (scale baby * pt).  The baby-step-sharded latency mode (fhespear_dist.bsgs_baby_sharded)
 * forms every giant group's partial inner product over a rank's share of the baby steps with it.
 * outs: B new ciphertexts. */
fhs_status fhs_bsgs_inner_products(fhs_context* ctx, const fhs_ciphertext* const* baby, int G,
                                   const fhs_plaintext* const* pts, int B, fhs_ciphertext** outs);
/* Extension (no reference symbol): the giant-step half of fhs_bsgs_multiply_accumulate (bg:478-483):
 * out = sum_j rot_{elts[j]}(inners[j]) for k 2-component ciphertexts at one chain index and scale, the k
 * key switches summed before one ModDown, NOT rescaled.  elts[0] may be 1 (unrotated term); no other.
 * The baby-step-sharded latency mode finishes a rank's giant groups with it.  out: 1 new ciphertext. */
fhs_status fhs_bsgs_giant_steps(fhs_context* ctx, const fhs_ciphertext* const* inners, int k, const uint64_t* elts,
                                const fhs_galois_keys* gk, fhs_ciphertext** out);
/* Extensions (no reference symbol): the two halves over caller device memory, for the grid-sharded
 * latency mode's reduce-scatter buffers -- fhs_bsgs_inner_products writing group g at dst + g 2 l N words,
 * and fhs_bsgs_giant_steps reading term j at src + j 2 l N words (l = L0 + 1 - chain_index).  Both are
 * ordered on the context's stream (fhs_context_stream); the caller orders its own streams around them. */
fhs_status fhs_bsgs_inner_products_device(fhs_context* ctx, const fhs_ciphertext* const* baby, int G,
                                          const fhs_plaintext* const* pts, int B, uint64_t* dst);
fhs_status fhs_bsgs_giant_steps_device(fhs_context* ctx, const uint64_t* src, int k, int chain_index, double scale,
                                       const uint64_t* elts, const fhs_galois_keys* gk, fhs_ciphertext** out);
/* Extension (no reference symbol): bg:198-203 + bg:361-432 on the device -- the D diagonals of the
 * D x D row-major matrix M1 (complex: M1 + i M2; M2 = NULL for real), group g = k / G rolled by g G,
 * tiled to N/2 slots, encoded at `scale` / `chain_index`.  Limb-identical to encode_*_vector_batch
 * of the host-prepared rows; uploads D^2 doubles instead of D x N/2.  out_array: D plaintexts. */
fhs_status fhs_encode_diagonals(fhs_context* ctx, const double* M1, const double* M2, int D, int G, double scale,
                                int chain_index, fhs_plaintext** out_array);
/* the same for a strided or transposed view: row r of the D x D block starts at A + r * ld (ld >= D);
 * trans = 1 means the block holds M^T (M[m][c] = A[c * ld + m]), e.g. numpy's W[:, lo:hi].T */
fhs_status fhs_encode_diagonals_ex(fhs_context* ctx, const double* A1, const double* A2, int64_t ld, int trans, int D,
                                   int G, double scale, int chain_index, fhs_plaintext** out_array);
/* only the diagonals rows[0..nrows) (indices < D, any order; out_array[k] is diagonal rows[k]): the rows one
 * rank of a sharded matvec needs (fhespear_dist giant_groups / grid_rows) -- limb-identical to the same
 * plaintexts of the full encode */
fhs_status fhs_encode_diagonals_rows(fhs_context* ctx, const double* A1, const double* A2, int64_t ld, int trans, int D,
                                     int G, double scale, int chain_index, const int* rows, int nrows,
                                     fhs_plaintext** out_array);
/* encode_complex_vector_batch with an extended-precision (long double) canonical-embedding FFT on the
 * host and exact 128-bit rounding: for constant plaintexts whose f64 encoding error (~2^-52 log n
 * relative) matters -- the bootstrap's CoeffToSlot / SlotToCoeff diagonals.  |values x scale| < 2^126. */
fhs_status fhs_encode_precise(fhs_context* ctx, const double* re_im, size_t count, size_t n, double scale,
                              int chain_index, fhs_plaintext** out_array);
/* out = a * c with the integer c = round(value * const_scale) (half away from zero, exact for any
 * finite double); out scale = a.scale * const_scale */
fhs_status fhs_multiply_const(fhs_context* ctx, const fhs_ciphertext* a, double value, double const_scale,
                              fhs_ciphertext** out);
/* out = a + round(value * a.scale) (added to component 0; scale unchanged) */
fhs_status fhs_add_const(fhs_context* ctx, const fhs_ciphertext* a, double value, fhs_ciphertext** out);
/* ModRaise: limb q0 of a (any level) lifted centred to all L0 data limbs; out at chain index 1,
 * same scale (decrypts to m + q0 I) */
fhs_status fhs_mod_raise(fhs_context* ctx, const fhs_ciphertext* a, fhs_ciphertext** out);
/* ckks_bootstrapper EvalMod (pyPhantom/bootstrap.py Bootstrapper._evalmod, the same op sequence):
 * cos / sin Chebyshev series cc, cs (ncoef coefficients each, scale-exact split, landing at chain
 * index y + cheb_depth at y's scale) on one basis, then r complex squarings; out = sin(2 pi K y) */
fhs_status fhs_bootstrap_evalmod(fhs_context* ctx, const fhs_ciphertext* y, const fhs_relin_key* rk,
                                 const double* cc, const double* cs, int ncoef, int r, int cheb_depth,
                                 fhs_ciphertext** out);

/* ---- measurement hooks (bench.py) ---- */
/* fill n plaintexts with i.i.d. uniform limbs mod q_i (SURVEY.md §8d throughput workload) */
fhs_status fhs_random_plaintexts(fhs_context* ctx, uint64_t seed, int count, int chain_index, double scale,
                                 fhs_plaintext** out_array);
/* HIP events on the context stream: record returns an opaque id usable with fhs_event_elapsed */
fhs_status fhs_event_record(fhs_context* ctx, void** ev);
fhs_status fhs_event_elapsed(void* start, void* stop, float* ms);
fhs_status fhs_event_destroy(void* ev);
/* Per-kernel device time from HIP events recorded on the context stream around each launch.
 * Kernel ids: 0 k_bsgs_inner (ct x pt Hadamard-accumulate), 1 k_modup (ModUp + NTT), 2 k_ks_ip
 * (key inner product), 3 k_moddown, 4 k_ks_intt, 5 k_ks_special_intt, 6 k_giant_sum,
 * 7 k_giant_final, 8 rescale.  arm(mask) enables ids (bit i); timer() reports kernel_id's
 * accumulated ms / launch count and optionally resets every accumulator. */
fhs_status fhs_kernel_timer_arm(fhs_context* ctx, uint32_t mask);
fhs_status fhs_kernel_timer(fhs_context* ctx, int kernel_id, float* ms, int* launches, int reset);
/* device-to-device copies of ciphertext limbs to / from caller-owned HBM (RCCL gather in bench.py) */
fhs_status fhs_ciphertext_copy_to_device(fhs_context* ctx, const fhs_ciphertext* ct, void* dst);
fhs_status fhs_ciphertext_from_device(fhs_context* ctx, const void* src, int ncomp, int chain_index, double scale,
                                      fhs_ciphertext** out);
/* Stream-ordered variants for callers that order their own streams against the context stream
 * (fhespear_dist: torch / RCCL buffers): the copy is enqueued on the context stream and the call
 * returns without waiting; the caller makes the context stream wait for the buffer's producer and
 * its own stream wait for the copy (HIP events; torch.cuda.ExternalStream on fhs_context_stream). */
fhs_status fhs_ciphertext_copy_to_device_async(fhs_context* ctx, const fhs_ciphertext* ct, void* dst);
fhs_status fhs_ciphertext_from_device_async(fhs_context* ctx, const void* src, int ncomp, int chain_index,
                                            double scale, fhs_ciphertext** out);
/* the context's HIP stream (hipStream_t), on which every library call is ordered */
fhs_status fhs_context_stream(fhs_context* ctx, void** stream);
/* staging-ring statistics: how often the pinned descriptor ring re-entered a segment, and how many of
 * those re-entries had to wait for the GPU (should stay 0: the host never drains the queue) */
fhs_status fhs_staging_stats(fhs_context* ctx, uint64_t* reentries, uint64_t* blocked);
/* Host-side diagnostic of the device reduction arithmetic (no GPU needed): reduces hi:lo mod q with
 * the pseudo-Mersenne folds the kernels use when q qualifies (*pm_used = 1), else *pm_used = 0 and
 * *out = (hi:lo) mod q.  Exists so the CPU test suite can check the fold bounds against big ints. */
fhs_status fhs_debug_reduce128(uint64_t q, uint64_t lo, uint64_t hi, uint64_t* out, int* pm_used);
/* Test hook: ModUp's X form (k_centered_x + modup_convert3x arithmetic, run on the host) of the 3-limb
 * digit residues y3 over primes q3 into target prime m; *out = the centred digit value mod m. */
fhs_status fhs_debug_modup_xform(const uint64_t* q3, const uint64_t* y3, uint64_t m, uint64_t* out);
/* Test hook: ModDown's X form (k_special_x + moddown_convert3x arithmetic, on the host): special residues y3
 * over primes p3 (< 2^59) into target prime q; *out = (sum_k y3[k] P/p3[k]) mod q. */
fhs_status fhs_debug_moddown_xform(const uint64_t* p3, const uint64_t* y3, uint64_t q, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif
