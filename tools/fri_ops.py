"""fhe_rwkv_inference.py's CKKS chain restated over any `pyPhantom`-shaped module (BASELINE configs[2]
names this caller; north_star: it must run unchanged on the MI355X backend).  The reference file
imports torch model weights that are absent here, and does not travel to the GPU box, so its FHE
part is restated (fri = /root/reference/fhe_rwkv_inference.py):

  CKKSContext          fri:29-54   N=32768, [60] + [40] x depth + [60], special_modulus_size 1, default
                                   (power-of-two + conjugation) Galois keys, public-key encryption
  ct_pt_dot            fri:66-76   multiply_plain + rescale, then a rotate-and-add tree over dim
  ct_pt_weighted_sum   fri:79-94   constant plaintexts mod-switched to `level`, multiply_plain,
                                   rescale, add
  ct_ct_square         fri:97-101  multiply + relinearize + rescale
  ffn_head             fri:111-160 run_inference's encrypted FFN + head on random weights (the
                                   reference's pass criterion: the argmax token matches plaintext)

`phantom` is the module (pyPhantom on the GPU, oracle.pyphantom_oracle on the CPU); `encoder`
overrides the CKKS encoder (the bit-exact GPU test encodes with the oracle so float64 encoding
drops out of the limb comparison)."""
import numpy as np


class CKKSContext:
    """fri:29-54 (seed: deterministic keys and encryptions, an extension used by the tests)."""

    def __init__(self, phantom, poly_modulus_degree=32768, depth=9, prime_bits=40, seed=None, encoder=None):
        self.phantom = phantom
        bit_sizes = [60] + [prime_bits] * depth + [60]
        params = phantom.params(phantom.scheme_type.ckks)
        params.set_poly_modulus_degree(poly_modulus_degree)
        params.set_coeff_modulus(phantom.create_coeff_modulus(poly_modulus_degree, bit_sizes))
        params.set_special_modulus_size(1)
        self.ctx = phantom.context(params)
        self.sk = phantom.secret_key(self.ctx, seed=seed)
        self.pk = self.sk.gen_publickey(self.ctx)
        self.rlk = self.sk.gen_relinkey(self.ctx)
        self.gk = self.sk.create_galois_keys(self.ctx)
        self.encoder = encoder if encoder is not None else phantom.ckks_encoder(self.ctx)
        self.decoder = phantom.ckks_encoder(self.ctx)
        self.scale = 2.0 ** prime_bits
        self.slots = poly_modulus_degree // 2
        self.depth = depth

    def encrypt(self, vec):
        padded = list(vec) + [0.0] * (self.slots - len(vec))
        pt = self.encoder.encode_double_vector(self.ctx, padded, self.scale)
        return self.pk.encrypt_asymmetric(self.ctx, pt)

    def decrypt_slot0(self, ct):
        pt = self.sk.decrypt(self.ctx, ct)
        return self.decoder.decode_double_vector(self.ctx, pt)[0]


def ct_pt_dot(ckks, ct, weights, dim):
    ph = ckks.phantom
    w_padded = list(weights) + [0.0] * (ckks.slots - dim)
    w_pt = ckks.encoder.encode_double_vector(ckks.ctx, w_padded, ckks.scale)
    prod = ph.multiply_plain(ckks.ctx, ct, w_pt)
    prod = ph.rescale_to_next(ckks.ctx, prod)
    step = 1
    while step < dim:
        rotated = ph.rotate(ckks.ctx, prod, step, ckks.gk)
        prod = ph.add(ckks.ctx, prod, rotated)
        step *= 2
    return prod


def ct_pt_weighted_sum(ckks, ct_list, weights, level):
    ph = ckks.phantom
    result = None
    for j, ct in enumerate(ct_list):
        w_pt = ckks.encoder.encode_double_vector(ckks.ctx, [weights[j]] * ckks.slots, ckks.scale)
        w_pt = ph.mod_switch_to(ckks.ctx, w_pt, level)
        term = ph.rescale_to_next(ckks.ctx, ph.multiply_plain(ckks.ctx, ct, w_pt))
        result = term if result is None else ph.add(ckks.ctx, result, term)
    return result


def ct_ct_square(ckks, ct):
    ph = ckks.phantom
    sq = ph.multiply(ckks.ctx, ct, ct)
    sq = ph.relinearize(ckks.ctx, sq, ckks.rlk)
    return ph.rescale_to_next(ckks.ctx, sq)


def ffn_head(ckks, x, W_key, W_val, W_head):
    """fri:128-160: Enc(x) -> ffn_dim dot products -> squares -> embed_dim weighted sums at level 3
    -> vocab_dim weighted sums at level 4 -> decrypted logits (slot 0 of each)."""
    embed_dim, ffn_dim = W_key.shape
    vocab_dim = W_head.shape[1]
    ct_x = ckks.encrypt(x)
    ct_k = [ct_pt_dot(ckks, ct_x, W_key[:, j], embed_dim) for j in range(ffn_dim)]
    ct_k_sq = [ct_ct_square(ckks, c) for c in ct_k]
    ct_v = [ct_pt_weighted_sum(ckks, ct_k_sq, W_val[:, i], level=3) for i in range(embed_dim)]
    ct_logits = [ct_pt_weighted_sum(ckks, ct_v, W_head[:, i], level=4) for i in range(vocab_dim)]
    return ct_x, ct_logits, np.array([ckks.decrypt_slot0(c) for c in ct_logits])


def normalize_columns(W):
    """fri:57-63"""
    W = W.copy()
    s = W.std(axis=0)
    W[:, s > 1e-6] /= s[s > 1e-6]
    return W
