"""fhe_rwkv_inference.py's ring and op chain: CKKSContext(depth=9) = N=32768,
[60] + [40] x 9 + [60] primes, special_modulus_size 1, default Galois keys (no set_galois_elts),
encrypt_asymmetric; ct_pt_dot / ct_pt_weighted_sum / ct_ct_square (fri:29-101) chained as
run_inference does (fri:128-160), restated in tools/fri_ops.py.

- CPU: the restated chain on the oracle passes the reference's criterion (argmax token matches
  the plaintext FFN + head).
- GPU, N = 4096 with the same bit pattern: every ciphertext (the public-key encryption, the
  rotate-and-sum dot products, squares, level-3/4 weighted sums) bit-exact against the oracle,
  float64 encoding taken out of the comparison by encoding with the oracle on both sides.
- GPU, N = 32768 (the configuration itself): decrypted logits against the plaintext chain."""
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))

import fri_ops  # noqa: E402


def _weights(seed, embed, ffn, vocab):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(embed) * 0.3
    return (x, rng.standard_normal((embed, ffn)) / np.sqrt(embed), rng.standard_normal((ffn, embed)) / np.sqrt(ffn),
            rng.standard_normal((embed, vocab)) / np.sqrt(embed))


def _plain(x, Wk, Wv, Wh):
    return ((x @ Wk) ** 2 @ Wv) @ Wh


def test_fri_chain_on_the_oracle_matches_plaintext():
    from oracle import pyphantom_oracle as php
    x, Wk, Wv, Wh = _weights(3, 8, 8, 4)
    ck = fri_ops.CKKSContext(php, poly_modulus_degree=1024, depth=9, seed=77)
    _, _, logits = fri_ops.ffn_head(ck, x, Wk, Wv, Wh)
    ref = _plain(x, Wk, Wv, Wh)
    assert np.max(np.abs(logits - ref)) < 1e-3
    assert int(np.argmax(logits)) == int(np.argmax(ref))


class _OracleEncoder:
    """ckks_encoder stand-in for the GPU context: the oracle's float64 encode, imported as limbs."""

    def __init__(self, ph, ctx, o):
        self.ph, self.ctx, self.o = ph, ctx, o

    def encode_double_vector(self, ctx, values, scale, chain_index=1):
        limbs = self.o.encode(np.asarray(values, dtype=np.float64), scale, self.o.L0 + 1 - chain_index)
        return self.ph.plaintext_from_numpy(self.ctx, limbs, chain_index, scale)


@pytest.mark.gpu
def test_fri_chain_bit_exact_vs_oracle_n4096(require_gpu):
    import pyPhantom as ph
    from oracle import pyphantom_oracle as php
    from oracle.oracle import Oracle
    x, Wk, Wv, Wh = _weights(4, 8, 8, 4)
    ref_ck = fri_ops.CKKSContext(php, poly_modulus_degree=4096, depth=9, seed=91)
    gpu_ck = fri_ops.CKKSContext(ph, poly_modulus_degree=4096, depth=9, seed=91)
    primes = [int(q) for q in ph.create_coeff_modulus(4096, [60] + [40] * 9 + [60])]
    assert primes == [int(q) for q in ref_ck.ctx.primes]
    assert max(q.bit_length() for q in primes) == 60 and min(q.bit_length() for q in primes) == 40
    gpu_ck.encoder = _OracleEncoder(ph, gpu_ck.ctx, Oracle(4096, primes, 1))
    assert sorted(gpu_ck.ctx.galois_elts()) == sorted(ref_ck.gk.keys)     # default keys: +-2^k, conjugation
    r_x, r_logits, r_dec = fri_ops.ffn_head(ref_ck, x, Wk, Wv, Wh)
    g_x, g_logits, g_dec = fri_ops.ffn_head(gpu_ck, x, Wk, Wv, Wh)
    assert np.array_equal(g_x.to_numpy(), r_x.data)                       # public-key encryption
    for i, (g, r) in enumerate(zip(g_logits, r_logits)):
        assert g.chain_index() == r.chain_index() == 5
        assert np.array_equal(g.to_numpy(), r.data), f"logit {i}: limbs differ from the oracle"
    assert np.max(np.abs(g_dec - r_dec)) < 1e-9


@pytest.mark.gpu
def test_fri_chain_full_ring_n32768(require_gpu):
    import pyPhantom as ph
    x, Wk, Wv, Wh = _weights(5, 32, 32, 8)
    ck = fri_ops.CKKSContext(ph, poly_modulus_degree=32768, depth=9)
    _, cts, logits = fri_ops.ffn_head(ck, x, Wk, Wv, Wh)
    ref = _plain(x, Wk, Wv, Wh)
    assert cts[0].chain_index() == 5
    assert np.max(np.abs(logits - ref)) < 1e-2 * max(1.0, float(np.max(np.abs(ref))))
    assert int(np.argmax(logits)) == int(np.argmax(ref))
