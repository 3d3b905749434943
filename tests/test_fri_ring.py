"""fhe_rwkv_inference.py (fri) replayed from traces the REFERENCE itself produced.

tests/golden/make_fri_trace.py imports /root/reference/fhe_rwkv_inference.py with the C oracle as
`pyPhantom` and runs its own CKKSContext (N, [60] + [40] x 9 + [60], special_modulus_size 1, default
Galois keys, public-key encryption; fri:29-54), run_inference (ct_pt_dot rotate-and-sum, ct_ct_square,
ct_pt_weighted_sum at levels 3 and 4; fri:66-166) and run_multilayer_residual_inference (2 blocks, +
mod_switch_to_next, set_scale, residual add; fri:294-395), recording every pyPhantom call and the limb
digest of every ciphertext / plaintext it returned (tests/golden/fri_trace.json).  tools/fri_replay.py
issues the same calls:
- CPU: on the oracle shim -- the replay driver reproduces the reference run object for object;
- GPU: on the MI355X pyPhantom, at N = 4096 (both functions) and N = 32768 (the configuration itself) --
  every ciphertext limb-identical to the reference run (plaintexts encoded with the oracle on both sides,
  so float64 encoding drops out), decrypted logits equal, the reference's criterion (argmax) holds."""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))

import fri_replay  # noqa: E402

TRACE = json.loads((REPO / "tests" / "golden" / "fri_trace.json").read_text())["cases"]


def test_fri_traces_are_the_reference_criterion():
    for name, case in TRACE.items():
        assert case["token_match"] and case["corr"] > 0.999, name
        assert case["bit_sizes"] == [60] + [40] * case["depth"] + [60] and case["special_modulus_size"] == 1
        ops = {op for op, *_ in case["ops"]}
        assert {"encrypt_asymmetric", "multiply_plain", "rescale_to_next", "rotate", "add", "mod_switch_to",
                "multiply", "relinearize", "decrypt"} <= ops, name
    assert {op for op, *_ in TRACE["residual2_n4096"]["ops"]} >= {"mod_switch_to_next", "set_scale"}


@pytest.mark.parametrize("name", ["inference_n4096", "residual2_n4096"])
def test_fri_replay_on_the_oracle_reproduces_the_reference_run(name):
    from oracle import pyphantom_oracle as php
    case = TRACE[name]

    def encode(ctx, v, scale, ci):
        return php.ckks_encoder(ctx).encode_double_vector(ctx, v, scale, ci)
    res = fri_replay.replay(php, case, encode)
    assert res["objects_checked"] == len({o for _, o, _, _ in case["ops"] if o is not None})
    assert all(got == want for got, want in res["slot0"])


class _OracleEncoder:
    """Plaintexts for the GPU context encoded by the oracle (the reference run's encoder) and imported as
    limbs: float64 encoding is not part of the limb comparison."""

    def __init__(self, ph, N, primes):
        from oracle.oracle import Oracle
        self.ph, self.o = ph, Oracle(N, primes, 1)

    def __call__(self, ctx, values, scale, chain_index):
        limbs = self.o.encode(np.asarray(values, dtype=np.float64), scale, self.o.L0 + 1 - chain_index)
        return self.ph.plaintext_from_numpy(ctx, limbs, chain_index, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["inference_n4096", "residual2_n4096", "inference_n32768"])
def test_fri_replay_on_the_gpu_is_limb_identical(require_gpu, name):
    import pyPhantom as ph
    case = TRACE[name]
    primes = [int(q) for q in ph.create_coeff_modulus(case["N"], case["bit_sizes"])]
    res = fri_replay.replay(ph, case, _OracleEncoder(ph, case["N"], primes))
    assert res["objects_checked"] == len({o for _, o, _, _ in case["ops"] if o is not None})
    got = np.array([g for g, _ in res["slot0"]])
    want = np.array([w for _, w in res["slot0"]])
    assert np.max(np.abs(got - want)) < 1e-9 * max(1.0, float(np.max(np.abs(want))))


@pytest.mark.gpu
def test_fri_default_keys_and_gpu_encoder(require_gpu):
    """The context fri builds without set_galois_elts gets SEAL/Phantom's default key set (the trace's
    recorded elements), and the same call sequence with the GPU's own float64 encoder (which rounds its own
    way, so limbs are not compared) decrypts to the reference run's logits within CKKS precision."""
    import pyPhantom as ph
    case = TRACE["inference_n32768"]
    ctx, *_ = fri_replay.make_context(ph, case)
    assert sorted(int(e) for e in ctx.galois_elts()) == case["galois_elts"]
    del ctx

    def gpu_encode(c, v, scale, ci):
        pt = ph.ckks_encoder(c).encode_double_vector(c, v, scale)
        return ph.mod_switch_to(c, pt, ci) if ci != 1 else pt
    res = fri_replay.replay(ph, case, gpu_encode, check_limbs=False)
    got = np.array([g for g, _ in res["slot0"]])
    want = np.array([w for _, w in res["slot0"]])
    assert np.max(np.abs(got - want)) < 1e-4 * max(1.0, float(np.max(np.abs(want))))
    assert int(np.argmax(got)) == int(np.argmax(want))
