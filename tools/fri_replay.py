"""Replay driver for the reference-executed fhe_rwkv_inference.py traces (tests/golden/fri_trace.json,
made by tests/golden/make_fri_trace.py from the reference's own CKKSContext / run_inference /
run_multilayer_residual_inference running on the C oracle).

`replay(phantom, case, encode)` rebuilds the case's context the way fri:29-54 does (N, [60] + [40] x depth +
[60], special_modulus_size 1, default Galois keys, public-key encryption) with the recorded secret-key
seed, then issues the recorded pyPhantom calls in order through `phantom` (the MI355X pyPhantom on the GPU,
oracle.pyphantom_oracle on the CPU) and checks every ciphertext and plaintext it produces against the
reference run: limbs (SHA-256; check_limbs=False: chain index and scale only), chain index and scale.  `encode(ctx, values, scale, chain_index)` makes the
plaintexts (the tests encode with the oracle so float64 encoding drops out of the limb comparison).
Returns a summary; the first mismatch raises AssertionError naming the op."""
import hashlib

import numpy as np


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:32]


def _limbs(x):
    return x.to_numpy() if hasattr(x, "to_numpy") else x.data


def make_context(phantom, case):
    params = phantom.params(phantom.scheme_type.ckks)
    params.set_poly_modulus_degree(case["N"])
    params.set_coeff_modulus(phantom.create_coeff_modulus(case["N"], case["bit_sizes"]))
    params.set_special_modulus_size(case["special_modulus_size"])
    ctx = phantom.context(params)
    sk = phantom.secret_key(ctx, seed=case["sk_seed"])
    return ctx, sk, sk.gen_publickey(ctx), sk.gen_relinkey(ctx), sk.create_galois_keys(ctx)


def replay(phantom, case, encode, check_limbs=True):
    ctx, sk, pk, rlk, gk = make_context(phantom, case)
    objs, want = {}, case["objects"]
    checked, slot0 = 0, []

    def check(oid, x, op):
        nonlocal checked
        w = want[oid]
        assert x.chain_index() == w["ci"], f"{op} -> object {oid}: chain index {x.chain_index()} != {w['ci']}"
        if check_limbs:
            assert _sha(_limbs(x)) == w["sha"], f"{op} -> object {oid}: limbs differ from the reference run"
            checked += 1

    for i, (op, out, ins, extra) in enumerate(case["ops"]):
        a = [objs[k] for k in ins]
        tag = f"op {i} ({op})"
        if op == "encode":
            v = np.full(extra["n"], extra["const"]) if "const" in extra else \
                np.concatenate([np.asarray(extra["prefix"], dtype=np.float64), np.zeros(extra["n"] - len(extra["prefix"]))])
            r = encode(ctx, v, extra["scale"], extra["chain_index"])
        elif op == "encrypt_asymmetric":
            r = pk.encrypt_asymmetric(ctx, a[0])
        elif op == "multiply_plain":
            r = phantom.multiply_plain(ctx, a[0], a[1])
        elif op == "add_plain":
            r = phantom.add_plain(ctx, a[0], a[1])
        elif op == "rescale_to_next":
            r = phantom.rescale_to_next(ctx, a[0])
        elif op == "rotate":
            r = phantom.rotate(ctx, a[0], extra["step"], gk)
        elif op == "add":
            r = phantom.add(ctx, a[0], a[1])
        elif op == "mod_switch_to":
            r = phantom.mod_switch_to(ctx, a[0], extra["chain_index"])
        elif op == "mod_switch_to_next":
            r = phantom.mod_switch_to_next(ctx, a[0])
        elif op == "multiply":
            r = phantom.multiply(ctx, a[0], a[1])
        elif op == "relinearize":
            r = phantom.relinearize(ctx, a[0], rlk)
        elif op == "set_scale":
            a[0].set_scale(extra["scale"])
            continue
        elif op == "decrypt":
            r = sk.decrypt(ctx, a[0])
        elif op == "decode":
            slot0.append((phantom.ckks_encoder(ctx).decode_double_vector(ctx, a[0])[0], extra["slot0"]))
            continue
        else:
            raise ValueError(f"{tag}: unknown op")
        if out in objs and objs[out] is not r and out not in ins:
            raise AssertionError(f"{tag}: object {out} produced twice")
        objs[out] = r
        check(out, r, tag)
        if abs(r.scale() - want[out]["scale"]) > 1e-9 * abs(want[out]["scale"]) and op != "encode":
            # scales are compared at creation (set_scale changes them later, as recorded)
            raise AssertionError(f"{tag}: scale {r.scale()} != {want[out]['scale']}")
    return {"ops": len(case["ops"]), "objects_checked": checked, "slot0": slot0}
