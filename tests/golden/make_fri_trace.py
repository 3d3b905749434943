"""Record the REFERENCE's fhe_rwkv_inference.py (fri) running on the C parity oracle, op by op, as a
replayable trace (n1 pinned by reference-executed fixtures, not by a restatement).

/root/reference/fhe_rwkv_inference.py is imported read-only (bytecode writing off) with the oracle
installed as `pyPhantom` (oracle/pyphantom_oracle.py), and its own functions run unchanged:
  - CKKSContext(poly_modulus_degree=N, depth=9)              fri:29-54
  - run_inference(embed, ffn, vocab, ckks, w)                fri:111-166 (ct_pt_dot, ct_ct_square,
                                                             ct_pt_weighted_sum at levels 3 and 4)
  - run_multilayer_residual_inference(..., num_blocks=2)     fri:294-395 (+ mod_switch_to_next, set_scale,
                                                             residual add)
with synthetic weights in the layout load_weights() returns (fri:18-26; the model checkpoint is absent).
Every pyPhantom call the reference makes is recorded: its operation, operand ids and arguments, and for
every ciphertext / plaintext it returns the SHA-256 of its limbs, its chain index and scale; decrypted
values are kept.  tests/test_fri_ring.py replays the trace through the MI355X pyPhantom
(tools/fri_replay.py) and compares every object's limbs to the reference run.  Run in the build container
only (the reference does not travel to the GPU box):

    python tests/golden/make_fri_trace.py          -> tests/golden/fri_trace.json
"""
import hashlib
import json
import sys
from pathlib import Path

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from oracle import pyphantom_oracle as php  # noqa: E402

sys.modules["pyPhantom"] = php
sys.path.insert(0, str(REF))
import fhe_rwkv_inference as fri  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:32]


class Recorder:
    """Wraps the shim's functions and methods the reference calls; nested shim calls (mod_switch_to ->
    mod_switch_to_next) are not recorded twice."""

    def __init__(self):
        self.ops, self.objs, self.ids, self.keep, self.depth = [], [], {}, [], 0

    def oid(self, x):
        k = id(x)
        if k not in self.ids:
            self.ids[k] = len(self.objs)
            self.keep.append(x)
            kind = "ct" if isinstance(x, php.ciphertext) else "pt"
            self.objs.append({"kind": kind, "sha": sha(x.data), "ci": x.chain_index(), "scale": x.scale(),
                              "shape": list(x.data.shape)})
        return self.ids[k]

    def wrap_fn(self, mod, name, argspec):
        orig = getattr(mod, name)

        def fn(*a, **k):
            self.depth += 1
            try:
                out = orig(*a, **k)
            finally:
                self.depth -= 1
            if self.depth == 0:
                ins, extra = [], {}
                for i, v in enumerate(a[1:]):   # a[0] is the context
                    if isinstance(v, (php.ciphertext, php.plaintext)):
                        ins.append(self.oid(v))
                    elif isinstance(v, php.galois_key) or isinstance(v, php.relin_key):
                        extra["key"] = "galois" if isinstance(v, php.galois_key) else "relin"
                    else:
                        extra[argspec[i]] = v
                self.ops.append([name, self.oid(out), ins, extra])
            return out
        setattr(mod, name, fn)

    def install(self):
        for name, spec in (("multiply_plain", ["a", "b"]), ("rescale_to_next", ["a"]), ("rotate", ["a", "step", "gk"]),
                           ("add", ["a", "b"]), ("mod_switch_to", ["a", "chain_index"]),
                           ("mod_switch_to_next", ["a"]), ("multiply", ["a", "b"]), ("relinearize", ["a", "rk"]),
                           ("add_plain", ["a", "b"])):
            self.wrap_fn(php, name, spec)
        rec = self
        enc = php.ckks_encoder.encode_double_vector

        def encode(self_, ctx, values, scale, chain_index=1):
            out = enc(self_, ctx, values, scale, chain_index)
            v = np.asarray(values, dtype=np.float64)
            if np.all(v == v[0]):
                desc = {"const": float(v[0]), "n": int(v.size)}
            else:
                nz = int(np.max(np.nonzero(v)[0])) + 1 if np.any(v) else 0
                desc = {"prefix": [float(t) for t in v[:nz]], "n": int(v.size)}
            rec.ops.append(["encode", rec.oid(out), [], dict(desc, scale=float(scale), chain_index=chain_index)])
            return out
        php.ckks_encoder.encode_double_vector = encode
        enc_a = php.public_key.encrypt_asymmetric

        def encrypt(self_, ctx, pt):
            out = enc_a(self_, ctx, pt)
            rec.ops.append(["encrypt_asymmetric", rec.oid(out), [rec.oid(pt)], {}])
            return out
        php.public_key.encrypt_asymmetric = encrypt
        dec = php.secret_key.decrypt

        def decrypt(self_, ctx, ct):
            out = dec(self_, ctx, ct)
            rec.ops.append(["decrypt", rec.oid(out), [rec.oid(ct)], {}])
            return out
        php.secret_key.decrypt = decrypt
        dcd = php.ckks_encoder.decode_double_vector

        def decode(self_, ctx, pt):
            out = dcd(self_, ctx, pt)
            rec.ops.append(["decode", None, [rec.oid(pt)], {"slot0": float(out[0])}])
            return out
        php.ckks_encoder.decode_double_vector = decode
        ss = php.ciphertext.set_scale

        def set_scale(self_, s):
            # set_scale changes the object in place: record it against the object's id; the scale the
            # object then carries is what the replay must set
            rec.ops.append(["set_scale", None, [rec.oid(self_)], {"scale": float(s)}])
            return ss(self_, s)
        php.ciphertext.set_scale = set_scale


def synthetic_weights(seed, embed, ffn, vocab, blocks, emb_std):
    """torch tensors in load_weights()'s layout (fri:18-26: key/value/head weights transposed)."""
    g = torch.Generator().manual_seed(seed)
    w = {"emb.weight": torch.randn(vocab, embed, generator=g, dtype=torch.float64) * emb_std,
         "head.weight": torch.randn(embed, vocab, generator=g, dtype=torch.float64)}
    for b in range(blocks):
        w[f"blocks.{b}.ffn.key.weight"] = torch.randn(embed, ffn, generator=g, dtype=torch.float64)
        w[f"blocks.{b}.ffn.value.weight"] = torch.randn(ffn, embed, generator=g, dtype=torch.float64)
    return w


REC = Recorder()
REC.install()


def run_case(name, fn, N, depth, embed, ffn, vocab, blocks, seed, emb_std):
    rec = REC
    rec.ops, rec.objs, rec.ids, rec.keep = [], [], {}, []   # one trace per case (wrappers installed once)
    ckks = fri.CKKSContext(poly_modulus_degree=N, depth=depth)
    w = synthetic_weights(seed, embed, ffn, vocab, blocks, emb_std)
    if fn == "run_inference":
        res = fri.run_inference(embed, ffn, vocab, ckks, w=w)
    else:
        res = fri.run_multilayer_residual_inference(embed, ffn, vocab, blocks, ckks, w=w)
    match, corr, _ = res
    print(f"[{name}] {fn} N={N} {embed}x{ffn}x{vocab} blocks={blocks}: match={match} corr={corr:.6f} "
          f"ops={len(rec.ops)} objects={len(rec.objs)}")
    assert match, f"{name}: the reference's own criterion (argmax token) failed"
    return {"function": fn, "reference": {"run_inference": "fhe_rwkv_inference.py:111-166",
                                          "run_multilayer_residual_inference": "fhe_rwkv_inference.py:294-395"}[fn],
            "N": N, "depth": depth, "bit_sizes": [60] + [40] * depth + [60], "special_modulus_size": 1,
            "embed": embed, "ffn": ffn, "vocab": vocab, "blocks": blocks, "weight_seed": seed,
            "sk_seed": ckks.sk.seed, "galois_elts": sorted(int(e) for e in ckks.gk.keys),
            "token_match": bool(match), "corr": float(corr), "ops": rec.ops, "objects": rec.objs}


def main():
    cases = {
        "inference_n4096": run_case("inference_n4096", "run_inference", 4096, 9, 8, 8, 4, 1, 21, 0.05),
        "residual2_n4096": run_case("residual2_n4096", "run_multilayer_residual_inference", 4096, 9, 8, 8, 4, 2,
                                    22, 0.01),
        "inference_n32768": run_case("inference_n32768", "run_inference", 32768, 9, 8, 8, 4, 1, 23, 0.05),
    }
    out = {"generator": "tests/golden/make_fri_trace.py",
           "reference": "fhe_rwkv_inference.py (fri), imported read-only with the C oracle as pyPhantom",
           "cases": cases}
    (OUT / "fri_trace.json").write_text(json.dumps(out, separators=(",", ":")))
    print("wrote", OUT / "fri_trace.json")


if __name__ == "__main__":
    main()
