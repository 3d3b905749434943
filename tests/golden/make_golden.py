"""Generate the committed golden fixtures by running the REFERENCE's own BSGS orchestration
(/root/reference/scripts/bootstrap_generation.py and test_fully_enc_bsgs.py, imported read-only,
bytecode writing disabled) on the C parity oracle, installed as `pyPhantom`
(oracle/pyphantom_oracle.py).  The oracle exports no fused symbols, so the reference executes
its pure-Python fallbacks: per-row encode + mod_switch_to (bg:385-391) and the BSGS loop
(bg:464-485).  Run in the build container only (the reference does not travel to the GPU box):

    python tests/golden/make_golden.py

Outputs tests/golden/*.npz + manifest.json (inputs, limbs, decrypted outputs, op counts).
"""
import hashlib
import json
import os
import sys
from pathlib import Path

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
from oracle import pyphantom_oracle as php  # noqa: E402

sys.modules["pyPhantom"] = php
sys.path.insert(0, str(REF))
sys.path.insert(0, str(REF / "scripts"))
import bootstrap_generation as bg  # noqa: E402
import test_fully_enc_bsgs as tf  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def reset_counts():
    php.OP_COUNTS.clear()


def bsgs_case(name, N, L0, P, D, seed, complex_pack=False):
    np.random.seed(seed)
    ckks = bg.CKKSBootstrapContext(poly_degree=N, L0=L0, prime_bits=59, special_mod_size=P,
                                   max_rot_dim=D, bsgs_dim=D, skip_bootstrap=True)
    G, B = bg.compute_bsgs_params(D)
    x = np.random.randn(D) * 0.1
    W1 = np.random.randn(D, D) * 0.02
    W2 = np.random.randn(D, D) * 0.02
    ct = ckks.encrypt_replicated(x)
    level = ct.chain_index()
    baby = bg._compute_baby_rotations(ckks, ct, G)
    if complex_pack:
        pts = bg._batch_encode_diags_complex(ckks, bg._extract_diagonals(W1, D), bg._extract_diagonals(W2, D),
                                             D, G, ckks.slots, level)
    else:
        pts = bg._batch_encode_diags_real(ckks, bg._extract_diagonals(W1, D), D, G, ckks.slots, level)
    reset_counts()
    if complex_pack:
        y = bg.fhe_matmul_bsgs_complex(ckks, ct, W1, W2, D, G, B, ct_baby=baby, preencoded=pts)
        dec = ckks.decrypt_vec_complex(y, D)
        ref = W1 @ x + 1j * (W2 @ x)
    else:
        y = bg.fhe_matmul_bsgs(ckks, ct, W1, D, G, B, ct_baby=baby, preencoded=pts)
        dec = ckks.decrypt_vec(y, D)
        ref = W1 @ x
    counts = dict(php.OP_COUNTS)
    err = float(np.max(np.abs(dec - ref)))
    print(f"[{name}] N={N} L0={L0} P={P} D={D} G={G} B={B} max|y-Mx|={err:.3e} ops={counts}")
    ctx = ckks.ctx
    np.savez_compressed(
        OUT / f"{name}.npz",
        primes=np.array(ctx.o.primes, dtype=np.uint64),
        x=x, W1=W1, W2=W2,
        ct_in=ct.data, baby=np.stack([b.data for b in baby]), pts=np.stack([p.data for p in pts]),
        out=y.data, dec=np.asarray(dec), ref=np.asarray(ref))
    giant_elts = [php.get_elt_from_step(g * G, N) for g in range(1, B)]
    return {
        "file": f"{name}.npz", "N": N, "L0": L0, "P": P, "D": D, "G": G, "B": B,
        "complex": complex_pack, "sk_seed": ckks.sk.seed, "enc_counter": 0,
        "scale": ckks.scale, "diag_scale": ckks.diag_scale,
        "chain_index_in": level, "chain_index_out": y.chain_index(), "scale_out": y.scale(),
        "max_err": err, "op_counts": counts,
        "giant_elts": giant_elts,
        "giant_key_sha256": {str(e): sha(ctx.o.gen_galois_key(ckks.sk.seed, ckks.sk.s, e)) for e in giant_elts[:2]},
        "secret_sha256": sha(ckks.sk.s),
        "out_sha256": sha(y.data),
    }


def ffn_case(name, N, L0, P, D, F, blocks, seed):
    """tf:main's random-weight path on a tiny shape, calling the reference's
    fully_encrypted_ffn_block (tf:26-118) unchanged."""
    np.random.seed(seed)
    W_keys = [np.random.randn(D, F) * 0.02 for _ in range(blocks)]
    W_vals_raw = [np.random.randn(F, D) * 0.02 for _ in range(blocks)]
    x_cal = np.random.randn(D) * 0.1
    W_vals, x_ref = [], x_cal.copy()
    for b in range(blocks):                                     # tf:181-196
        fk = x_ref @ W_keys[b]
        fv = (fk ** 2) @ W_vals_raw[b]
        ms = 1.0 / (np.max(np.abs(fv)) + 1e-12)
        W_vals.append(W_vals_raw[b] * ms)
        x_ref = x_ref + fv * ms
    x_pt = [x_cal.copy()]
    for b in range(blocks):
        x_pt.append(tf.plaintext_ffn_block(x_pt[-1], W_keys[b], W_vals[b]))
    ckks = bg.CKKSBootstrapContext(poly_degree=N, L0=L0, prime_bits=59, special_mod_size=P,
                                   max_rot_dim=max(D, F), bsgs_dim=[D, F], skip_bootstrap=True)
    ct = ckks.encrypt_replicated(x_cal)
    reset_counts()
    decs, cis = [], []
    for b in range(blocks):
        ct, _ = tf.fully_encrypted_ffn_block(ckks, ct, W_keys[b], W_vals[b], D, F, block_idx=b)
        decs.append(ckks.decrypt_vec(ct, D))
        cis.append(ct.chain_index())
    corr = [float(np.corrcoef(decs[b], x_pt[b + 1])[0, 1]) for b in range(blocks)]
    err = [float(np.max(np.abs(decs[b] - x_pt[b + 1]))) for b in range(blocks)]
    print(f"[{name}] corr={corr} max_err={err} ops={dict(php.OP_COUNTS)}")
    np.savez_compressed(OUT / f"{name}.npz", x=x_cal, W_keys=np.stack(W_keys), W_vals=np.stack(W_vals),
                        dec=np.stack(decs), ref=np.stack(x_pt[1:]), out_last=ct.data)
    return {"file": f"{name}.npz", "N": N, "L0": L0, "P": P, "D": D, "F": F, "blocks": blocks,
            "sk_seed": ckks.sk.seed, "corr": corr, "max_err": err, "chain_index": cis,
            "op_counts": dict(php.OP_COUNTS), "out_last_sha256": sha(ct.data)}


def main():
    man = {"generator": "tests/golden/make_golden.py",
           "reference": "scripts/bootstrap_generation.py:198-220,361-542; test_fully_enc_bsgs.py:26-125",
           "backend": "oracle/pyphantom_oracle.py over oracle/ckks_oracle.c", "cases": {}}
    man["cases"]["bsgs_real_n512"] = bsgs_case("bsgs_real_n512", 512, 6, 3, 16, 11)
    man["cases"]["bsgs_complex_n512"] = bsgs_case("bsgs_complex_n512", 512, 6, 3, 16, 12, complex_pack=True)
    man["cases"]["bsgs_real_n1024_p1"] = bsgs_case("bsgs_real_n1024_p1", 1024, 4, 1, 32, 13)
    man["cases"]["ffn_n1024"] = ffn_case("ffn_n1024", 1024, 9, 3, 16, 32, 2, 14)
    (OUT / "manifest.json").write_text(json.dumps(man, indent=1, sort_keys=True))
    print("wrote", OUT / "manifest.json")


if __name__ == "__main__":
    main()
