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


# ------------------------------------------------------------------ recording of the reference's BSGS calls
PT_SRC = {}      # id(plaintext) -> (slot values, scale, complex) it was encoded from
CALLS = []       # every fhe_matmul_bsgs[_complex] call: input ct, plaintext rows, output ct


def _install_recorders():
    """Wrap the shim's encoder / plaintext mod-switch (to know each plaintext's slot values) and the
    reference's two BSGS entry points (bg:435, bg:488; tf imports the first by name) to record, per
    call, the input ciphertext limbs, the rows of the D plaintexts the loop multiplies (in diagonal
    order) and the output limbs.  The GPU replay test re-encodes the rows with the same oracle
    encoder (deterministic), imports the input limbs and compares every output limb."""
    enc = php.ckks_encoder
    o_real, o_cplx = enc.encode_double_vector, enc.encode_complex_vector

    def e_real(self, ctx, values, scale, chain_index=1):
        pt = o_real(self, ctx, values, scale, chain_index)
        PT_SRC[id(pt)] = (np.asarray(values, dtype=np.float64), float(scale), False)
        return pt

    def e_cplx(self, ctx, values, scale, chain_index=1):
        pt = o_cplx(self, ctx, values, scale, chain_index)
        PT_SRC[id(pt)] = (np.asarray(values, dtype=np.complex128), float(scale), True)
        return pt
    enc.encode_double_vector, enc.encode_complex_vector = e_real, e_cplx
    o_msn = php.mod_switch_to_next

    def msn(ctx, x):
        y = o_msn(ctx, x)
        if id(x) in PT_SRC:
            PT_SRC[id(y)] = PT_SRC[id(x)]
        return y
    php.mod_switch_to_next = msn

    def wrap(fn, kind):
        def rec(ckks, ct, *a, **k):
            log0 = len(ENC_ORDER)
            out = fn(ckks, ct, *a, **k)
            pre = k.get("preencoded")
            pts = pre if pre is not None else ENC_ORDER[log0:]
            srcs = [PT_SRC[id(p)] for p in pts]
            CALLS.append(dict(kind=kind, ct_in=ct.data.copy(), ci_in=ct.chain_index(), scale_in=ct.scale(),
                              rows=np.stack([v for v, _, _ in srcs]), pt_scale=srcs[0][1], pt_complex=srcs[0][2],
                              pt_level=pts[0].chain_index(), pt_sha256=sha(np.stack([p.data for p in pts])),
                              out=out.data.copy(), ci_out=out.chain_index(), scale_out=out.scale()))
            return out
        return rec
    bg.fhe_matmul_bsgs = wrap(bg.fhe_matmul_bsgs, "real")
    bg.fhe_matmul_bsgs_complex = wrap(bg.fhe_matmul_bsgs_complex, "complex")
    tf.fhe_matmul_bsgs = bg.fhe_matmul_bsgs
    # plaintexts made inside a BSGS call (tf's non-pre-encoded path) in creation order
    o_mst = php.mod_switch_to

    def mst(ctx, x, ci):
        y = o_mst(ctx, x, ci)
        if id(x) in PT_SRC:
            PT_SRC[id(y)] = PT_SRC[id(x)]
            ENC_ORDER.append(y)
        return y
    php.mod_switch_to = mst
    bg.ph = php


ENC_ORDER = []


def _save_calls(name, calls, extra):
    arrs = {}
    for i, c in enumerate(calls):
        for k in ("ct_in", "rows", "out"):
            arrs[f"c{i}_{k}"] = c[k]
    np.savez_compressed(OUT / f"{name}.npz", **arrs, **extra)
    return [{k: v for k, v in c.items() if k not in ("ct_in", "rows", "out")} | {"out_sha256": sha(c["out"])}
            for c in calls]


def _random_rwkv_state_dict(rng, D, F, n_head, head_size):
    """Random RWKV-7 block-0 tensors with the names and shapes RWKVBlockWeights reads (bg:662-716)."""
    import torch

    def t(*shape, s=1.0, off=0.0):
        return torch.tensor(off + s * rng.standard_normal(shape))
    b = "blocks.0."
    w = {}
    for k in ("ln1", "ln2", "att.ln_x"):
        w[b + k + ".weight"], w[b + k + ".bias"] = t(D, s=0.1, off=1.0), t(D, s=0.1)
    for k in ("x_r", "x_k", "x_v", "x_g", "x_w", "x_a", "k_k", "k_a"):
        w[b + "att." + k] = torch.tensor(rng.uniform(0, 1, (1, 1, D)))
    w[b + "ffn.x_k"] = torch.tensor(rng.uniform(0, 1, (1, 1, D)))
    for k, r in (("w", 16), ("a", 16), ("v", 8)):
        w[b + f"att.{k}0"], w[b + f"att.{k}1"], w[b + f"att.{k}2"] = t(D, s=0.5), t(D, r, s=0.1), t(r, D, s=0.1)
    w[b + "att.r_k"] = t(n_head, head_size, s=0.1)
    w[b + "att.g1"], w[b + "att.g2"] = t(D, 8, s=D ** -0.5), t(8, D, s=8 ** -0.5)
    for k in ("receptance", "key", "value", "output"):
        w[b + f"att.{k}.weight"] = t(D, D, s=D ** -0.5)
    w[b + "ffn.key.weight"] = t(D, F, s=D ** -0.5)
    w[b + "ffn.value.weight"] = t(F, D, s=0.25 * F ** -0.5)
    return w


def client_aided_case(name, N, L0, P, D, F, head_size, seed):
    """The reference's client_aided_block (bg:756-899) with use_bsgs and pre-encoded diagonals
    (bg:265-333): every server BSGS (r, k, v, o, FFN key pairs with shared baby steps, FFN value
    pairs via the conjugate trick) is recorded with its input, plaintext rows and output."""
    rng = np.random.default_rng(seed)
    n_head = D // head_size
    blk = bg.RWKVBlockWeights(_random_rwkv_state_dict(rng, D, F, n_head, head_size), 0, D, F, n_head, head_size)
    ckks = bg.CKKSBootstrapContext(poly_degree=N, L0=L0, prime_bits=59, special_mod_size=P,
                                   max_rot_dim=D, bsgs_dim=D, skip_bootstrap=True)
    pe = bg.pre_encode_block(ckks, blk, D, F)
    x = rng.standard_normal(D)
    st = (x, np.zeros(D), np.zeros(D), np.zeros((n_head, head_size, head_size)), None)
    CALLS.clear()
    reset_counts()
    out = bg.client_aided_block(ckks, blk, *st, use_bsgs=True, preencoded_block=pe)
    ref = bg.plaintext_block(blk, *st)
    err = float(np.max(np.abs(out[0] - ref[0])))
    names = ["r", "k", "v", "o"] + [f"ffn_key_{p}" for p in range(F // D // 2)] + \
            [f"ffn_val_{p}" for p in range(F // D // 2)]
    assert len(CALLS) == len(names), len(CALLS)
    print(f"[{name}] N={N} L0={L0} P={P} D={D} F={F} calls={len(CALLS)} max|x-plain|={err:.3e} "
          f"ops={dict(php.OP_COUNTS)}")
    calls = _save_calls(name, CALLS, dict(primes=np.array(ckks.ctx.o.primes, dtype=np.uint64), x=x,
                                          x_out=out[0], x_ref=ref[0]))
    for c, n in zip(calls, names):
        c["projection"] = n
    return {"file": f"{name}.npz", "N": N, "L0": L0, "P": P, "D": D, "F": F, "head_size": head_size,
            "sk_seed": ckks.sk.seed, "diag_scale": ckks.diag_scale, "max_err_vs_plaintext": err,
            "op_counts": dict(php.OP_COUNTS), "calls": calls,
            "reference": "scripts/bootstrap_generation.py:545-659 (fhe_projection_bsgs), 756-899 "
                         "(client_aided_block), 265-333 (pre_encode_block)"}


def ffn_replay_case(name, N, L0, P, D, F, blocks, seed):
    """tf's fully_encrypted_ffn_block (tf:26-118) chained over `blocks` blocks, every BSGS call
    (re-encoded diagonals at the ciphertext's level, tf:48, 76) recorded, plus each block's output."""
    np.random.seed(seed)
    W_keys = [np.random.randn(D, F) * 0.02 for _ in range(blocks)]
    W_vals = [np.random.randn(F, D) * 0.02 * 25 for _ in range(blocks)]
    x = np.random.randn(D) * 0.1
    ckks = bg.CKKSBootstrapContext(poly_degree=N, L0=L0, prime_bits=59, special_mod_size=P,
                                   max_rot_dim=max(D, F), bsgs_dim=[D, F], skip_bootstrap=True)
    ct = ckks.encrypt_replicated(x)
    ct_in = ct.data.copy()
    CALLS.clear()
    ENC_ORDER.clear()
    reset_counts()
    outs, ref = {}, x.copy()
    for b in range(blocks):
        ct, _ = tf.fully_encrypted_ffn_block(ckks, ct, W_keys[b], W_vals[b], D, F, block_idx=b)
        outs[f"block{b}_out"] = ct.data.copy()
        ref = tf.plaintext_ffn_block(ref, W_keys[b], W_vals[b])
    dec = ckks.decrypt_vec(ct, D)
    err = float(np.max(np.abs(dec - ref)))
    print(f"[{name}] N={N} L0={L0} P={P} D={D} F={F} blocks={blocks} calls={len(CALLS)} max_err={err:.3e}")
    calls = _save_calls(name, CALLS, dict(primes=np.array(ckks.ctx.o.primes, dtype=np.uint64), x=x,
                                          W_keys=np.stack(W_keys), W_vals=np.stack(W_vals), ct_in=ct_in,
                                          **outs))
    return {"file": f"{name}.npz", "N": N, "L0": L0, "P": P, "D": D, "F": F, "blocks": blocks,
            "sk_seed": ckks.sk.seed, "scale": ckks.scale, "max_err": err, "calls": calls,
            "block_out_sha256": [sha(outs[f"block{b}_out"]) for b in range(blocks)],
            "block_chain_index": [None] * blocks,
            "reference": "test_fully_enc_bsgs.py:26-118 (fully_encrypted_ffn_block)"}


def main():
    man = {"generator": "tests/golden/make_golden.py",
           "reference": "scripts/bootstrap_generation.py:198-220,361-542; test_fully_enc_bsgs.py:26-125",
           "backend": "oracle/pyphantom_oracle.py over oracle/ckks_oracle.c", "cases": {}}
    man["cases"]["bsgs_real_n512"] = bsgs_case("bsgs_real_n512", 512, 6, 3, 16, 11)
    man["cases"]["bsgs_complex_n512"] = bsgs_case("bsgs_complex_n512", 512, 6, 3, 16, 12, complex_pack=True)
    man["cases"]["bsgs_real_n1024_p1"] = bsgs_case("bsgs_real_n1024_p1", 1024, 4, 1, 32, 13)
    man["cases"]["ffn_n1024"] = ffn_case("ffn_n1024", 1024, 9, 3, 16, 32, 2, 14)
    _install_recorders()
    man["cases"]["client_aided_n256"] = client_aided_case("client_aided_n256", 256, 4, 2, 8, 32, 4, 15)
    man["cases"]["ffn_replay_n256"] = ffn_replay_case("ffn_replay_n256", 256, 8, 2, 8, 16, 2, 16)
    (OUT / "manifest.json").write_text(json.dumps(man, indent=1, sort_keys=True))
    print("wrote", OUT / "manifest.json")


if __name__ == "__main__":
    main()
