"""Replays of the reference's own orchestration, limb for limb, on the GPU.

tests/golden/make_golden.py ran, with the C oracle installed as `pyPhantom`, the reference's
  - client_aided_block (scripts/bootstrap_generation.py:756-899) with pre-encoded diagonals
    (bg:265-333): its 8 server BSGS calls through fhe_projection_bsgs (bg:545-659) -- r, k, v, o (D -> D),
    the FFN key pairs (D -> F, complex-packed output chunks sharing one set of baby steps, bg:558-606)
    and the FFN value pairs (F -> D, conjugate trick, bg:608-659);
  - test_fully_enc_bsgs.py's fully_encrypted_ffn_block (tf:26-118) over two chained blocks (BSGS,
    CT x CT square + relinearize + rescale, mod-switch alignment, set_scale, residual add);
and recorded every BSGS call's input ciphertext, the slot values of its D plaintexts and its output.

Here the same plaintexts are rebuilt with the same oracle encoder (deterministic; float64 encode is
thereby out of the comparison -- its SHA-256 is checked against the recording), the recorded inputs
are imported, keys are regenerated on the GPU from the recorded seed, and the MI355X restatements of
those callers (tools/rwkv_block.py BlockRunner, tools/ffn_block.py ffn_block) must reproduce every
output ciphertext exactly (np.array_equal)."""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
GOLD = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO / "tools"))


def _case(name):
    man = json.loads((GOLD / "manifest.json").read_text())["cases"][name]
    return man, np.load(GOLD / man["file"])


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _oracle_pts(ph, ctx, o, call, rows):
    """The call's D plaintexts: oracle encode of the recorded slot values at the recorded level."""
    l = o.L0 + 1 - call["pt_level"]
    limbs = np.stack([o.encode(r, call["pt_scale"], l) for r in rows])
    assert _sha(limbs) == call["pt_sha256"], "oracle re-encode differs from the recording"
    return [ph.plaintext_from_numpy(ctx, p, call["pt_level"], call["pt_scale"]) for p in limbs]


@pytest.fixture(scope="module")
def ph(require_gpu):
    import pyPhantom
    return pyPhantom


@pytest.mark.gpu
def test_client_aided_block_server_calls_bit_exact(ph):
    """bg:756-899 server side: 8 BSGS projections in 4 stages, reference limbs reproduced."""
    import rwkv_block as rb
    from oracle.oracle import Oracle
    man, z = _case("client_aided_n256")
    N, L0, P, D, F = man["N"], man["L0"], man["P"], man["D"], man["F"]
    srv = rb.Server(ph, N, L0, P, D, seed=man["sk_seed"])
    assert [int(q) for q in ph.create_coeff_modulus(N, [59] * (L0 + P))] == [int(q) for q in z["primes"]]
    o = Oracle(N, [int(q) for q in z["primes"]], P)
    block = rb.BlockWeights(np.random.default_rng(0), 0, D, F, D // man["head_size"])
    run = rb.BlockRunner(srv, block, False)
    calls = {c["projection"]: (i, c) for i, c in enumerate(man["calls"])}
    run.pre = True
    run.pts = {n: _oracle_pts(ph, srv.ctx, o, c, z[f"c{i}_rows"]) for n, (i, c) in calls.items()}

    def ct_in(n):
        i, c = calls[n]
        return ph.ciphertext_from_numpy(srv.ctx, z[f"c{i}_ct_in"], c["ci_in"], c["scale_in"])
    n_pairs = F // D // 2
    # the FFN key pairs share one input (and its baby steps, bg:563): the recording must say so too
    key_in = [z[f"c{calls[f'ffn_key_{p}'][0]}_ct_in"] for p in range(n_pairs)]
    assert all(np.array_equal(key_in[0], k) for k in key_in)
    shared = ct_in("ffn_key_0")
    stages = [{n: (ct_in(n), n) for n in ("r", "k", "v")}, {"o": (ct_in("o"), "o")},
              {f"ffn_key_{p}": (shared, "x_k_ffn") for p in range(n_pairs)},
              {f"ffn_val_{p}": (ct_in(f"ffn_val_{p}"), f"v{p}") for p in range(n_pairs)}]
    checked = 0
    for idx, ins in enumerate(stages):
        outs = run.stage(idx, ins)
        for n, ct in outs.items():
            i, c = calls[n]
            assert ct.chain_index() == c["ci_out"] and ct.scale() == pytest.approx(c["scale_out"], rel=1e-12)
            assert np.array_equal(ct.to_numpy(), z[f"c{i}_out"]), f"projection {n}: limbs differ from the reference"
            checked += 1
    assert checked == len(man["calls"]) == 8


@pytest.mark.gpu
def test_fully_encrypted_ffn_chain_bit_exact(ph):
    """tf:26-118 over two blocks: every BSGS input and output and each block's output, limb for limb."""
    import ffn_block as fb
    from oracle.oracle import Oracle
    man, z = _case("ffn_replay_n256")
    N, L0, P, D, F = man["N"], man["L0"], man["P"], man["D"], man["F"]
    ck = fb.Ckks(ph, N, L0, P, D, seed=man["sk_seed"])
    o = Oracle(N, [int(q) for q in z["primes"]], P)
    calls = list(enumerate(man["calls"]))
    seen = []

    def replay_matmul(ck_, ct, M, D_, baby):
        i, c = calls[len(seen)]
        seen.append(i)
        assert ct.chain_index() == c["ci_in"]
        assert np.array_equal(ct.to_numpy(), z[f"c{i}_ct_in"]), f"BSGS call {i}: input differs from the reference"
        G, B = fb.bsgs_params(D_)
        pts = _oracle_pts(ph, ck_.ctx, o, c, z[f"c{i}_rows"])
        y = ph.bsgs_multiply_accumulate(ck_.ctx, baby, pts, G, B, D_, ck_.gk)
        assert np.array_equal(y.to_numpy(), z[f"c{i}_out"]), f"BSGS call {i}: output differs from the reference"
        return y

    orig = fb.matmul
    fb.matmul = replay_matmul
    try:
        ct = ph.ciphertext_from_numpy(ck.ctx, z["ct_in"], 1, man["scale"])
        for b in range(man["blocks"]):
            ct = fb.ffn_block(ck, ct, z["W_keys"][b], z["W_vals"][b], D, F)
            assert np.array_equal(ct.to_numpy(), z[f"block{b}_out"]), f"block {b}: output differs from the reference"
    finally:
        fb.matmul = orig
    assert len(seen) == len(calls)


@pytest.mark.gpu
def test_client_aided_block_server_calls_half_limb_vs_oracle(ph):
    """The same 8 server calls (bg:545-659 through tools/rwkv_block.py BlockRunner) at N = 16384, where
    the GPU runs its half-limb NTT workgroup forms (k_ks_intt_h, k_modup_h, k_moddown_h) that the N=256
    recordings never reach (VERDICT r2 missing #6): every projection's output is compared limb for limb
    with the oracle's own baby steps (bg:215-220, one rotation at a time) and BSGS loop (bg:464-485) on
    the same oracle-encrypted input and oracle-encoded diagonals.  L0 = 6 keeps the oracle fast; the
    kernel forms depend on N only."""
    import rwkv_block as rb
    import fhespear_dist
    from oracle.oracle import Oracle, galois_elt
    N, L0, P, D, F, S = 16384, 6, 3, 32, 128, 77
    srv = rb.Server(ph, N, L0, P, D, seed=S)
    primes = [int(q) for q in ph.create_coeff_modulus(N, [59] * (L0 + P))]
    o = Oracle(N, primes, P)
    s = o.gen_secret(S)
    G, B = srv.G, srv.B
    baby_keys = {b: o.gen_galois_key(S, s, galois_elt(b, N)) for b in range(1, G)}
    giant_keys = [None] + [o.gen_galois_key(S, s, galois_elt(g * G, N)) for g in range(1, B)]
    block = rb.BlockWeights(np.random.default_rng(3), 0, D, F, 2)
    run = rb.BlockRunner(srv, block, False)
    run.pre = True
    run.pts, opts = {}, {}
    for name, (kind, ms) in run.mats.items():
        rows = rb._diag_rows(ms[0], D, G, srv.slots)
        if kind == "complex":
            rows = rows + 1j * rb._diag_rows(ms[1], D, G, srv.slots)
        opts[name] = [o.encode(r, srv.diag_scale, L0) for r in rows]
        run.pts[name] = [ph.plaintext_from_numpy(srv.ctx, p, srv.level, srv.diag_scale) for p in opts[name]]
    rng = np.random.default_rng(4)
    inputs, counter = {}, 0

    def enc(key, complex_):
        nonlocal counter
        if key not in inputs:
            z = rng.standard_normal(D) + (1j * rng.standard_normal(D) if complex_ else 0)
            pt = o.encode(np.tile(z, srv.slots // D), srv.scale, L0)
            counter += 1
            inputs[key] = o.encrypt_symmetric(S, counter, s, pt)
        return ph.ciphertext_from_numpy(srv.ctx, inputs[key], srv.level, srv.scale), key
    n_pairs = F // D // 2
    stages = [{n: enc(n, False) for n in ("r", "k", "v")}, {"o": enc("o", False)},
              {f"ffn_key_{p}": enc("x_k_ffn", False) for p in range(n_pairs)},
              {f"ffn_val_{p}": enc(f"v{p}", True) for p in range(n_pairs)}]
    assert [sorted(st) for st in stages] == [sorted(n) for n in fhespear_dist.RWKV_BLOCK_STAGES]
    checked = 0
    for idx, ins in enumerate(stages):
        outs = run.stage(idx, ins)
        for n, (_, key) in ins.items():
            ct = inputs[key]
            baby = [ct] + [o.rotate(ct, baby_keys[b], b) for b in range(1, G)]
            want = o.bsgs_loop(baby, opts[n], giant_keys, G, B, D)
            assert np.array_equal(outs[n].to_numpy(), want), f"projection {n}: limbs differ from the oracle"
            checked += 1
    assert checked == 8
