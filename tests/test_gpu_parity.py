"""GPU parity: libfhespear_hip (through the pyPhantom ctypes shim) vs the CPU oracle, bit-exact on
limbs, plus the committed golden fixtures produced by the reference's own BSGS orchestration
(tests/golden/make_golden.py).  Every test here needs an MI355X: -m gpu."""
import json
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).resolve().parent / "golden"
REPO = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def ph(require_gpu):
    import pyPhantom
    return pyPhantom


def make_ctx(ph, N, L0, P, steps=(), bits=59, seed=99):
    primes = ph.create_coeff_modulus(N, [bits] * (L0 + P))
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(P)
    if steps:
        parms.set_galois_elts(sorted(set(ph.get_elts_from_steps(list(steps), N))))
    parms.set_coeff_modulus(primes)
    ctx = ph.context(parms)
    sk = ph.secret_key(ctx, seed=seed)
    return ctx, sk, [int(q) for q in primes]


def oracle_for(primes, N, P):
    from oracle.oracle import Oracle
    return Oracle(N, primes, P)


def rand_ct(o, rng, ncomp, l):
    return np.stack([np.stack([rng.integers(0, o.primes[i], o.N, dtype=np.uint64) for i in range(l)])
                     for _ in range(ncomp)])


def rand_pt(o, rng, l):
    return np.stack([rng.integers(0, o.primes[i], o.N, dtype=np.uint64) for i in range(l)])


PARAMS = [(1024, 6, 3), (2048, 4, 1), (4096, 6, 2), (32768, 3, 1)]   # N = 32768: half-limb NTT forms


@pytest.mark.parametrize("N,L0,P", PARAMS)
def test_keys_and_encryption_match_oracle(ph, N, L0, P):
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=[1, 5, -3], seed=1234)
    o = oracle_for(primes, N, P)
    s = o.gen_secret(1234)
    assert np.array_equal(sk.export(), s)
    gk = sk.create_galois_keys(ctx)
    for st in (1, 5, -3):
        elt = ph.get_elt_from_step(st, N)
        assert np.array_equal(gk.export(elt), o.gen_galois_key(1234, s, elt)), f"galois key step {st}"
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(0)
    pt = ph.plaintext_from_numpy(ctx, rand_pt(o, rng, L0), 1, 2.0 ** 40)
    ct = sk.encrypt_symmetric(ctx, pt)
    assert np.array_equal(ct.to_numpy(), o.encrypt_symmetric(1234, 0, s, pt.to_numpy()))
    pk = sk.gen_publickey(ctx)
    cta = pk.encrypt_asymmetric(ctx, pt)
    pk_o = o.gen_public_key(1234, s)
    assert np.array_equal(cta.to_numpy(), o.encrypt_asymmetric(1234, 1 << 20, pk_o, pt.to_numpy()))
    # decrypt parity
    assert np.array_equal(sk.decrypt(ctx, ct).to_numpy(), o.decrypt(s, ct.to_numpy()))
    del enc


@pytest.mark.parametrize("N,L0,P", PARAMS)
def test_elementwise_ops_match_oracle(ph, N, L0, P):
    ctx, sk, primes = make_ctx(ph, N, L0, P)
    o = oracle_for(primes, N, P)
    rng = np.random.default_rng(N + L0)
    for l in (L0, max(2, L0 - 1)):
        ci = L0 + 1 - l
        a, b = rand_ct(o, rng, 2, l), rand_ct(o, rng, 2, l)
        p = rand_pt(o, rng, l)
        A = ph.ciphertext_from_numpy(ctx, a, ci, 2.0 ** 40)
        Bc = ph.ciphertext_from_numpy(ctx, b, ci, 2.0 ** 40)
        Pp = ph.plaintext_from_numpy(ctx, p, ci, 2.0 ** 40)
        assert np.array_equal(ph.add(ctx, A, Bc).to_numpy(), o.add(a, b))
        assert np.array_equal(ph.sub(ctx, A, Bc).to_numpy(), o.sub(a, b))
        assert np.array_equal(ph.sub(ctx, A, Bc, True).to_numpy(), o.sub(b, a))
        assert np.array_equal(ph.negate(ctx, A).to_numpy(), o.negate(a))
        assert np.array_equal(ph.multiply_plain(ctx, A, Pp).to_numpy(), o.multiply_plain(a, p))
        assert np.array_equal(ph.add_plain(ctx, A, Pp).to_numpy(), o.add_plain(a, p))
        m = ph.multiply(ctx, A, Bc)
        assert m.size() == 3 and np.array_equal(m.to_numpy(), o.multiply(a, b))
        r = ph.rescale_to_next(ctx, A)
        assert r.chain_index() == ci + 1 and np.array_equal(r.to_numpy(), o.rescale(a))
        d = ph.mod_switch_to_next(ctx, A)
        assert np.array_equal(d.to_numpy(), a[:, :-1])
        assert ph.multiply_plain(ctx, A, Pp).scale() == 2.0 ** 80


@pytest.mark.parametrize("N,L0,P", PARAMS)
def test_rotate_and_relinearize_match_oracle(ph, N, L0, P):
    steps = [1, 2, 7, -1]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, seed=77)
    o = oracle_for(primes, N, P)
    s = o.gen_secret(77)
    gk = sk.create_galois_keys(ctx)
    rlk = sk.gen_relinkey(ctx)
    rng = np.random.default_rng(5)
    for l in (L0, 2):
        ci = L0 + 1 - l
        a = rand_ct(o, rng, 2, l)
        A = ph.ciphertext_from_numpy(ctx, a, ci, 2.0 ** 40)
        # several rotations queued back to back -> one batched key-switch launch
        outs = [ph.rotate(ctx, A, st, gk) for st in steps]
        for st, out in zip(steps, outs):
            want = o.rotate_elt(a, o.gen_galois_key(77, s, ph.get_elt_from_step(st, N)), ph.get_elt_from_step(st, N))
            assert np.array_equal(out.to_numpy(), want), f"rotate step {st} at l={l}"
        c3 = rand_ct(o, rng, 3, l)
        C3 = ph.ciphertext_from_numpy(ctx, c3, ci, 2.0 ** 40)
        assert np.array_equal(ph.relinearize(ctx, C3, rlk).to_numpy(), o.relinearize(c3, o.gen_relin_key(77, s)))


def test_encode_decode_and_rotation_semantics(ph):
    N, L0, P = 2048, 6, 3
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=[1, 3, -2])
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(3)
    x = rng.normal(0, 1, N // 2)
    pt = enc.encode_double_vector(ctx, x, 2.0 ** 40)
    assert np.max(np.abs(np.array(enc.decode_double_vector(ctx, pt)) - x)) < 1e-6
    z = rng.normal(0, 1, N // 2) + 1j * rng.normal(0, 1, N // 2)
    ptc = enc.encode_complex_vector(ctx, z, 2.0 ** 40)
    assert np.max(np.abs(np.array(enc.decode_complex_vector(ctx, ptc)) - z)) < 1e-6
    # oracle encoder agrees to within rounding of the f64 FFT
    o = oracle_for(primes, N, P)
    dec_o = o.decode(pt.to_numpy(), 2.0 ** 40).real
    assert np.max(np.abs(dec_o - x)) < 1e-6
    gk = sk.create_galois_keys(ctx)
    ct = sk.encrypt_symmetric(ctx, pt)
    for st in (1, 3, -2):
        r = ph.rotate(ctx, ct, st, gk)
        d = np.array(enc.decode_double_vector(ctx, sk.decrypt(ctx, r)))
        assert np.max(np.abs(d - np.roll(x, -st))) < 1e-5, st   # left rotation, pb:203
    # batch encode == single encode
    mats = rng.normal(0, 0.1, (3, N // 2))
    batch = enc.encode_double_vector_batch(ctx, mats, 2.0 ** 40, chain_index=2)
    for i in range(3):
        assert batch[i].chain_index() == 2
        assert np.array_equal(batch[i].to_numpy(), enc.encode_double_vector(ctx, mats[i], 2.0 ** 40, 2).to_numpy())


def _load_golden(name):
    man = json.loads((GOLDEN / "manifest.json").read_text())
    return man["cases"][name], np.load(GOLDEN / man["cases"][name]["file"])


@pytest.mark.parametrize("case", ["bsgs_real_n512", "bsgs_complex_n512", "bsgs_real_n1024_p1"])
def test_bsgs_fused_matches_reference_loop_golden(ph, case):
    """Golden fixture = reference bg:464-485 loop executed on the oracle; the fused GPU op must
    reproduce its output limbs exactly from the same baby steps, diagonals and keys."""
    meta, z = _load_golden(case)
    N, L0, P, D, G, B = (meta[k] for k in ("N", "L0", "P", "D", "G", "B"))
    primes = [int(q) for q in z["primes"]]
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(P)
    parms.set_galois_elts(meta["giant_elts"])
    parms.set_coeff_modulus(primes)
    ctx = ph.context(parms)
    sk = ph.secret_key(ctx, seed=meta["sk_seed"])
    gk = sk.create_galois_keys(ctx)
    import hashlib
    for elt, digest in meta["giant_key_sha256"].items():
        assert hashlib.sha256(gk.export(int(elt)).tobytes()).hexdigest() == digest
    ci = meta["chain_index_in"]
    baby = [ph.ciphertext_from_numpy(ctx, z["baby"][b], ci, meta["scale"]) for b in range(G)]
    pts = [ph.plaintext_from_numpy(ctx, z["pts"][k], ci, meta["diag_scale"]) for k in range(D)]
    y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    assert y.chain_index() == meta["chain_index_out"]
    assert np.isclose(y.scale(), meta["scale_out"], rtol=1e-12)
    assert np.array_equal(y.to_numpy(), z["out"])
    # streamed-from-host variant (bg:449) is the same computation
    data, cci, sc, cms, pmd = ph.offload_plaintexts(pts)
    y2 = ph.bsgs_from_cpu(ctx, baby, data, cci, sc, cms, pmd, G, B, D, gk)
    assert np.array_equal(y2.to_numpy(), z["out"])
    up = ph.upload_plaintexts(data, cci, sc, cms, pmd)
    assert np.array_equal(up[3].to_numpy(), z["pts"][3])


def test_bsgs_fused_equals_op_by_op_loop(ph):
    """Fused bsgs_multiply_accumulate == the bg:464-485 loop issued op by op through pyPhantom."""
    N, L0, P, D = 2048, 6, 3, 64
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, seed=5)
    gk = sk.create_galois_keys(ctx)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(8)
    x = rng.normal(0, 0.1, D)
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(x, (N // 2) // D), 2.0 ** 59))
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    pts = ph.random_plaintexts(ctx, 3, D, ct.chain_index(), 2.0 ** 59)
    res = None
    for g in range(B):
        inner = None
        for b in range(G):
            k = g * G + b
            if k >= D:
                continue
            term = ph.multiply_plain(ctx, baby[b], pts[k])
            inner = term if inner is None else ph.add(ctx, inner, term)
        if g > 0:
            inner = ph.rotate(ctx, inner, g * G, gk)
        res = inner if res is None else ph.add(ctx, res, inner)
    res = ph.rescale_to_next(ctx, res)
    fused = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    assert np.array_equal(fused.to_numpy(), res.to_numpy())


def test_bsgs_complete_from_cpu_thread_pool(ph):
    """bg:226-249 _parallel_bsgs_projections: ph.bsgs_complete_from_cpu (baby steps + host-streamed
    BSGS in one call) issued from a 4-worker thread pool on one context equals the sequential
    rotate + bsgs_multiply_accumulate for each input, limb for limb."""
    from concurrent.futures import ThreadPoolExecutor
    N, L0, P, D = 2048, 6, 3, 64
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, seed=6)
    gk = sk.create_galois_keys(ctx)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(9)
    cts = [sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(rng.normal(0, 0.1, D), (N // 2) // D),
                                                              2.0 ** 59)) for _ in range(4)]
    pts = [ph.random_plaintexts(ctx, 10 + i, D, cts[0].chain_index(), 2.0 ** 59) for i in range(4)]
    host = [ph.offload_plaintexts(p) for p in pts]
    with ThreadPoolExecutor(max_workers=4) as pool:
        futs = [pool.submit(ph.bsgs_complete_from_cpu, ctx, ct, *h, G, B, D, gk) for ct, h in zip(cts, host)]
        got = [f.result() for f in futs]
    for ct, p, y in zip(cts, pts, got):
        baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
        assert np.array_equal(y.to_numpy(), ph.bsgs_multiply_accumulate(ctx, baby, p, G, B, D, gk).to_numpy())


def test_bsgs_decrypts_to_matvec(ph):
    """Accuracy contract of tf:272-298 (corr > 0.999) on the reference's diagonal layout."""
    import __graft_entry__ as ge
    N, L0, P, D = 4096, 6, 3, 128
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps)
    gk = sk.create_galois_keys(ctx)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(42)
    x = rng.normal(0, 0.1, D)
    W = rng.normal(0, 0.02, (D, D))
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(x, (N // 2) // D), 2.0 ** 59))
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    pts = enc.encode_double_vector_batch(ctx, ge._rolled_diagonals(W, D, G, N // 2), 2.0 ** 59,
                                         chain_index=ct.chain_index())
    y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    dec = np.array(enc.decode_double_vector(ctx, sk.decrypt(ctx, y)))[:D]
    ref = W @ x
    assert np.corrcoef(dec, ref)[0, 1] > 0.999999
    assert np.max(np.abs(dec - ref)) < 1e-8


def test_errors(ph):
    ctx, sk, primes = make_ctx(ph, 1024, 6, 3, steps=[1])
    gk = sk.create_galois_keys(ctx)
    enc = ph.ckks_encoder(ctx)
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, [1.0], 2.0 ** 40))
    with pytest.raises(ValueError):
        ph.rotate(ctx, ct, 2, gk)      # no key for step 2
    low = ph.mod_switch_to_next(ctx, ct)
    with pytest.raises(ValueError):
        ph.add(ctx, ct, low)           # chain index mismatch
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(1024)
    parms.set_special_modulus_size(3)
    parms.set_coeff_modulus(ph.create_coeff_modulus(1024, [59] * 8))   # L0 = 5, not a multiple of 3
    with pytest.raises(ValueError):
        ph.context(parms)


@pytest.mark.parametrize("N,L0,P,D", [(8192, 24, 3, 1024), (16384, 36, 3, 2048)])
def test_fused_bsgs_equals_loop_at_baseline_configs(ph, N, L0, P, D):
    """BASELINE configs[0] / configs[1] at full size (d=1024 N=8192 L0=24; d=2048 N=16384 L0=36):
    the fused bsgs_multiply_accumulate equals the reference loop bg:464-485 issued op by op
    (D multiply_plain, D-1 add, B-1 rotate, 1 rescale) limb for limb, and the decrypted result is
    the matvec (tf:272-298's corr criterion, tighter)."""
    import __graft_entry__ as ge
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, seed=13)
    enc = ph.ckks_encoder(ctx)
    gk = sk.create_galois_keys(ctx)
    rng = np.random.default_rng(14)
    x = rng.normal(0, 0.1, D)
    W = rng.normal(0, 0.02, (D, D))
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(x, (N // 2) // D), 2.0 ** 59))
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    pts = enc.encode_double_vector_batch(ctx, ge._rolled_diagonals(W, D, G, N // 2), 2.0 ** 59,
                                         chain_index=ct.chain_index())
    res = None
    for g in range(B):
        inner = None
        for b in range(G):
            k = g * G + b
            if k >= D:
                continue
            term = ph.multiply_plain(ctx, baby[b], pts[k])
            inner = term if inner is None else ph.add(ctx, inner, term)
        if g > 0:
            inner = ph.rotate(ctx, inner, g * G, gk)
        res = inner if res is None else ph.add(ctx, res, inner)
    res = ph.rescale_to_next(ctx, res)
    fused = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    assert np.array_equal(fused.to_numpy(), res.to_numpy())
    dec = np.array(enc.decode_double_vector(ctx, sk.decrypt(ctx, fused)))[:D]
    ref = W @ x
    assert np.corrcoef(dec, ref)[0, 1] > 0.999999
    assert np.max(np.abs(dec - ref)) < 1e-8


_DECODE_SCRIPT = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[2])
import pyPhantom as ph
N, L0, P = 4096, 12, 3
parms = ph.params(ph.scheme_type.ckks)
parms.set_poly_modulus_degree(N); parms.set_special_modulus_size(P)
parms.set_galois_elts(ph.get_elts_from_steps([1], N))
parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (L0 + P)))
ctx = ph.context(parms); sk = ph.secret_key(ctx, seed=4); enc = ph.ckks_encoder(ctx)
rng = np.random.default_rng(6)
x = rng.normal(0, 1, N // 2)
pt = enc.encode_double_vector(ctx, x, 2.0 ** 40)
ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, x, 2.0 ** 59))
prod = ph.multiply(ctx, ct, ct)                       # scale 2^118, 3 components
rk = sk.gen_relinkey(ctx)
sq = ph.relinearize(ctx, prod, rk)
q = [int(v) for v in ph.create_coeff_modulus(N, [59] * (L0 + P))][:L0]
junk = ph.plaintext_from_numpy(ctx, np.stack([rng.integers(0, q[i], N, dtype=np.uint64) for i in range(L0)]), 1, 2.0 ** 40)
out = [np.array(enc.decode_complex_vector(ctx, p)) for p in (pt, sk.decrypt(ctx, ct), sk.decrypt(ctx, sq), junk)]
# an alias the magnitude heuristic could not see: x = Q_3 M + s with small s looks small on the first
# 3 limbs (the ones composed at scale 2^40) -- only the check against the other limbs catches it
sys.path.insert(0, sys.argv[3])
from oracle.oracle import Oracle
o = Oracle(N, [int(v) for v in ctx.primes], P)
Q3 = q[0] * q[1] * q[2]
M = rng.integers(1, 2 ** 60, N)
sm = rng.integers(-2 ** 40, 2 ** 40, N)
xs = [Q3 * int(M[n]) + int(sm[n]) for n in range(N)]
alias = ph.plaintext_from_numpy(ctx, np.stack([o.ntt(np.array([v % q[i] for v in xs], dtype=np.uint64), i)
                                               for i in range(L0)]), 1, 2.0 ** 40)
out.append(np.array(enc.decode_complex_vector(ctx, alias)))
# a 7-limb ring: uniform limbs take the all-limb fallback through the widest GPU composition
parms7 = ph.params(ph.scheme_type.ckks)
parms7.set_poly_modulus_degree(N); parms7.set_special_modulus_size(1)
parms7.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * 8))
ctx7 = ph.context(parms7); enc7 = ph.ckks_encoder(ctx7)
q7 = [int(v) for v in ctx7.primes][:7]
for scale in (2.0 ** 40, 2.0 ** 100):
    junk7 = ph.plaintext_from_numpy(ctx7, np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in q7]), 1, scale)
    out.append(np.array(enc7.decode_complex_vector(ctx7, junk7)))
np.save(sys.argv[1], np.stack(out))
'''


def test_decode_shortcut_equals_full_crt(require_gpu, tmp_path):
    """fhs_decode composes the centred CRT from the first k limbs (+1 as a check, full fallback);
    its output must be bitwise identical to composing all limbs (FHESPEAR_DECODE_FULL=1), and the
    GPU composition (k_crt_compose, up to 7 limbs) to the host's (FHESPEAR_DECODE_HOST_CRT=1): a
    plaintext at 2^40, a fresh decryption at 2^59, a squared one at 2^118, uniformly random limbs
    (|x| ~ Q/2, which takes the fallback) and coefficients Q_3 M + s that alias to small values on the
    composed limbs (caught by the check against the remaining limbs)."""
    import os
    import subprocess
    import sys as _sys
    script = tmp_path / "dec.py"
    script.write_text(_DECODE_SCRIPT)
    pyp = str(REPO / "fhe-spear_amd" / "python")
    outs = []
    for i, knob in enumerate((None, "FHESPEAR_DECODE_FULL", "FHESPEAR_DECODE_HOST_CRT")):
        env = dict(os.environ)
        env.pop("FHESPEAR_DECODE_FULL", None)
        env.pop("FHESPEAR_DECODE_HOST_CRT", None)
        if knob:
            env[knob] = "1"
        f = tmp_path / f"dec_{i}.npy"
        r = subprocess.run([_sys.executable, str(script), str(f), pyp, str(REPO)], env=env, capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(np.load(f))
    assert np.array_equal(outs[0].view(np.uint64), outs[1].view(np.uint64))
    assert np.array_equal(outs[0].view(np.uint64), outs[2].view(np.uint64))


_ENCODE_SCRIPT = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[2])
import pyPhantom as ph
out = []
for N, L0 in ((4096, 8), (32768, 3)):
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N); parms.set_special_modulus_size(1)
    parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (L0 + 1)))
    ctx = ph.context(parms); enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(N)
    r = enc.encode_double_vector_batch(ctx, rng.normal(0, 3, (3, N // 2)), 2.0 ** 59, chain_index=1)
    z = rng.normal(0, 3, (2, N // 2)) + 1j * rng.normal(0, 3, (2, N // 2))
    c = enc.encode_complex_vector_batch(ctx, z, 2.0 ** 70, chain_index=2)
    # periodic rows (the sparse form, t = 2, 4, 8 in one batch, and complex t = 4)
    per = [np.tile(rng.normal(0, 3, N // 2 // t), t) for t in (2, 4, 8, 16)]
    rp = enc.encode_double_vector_batch(ctx, np.stack(per), 2.0 ** 59, chain_index=1)
    cp = enc.encode_complex_vector_batch(ctx, np.tile(z[:, :N // 8], (1, 4)), 2.0 ** 70, chain_index=2)
    out += [p.to_numpy().ravel() for p in r + c + rp + cp]
np.save(sys.argv[1], np.concatenate(out))
'''


def test_encode_fused_ntt_equals_unfused(require_gpu, tmp_path):
    """The encoder's fused exact-reduction + NTT (k_ntt_fwd_from_dbl) gives the same limbs as
    reducing into every limb and transforming in place (FHESPEAR_ENCODE_UNFUSED=1), at N = 4096 and
    at N = 32768 (split FFT, half-limb NTT), real and complex, scales 2^59 and 2^70 -- and for periodic rows
    the (N/t)-point NTTs of the sparse form (k_ntt_fwd_from_dbl_sp, t = 2, 4, 8) give the limbs of the N-point NTT
    of the spread coefficients (the unfused path)."""
    import os
    import subprocess
    import sys as _sys
    script = tmp_path / "enc.py"
    script.write_text(_ENCODE_SCRIPT)
    pyp = str(REPO / "fhe-spear_amd" / "python")
    outs = []
    for unfused in (False, True):
        env = dict(os.environ)
        env.pop("FHESPEAR_ENCODE_UNFUSED", None)
        if unfused:
            env["FHESPEAR_ENCODE_UNFUSED"] = "1"
        f = tmp_path / f"enc_{int(unfused)}.npy"
        r = subprocess.run([_sys.executable, str(script), str(f), pyp], env=env, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(np.load(f))
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("N,t", [(4096, 2), (4096, 16), (16384, 4), (32768, 8)])
def test_encode_periodic_rows_take_the_sparse_form(ph, N, t):
    """Tiled rows (np.tile of an (N/2t)-vector: the reference's diagonals, bg:361-378, and replicated inputs,
    bg:53-58) are encoded as p(X^t'), t' = min(t, 8) (fhs_kernels.hip k_enc_period): in coefficient form (the
    oracle's INTT of every limb) the coefficients off the multiples of t' are exact zeros, in NTT form every value
    repeats t' times, and the slots decode to the input as closely as the dense encoder's do.  A row that breaks the
    period in one value keeps the dense form."""
    ctx, _, primes = make_ctx(ph, N, 3, 1, seed=31)
    enc = ph.ckks_encoder(ctx)
    o = oracle_for(primes, N, 1)
    rng = np.random.default_rng(N + t)
    d, tt = N // 2 // t, min(t, 8)
    x = rng.normal(0, 1, d)
    z = rng.normal(0, 1, d) + 1j * rng.normal(0, 1, d)
    off = np.arange(N) % tt != 0
    for want, pt in ((np.tile(x, t), enc.encode_double_vector(ctx, np.tile(x, t), 2.0 ** 40)),
                     (np.tile(z, t), enc.encode_complex_vector(ctx, np.tile(z, t), 2.0 ** 40))):
        limbs = pt.to_numpy()
        assert (limbs.reshape(limbs.shape[0], N // tt, tt) == limbs[:, ::tt, None]).all()
        for i in range(limbs.shape[0]):
            assert not o.intt(limbs[i], i)[off].any(), f"limb {i}: nonzero coefficient off the multiples of {tt}"
        if np.iscomplexobj(want):
            dec = np.array(enc.decode_complex_vector(ctx, pt))
        else:
            dec = np.array(enc.decode_double_vector(ctx, pt))
        assert np.max(np.abs(dec - want)) < 1e-6
        # the oracle's decoder (CRT + its own FFT) reads the same slots from these limbs
        dec_o = o.decode(limbs, 2.0 ** 40)
        assert np.max(np.abs((dec_o if np.iscomplexobj(want) else dec_o.real) - want)) < 1e-6
    y = np.tile(x, t)
    y[-1] += 1.0
    limbs = enc.encode_double_vector(ctx, y, 2.0 ** 40).to_numpy()
    assert o.intt(limbs[0], 0)[off].any()
    assert np.max(np.abs(np.array(enc.decode_double_vector(ctx, enc.encode_double_vector(ctx, y, 2.0 ** 40))) - y)) < 1e-6


@pytest.mark.parametrize("N,D,L0", [(4096, 1024, 4), (16384, 2048, 3), (32768, 2048, 3), (32768, 8192, 2)])
def test_bsgs_compact_diagonals_equal_dense(ph, N, D, L0):
    """Tiled diagonals (encode_matrix_diagonals, bg:361-378) carry a compact shadow (word e >> t of each limb
    holds dense word e, t = log2 of the tiling, at most 3) that the fused BSGS's Hadamard reads instead of the
    dense limbs (k_bsgs_inner<..., TL>): the matvec, the inner products alone and the linear transform give the
    limbs of the same call on dense copies of the same plaintexts (plaintext_from_numpy: no shadow).  D = 8192
    (G = 91) takes the baby-step windows (G > 64) on compact diagonals."""
    G = int(np.ceil(np.sqrt(D)))
    B = -(-D // G)
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, _ = make_ctx(ph, N, L0, 1, steps=steps, seed=41)
    gk = sk.create_galois_keys(ctx)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(N + D)
    x = rng.normal(0, 0.1, D)
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(x, N // 2 // D), 2.0 ** 50))
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    W = rng.normal(0, 0.02, (D, D))
    pts = enc.encode_matrix_diagonals(ctx, W, G, 2.0 ** 50, chain_index=ct.chain_index())
    dense = [ph.plaintext_from_numpy(ctx, p.to_numpy(), p.chain_index(), p.scale()) for p in pts]
    got = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk).to_numpy()
    want = ph.bsgs_multiply_accumulate(ctx, baby, dense, G, B, D, gk).to_numpy()
    assert np.array_equal(got, want)
    if D == 2048 and N == 16384:
        dec = np.array(enc.decode_double_vector(ctx, sk.decrypt(ctx, ph.bsgs_multiply_accumulate(
            ctx, baby, pts, G, B, D, gk))))[:D]
        assert np.max(np.abs(dec - W @ x)) < 1e-4
        Bi = 3
        gi = [c.to_numpy() for c in ph.bsgs_inner_products(ctx, baby, pts[:Bi * G], G, Bi)]
        wi = [c.to_numpy() for c in ph.bsgs_inner_products(ctx, baby, dense[:Bi * G], G, Bi)]
        assert all(np.array_equal(a, b) for a, b in zip(gi, wi))


def test_compact_plaintexts_behave_as_dense(ph):
    """A batch of >= 32 periodic rows is stored compact only (fhs_host.hip new_pts_compact): every op other than the
    fused BSGS's Hadamard expands it on first use (pt_dense), so multiply_plain / add_plain, decode, encryption,
    plain mod_switch, export and offload_plaintexts see the limbs of the same rows encoded one at a time (dense)."""
    N, L0 = 4096, 4
    ctx, sk, _ = make_ctx(ph, N, L0, 1, seed=61)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(62)
    rows = np.tile(rng.normal(0, 1, (40, N // 8)), (1, 4))
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, rng.normal(0, 1, N // 2), 2.0 ** 40, 2))

    def fresh():
        return enc.encode_double_vector_batch(ctx, rows, 2.0 ** 40, chain_index=2)
    single = [enc.encode_double_vector(ctx, rows[k], 2.0 ** 40, 2) for k in (0, 7, 39)]
    for op in (ph.multiply_plain, ph.add_plain):   # the first use of each compact plaintext is the op itself
        b = fresh()
        for k, s in zip((0, 7, 39), single):
            assert np.array_equal(op(ctx, ct, b[k]).to_numpy(), op(ctx, ct, s).to_numpy())
    b = fresh()
    assert np.array_equal(np.array(enc.decode_double_vector(ctx, b[7])), np.array(enc.decode_double_vector(ctx, single[1])))
    b = fresh()
    assert np.array_equal(ph.mod_switch_to_next(ctx, b[39]).to_numpy(), ph.mod_switch_to_next(ctx, single[2]).to_numpy())
    b = fresh()
    dec = np.array(enc.decode_double_vector(ctx, sk.decrypt(ctx, sk.encrypt_symmetric(ctx, b[0]))))
    assert np.max(np.abs(dec - rows[0])) < 1e-6
    b = fresh()
    data = ph.offload_plaintexts(b)
    assert np.array_equal(np.asarray(data[0])[7], single[1].to_numpy())
    assert all(np.array_equal(b[k].to_numpy(), s.to_numpy()) for k, s in zip((0, 7, 39), single))


def _bg_rows(W, D, G, slots):
    """numpy restatement of bg:198-203 (_extract_diagonals) + bg:361-378 (roll, tile, remainder)"""
    j = np.arange(D)
    d = W[j[None, :], (j[None, :] + j[:, None]) % D]
    r = d.copy()
    for g in range(1, (D + G - 1) // G):
        s, e = g * G, min((g + 1) * G, D)
        r[s:e, g * G:] = d[s:e, :D - g * G]
        r[s:e, :g * G] = d[s:e, D - g * G:]
    reps, rem = divmod(slots, D)
    return np.concatenate([np.tile(r, (1, reps)), r[:, :rem]], axis=1) if rem else np.tile(r, (1, reps))


@pytest.mark.parametrize("N,D", [(1024, 32), (1024, 48), (16384, 2048)])
def test_encode_matrix_diagonals_equals_host_rows(ph, N, D):
    """Extension fhs_encode_diagonals (diagonal extraction, roll, tiling on the GPU) yields the same
    plaintext limbs as the batch encoder fed the reference caller's numpy rows (real and complex,
    slot count a multiple of D or not)."""
    G = int(np.ceil(np.sqrt(D)))
    ctx, sk, primes = make_ctx(ph, N, 6 if N < 16384 else 36, 3, seed=17)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(18)
    W1, W2 = rng.normal(0, 0.02, (D, D)), rng.normal(0, 0.02, (D, D))
    slots = N // 2
    got = enc.encode_matrix_diagonals(ctx, W1, G, 2.0 ** 59, chain_index=2)
    want = enc.encode_double_vector_batch(ctx, _bg_rows(W1, D, G, slots), 2.0 ** 59, chain_index=2)
    for k in (0, 1, G - 1, G, D // 2, D - 1):
        assert np.array_equal(got[k].to_numpy(), want[k].to_numpy()), f"real diagonal {k}"
    gotc = enc.encode_matrix_diagonals(ctx, W1, G, 2.0 ** 59, chain_index=2, M2=W2)
    wantc = enc.encode_complex_vector_batch(ctx, _bg_rows(W1, D, G, slots) + 1j * _bg_rows(W2, D, G, slots),
                                            2.0 ** 59, chain_index=2)
    for k in (0, G, D - 1):
        assert np.array_equal(gotc[k].to_numpy(), wantc[k].to_numpy()), f"complex diagonal {k}"
    # strided and transposed numpy views are read in place (fhs_encode_diagonals_ex)
    big = rng.normal(0, 0.02, (D, 2 * D + 3))
    for view in (big[:, 3:3 + D], big[:, 3:3 + D].T):
        gv = enc.encode_matrix_diagonals(ctx, view, G, 2.0 ** 59, chain_index=2)
        wv = enc.encode_double_vector_batch(ctx, _bg_rows(np.ascontiguousarray(view), D, G, slots), 2.0 ** 59,
                                            chain_index=2)
        for k in (0, G, D - 1):
            assert np.array_equal(gv[k].to_numpy(), wv[k].to_numpy()), f"view diagonal {k}"
    # a sharded matvec's rank encodes only its rows (fhs_encode_diagonals_rows): a giant column's
    # contiguous range and a grid rank's scattered baby share, real and complex, same limbs as the full set
    import fhespear_dist as fd
    B = -(-D // G)
    for rows in (list(range(G, min(D, 3 * G))), fd.grid_rows(G, B, D, 4, 2, 3), [D - 1, 0, G]):
        sub = enc.encode_matrix_diagonals(ctx, W1, G, 2.0 ** 59, chain_index=2, rows=rows)
        subc = enc.encode_matrix_diagonals(ctx, W1, G, 2.0 ** 59, chain_index=2, M2=W2, rows=rows)
        assert len(sub) == len(rows)
        for p, pc, k in zip(sub, subc, rows):
            assert np.array_equal(p.to_numpy(), got[k].to_numpy()), f"row subset, diagonal {k}"
            assert np.array_equal(pc.to_numpy(), gotc[k].to_numpy()), f"complex row subset, diagonal {k}"
    with pytest.raises(ValueError):
        enc.encode_matrix_diagonals(ctx, W1, G, 2.0 ** 59, chain_index=2, rows=[D])


def test_bsgs_matches_oracle_on_cfg2_ring(ph):
    """The cfg2 ring and chain (N = 16384, 36 + 3 primes) with a small D = 16 so the C oracle
    finishes in seconds: keys, encryption, hoisted baby rotations and the fused BSGS are
    bit-identical to the oracle's restatement of bg:215-220 + bg:464-485 at full size."""
    N, L0, P, D, seed = 16384, 36, 3, 16, 31
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, seed=seed)
    gk = sk.create_galois_keys(ctx)
    o = oracle_for(primes, N, P)
    s = o.gen_secret(seed)
    rng = np.random.default_rng(15)
    a = rand_ct(o, rng, 2, L0)
    ct = ph.ciphertext_from_numpy(ctx, a, 1, 2.0 ** 59)
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    bkeys = {b: o.gen_galois_key(seed, s, ph.get_elt_from_step(b, N)) for b in range(1, G)}
    want_baby = [a] + [o.rotate_elt(a, bkeys[b], ph.get_elt_from_step(b, N)) for b in range(1, G)]
    for b in range(G):
        assert np.array_equal(baby[b].to_numpy(), want_baby[b]), f"baby step {b}"
    pts = ph.random_plaintexts(ctx, 16, D, 1, 2.0 ** 59)
    y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    gkeys = [None] + [o.gen_galois_key(seed, s, ph.get_elt_from_step(g * G, N)) for g in range(1, B)]
    want = o.bsgs_loop(want_baby, [p.to_numpy() for p in pts], gkeys, G, B, D)
    assert np.array_equal(y.to_numpy(), want)


def test_cfg5_ring_matches_oracle(ph):
    """BASELINE configs[4]'s ring and chain (N = 32768, 36 + 3 primes of 59 bits: tf --N 32768 --L0 36 --P 3, tf:134,
    tf:209-218) with D = 16 so the C oracle finishes in seconds: the secret, Galois keys,
    symmetric encryption, the hoisted baby rotations (bg:215-220), the fused BSGS (bg:464-485), the FFN's square
    (tf:57-61: multiply + relinearize + rescale_to_next) and mod_switch_to_next, each bit-identical to the oracle.
    Every NTT of this ring runs in its half-limb form with the radix-8 global stages and the lazy encoder NTTs
    of round 5."""
    N, L0, P, D, seed = 32768, 36, 3, 16, 53
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, seed=seed)
    o = oracle_for(primes, N, P)
    s = o.gen_secret(seed)
    assert np.array_equal(sk.export(), s)
    gk = sk.create_galois_keys(ctx)
    rlk = sk.gen_relinkey(ctx)
    keys = {st: o.gen_galois_key(seed, s, ph.get_elt_from_step(st, N)) for st in steps}
    for st in (1, G):
        assert np.array_equal(gk.export(ph.get_elt_from_step(st, N)), keys[st]), f"galois key step {st}"
    rng = np.random.default_rng(29)
    pt = ph.plaintext_from_numpy(ctx, rand_pt(o, rng, L0), 1, 2.0 ** 59)
    ct = sk.encrypt_symmetric(ctx, pt)
    a = o.encrypt_symmetric(seed, 0, s, pt.to_numpy())
    assert np.array_equal(ct.to_numpy(), a)
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    want_baby = [a] + [o.rotate_elt(a, keys[b], ph.get_elt_from_step(b, N)) for b in range(1, G)]
    for b in range(G):
        assert np.array_equal(baby[b].to_numpy(), want_baby[b]), f"baby step {b}"
    pts = ph.random_plaintexts(ctx, 23, D, 1, 2.0 ** 59)
    y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    yw = o.bsgs_loop(want_baby, [p.to_numpy() for p in pts], [None] + [keys[g * G] for g in range(1, B)], G, B, D)
    assert np.array_equal(y.to_numpy(), yw)
    sq = ph.rescale_to_next(ctx, ph.relinearize(ctx, ph.multiply(ctx, y, y), rlk))
    sqw = o.rescale(o.relinearize(o.multiply(yw, yw), o.gen_relin_key(seed, s)))
    assert sq.chain_index() == 3 and np.array_equal(sq.to_numpy(), sqw)
    assert np.array_equal(ph.mod_switch_to_next(ctx, sq).to_numpy(), sqw[:, :-1])


@pytest.mark.parametrize("D,bits", [(8192, 59), (4290, 60)])
def test_bsgs_g_above_64_matches_oracle(ph, D, bits):
    """D = 8192 at N = 16384 (tf --D 8192: G = B = 91, D <= slots): the fused BSGS's Hadamard runs in two
    baby-step windows (64 + 27 baby steps; the second adds its sums to the first's), bit-identical to the
    oracle's restatement of the reference loop bg:464-485 (before round 6 this shape was
    rejected with hipErrorInvalidValue).  The inner products alone (the latency modes' half) are checked
    against the oracle's sums too.  D = 4290 on 60-bit primes: G = 66 (a 2-step second window), a short last
    giant group, and the 8-products-per-fold accumulator variant of both windows."""
    N, L0, P, seed = 16384, 3, 1, 61
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    assert (G, B) == ((91, 91) if D == 8192 else (66, 65))
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, bits=bits, seed=seed)
    gk = sk.create_galois_keys(ctx)
    o = oracle_for(primes, N, P)
    s = o.gen_secret(seed)
    rng = np.random.default_rng(91)
    a = rand_ct(o, rng, 2, L0)
    ct = ph.ciphertext_from_numpy(ctx, a, 1, 2.0 ** 40)
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    want_baby = [a] + [o.rotate_elt(a, o.gen_galois_key(seed, s, ph.get_elt_from_step(b, N)), ph.get_elt_from_step(b, N))
                       for b in range(1, G)]
    for b in (1, 63, 64, G - 1):
        assert np.array_equal(baby[b].to_numpy(), want_baby[b]), f"baby step {b}"
    pts = ph.random_plaintexts(ctx, 19, D, 1, 2.0 ** 40)
    pn = [p.to_numpy() for p in pts]
    y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    gkeys = [None] + [o.gen_galois_key(seed, s, ph.get_elt_from_step(g * G, N)) for g in range(1, B)]
    assert np.array_equal(y.to_numpy(), o.bsgs_loop(want_baby, pn, gkeys, G, B, D))
    zero = ph.plaintext_from_numpy(ctx, np.zeros((L0, N), dtype=np.uint64), 1, 2.0 ** 40)
    inner = ph.bsgs_inner_products(ctx, baby, list(pts) + [zero] * (G * B - D), G, B)
    for g in (0, 1, B - 1):
        acc = None
        for b in range(G):
            if g * G + b < D:
                t = o.multiply_plain(want_baby[b], pn[g * G + b])
                acc = t if acc is None else o.add(acc, t)
        assert np.array_equal(inner[g].to_numpy(), acc), f"inner product of giant group {g}"


def test_exact_p1_all_59_bit_rotations_match_oracle(ph):
    """Exact (default) key switching with P = 1 on an all-59-bit chain at N = 16384, L0 = 36 (the cfg2seal ring in
    the default convention): one-prime digits take the radix-4 ModUp conversion (modup_convert1_r4, all_b59) and
    the centred v = 1 branch -- a batch of hoisted rotations and a relinearisation, bit-identical to the oracle
    (this path was covered only by the bench digest)."""
    N, L0, P, seed = 16384, 36, 1, 83
    steps = [1, 5, -7]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, seed=seed)
    assert all(q < 2 ** 59 for q in primes)
    o = oracle_for(primes, N, P)
    s = o.gen_secret(seed)
    gk = sk.create_galois_keys(ctx)
    rlk = sk.gen_relinkey(ctx)
    rng = np.random.default_rng(37)
    for l in (L0, 20):
        a = rand_ct(o, rng, 2, l)
        A = ph.ciphertext_from_numpy(ctx, a, L0 + 1 - l, 2.0 ** 40)
        outs = [ph.rotate(ctx, A, st, gk) for st in steps]
        for st, out in zip(steps, outs):
            e = ph.get_elt_from_step(st, N)
            assert np.array_equal(out.to_numpy(), o.rotate_elt(a, o.gen_galois_key(seed, s, e), e)), f"step {st}, l={l}"
    c3 = rand_ct(o, rng, 3, L0)
    C3 = ph.ciphertext_from_numpy(ctx, c3, 1, 2.0 ** 40)
    assert np.array_equal(ph.relinearize(ctx, C3, rlk).to_numpy(), o.relinearize(c3, o.gen_relin_key(seed, s)))


@pytest.mark.parametrize("bits", [59, 60])
def test_bsgs_full_batches_match_oracle(ph, bits):
    """Shapes the small oracle tests above miss: G = 23 (two full 8-diagonal batches plus a tail per giant
    group, the Hadamard's rolling refill) and B = 23 (waves with two giant groups, the next group's
    first batch requested after a group's stores), with 59-bit primes (16 products per fold, lazy NTT)
    and 60-bit ones (8 per fold and batch-at-a-time loads, Harvey NTT, the X form at b = 60) -- the
    hoisted baby steps and the fused BSGS bit-identical to the oracle's loop (bg:215-220, bg:464-485)."""
    N, L0, P, D, seed = 1024, 6, 3, 512, 41
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    assert (G, B) == (23, 23)
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, bits=bits, seed=seed)
    gk = sk.create_galois_keys(ctx)
    o = oracle_for(primes, N, P)
    s = o.gen_secret(seed)
    rng = np.random.default_rng(bits)
    a = rand_ct(o, rng, 2, L0)
    ct = ph.ciphertext_from_numpy(ctx, a, 1, 2.0 ** 40)
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    bkeys = {b: o.gen_galois_key(seed, s, ph.get_elt_from_step(b, N)) for b in range(1, G)}
    want_baby = [a] + [o.rotate_elt(a, bkeys[b], ph.get_elt_from_step(b, N)) for b in range(1, G)]
    for b in range(G):
        assert np.array_equal(baby[b].to_numpy(), want_baby[b]), f"baby step {b}"
    pts = ph.random_plaintexts(ctx, 17, D, 1, 2.0 ** 40)
    y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    gkeys = [None] + [o.gen_galois_key(seed, s, ph.get_elt_from_step(g * G, N)) for g in range(1, B)]
    want = o.bsgs_loop(want_baby, [p.to_numpy() for p in pts], gkeys, G, B, D)
    assert np.array_equal(y.to_numpy(), want)


def test_n32768_encode_bsgs_and_fused_equals_loop(ph):
    """cfg5's ring size (N = 32768, BASELINE configs[4]): every NTT runs in its half-limb form and
    the encoder FFT in its split form; decode accuracy, fused BSGS == op-by-op loop, and the
    decrypted matvec."""
    import __graft_entry__ as ge
    N, L0, P, D = 32768, 3, 1, 64
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    ctx, sk, primes = make_ctx(ph, N, L0, P, steps=steps, seed=11)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(12)
    z = rng.normal(0, 1, N // 2) + 1j * rng.normal(0, 1, N // 2)
    assert np.max(np.abs(np.array(enc.decode_complex_vector(ctx, enc.encode_complex_vector(ctx, z, 2.0 ** 40))) - z)) < 1e-6
    gk = sk.create_galois_keys(ctx)
    x = rng.normal(0, 0.1, D)
    W = rng.normal(0, 0.02, (D, D))
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(x, (N // 2) // D), 2.0 ** 59))
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    pts = enc.encode_double_vector_batch(ctx, ge._rolled_diagonals(W, D, G, N // 2), 2.0 ** 59,
                                         chain_index=ct.chain_index())
    res = None
    for g in range(B):
        inner = None
        for b in range(G):
            k = g * G + b
            if k >= D:
                continue
            term = ph.multiply_plain(ctx, baby[b], pts[k])
            inner = term if inner is None else ph.add(ctx, inner, term)
        if g > 0:
            inner = ph.rotate(ctx, inner, g * G, gk)
        res = inner if res is None else ph.add(ctx, res, inner)
    res = ph.rescale_to_next(ctx, res)
    fused = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    assert np.array_equal(fused.to_numpy(), res.to_numpy())
    dec = np.array(enc.decode_double_vector(ctx, sk.decrypt(ctx, fused)))[:D]
    ref = W @ x
    assert np.corrcoef(dec, ref)[0, 1] > 0.999999
    assert np.max(np.abs(dec - ref)) < 1e-8


def test_ffn_block_ct_ct_chain(ph):
    """tf:26-118's FFN block (BSGS key chunks, CT x CT square + relinearize +
    rescale, value chunks, mod_switch alignment, set_scale, residual add) decrypts to the plaintext
    FFN (tf:272-298 pass criterion corr > 0.999) over two blocks."""
    sys_path = str(Path(__file__).resolve().parents[1] / "tools")
    import sys
    if sys_path not in sys.path:
        sys.path.insert(0, sys_path)
    import ffn_block as fb
    N, L0, P, D, F = 4096, 12, 3, 64, 128
    rng = np.random.default_rng(7)
    ck = fb.Ckks(ph, N, L0, P, D, seed=3)
    x = rng.normal(0, 0.1, D)
    ct = ck.encrypt_replicated(x)
    ref = x.copy()
    for _ in range(2):
        Wk = rng.normal(0, 0.02, (D, F))
        Wv = rng.normal(0, 0.02, (F, D))
        ct = fb.ffn_block(ck, ct, Wk, Wv, D, F)
        ref = fb.plain_ffn(ref, Wk, Wv)
        dec = ck.decrypt(ct, D)
        assert np.corrcoef(dec, ref)[0, 1] > 0.999
        assert np.max(np.abs(dec - ref)) < 1e-6


_RNG_PROBE = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import pyPhantom as ph
p = ph.params(ph.scheme_type.ckks)
p.set_poly_modulus_degree(1024)
p.set_special_modulus_size(1)
p.set_coeff_modulus(ph.create_coeff_modulus(1024, [59, 59, 59]))
ctx = ph.context(p)
enc = ph.ckks_encoder(ctx)
pt = enc.encode_double_vector(ctx, np.linspace(0, 1, 16), 2.0 ** 40)
a, b = ph.secret_key(ctx, seed=5), ph.secret_key(ctx, seed=5)
sym = np.array_equal(a.encrypt_symmetric(ctx, pt).to_numpy(), b.encrypt_symmetric(ctx, pt).to_numpy())
asym = np.array_equal(a.gen_publickey(ctx).encrypt_asymmetric(ctx, pt).to_numpy(),
                      b.gen_publickey(ctx).encrypt_asymmetric(ctx, pt).to_numpy())
dec = np.array(enc.decode_double_vector(ctx, b.decrypt(ctx, a.gen_publickey(ctx).encrypt_asymmetric(ctx, pt))))[:16]
print("RESULT", int(sym), int(asym), float(np.max(np.abs(dec - np.linspace(0, 1, 16)))))
"""


def test_encryption_randomness_fresh_outside_parity_mode(require_gpu):
    """outside parity mode, two secret keys made from the same 32 key bytes (as in two
    processes) never repeat a symmetric-encryption mask, and their public keys never share a mask
    stream; with FHESPEAR_PARITY_RNG (the tests' and the bench's setting) they reproduce each other,
    which is what makes oracle parity of seeded encryptions possible.  Decryption works either way."""
    import os
    import subprocess
    import sys
    py = str(REPO / "fhe-spear_amd" / "python")
    res = {}
    for mode in ("parity", "fresh"):
        env = dict(os.environ)
        env.pop("FHESPEAR_PARITY_RNG", None)
        if mode == "parity":
            env["FHESPEAR_PARITY_RNG"] = "1"
        out = subprocess.run([sys.executable, "-c", _RNG_PROBE, py], env=env, capture_output=True, text=True,
                             timeout=120)
        assert out.returncode == 0, out.stderr[-2000:]
        line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")][-1].split()
        res[mode] = (int(line[1]), int(line[2]), float(line[3]))
    assert res["parity"][:2] == (1, 1), res
    assert res["fresh"][:2] == (0, 0), res
    assert res["parity"][2] < 1e-6 and res["fresh"][2] < 1e-6, res


_DECODE_PROBE = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import pyPhantom as ph
out = []
for N in (1024, 16384, 32768):   # 32768: the split FFT (two halves in LDS, last stage from registers)
    p = ph.params(ph.scheme_type.ckks)
    p.set_poly_modulus_degree(N)
    p.set_special_modulus_size(1)
    primes = ph.create_coeff_modulus(N, [59, 59, 59, 59])
    p.set_coeff_modulus(primes)
    ctx = ph.context(p)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(N)
    z = rng.normal(0, 1, N // 2) + 1j * rng.normal(0, 1, N // 2)
    pts = [enc.encode_complex_vector(ctx, z, 2.0 ** 45), enc.encode_double_vector(ctx, z.real[:100], 2.0 ** 30, 2)]
    qs = [int(q) for q in primes[:3]]
    limbs = np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in qs])
    pts.append(ph.plaintext_from_numpy(ctx, limbs, 1, 2.0 ** 40))   # aliased: the all-limb composition
    out.append(np.array(enc.decode_complex_vector(ctx, pts[0])))
    out.append(enc.decode_batch(ctx, pts, 64).ravel())
np.save(sys.argv[2], np.concatenate(out))
"""


def test_gpu_slot_fft_equals_host_fft(require_gpu, tmp_path):
    """The decoder's slot FFT on the GPU (k_decode_fft + gather, contraction off) gives the same doubles
    as the host FFT it replaced (FHESPEAR_DECODE_HOST_FFT=1, decode_slots): N = 1024, 16384 and 32768 (the
    split form), single and batched decodes, and an aliased plaintext (all-limb composition path)."""
    import os
    import subprocess
    import sys
    py = str(REPO / "fhe-spear_amd" / "python")
    got = {}
    for mode in ("gpu", "host"):
        env = dict(os.environ)
        env.pop("FHESPEAR_DECODE_HOST_FFT", None)
        if mode == "host":
            env["FHESPEAR_DECODE_HOST_FFT"] = "1"
        f = tmp_path / f"{mode}.npy"
        r = subprocess.run([sys.executable, "-c", _DECODE_PROBE, py, str(f)], env=env, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        got[mode] = np.load(f)
    assert got["gpu"].shape == got["host"].shape
    assert np.array_equal(got["gpu"].view(np.uint64), got["host"].view(np.uint64))


def test_encrypt_symmetric_batch_equals_single_encryptions(ph):
    """fhs_encrypt_symmetric_batch (the client's stage inputs in one pass: one sampler launch per
    distribution and one NTT over the batch) gives limb for limb the ciphertexts of encrypt_symmetric
    called in order with a key made from the same seed, and keeps the key's counter in step; a batch of
    mixed levels goes one at a time."""
    N, L0, P = 2048, 6, 2
    ctx, _, _ = make_ctx(ph, N, L0, P, seed=41)
    a, b = ph.secret_key(ctx, seed=42), ph.secret_key(ctx, seed=42)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(43)
    pts = enc.encode_double_vector_batch(ctx, rng.normal(0, 1, (3, N // 2)), 2.0 ** 40)
    for batch in (pts, [pts[0], enc.encode_double_vector(ctx, rng.normal(0, 1, 8), 2.0 ** 40, 2), pts[2]], pts[:1]):
        want = [a.encrypt_symmetric(ctx, p) for p in batch]
        got = b.encrypt_symmetric_batch(ctx, batch)
        assert len(got) == len(want)
        for g, w in zip(got, want):
            assert np.array_equal(g.to_numpy(), w.to_numpy())
    # counters in step afterwards
    assert np.array_equal(a.encrypt_symmetric(ctx, pts[1]).to_numpy(), b.encrypt_symmetric(ctx, pts[1]).to_numpy())
    assert b.encrypt_symmetric_batch(ctx, []) == []


def test_fused_client_calls_equal_separate_calls(ph):
    """encode_encrypt_batch (the message's rounded coefficients go into the error's NTT) gives the
    ciphertexts of encode_*_vector_batch + encrypt_symmetric_batch, limb for limb, real and complex rows at
    two chain indices; decrypt_decode_batch (decrypted straight into the decoder's INTT buffer) gives the
    doubles of decrypt + decode_batch, including a ciphertext whose decryption aliases (all-limb path)."""
    N, L0, P = 2048, 6, 2
    ctx, _, primes = make_ctx(ph, N, L0, P, seed=51)
    a, b = ph.secret_key(ctx, seed=52), ph.secret_key(ctx, seed=52)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(53)
    real = rng.normal(0, 1, (3, N // 2))
    cplx = rng.normal(0, 1, (2, 100)) + 1j * rng.normal(0, 1, (2, 100))
    # periodic rows (encode_*_batch's sparse form): the fused call must detect them the same way
    tiled = np.concatenate([np.tile(rng.normal(0, 1, (2, N // 16)), (1, 8)), real[:1]])
    tiledc = np.tile(rng.normal(0, 1, (2, N // 4)) + 1j * rng.normal(0, 1, (2, N // 4)), (1, 2))
    for rows, ci in ((real, 1), (cplx, 1), (real[:1], 3), (cplx, 2), (tiled, 1), (tiledc, 2)):
        batch = enc.encode_complex_vector_batch if np.iscomplexobj(rows) else enc.encode_double_vector_batch
        want = a.encrypt_symmetric_batch(ctx, batch(ctx, rows, 2.0 ** 40, ci))
        got = b.encode_encrypt_batch(ctx, rows, 2.0 ** 40, ci)
        assert len(got) == len(want)
        for g, w in zip(got, want):
            assert g.chain_index() == w.chain_index() and g.scale() == w.scale()
            assert np.array_equal(g.to_numpy(), w.to_numpy())
    cts = a.encode_encrypt_batch(ctx, real, 2.0 ** 40) + a.encode_encrypt_batch(ctx, cplx, 2.0 ** 40, 2)[:1]
    o = oracle_for(primes, N, P)
    cts.append(ph.ciphertext_from_numpy(ctx, np.stack([rand_pt(o, rng, L0), rand_pt(o, rng, L0)]), 1, 2.0 ** 40))
    for group in (cts[:3], cts[3:], cts):
        for n in (N // 2, 64):
            want = enc.decode_batch(ctx, [a.decrypt(ctx, c) for c in group], n)
            got = a.decrypt_decode_batch(ctx, group, n)
            assert np.array_equal(got, want), n


def test_decode_batch_equals_single_decodes(ph):
    """fhs_decode_batch (the client's decrypt_vec of a block stage in one synchronisation) returns the
    same doubles as fhs_decode one plaintext at a time: real and complex encodings at two levels, and a
    plaintext whose coefficients exceed the first limbs' range (the aliased case that falls back to the
    all-limb composition)."""
    N, L0, P = 4096, 8, 2
    ctx, sk, primes = make_ctx(ph, N, L0, P, seed=31)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(32)
    pts = [enc.encode_double_vector(ctx, rng.normal(0, 1, N // 2), 2.0 ** 59),
           enc.encode_complex_vector(ctx, rng.normal(0, 1, N // 2) + 1j * rng.normal(0, 1, N // 2), 2.0 ** 59, 3),
           sk.decrypt(ctx, sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, rng.normal(0, 1, 64), 2.0 ** 50)))]
    o = oracle_for(primes, N, P)
    pts.append(ph.plaintext_from_numpy(ctx, rand_pt(o, rng, L0), 1, 2.0 ** 40))   # aliased: all-limb fallback
    for n in (N // 2, 64):
        got = enc.decode_batch(ctx, pts, n)
        assert got.shape == (len(pts), n)
        for i, p in enumerate(pts):
            want = np.array(enc.decode_complex_vector(ctx, p))[:n]
            assert np.array_equal(got[i], want), (i, n)
