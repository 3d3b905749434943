"""SEAL-convention key switching and key import.

north_star asks for limbs bit-exact with TenSEAL/SEAL on identical (N, L0, q_i, Galois keys).  SEAL's
switch_key_inplace (P = 1, evaluator.cpp, the published algorithm) differs from this engine's default
(exact centred ModUp, ModDown without rounding, hoistable):
  1. every data limb of the automorphed target is lifted to the other primes as its residue in
     [0, q_I) -- no centring -- so rotations cannot share one decomposition (no hoisting);
  2. the ModDown adds floor(p/2) to the special limb before converting it and subtracts floor(p/2)
     mod q_J after: round(acc / p) instead of a floor.
The context's key_switch_mode('seal') selects it (oracle: Oracle.set_key_switch_mode).  Imported keys
(galois_keys_from_numpy, relin_key_from_numpy, secret_key_from_numpy) express "identical keys".

Pinned here: the oracle's SEAL mode against a direct Python transcription of the published algorithm
(CPU); the GPU in SEAL mode bit-exact against the oracle for rotations (single, and batched: one
decomposition shared by the rotations of an input, corrected per Galois key to SEAL's per-rotation
lift -- or SEAL's own per-rotation path when a digit coefficient is 0), relinearize and the fused BSGS; imported keys reproduce the exporting
context's rotations.  Parity against SEAL itself stays unpinned: SEAL/TenSEAL are not importable here
(SURVEY.md §8c), and SEAL's rotation group generator is 3 where the reference (bg:24) and Phantom use 5."""
import numpy as np
import pytest


def _primes(orc, N, bits):
    return [int(q) for q in orc.create_coeff_modulus(N, bits)]


def _seal_switch_key_reference(o, a, key):
    """SEAL switch_key_inplace on `a` (NTT form, l data limbs) with key [l'][2][K][N] (P = 1), in
    Python integers: the transcription the oracle's 'seal' mode is checked against."""
    l, N = a.shape
    K, L0 = o.K, o.L0
    qs = o.primes
    p = qs[L0]
    targets = list(range(l)) + [L0]                      # data limbs of the level, then the special prime
    acc = {(k, J): np.zeros(N, dtype=object) for k in (0, 1) for J in targets}
    for I in range(l):
        t = [int(v) for v in o.intt(a[I], I)]            # coefficient form in [0, q_I)
        for J in targets:
            x = o.ntt(np.array([v % qs[J] for v in t], dtype=np.uint64), J)   # lift without centring
            for k in (0, 1):
                acc[(k, J)] = (acc[(k, J)] + x.astype(object) * key[I, k, J].astype(object)) % qs[J]
    out = np.empty((2, l, N), dtype=np.uint64)
    half = p >> 1
    for k in (0, 1):
        y = [(int(v) + half) % p for v in o.intt(np.array(acc[(k, L0)], dtype=np.uint64), L0)]
        for J in range(l):
            z = o.ntt(np.array([(v % qs[J] - half) % qs[J] for v in y], dtype=np.uint64), J)
            pinv = pow(p, -1, qs[J])
            out[k, J] = ((acc[(k, J)] - z.astype(object)) * pinv) % qs[J]
    return out


def test_oracle_seal_mode_is_seals_switch_key(orc):
    N = 256
    primes = _primes(orc, N, [59, 59, 59, 60])
    o = orc.Oracle(N, primes, 1)
    o.set_key_switch_mode("seal")
    rng = np.random.default_rng(3)
    for l in (3, 2):
        a = np.stack([rng.integers(0, primes[i], N, dtype=np.uint64) for i in range(l)])
        key = np.stack([np.stack([np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in primes])
                                  for _ in range(2)]) for _ in range(o.dnum)])
        got = o.keyswitch(a, key)
        want = _seal_switch_key_reference(o, a, key)
        assert np.array_equal(np.stack(got), want)


def test_oracle_seal_mode_rotation_decrypts_and_differs_from_exact(orc):
    N = 1024
    primes = _primes(orc, N, [59] * 4 + [60])
    o = orc.Oracle(N, primes, 1)
    s = o.gen_secret(21)
    key = o.gen_galois_key(21, s, orc.galois_elt(3, N))
    x = np.random.default_rng(1).normal(0, 0.1, N // 2)
    ct = o.encrypt_symmetric(21, 0, s, o.encode(x, 2.0 ** 40, 4))
    exact = o.rotate(ct, key, 3)
    o.set_key_switch_mode("seal")
    seal = o.rotate(ct, key, 3)
    assert not np.array_equal(exact, seal)
    for r in (exact, seal):
        assert np.max(np.abs(o.decode(o.decrypt(s, r), 2.0 ** 40).real - np.roll(x, -3))) < 1e-6
    with pytest.raises(ValueError):
        orc.Oracle(N, _primes(orc, N, [59] * 6), 2).set_key_switch_mode("seal")


@pytest.fixture(scope="module")
def ph(require_gpu):
    import pyPhantom
    return pyPhantom


def _gpu_ctx(ph, N, bits, P, elts=None):
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(P)
    if elts:
        parms.set_galois_elts(elts)
    parms.set_coeff_modulus(ph.create_coeff_modulus(N, bits))
    return ph.context(parms)


@pytest.mark.gpu
@pytest.mark.parametrize("N,L0,sp", [(1024, 4, 60), (8192, 24, 60), (16384, 26, 60), (16384, 36, 59)])
def test_gpu_seal_mode_bit_exact_vs_oracle(ph, orc, N, L0, sp):
    """Rotations (a batch of 5 of one input: each decomposed after its automorphism), relinearize and
    the fused BSGS (its giant steps too) in SEAL mode, limb for limb against the oracle.  (16384, 26): a limb's
    extension (26 one-limb digits x 128 KiB) exceeds 3 MiB, so the hoisted key inner product runs half-major
    (FHS_KSIP_HALVES), at both levels.  sp = 59: every prime 59-bit, the bench's cfg2seal ring, where the ModUp
    takes its radix-4 one-prime conversion (modup_convert1_r4, all_b59)."""
    bits = [59] * L0 + [sp]
    D = 32
    G, B = 6, 6
    steps = list(range(1, G)) + [g * G for g in range(1, B)]
    elts = sorted(set(ph.get_elts_from_steps(steps, N)))
    ctx = _gpu_ctx(ph, N, bits, 1, elts)
    ctx.set_key_switch_mode("seal")
    assert ctx.key_switch_mode() == "seal"
    primes = [int(q) for q in ctx.primes]
    o = orc.Oracle(N, primes, 1)
    o.set_key_switch_mode("seal")
    sk = ph.secret_key(ctx, seed=33)
    gk = sk.create_galois_keys(ctx)
    rk = sk.gen_relinkey(ctx)
    s = o.gen_secret(33)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(4)
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(rng.normal(0, 0.1, D), N // 2 // D), 2.0 ** 40))
    c_np = ct.to_numpy()
    okeys = {e: o.gen_galois_key(33, s, e) for e in elts}
    h0 = ctx.seal_hoist_stats()
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    for b in range(1, G):
        assert np.array_equal(baby[b].to_numpy(), o.rotate(c_np, okeys[ph.get_elt_from_step(b, N)], b)), f"rotation {b}"
    h1 = ctx.seal_hoist_stats()
    assert h1[0] == h0[0] + 1 and h1[1] == h0[1], "the batch of rotations of one input took the hoisted path"
    # a lower level: the corrections are per (key, level)
    low = ph.mod_switch_to_next(ctx, ct)
    lows = [ph.rotate(ctx, low, b, gk) for b in (1, 2, 3)]
    for b, r in zip((1, 2, 3), lows):
        assert np.array_equal(r.to_numpy(), o.rotate(low.to_numpy(), okeys[ph.get_elt_from_step(b, N)], b))
    assert ctx.seal_hoist_stats()[0] == h1[0] + 1
    sq = ph.multiply(ctx, ct, ct)
    got = ph.relinearize(ctx, sq, rk).to_numpy()
    assert np.array_equal(got, o.relinearize(sq.to_numpy(), o.gen_relin_key(33, s)))
    pts = ph.random_plaintexts(ctx, 9, D, ct.chain_index(), 2.0 ** 40)
    y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    want = o.bsgs_loop([b_.to_numpy() for b_ in baby], [p.to_numpy() for p in pts],
                       [None] + [okeys[ph.get_elt_from_step(g * G, N)] for g in range(1, B)], G, B, D)
    assert np.array_equal(y.to_numpy(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("N,L0,sp", [(1024, 4, 60), (8192, 24, 60), (16384, 36, 59)])
def test_gpu_seal_hoisting_with_a_zero_digit_coefficient(ph, orc, N, L0, sp):
    """SEAL lifts the automorphed digit without centring: at a coefficient sigma negates, -y lifts to
    q_j - y, which the hoisted path's correction reproduces only for y != 0.  A ciphertext whose digit has
    coefficient 0 at a position the first rotation negates (and, in a second digit, one it does not)
    must take SEAL's per-rotation path and still match the oracle limb for limb; the same rotations of
    an unmodified ciphertext take the hoisted path.  sp = 59: the all-59-bit chain (radix-4 ModUp path)."""
    bits = [59] * L0 + [sp]
    steps = [1, 2, 3, 7]
    elts = sorted(set(ph.get_elts_from_steps(steps, N)))
    ctx = _gpu_ctx(ph, N, bits, 1, elts)
    ctx.set_key_switch_mode("seal")
    primes = [int(q) for q in ctx.primes]
    o = orc.Oracle(N, primes, 1)
    o.set_key_switch_mode("seal")
    sk = ph.secret_key(ctx, seed=71)
    gk = sk.create_galois_keys(ctx)
    s = o.gen_secret(71)
    okeys = {e: o.gen_galois_key(71, s, e) for e in elts}
    enc = ph.ckks_encoder(ctx)
    x = np.random.default_rng(8).normal(0, 0.1, N // 2)
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, x, 2.0 ** 40))
    c = ct.to_numpy().copy()
    l = c.shape[1]
    e1 = ph.get_elt_from_step(1, N)
    neg = [i for i in range(N) if (i * e1) % (2 * N) >= N]
    pos = [i for i in range(N) if (i * e1) % (2 * N) < N]
    for limb, i in ((0, neg[5]), (l - 1, neg[-3]), (1, pos[7])):
        coef = np.array(o.intt(c[1, limb], limb), dtype=np.uint64)
        coef[i] = 0
        c[1, limb] = o.ntt(coef, limb)
    bad = ph.ciphertext_from_numpy(ctx, c, ct.chain_index(), ct.scale())
    for src, path in ((bad, 1), (ct, 0)):
        h0 = ctx.seal_hoist_stats()
        rots = ph.hoisting(ctx, src, gk, steps)
        s_np = src.to_numpy()
        for st, r in zip(steps, rots):
            assert np.array_equal(r.to_numpy(), o.rotate(s_np, okeys[ph.get_elt_from_step(st, N)], st)), st
        h1 = ctx.seal_hoist_stats()
        assert h1[path] == h0[path] + 1 and h1[1 - path] == h0[1 - path]


@pytest.mark.gpu
def test_gpu_exact_mode_unchanged_and_seal_needs_p1(ph):
    ctx = _gpu_ctx(ph, 1024, [59] * 6 + [59] * 3, 3, [ph.get_elt_from_step(1, 1024)])
    assert ctx.key_switch_mode() == "exact"
    with pytest.raises(ValueError):
        ctx.set_key_switch_mode("seal")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["exact", "seal"])
def test_gpu_imported_keys_reproduce_rotations(ph, orc, mode):
    """Keys generated by the oracle (standing in for keys made elsewhere) imported into the GPU
    context: rotation and relinearization limbs equal the oracle's with those very keys, and a
    GPU-generated key exported and re-imported rotates identically."""
    N, L0 = 2048, 6
    bits = [59] * L0 + [60]
    steps = [1, 5, -3]
    elts = sorted(set(ph.get_elts_from_steps(steps, N)))
    ctx = _gpu_ctx(ph, N, bits, 1, elts)
    ctx.set_key_switch_mode(mode)
    o = orc.Oracle(N, [int(q) for q in ctx.primes], 1)
    o.set_key_switch_mode(mode)
    s = o.gen_secret(1234)
    okeys = {e: o.gen_galois_key(1234, s, e) for e in elts}
    sk = ph.secret_key_from_numpy(ctx, s)
    gk = ph.galois_keys_from_numpy(ctx, okeys)
    rk = ph.relin_key_from_numpy(ctx, o.gen_relin_key(1234, s))
    enc = ph.ckks_encoder(ctx)
    x = np.random.default_rng(6).normal(0, 0.1, N // 2)
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, x, 2.0 ** 40))
    c_np = ct.to_numpy()
    for st in steps:
        r = ph.rotate(ctx, ct, st, gk)
        assert np.array_equal(r.to_numpy(), o.rotate(c_np, okeys[ph.get_elt_from_step(st, N)], st))
        assert np.max(np.abs(np.array(enc.decode_double_vector(ctx, sk.decrypt(ctx, r))) - np.roll(x, -st))) < 1e-6
    # the same rotations batched (one decomposition; in SEAL mode the corrections from the imported a_j)
    for st, r in zip(steps, ph.hoisting(ctx, ct, gk, steps)):
        assert np.array_equal(r.to_numpy(), o.rotate(c_np, okeys[ph.get_elt_from_step(st, N)], st))
    sq = ph.multiply(ctx, ct, ct)
    assert np.array_equal(ph.relinearize(ctx, sq, rk).to_numpy(), o.relinearize(sq.to_numpy(), o.gen_relin_key(1234, s)))
    assert np.array_equal(gk.export(elts[0]), okeys[elts[0]])
    # round trip of a generated key
    sk2 = ph.secret_key(ctx, seed=99)
    gk2 = sk2.create_galois_keys(ctx)
    gk3 = ph.galois_keys_from_numpy(ctx, {e: gk2.export(e) for e in elts})
    ct2 = sk2.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, x, 2.0 ** 40))
    assert np.array_equal(ph.rotate(ctx, ct2, 5, gk2).to_numpy(), ph.rotate(ctx, ct2, 5, gk3).to_numpy())
    with pytest.raises(ValueError):
        bad = {elts[0]: np.full_like(okeys[elts[0]], np.iinfo(np.uint64).max)}
        ph.galois_keys_from_numpy(ctx, bad)
    # shapes are checked before the C side reads dnum (L0+P) N words from the pointer: a key made for
    # another dnum / P / N raises instead of being read out of bounds
    k0 = okeys[elts[0]]
    for bad_shape in (k0[:-1], k0[:, :, :-1], k0[..., : N // 2], k0[0]):
        with pytest.raises(ValueError, match="shape"):
            ph.galois_keys_from_numpy(ctx, {elts[0]: bad_shape})
        with pytest.raises(ValueError, match="shape"):
            ph.relin_key_from_numpy(ctx, bad_shape)
    with pytest.raises(ValueError, match="shape"):
        ph.secret_key_from_numpy(ctx, s[:-1])
    with pytest.raises(ValueError, match="shape"):
        ph.secret_key_from_numpy(ctx, s[:, : N // 2])
