"""A `pyPhantom`-shaped module backed by the C parity oracle.

TEST INFRASTRUCTURE ONLY.  tests/golden/make_golden.py installs it as sys.modules['pyPhantom']
so that the reference's OWN orchestration (scripts/bootstrap_generation.py: diagonal extraction
bg:198-203, roll/tile bg:361-432, baby steps bg:215-220 and the fallback BSGS loop bg:464-485)
runs verbatim on oracle arithmetic.  It deliberately does NOT export the fork-only fused symbols
(bsgs_multiply_accumulate, encode_*_vector_batch, ...), so the reference takes its pure-Python
fallback paths (bg:384-391, bg:461-485), which are the executable specification of the fused op.

Surface mirrors gpu/phantom_binding.cu:48-206.  Chain-index convention (pb:144, tf:33): a fresh
ciphertext is at chain_index 1 with L0 data limbs; chain_index c holds L0+1-c limbs.
"""
from __future__ import annotations

import enum
import itertools

import numpy as np

from .oracle import Oracle, create_coeff_modulus as _ccm, galois_elt as _gelt

OP_COUNTS = {}


def _count(name):
    OP_COUNTS[name] = OP_COUNTS.get(name, 0) + 1


class scheme_type(enum.Enum):
    none = 0
    bgv = 1
    bfv = 2
    ckks = 3


class modulus(int):
    pass


def create_coeff_modulus(N, bits):
    return [modulus(q) for q in _ccm(N, bits)]


def get_elt_from_step(step, N):
    return _gelt(step, N)


def get_elts_from_steps(steps, N):
    return [_gelt(s, N) for s in steps]


class params:
    def __init__(self, scheme):
        self.scheme = scheme
        self.N = None
        self.special = 1
        self.galois_elts = None
        self.coeff = None

    def set_poly_modulus_degree(self, N):
        self.N = int(N)

    def set_special_modulus_size(self, p):
        self.special = int(p)

    def set_galois_elts(self, elts):
        self.galois_elts = [int(e) for e in elts]

    def set_coeff_modulus(self, mods):
        self.coeff = [int(q) for q in mods]


_seed_counter = itertools.count(1000)


class context:
    def __init__(self, p: params):
        L0 = len(p.coeff) - p.special
        if L0 % p.special != 0:
            raise ValueError("L0 % special_modulus_size != 0 is not supported (README.md:59)")
        self.o = Oracle(p.N, p.coeff, p.special)
        self.primes = list(p.coeff)
        self.params = p
        self.N = p.N
        self.L0 = L0

    def limbs(self, chain_index):
        return self.L0 + 1 - chain_index


class plaintext:
    def __init__(self, data=None, chain_index=1, scale=1.0):
        self.data = data
        self._ci = chain_index
        self._scale = scale

    def chain_index(self):
        return self._ci

    def scale(self):
        return self._scale


class ciphertext:
    def __init__(self, data=None, chain_index=1, scale=1.0):
        self.data = data
        self._ci = chain_index
        self._scale = scale

    def chain_index(self):
        return self._ci

    def scale(self):
        return self._scale

    def set_scale(self, s):
        self._scale = float(s)

    def coeff_modulus_size(self):
        return self.data.shape[1]

    def size(self):
        return self.data.shape[0]


class public_key:
    def __init__(self, ctx=None, data=None, seed=0):
        self.ctx, self.data, self.seed = ctx, data, seed
        self._ctr = itertools.count(1 << 20)

    def encrypt_asymmetric(self, ctx, pt):
        ct = ctx.o.encrypt_asymmetric(self.seed, next(self._ctr), self.data, pt.data)
        return ciphertext(ct, pt.chain_index(), pt.scale())


class relin_key:
    def __init__(self, data=None):
        self.data = data


class galois_key:
    def __init__(self, keys=None):
        self.keys = keys or {}


class secret_key:
    def __init__(self, ctx, seed=None):
        self.seed = int(seed) if seed is not None else next(_seed_counter)
        self.s = ctx.o.gen_secret(self.seed)
        self._ctr = itertools.count(0)

    def gen_publickey(self, ctx):
        return public_key(ctx, ctx.o.gen_public_key(self.seed, self.s), self.seed)

    def gen_relinkey(self, ctx):
        return relin_key(ctx.o.gen_relin_key(self.seed, self.s))

    def create_galois_keys(self, ctx, elts=None):
        elts = elts or ctx.params.galois_elts
        if elts is None:
            N = ctx.N
            steps = []
            k = 1
            while k < N // 2:
                steps += [k, -k]
                k *= 2
            elts = sorted(set(get_elts_from_steps(steps, N)) | {2 * N - 1})
        return galois_key({e: ctx.o.gen_galois_key(self.seed, self.s, e) for e in elts})

    def encrypt_symmetric(self, ctx, pt):
        ct = ctx.o.encrypt_symmetric(self.seed, next(self._ctr), self.s, pt.data)
        return ciphertext(ct, pt.chain_index(), pt.scale())

    def decrypt(self, ctx, ct):
        return plaintext(ctx.o.decrypt(self.s, ct.data), ct.chain_index(), ct.scale())


class ckks_encoder:
    def __init__(self, ctx):
        self.ctx = ctx

    def slot_count(self):
        return self.ctx.N // 2

    def encode_double_vector(self, ctx, values, scale, chain_index=1):
        _count("encode")
        return plaintext(ctx.o.encode(np.asarray(values, dtype=np.float64), scale, ctx.limbs(chain_index)),
                         chain_index, scale)

    def encode_complex_vector(self, ctx, values, scale, chain_index=1):
        _count("encode")
        return plaintext(ctx.o.encode(np.asarray(values, dtype=np.complex128), scale, ctx.limbs(chain_index)),
                         chain_index, scale)

    def encode_complex_vector_batch(self, ctx, mat, scale, chain_index=1, precise=False):
        return [self.encode_complex_vector(ctx, row, scale, chain_index) for row in np.asarray(mat)]

    def decode_double_vector(self, ctx, pt):
        return list(ctx.o.decode(pt.data, pt.scale()).real)

    def decode_complex_vector(self, ctx, pt):
        return list(ctx.o.decode(pt.data, pt.scale()))


def _check_same(a, b):
    if a.chain_index() != b.chain_index():
        raise ValueError("operands at different chain indices")


def add(ctx, a, b):
    _count("add")
    _check_same(a, b)
    if not np.isclose(a.scale(), b.scale(), rtol=1e-9):
        raise ValueError("scale mismatch")
    return ciphertext(ctx.o.add(a.data, b.data), a.chain_index(), a.scale())


def sub(ctx, a, b, negate=False):
    _check_same(a, b)
    r = ctx.o.sub(a.data, b.data)
    if negate:
        r = ctx.o.negate(r)
    return ciphertext(r, a.chain_index(), a.scale())


def negate(ctx, a):
    return ciphertext(ctx.o.negate(a.data), a.chain_index(), a.scale())


def add_plain(ctx, ct, pt):
    _check_same(ct, pt)
    return ciphertext(ctx.o.add_plain(ct.data, pt.data), ct.chain_index(), ct.scale())


def multiply_plain(ctx, ct, pt):
    _count("multiply_plain")
    _check_same(ct, pt)
    return ciphertext(ctx.o.multiply_plain(ct.data, pt.data), ct.chain_index(), ct.scale() * pt.scale())


def multiply(ctx, a, b):
    _count("multiply")
    _check_same(a, b)
    return ciphertext(ctx.o.multiply(a.data, b.data), a.chain_index(), a.scale() * b.scale())


def relinearize(ctx, ct, rlk):
    _count("relinearize")
    return ciphertext(ctx.o.relinearize(ct.data, rlk.data), ct.chain_index(), ct.scale())


def rescale_to_next(ctx, ct):
    _count("rescale_to_next")
    q_last = ctx.o.primes[ct.data.shape[1] - 1]
    return ciphertext(ctx.o.rescale(ct.data), ct.chain_index() + 1, ct.scale() / q_last)


def mod_switch_to_next(ctx, x):
    data = np.ascontiguousarray(x.data[..., :-1, :]) if isinstance(x, ciphertext) else np.ascontiguousarray(x.data[:-1])
    return type(x)(data, x.chain_index() + 1, x.scale())


def mod_switch_to(ctx, x, chain_index):
    while x.chain_index() < chain_index:
        x = mod_switch_to_next(ctx, x)
    return x


def rotate(ctx, ct, step, gk):
    _count("rotate")
    elt = _gelt(step, ctx.N)
    if elt not in gk.keys:
        raise ValueError(f"galois key for step {step} (elt {elt}) not present")
    return ciphertext(ctx.o.rotate_elt(ct.data, gk.keys[elt], elt), ct.chain_index(), ct.scale())


def apply_galois(ctx, ct, elt, gk):
    _count("rotate")
    return ciphertext(ctx.o.rotate_elt(ct.data, gk.keys[int(elt)], int(elt)), ct.chain_index(), ct.scale())


def hoisting(ctx, ct, gk, steps):
    return [rotate(ctx, ct, s, gk) for s in steps]


# ---- bootstrapping primitives (ckks_bootstrapper; restated in ckks_oracle.c / below) ----
def _round_half_away(p):
    """std::round of the double p, exactly (the library's constant rule, fhs_host.hip scalar_consts)."""
    from fractions import Fraction
    import math
    f = Fraction(float(p))
    return math.floor(f + Fraction(1, 2)) if f >= 0 else -math.floor(-f + Fraction(1, 2))


def multiply_const(ctx, ct, value, const_scale=1.0):
    k = _round_half_away(float(value) * float(const_scale))
    return ciphertext(ctx.o.scalar(ct.data, k, add=False), ct.chain_index(), ct.scale() * float(const_scale))


def add_const(ctx, ct, value):
    k = _round_half_away(float(value) * ct.scale())
    return ciphertext(ctx.o.scalar(ct.data, k, add=True), ct.chain_index(), ct.scale())


def mod_raise(ctx, ct):
    return ciphertext(ctx.o.mod_raise(ct.data), 1, ct.scale())


def linear_transform(ctx, babies, pts, G, giant_elts, gk, rescale=True):
    """Loop form of the fused linear transform: sum_g galois_g(sum_b baby[b] * pt[gG+b]), then rescale."""
    acc = None
    for g, elt in enumerate(giant_elts):
        inner = None
        for b in range(G):
            t = multiply_plain(ctx, babies[b], pts[g * G + b])
            inner = t if inner is None else ciphertext(ctx.o.add(inner.data, t.data), t.chain_index(), t.scale())
        if int(elt) != 1:
            inner = apply_galois(ctx, inner, elt, gk)
        acc = inner if acc is None else ciphertext(ctx.o.add(acc.data, inner.data), acc.chain_index(), acc.scale())
    return rescale_to_next(ctx, acc) if rescale else acc
