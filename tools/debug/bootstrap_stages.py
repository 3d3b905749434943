"""Per-stage error audit of ckks_bootstrapper on the GPU (diagnostic, not a test): decrypts after
every stage of bootstrap() and compares with the exact float expectation derived from the
ModRaised plaintext.  Usage: python tools/debug/bootstrap_stages.py [N] [L0]"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))
sys.path.insert(0, str(REPO))
import pyPhantom as ph  # noqa: E402
from pyPhantom import bootstrap as bt  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
L0 = int(sys.argv[2]) if len(sys.argv) > 2 else 36
P, budget = 3, [2, 2]
elts = ph.ckks_bootstrapper.get_galois_elements(N, 0, budget)
parms = ph.params(ph.scheme_type.ckks)
parms.set_poly_modulus_degree(N)
parms.set_special_modulus_size(P)
parms.set_galois_elts(elts)
primes = ph.create_coeff_modulus(N, [59] * (L0 + P))
parms.set_coeff_modulus(primes)
ctx = ph.context(parms)
sk = ph.secret_key(ctx, seed=21)
enc = ph.ckks_encoder(ctx)
b = ph.ckks_bootstrapper(enc)
b.setup(ctx, budget)
b.keygen(ctx, sk)
o = Oracle(N, [int(q) for q in primes], P)
n = N // 2
br = bt.bitrev_perm(n)
z = np.random.default_rng(6).uniform(-4, 4, n)
ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, z, 2.0 ** 59))
while ct.coeff_modulus_size() > 2:
    ct = ph.mod_switch_to_next(ctx, ct)


def dec(c):
    return np.array(enc.decode_complex_vector(ctx, sk.decrypt(ctx, c)))


def coeffs(c):
    """exact centred integer coefficients of decrypt(c), via CRT of limbs 0, 1"""
    limbs = sk.decrypt(ctx, c).to_numpy()
    a0 = o.intt(limbs[0], 0).astype(object)
    a1 = o.intt(limbs[1], 1).astype(object)
    q0, q1 = int(primes[0]), int(primes[1])
    inv = pow(q0, -1, q1)
    t = a0 + q0 * (((a1 - a0) * inv) % q1)
    Q = q0 * q1
    return np.array([int(v) - Q if v > Q // 2 else int(v) for v in t], dtype=object)


q0, q1 = int(primes[0]), int(primes[1])
x = b._prescale(ct)
print("prescale: scale 2^%.3f  decode err %.3e" % (np.log2(x.scale()), np.abs(dec(x).real - z).max()))
d_prime = x.scale()
x = b._mod_raise(x)
t = coeffs(x)
xs = np.array([float(v) / q0 for v in t])
I = np.round(xs)
print("modraise: max|I| %d (K %d)  max|frac| %.3e  (expected ~|m| 2^-k)" % (np.abs(I).max(), b.K, np.abs(xs - I).max()))
v = (xs[:n] + 1j * xs[n:])[br]
x = b._coeff_to_slot(x)
u = dec(x)
print("CtS: scale 2^%.3f ci %d  err (x units) %.3e" % (np.log2(x.scale()), x.chain_index(),
                                                      np.abs(u - v / (2 * b.K)).max() * 2 * b.K))
import time
for name, fn in (("prescale", lambda: b._prescale(ct)), ("cts", lambda: b._coeff_to_slot(b._mod_raise(b._prescale(ct)))),
                 ("evalmod", lambda: b._evalmod(b._split(x)[0])), ("full", lambda: b.bootstrap(ctx, ct))):
    fn(); ctx.synchronize(); t0 = time.perf_counter(); fn(); ctx.synchronize()
    print("  time %-8s %.1f ms" % (name, 1e3 * (time.perf_counter() - t0)))
re, im = b._split(x)
print("split: re err (x units) %.3e  im err %.3e" % (np.abs(dec(re).real - v.real / b.K).max() * b.K,
                                                    np.abs(dec(im).real - v.imag / b.K).max() * b.K))
r2 = b._evalmod(re)
i2 = b._evalmod(im)
want = np.sin(2 * np.pi * v.real)
got = dec(r2).real
print("EvalMod: scale 2^%.3f ci %d  err %.3e  (msg units x 2^k/2pi: %.3e)" % (
    np.log2(r2.scale()), r2.chain_index(), np.abs(got - want).max(),
    np.abs(got - want).max() * 2 ** bt.PRESCALE_BITS / (2 * np.pi)))
y = b._slot_to_coeff(r2, i2, d_prime)
print("final: ci %d scale 2^%.3f err %.3e" % (y.chain_index(), np.log2(y.scale()), np.abs(dec(y).real - z).max()))
