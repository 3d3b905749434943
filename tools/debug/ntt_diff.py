"""Debug helper (GPU box): compare the library's NTT'd secret key with the oracle's, limb by limb,
and classify mismatches (non-canonical but congruent vs. wrong residue)."""
import sys
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO)); sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))
import pyPhantom as ph
from oracle.oracle import Oracle
for N, L0, P in ((1024, 6, 3), (16384, 6, 3)):
    primes = ph.create_coeff_modulus(N, [59] * (L0 + P))
    parms = ph.params(ph.scheme_type.ckks); parms.set_poly_modulus_degree(N); parms.set_special_modulus_size(P)
    parms.set_coeff_modulus(primes)
    ctx = ph.context(parms)
    sk = ph.secret_key(ctx, seed=1234)
    a = sk.export()
    o = Oracle(N, [int(q) for q in primes], P)
    b = o.gen_secret(1234)
    for i, q in enumerate(primes):
        q = int(q)
        d = a[i] != b[i]
        nc = (a[i] >= q).sum()
        cong = ((a[i].astype(object) - b[i].astype(object)) % q == 0)
        print(N, i, "mismatch", int(d.sum()), "noncanon", int(nc), "congruent", int(cong.sum()), "first", np.flatnonzero(d)[:8])
    # coefficient-domain view of the library's key
    for i in range(2):
        c = o.intt(a[i].copy(), i)
        if c is not None:
            v = np.asarray(c).ravel()
            q = int(primes[i])
            print("  limb", i, "coeffs ternary:", bool(np.all((v == 0) | (v == 1) | (v == q - 1))), v[:6])
