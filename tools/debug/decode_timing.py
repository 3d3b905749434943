"""Client-side cost per projection at the cfg3 ring: encrypt_replicated, decrypt, decode (list and raw)."""
import sys, time
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "fhe-spear_amd" / "python"))
import pyPhantom as ph

N, L0, P = 16384, 36, 3
parms = ph.params(ph.scheme_type.ckks)
parms.set_poly_modulus_degree(N)
parms.set_special_modulus_size(P)
parms.set_galois_elts([ph.get_elt_from_step(1, N)])
parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (L0 + P)))
ctx = ph.context(parms)
sk = ph.secret_key(ctx, seed=1)
enc = ph.ckks_encoder(ctx)
x = np.random.default_rng(0).normal(0, 1, 2048)
def t(f, n=20):
    f(); ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        r = f()
    ctx.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, r
ms_enc, ct = t(lambda: sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(x, 4), 2.0 ** 59)))
ct2 = ph.rescale_to_next(ctx, ph.multiply_plain(ctx, ct, enc.encode_double_vector(ctx, np.ones(N // 2), 2.0 ** 59)))
ms_dec, pt = t(lambda: sk.decrypt(ctx, ct2))
ms_decode, v = t(lambda: enc.decode_double_vector(ctx, pt))
ms_decode_c, v = t(lambda: enc.decode_complex_vector(ctx, pt))
ms_raw, v = t(lambda: enc._decode(ctx, pt))
print(f"encode+encrypt {ms_enc:.3f} ms, decrypt {ms_dec:.3f} ms, decode_double (list) {ms_decode:.3f} ms, "
      f"decode_complex (list) {ms_decode_c:.3f} ms, raw decode {ms_raw:.3f} ms")
