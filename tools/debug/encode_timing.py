"""Throughput of batched CKKS encoding of BSGS diagonals, GPU box."""
import sys, time
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO)); sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))
import pyPhantom as ph
N, L0, P, D = 16384, 36, 3, 2048
primes = ph.create_coeff_modulus(N, [59] * (L0 + P))
parms = ph.params(ph.scheme_type.ckks); parms.set_poly_modulus_degree(N); parms.set_special_modulus_size(P)
parms.set_coeff_modulus(primes)
ctx = ph.context(parms)
enc = ph.ckks_encoder(ctx)
rng = np.random.default_rng(0)
vals = rng.normal(0, 0.02, (D, N // 2))
for it in range(3):
    t0 = time.perf_counter()
    pts = enc.encode_double_vector_batch(ctx, vals, 2.0 ** 59, chain_index=1)
    ctx.synchronize()
    t1 = time.perf_counter()
    print(f"encode_double_vector_batch D={D} N={N} l={L0}: {1e3 * (t1 - t0):.1f} ms  ({D / (t1 - t0):.0f} diag/s)")
    del pts
