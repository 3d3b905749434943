"""Host-side latency of each API call in the bench step while the GPU is busy (GPU box)."""
import sys, time
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO)); sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))
import pyPhantom as ph
import bench
N, L0, P, D = 16384, 36, 3, 2048
G, B = bench.bsgs_params(D)
steps = list(range(1, G)) + [g * G for g in range(1, B)]
primes = ph.create_coeff_modulus(N, [59] * (L0 + P))
parms = ph.params(ph.scheme_type.ckks); parms.set_poly_modulus_degree(N); parms.set_special_modulus_size(P)
parms.set_galois_elts(sorted(set(ph.get_elts_from_steps(steps, N)))); parms.set_coeff_modulus(primes)
ctx = ph.context(parms); sk = ph.secret_key(ctx, seed=1); gk = sk.create_galois_keys(ctx)
enc = ph.ckks_encoder(ctx)
ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.zeros(8), 2.0 ** 59))
pts = ph.random_plaintexts(ctx, 2, D, ct.chain_index(), 2.0 ** 59)
ctx.synchronize()
for it in range(4):
    t = [time.perf_counter()]
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    t.append(time.perf_counter())
    y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
    t.append(time.perf_counter())
    del baby
    t.append(time.perf_counter())
    del y
    t.append(time.perf_counter())
    ctx.synchronize()
    t.append(time.perf_counter())
    d = np.diff(t) * 1e3
    print(f"iter {it}: rotates {d[0]:.2f} ms, bsgs call {d[1]:.2f} ms, del baby {d[2]:.2f} ms, del y {d[3]:.2f}, sync {d[4]:.2f}")
