"""Matvec rate of the three ways the reference feeds diagonals to the BSGS (cfg2 by default):

  resident   pre-encoded diagonals in HBM (bg:1124-1174 --preencoded; the bench.py workload)
  from_cpu   pinned host copies streamed per matvec (bg:336-358 offload, bg:449 bsgs_from_cpu):
             the PCIe-inclusive rate (9.66 GB of diagonals cross the link every matvec at cfg2)
  encode     float64 rolled diagonals (D x slots, from the host) encoded on the GPU per matvec, as
             test_fully_enc_bsgs.py does (tf:48, 76 via bg:382) -- the caller's numpy roll/tile is
             not included
  matrix     the D x D matrix itself uploaded (D^2 doubles) and its rolled, tiled diagonals built and
             encoded on the GPU (pyPhantom encode_matrix_diagonals, an extension): no caller numpy

    python tools/host_paths.py [--N 16384 --L0 36 --P 3 --D 2048 --reps 3]
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--L0", type=int, default=36)
    ap.add_argument("--P", type=int, default=3)
    ap.add_argument("--D", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import pyPhantom as ph
    N, D = a.N, a.D
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(a.P)
    parms.set_galois_elts(sorted(set(ph.get_elts_from_steps(list(range(1, G)) + [g * G for g in range(1, B)], N))))
    parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (a.L0 + a.P)))
    ctx = ph.context(parms)
    sk = ph.secret_key(ctx, seed=3)
    gk = sk.create_galois_keys(ctx)
    enc = ph.ckks_encoder(ctx)
    scale = 2.0 ** 59
    rng = np.random.default_rng(1)
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(rng.normal(0, 0.1, D), (N // 2) // D), scale))
    level = ct.chain_index()
    pts = ph.random_plaintexts(ctx, 2, D, level, scale)
    diag_f64 = rng.normal(0, 0.02, (D, N // 2))
    t0 = time.perf_counter()
    host = ph.offload_plaintexts(pts)
    t_off = time.perf_counter() - t0
    nbytes = host[0].nbytes

    def baby():
        return [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]

    def timed(fn):
        fn()
        ctx.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            fn()
        ctx.synchronize()
        return (time.perf_counter() - t) / a.reps

    t_res = timed(lambda: ph.bsgs_multiply_accumulate(ctx, baby(), pts, G, B, D, gk))
    t_cpu = timed(lambda: ph.bsgs_from_cpu(ctx, baby(), *host, G, B, D, gk))
    t_enc = timed(lambda: ph.bsgs_multiply_accumulate(
        ctx, baby(), enc.encode_double_vector_batch(ctx, diag_f64, scale, chain_index=level), G, B, D, gk))
    W = rng.normal(0, 0.02, (D, D))
    t_mat = timed(lambda: ph.bsgs_multiply_accumulate(
        ctx, baby(), enc.encode_matrix_diagonals(ctx, W, G, scale, chain_index=level), G, B, D, gk))
    print(f"N={N} L0={a.L0} P={a.P} D={D}: diagonals {nbytes / 1e9:.2f} GB (offload once: {t_off:.2f} s)")
    for name, t in (("resident", t_res), ("from_cpu", t_cpu), ("encode", t_enc), ("matrix", t_mat)):
        extra = f", {nbytes / (t - t_res) / 1e9:.1f} GB/s host->device beyond resident" if name == "from_cpu" else ""
        print(f"  {name:9s} {1e3 * t:8.2f} ms/matvec  {1.0 / t:7.2f} matvec/s{extra}", flush=True)


if __name__ == "__main__":
    main()
