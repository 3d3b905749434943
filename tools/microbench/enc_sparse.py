"""Diagonal encoding at cfg5's ring: encode_matrix_diagonals of a D x D matrix (bg:361-378 via the GPU pipeline:
k_diag_gather, k_enc_period, k_encode, k_ntt_fwd_from_dbl_sp) at N = 32768, L0 = 36, P = 3, D = 2048 (t = 8), at
the top level and two lower ones -- the encode the cfg5 chain runs inside every FFN matmul (tf:48, 76).

  python tools/microbench/enc_sparse.py [--reps R] [--out JSON]

Prints ms per call per level and a sha256 of the limbs of rows 0, 1, D-1 at every level (equal across kernel
variants means the same residues).  Run under rocprofv3 --kernel-trace --stats for per-kernel times."""
import argparse, hashlib, json, os, sys, time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fhe-spear_amd", "python"))
import pyPhantom as ph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--N", type=int, default=32768)
    ap.add_argument("--D", type=int, default=2048)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    N, D, L0, P = a.N, a.D, 36, 3
    G = int(np.ceil(np.sqrt(D)))
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(P)
    parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (L0 + P)))
    ctx = ph.context(parms)
    enc = ph.ckks_encoder(ctx)
    rng = np.random.default_rng(5)
    M = rng.normal(0, 1 / np.sqrt(D), (D, D))
    res = {"N": N, "D": D, "L0": L0, "levels": []}
    for ci in (1, 13, 25):
        pts = enc.encode_matrix_diagonals(ctx, M, G, 2.0 ** 40, chain_index=ci)
        ctx.synchronize()
        h = hashlib.sha256()
        for i in (0, 1, D - 1):
            h.update(np.ascontiguousarray(pts[i].to_numpy()).tobytes())
        l = pts[0].to_numpy().shape[0]
        del pts
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            pts = enc.encode_matrix_diagonals(ctx, M, G, 2.0 ** 40, chain_index=ci)
            ctx.synchronize()
            ts.append(time.perf_counter() - t0)
            del pts
        r = {"chain_index": ci, "limbs": l, "ms_median": round(1e3 * float(np.median(ts)), 3),
             "ms_min": round(1e3 * min(ts), 3), "sha256_rows_0_1_last": h.hexdigest()}
        res["levels"].append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
