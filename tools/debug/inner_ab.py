"""Same-placement A/B of k_bsgs_inner variants (round 6).  tools/debug/alloc_spread.py showed the Hadamard's time
moving 12-15 % with where its diagonal slab lands in HBM, so an A/B across two processes (two placements) cannot
resolve a few per cent.  Here one process holds one cfg2 workload (N=16384, L0=36, P=3, d=2048) and alternates the
variants ENV=0 / ENV=1 on the SAME allocation, REPS times, then re-allocates the diagonals (a torch spacer of a
different size first) and repeats, PLACEMENTS times.  Per (placement, variant): k_bsgs_inner's mean device time over
STEPS fused BSGS calls (kernel-timer events); the output limbs must be identical across variants.

    python tools/debug/inner_ab.py ENV VALUE [PLACEMENTS] [REPS] [STEPS]   (ENV=0 against ENV=VALUE, e.g.
    FHESPEAR_INNER_VAR 2)

The round-6 variants it measured (profiles/r06/ab_inner_same_placement/) were compiled in behind
FHESPEAR_INNER_VAR at commit 810c6ec and removed after the A/B; a new variant needs its own run-time knob read at
launch, as there.
"""
import hashlib
import os
import sys
from pathlib import Path

os.environ.setdefault("FHESPEAR_CACHE_BYTES", "0")
os.environ.setdefault("FHESPEAR_PARITY_RNG", "1")
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "fhe-spear_amd" / "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pyPhantom as ph  # noqa: E402


def main():
    env, val = sys.argv[1], sys.argv[2]
    placements = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    N, L0, P, D, G, B = 16384, 36, 3, 2048, 46, 45
    st = list(range(1, G)) + [g * G for g in range(1, B)]
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(P)
    parms.set_galois_elts(sorted(set(ph.get_elts_from_steps(st, N))))
    parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (L0 + P)))
    ctx = ph.context(parms)
    sk = ph.secret_key(ctx, seed=1000)
    gk = sk.create_galois_keys(ctx)
    ct = sk.encrypt_symmetric(ctx, ph.random_plaintexts(ctx, 10000, 1, 1, 2.0 ** 59)[0])
    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
    ctx.synchronize()
    table = {0: [], 1: []}
    digests = set()
    for pl in range(placements):
        spacer = torch.empty(int((0.5 + 1.7 * pl) * 2 ** 30), dtype=torch.uint8, device="cuda:0")
        pts = ph.random_plaintexts(ctx, 2, D, 1, 2.0 ** 59)
        row = {0: [], 1: []}
        for _ in range(reps):
            for var in (0, 1):
                os.environ[env] = val if var else "0"
                y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)   # warm
                ctx.synchronize()
                ph.kernel_timer_read(ctx, reset=True)
                ph.kernel_timer_arm(ctx, ["k_bsgs_inner"])
                for _ in range(steps):
                    y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
                ctx.synchronize()
                ms, n = ph.kernel_timer_read(ctx, reset=True)["k_bsgs_inner"]
                ph.kernel_timer_arm(ctx, [])
                row[var].append(ms / max(n, 1))
                digests.add(hashlib.sha256(np.ascontiguousarray(y.to_numpy()).tobytes()).hexdigest())
        for var in (0, 1):
            table[var].append(float(np.median(row[var])))
        print(f"placement {pl}: {env}=0 {table[0][-1]:.4f} ms, {env}={val} {table[1][-1]:.4f} ms "
              f"({100 * (table[1][-1] / table[0][-1] - 1):+.2f} %)  reps 0: {[round(v, 4) for v in row[0]]} "
              f"1: {[round(v, 4) for v in row[1]]}", flush=True)
        del pts, y, spacer
        torch.cuda.empty_cache()
        ctx.synchronize()
    rel = [b / a - 1 for a, b in zip(table[0], table[1])]
    print(f"{env}={val} vs 0 over {placements} placements: mean {100 * float(np.mean(rel)):+.2f} %, "
          f"min {100 * min(rel):+.2f} %, max {100 * max(rel):+.2f} %; output digests identical: {len(digests) == 1}")


if __name__ == "__main__":
    main()
