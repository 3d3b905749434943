"""Does the Hadamard's speed follow where its diagonals land in HBM?  (k_bsgs_inner ran 1.80 ms
on some boxes and 2.05 ms on others; round 6's clock samples show the same SCLK / MCLK in both states.)

One process, cfg2 (N=16384, L0=36, P=3, d=2048): keys, input and baby steps fixed; the 2048 diagonals (9.66 GB, one
slab) re-allocated TRIALS times, each time after a torch spacer allocation of a different size so the slab lands
elsewhere (the library's block cache is off: FHESPEAR_CACHE_BYTES=0).  Per trial: k_bsgs_inner's mean device time
over STEPS fused BSGS calls (kernel-timer events) and the slab's device address.  The output limbs are checked
to be identical across trials (same seeds).

    python tools/debug/alloc_spread.py [TRIALS] [STEPS]
"""
import hashlib
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("FHESPEAR_CACHE_BYTES", "0")
os.environ.setdefault("FHESPEAR_PARITY_RNG", "1")
REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pyPhantom as ph  # noqa: E402


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    N, L0, P, D = 16384, 36, 3, 2048
    G, B = 46, 45
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
    digests, rows = set(), []
    for t in range(trials):
        spacer = torch.empty(int((0.5 + 1.7 * t) * 2 ** 30), dtype=torch.uint8, device="cuda:0")
        pts = ph.random_plaintexts(ctx, 2, D, 1, 2.0 ** 59)
        addr = ph.plaintext_device_ptr(pts[0]) if hasattr(ph, "plaintext_device_ptr") else None
        y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)   # warm
        ctx.synchronize()
        ph.kernel_timer_read(ctx, reset=True)
        ph.kernel_timer_arm(ctx, ["k_bsgs_inner"])
        t0 = time.perf_counter()
        for _ in range(steps):
            y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
        ctx.synchronize()
        wall = time.perf_counter() - t0
        ms, n = ph.kernel_timer_read(ctx, reset=True)["k_bsgs_inner"]
        ph.kernel_timer_arm(ctx, [])
        digests.add(hashlib.sha256(np.ascontiguousarray(y.to_numpy()).tobytes()).hexdigest())
        per = ms / max(n, 1)
        rows.append(per)
        print(f"trial {t}: spacer {spacer.numel() / 2 ** 30:.1f} GiB, slab at {addr}, k_bsgs_inner {per:.4f} ms "
              f"({10.522e9 / (per * 1e-3) / 1e12:.2f} TB/s), giant-step wall {1e3 * wall / steps:.3f} ms/call", flush=True)
        del pts, y, spacer
        torch.cuda.empty_cache()
        ctx.synchronize()
    print(f"k_bsgs_inner over {trials} placements: min {min(rows):.4f} max {max(rows):.4f} ms "
          f"(spread {100 * (max(rows) / min(rows) - 1):.1f} %); output digests identical: {len(digests) == 1}")


if __name__ == "__main__":
    main()
