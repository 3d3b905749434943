"""Is the Hadamard's placement sensitivity a channel effect of the diagonals' stride?  cfg2's plaintexts sit
36 x 128 KiB apart in their slab, so the words one wave streams concurrently (the same limb and coefficient tile of
successive diagonals) share their low 19 address bits.  Here the same 2048 diagonals are allocated TRIALS times per
padding (FHESPEAR_PT_PAD_WORDS words between plaintexts, read per allocation), the paddings interleaved so each sees
a spread of placements, and k_bsgs_inner timed as in tools/debug/alloc_spread.py.  Output limbs must not change.

    python tools/debug/pad_spread.py [TRIALS] [STEPS] [PAD ...]
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
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    pads = [int(a) for a in sys.argv[3:]] or [0, 512, 2560, 16896]
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
    digests, res = set(), {p: [] for p in pads}
    k = 0
    for t in range(trials):
        for pad in pads:
            spacer = torch.empty(int((0.5 + 0.37 * k) * 2 ** 30), dtype=torch.uint8, device="cuda:0")
            k += 1
            os.environ["FHESPEAR_PT_PAD_WORDS"] = str(pad)
            pts = ph.random_plaintexts(ctx, 2, D, 1, 2.0 ** 59)
            y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)   # warm
            ctx.synchronize()
            ph.kernel_timer_read(ctx, reset=True)
            ph.kernel_timer_arm(ctx, ["k_bsgs_inner"])
            for _ in range(steps):
                y = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
            ctx.synchronize()
            ms, n = ph.kernel_timer_read(ctx, reset=True)["k_bsgs_inner"]
            ph.kernel_timer_arm(ctx, [])
            digests.add(hashlib.sha256(np.ascontiguousarray(y.to_numpy()).tobytes()).hexdigest())
            res[pad].append(ms / max(n, 1))
            print(f"trial {t} pad {pad:6d} words: k_bsgs_inner {res[pad][-1]:.4f} ms", flush=True)
            del pts, y, spacer
            torch.cuda.empty_cache()
            ctx.synchronize()
    os.environ.pop("FHESPEAR_PT_PAD_WORDS", None)
    for pad, v in res.items():
        print(f"pad {pad:6d}: min {min(v):.4f} mean {np.mean(v):.4f} max {max(v):.4f} ms over {len(v)} placements")
    print(f"output digests identical: {len(digests) == 1}")


if __name__ == "__main__":
    main()
