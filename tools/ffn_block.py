"""The fully-encrypted RWKV FFN block of test_fully_enc_bsgs.py:26-118, restated over pyPhantom for
GPU-side testing and timing of SURVEY.md §8(f) row 3 (CT x CT multiply + relinearize + rescale +
mod_switch / set_scale / add chain) around the fused BSGS.  The reference's own function runs
unchanged against this backend where the reference is present; this copy exists
because the reference does not travel to the GPU box.

    python tools/ffn_block.py [--N 16384 --L0 36 --D 2048 --F 4096 --blocks 2 [--bootstrap]]

--bootstrap runs tf's main loop (tf:233-298): magnitude calibration of W_val (tf:181-196), a
bootstrap whenever fewer than 4 levels remain (tf:239-266, ckks_bootstrapper + one rescale), and
per-block verification against the plaintext chain -- BASELINE configs[4] is
`--N 32768 --L0 36 --P 3 --D 2048 --F 4096 --blocks 24 --bootstrap`.
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))


def bsgs_params(D):
    G = int(np.ceil(np.sqrt(D)))
    return G, int(np.ceil(D / G))


def rolled_diagonals(M, D, G, slots):
    """bg:198-203 + bg:361-378: generalized diagonals d_k[j] = M[j, (j+k) mod D], rows of giant
    group g rolled by gG, tiled to the slot count."""
    j = np.arange(D)
    diags = M[j[None, :], (j[None, :] + j[:, None]) % D]
    for g in range(1, (D + G - 1) // G):
        s, e = g * G, min((g + 1) * G, D)
        diags[s:e] = np.roll(diags[s:e], g * G, axis=1)
    return np.tile(diags, (1, slots // D))


class Ckks:
    """The CKKSBootstrapContext members the block uses (bg:60-154)."""

    def __init__(self, ph, N, L0, P, D, seed=1, bootstrap=False, level_budget=(2, 2)):
        G, B = bsgs_params(D)
        steps = list(range(1, G)) + [g * G for g in range(1, B)]
        bsgs_elts = sorted(set(ph.get_elts_from_steps(steps, N)))
        boot_elts = ph.ckks_bootstrapper.get_galois_elements(N, 0, list(level_budget)) if bootstrap else []
        parms = ph.params(ph.scheme_type.ckks)
        parms.set_poly_modulus_degree(N)
        parms.set_special_modulus_size(P)
        parms.set_galois_elts(sorted(set(bsgs_elts) | set(boot_elts)))          # bg:86-97
        parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (L0 + P)))
        self.ph, self.N, self.L0 = ph, N, L0
        self.ctx = ph.context(parms)
        self.sk = ph.secret_key(self.ctx, seed=seed)
        self.encoder = ph.ckks_encoder(self.ctx)
        self.rlk = self.sk.gen_relinkey(self.ctx)
        self.gk = self.sk.create_galois_keys(self.ctx, bsgs_elts)
        self.scale = 2.0 ** 59
        self.slots = N // 2
        self.bt = None
        if bootstrap:                                                           # bg:110-116
            self.bt = ph.ckks_bootstrapper(self.encoder)
            self.bt.setup(self.ctx, list(level_budget))
            self.bt.keygen(self.ctx, self.sk)

    def bootstrap(self, ct):
        """bg:149-154"""
        while ct.coeff_modulus_size() > 2:
            ct = self.ph.mod_switch_to_next(self.ctx, ct)
        return self.bt.bootstrap(self.ctx, ct)

    def encrypt_replicated(self, x):
        pt = self.encoder.encode_double_vector(self.ctx, np.tile(x, self.slots // len(x)), self.scale)
        return self.sk.encrypt_symmetric(self.ctx, pt)

    def decrypt(self, ct, n):
        return np.array(self.encoder.decode_double_vector(self.ctx, self.sk.decrypt(self.ctx, ct)))[:n]


HOST_PREP_S = [0.0]   # numpy diagonal extraction / roll / tile (the reference caller's own work)
HOST_DIAGONALS = [False]   # --host-diagonals: prepare the rows with numpy as tf does (tf:48, 76)


def matmul(ck, ct, M, D, baby):
    """bg:435-485 through the fused path: encode the rolled diagonals at ct's level, then
    bsgs_multiply_accumulate (one rescale inside)."""
    ph = ck.ph
    G, B = bsgs_params(D)
    if HOST_DIAGONALS[0]:   # the reference caller's numpy roll/tile, then the batch encoder
        t0 = time.perf_counter()
        diags = rolled_diagonals(M, D, G, ck.slots)
        HOST_PREP_S[0] += time.perf_counter() - t0
        pts = ck.encoder.encode_double_vector_batch(ck.ctx, diags, ck.scale, chain_index=ct.chain_index())
    else:                   # the same rows built and encoded on the GPU (limb-identical)
        pts = ck.encoder.encode_matrix_diagonals(ck.ctx, M, G, ck.scale, chain_index=ct.chain_index())
    return ph.bsgs_multiply_accumulate(ck.ctx, baby, pts, G, B, D, ck.gk)


def baby_steps(ck, ct, G):
    return [ct] + [ck.ph.rotate(ck.ctx, ct, b, ck.gk) for b in range(1, G)]


def align(ph, ctx, a, b):
    while a.chain_index() < b.chain_index():
        a = ph.mod_switch_to_next(ctx, a)
    while b.chain_index() < a.chain_index():
        b = ph.mod_switch_to_next(ctx, b)
    return a, b


def ffn_block(ck, ct_x, W_key, W_val, D, F):
    """x -> x + (relu-free square FFN) W_val^T ((W_key^T x)^2), tf:26-118."""
    ph = ck.ph
    G, _ = bsgs_params(D)
    chunks = int(np.ceil(F / D))
    baby = baby_steps(ck, ct_x, G)
    keys = []
    for c in range(chunks):
        lo, hi = c * D, min(c * D + D, F)
        if hi - lo == D and not HOST_DIAGONALS[0]:
            M = W_key[:, lo:hi].T          # a view: the GPU encoder reads it strided, no host copy
        else:
            M = np.zeros((D, D))
            M[:hi - lo, :] = W_key[:, lo:hi].T
        keys.append(matmul(ck, ct_x, M, D, baby))
    sq = []
    for k in keys:   # tf:57-61
        s = ph.relinearize(ck.ctx, ph.multiply(ck.ctx, k, k), ck.rlk)
        sq.append(ph.rescale_to_next(ck.ctx, s))
    acc = None
    for c, s in enumerate(sq):   # tf:65-91
        lo, hi = c * D, min(c * D + D, F)
        if hi - lo == D and not HOST_DIAGONALS[0]:
            M = W_val[lo:hi, :].T
        else:
            M = np.zeros((D, D))
            M[:, :hi - lo] = W_val[lo:hi, :].T
        part = matmul(ck, s, M, D, baby_steps(ck, s, G))
        if acc is None:
            acc = part
        else:
            acc, part = align(ph, ck.ctx, acc, part)
            acc = ph.add(ck.ctx, acc, part)
    xa, acc = align(ph, ck.ctx, ct_x, acc)   # tf:96-109
    acc.set_scale(xa.scale())
    return ph.add(ck.ctx, xa, acc)


def plain_ffn(x, W_key, W_val):
    return x + (x @ W_key) ** 2 @ W_val


def calibrated_weights(rng, D, F, blocks):
    """tf:172-196: random weights, W_val scaled so every block adds an update of max magnitude 1."""
    W_keys = [rng.standard_normal((D, F)) * 0.02 for _ in range(blocks)]
    W_raw = [rng.standard_normal((F, D)) * 0.02 for _ in range(blocks)]
    x_cal = rng.standard_normal(D) * 0.1
    W_vals, x = [], x_cal.copy()
    for b in range(blocks):
        fv = (x @ W_keys[b]) ** 2 @ W_raw[b]
        ms = 1.0 / (np.max(np.abs(fv)) + 1e-12)
        W_vals.append(W_raw[b] * ms)
        x = x + fv * ms
    return x_cal, W_keys, W_vals


def run_chain(ck, x_cal, W_keys, W_vals, D, F, use_bootstrap, log=print):
    """tf:233-298: blocks in sequence, a bootstrap (+ one rescale) whenever fewer than 4 levels
    remain; returns per-block records (seconds, chain index, corr, max_err, bootstrapped)."""
    ph = ck.ph
    ct = ck.encrypt_replicated(x_cal)
    ref = x_cal.copy()
    out = []
    for b in range(len(W_keys)):
        boot_s = None
        if (ck.L0 - 1) - ct.chain_index() < 4:
            if not use_bootstrap:
                log(f"  *** OUT OF LEVELS at block {b}")
                break
            ck.ctx.synchronize()
            t0 = time.perf_counter()
            ct = ph.rescale_to_next(ck.ctx, ck.bootstrap(ct))
            ck.ctx.synchronize()
            boot_s = time.perf_counter() - t0
            err = np.max(np.abs(ck.decrypt(ct, D) - ref))
            log(f"  >>> bootstrap before block {b}: {1e3 * boot_s:.1f} ms, chain_index={ct.chain_index()}, "
                f"err vs ref={err:.2e}")
        ck.ctx.synchronize()
        t0 = time.perf_counter()
        ct = ffn_block(ck, ct, W_keys[b], W_vals[b], D, F)
        ck.ctx.synchronize()
        dt = time.perf_counter() - t0
        ref = plain_ffn(ref, W_keys[b], W_vals[b])
        dec = ck.decrypt(ct, D)
        rec = dict(block=b, seconds=dt, bootstrap_seconds=boot_s, chain_index=ct.chain_index(),
                   corr=float(np.corrcoef(dec, ref)[0, 1]), max_err=float(np.max(np.abs(dec - ref))),
                   mag=float(np.max(np.abs(ref))))
        out.append(rec)
        log(f"block {b}: {1e3 * dt:.1f} ms  chain_index={rec['chain_index']}  corr={rec['corr']:.10f}  "
            f"max_err={rec['max_err']:.3e}  |ref|={rec['mag']:.3f}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--L0", type=int, default=36)
    ap.add_argument("--P", type=int, default=3)
    ap.add_argument("--D", type=int, default=2048)
    ap.add_argument("--F", type=int, default=4096)
    ap.add_argument("--blocks", type=int, default=2)
    ap.add_argument("--bootstrap", action="store_true")
    ap.add_argument("--host-diagonals", action="store_true",
                    help="numpy diagonal prep as the reference caller does (default: pyPhantom encode_matrix_diagonals)")
    a = ap.parse_args()
    HOST_DIAGONALS[0] = a.host_diagonals
    import pyPhantom as ph
    rng = np.random.default_rng(42)
    if a.bootstrap:
        t0 = time.perf_counter()
        ck = Ckks(ph, a.N, a.L0, a.P, a.D, bootstrap=True)
        ck.ctx.synchronize()
        print(f"setup (keys, bootstrapper): {time.perf_counter() - t0:.2f} s")
        x_cal, Wk, Wv = calibrated_weights(rng, a.D, a.F, a.blocks)
        recs = run_chain(ck, x_cal, Wk, Wv, a.D, a.F, True)
        bl = [r["seconds"] for r in recs]
        bs = [r["bootstrap_seconds"] for r in recs if r["bootstrap_seconds"]]
        print(f"blocks completed {len(recs)}/{a.blocks}, bootstraps {len(bs)}, mean block {1e3 * np.mean(bl):.1f} ms, "
              f"mean bootstrap {1e3 * np.mean(bs) if bs else 0:.1f} ms, final corr {recs[-1]['corr']:.10f}, "
              f"max_err {recs[-1]['max_err']:.3e}")
        return
    ck = Ckks(ph, a.N, a.L0, a.P, a.D)
    x = rng.normal(0, 0.1, a.D)
    ct = ck.encrypt_replicated(x)
    ref = x.copy()
    for b in range(a.blocks):
        Wk = rng.normal(0, 0.02, (a.D, a.F))
        Wv = rng.normal(0, 0.02, (a.F, a.D))
        ck.ctx.synchronize()
        HOST_PREP_S[0] = 0.0
        t0 = time.perf_counter()
        ct = ffn_block(ck, ct, Wk, Wv, a.D, a.F)
        ck.ctx.synchronize()
        dt = time.perf_counter() - t0
        print(f"  numpy diagonal prep (caller side): {1e3 * HOST_PREP_S[0]:.1f} ms, backend: {1e3 * (dt - HOST_PREP_S[0]):.1f} ms")
        ref = plain_ffn(ref, Wk, Wv)
        dec = ck.decrypt(ct, a.D)
        print(f"block {b}: {1e3 * dt:.1f} ms  chain_index={ct.chain_index()}  "
              f"corr={np.corrcoef(dec, ref)[0, 1]:.8f}  max_err={np.max(np.abs(dec - ref)):.3e}")


if __name__ == "__main__":
    main()
