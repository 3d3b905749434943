"""The fully-encrypted RWKV FFN block of test_fully_enc_bsgs.py:26-118, restated over pyPhantom for
GPU-side testing and timing of SURVEY.md §8(f) row 3 (CT x CT multiply + relinearize + rescale +
mod_switch / set_scale / add chain) around the fused BSGS.  The reference's own function runs
unchanged against this backend where the reference is present; this copy exists
because the reference does not travel to the GPU box.

    python tools/ffn_block.py [--N 16384 --L0 36 --D 2048 --F 4096 --blocks 2 [--bootstrap]]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/ffn_block.py --dist [--shard giant|grid|baby]

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
# chain_over_ranks(record_first=True): the first one-rank BSGS call's input ciphertext, diagonals and output are
# kept here (device objects: nothing is copied inside the timed blocks) for a limb check after the chain
RECORD = [None]


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
    out = ph.bsgs_multiply_accumulate(ck.ctx, baby, pts, G, B, D, ck.gk)
    if RECORD[0] is not None and "ct_out" not in RECORD[0]:
        RECORD[0].update(ct_in=ct, pts=pts, ct_out=out)
    return out


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


# ------------------------------------------------------------------ over ranks (Config 5)
class FfnRanks:
    """The FFN block's chunks over the ranks of one node (tf:26-118 sharded; BASELINE configs[4] on 8
    GPUs).  Every rank holds the same keys (the client's seed) so that any rank's partial work is a
    valid share; rank 0 is where the chain's ciphertext lives between blocks (and the client decrypts).

    * chunk c of the F/D key chunks (and of the value chunks) gets a contiguous, balanced rank group
      (fhespear_dist.stage_groups; with fewer ranks than chunks the chunks are dealt round-robin);
    * the key chunks share one input, hence one set of baby steps: baby_mode "recompute" has every
      rank rotate its share itself, "broadcast" has rank 0 compute the G baby steps once and broadcast
      them (north_star "baby steps computed once and broadcast"; giant shard only);
    * inside a group each chunk's BSGS is sharded by shard="giant" (giant groups, fhespear_dist.
      bsgs_giant_sharded), "grid" (rb baby shares x giant columns, bsgs_grid_sharded; rb = the caller's
      when it divides the group, else fhespear_dist.grid_rb) or "baby" (rb = group size); each rank
      encodes only the diagonal rows it needs (encode_matrix_diagonals rows=);
    * the square / relinearize / rescale of key chunk c run on its group root, which then broadcasts
      the squared chunk to its group for the value matmul; the value chunks' rescaled outputs come to
      rank 0 and are added there in chunk order, then the residual (tf:96-109).
    Every term is the one-rank chain's: the output limbs are identical (tests/test_ffn_dist.py)."""

    def __init__(self, ck, D, F, dist, rank, world, shard="giant", rb=None, baby_mode="recompute", device="cuda:0"):
        import fhespear_dist as fd
        if shard not in ("giant", "grid", "baby"):
            raise ValueError(f"shard {shard!r}: 'giant', 'grid' or 'baby'")
        if baby_mode not in ("recompute", "broadcast"):
            raise ValueError(f"baby_mode {baby_mode!r}: 'recompute' or 'broadcast'")
        self.ck, self.D, self.F, self.dist, self.rank, self.world = ck, D, F, dist, rank, world
        self.shard, self.baby_mode, self.device = shard, baby_mode, device
        self.G, self.B = bsgs_params(D)
        self.chunks = int(np.ceil(F / D))
        groups = fd.stage_groups(self.chunks, world)
        self.groups = groups if groups is not None else [[c % world] for c in range(self.chunks)]
        # process groups, made by every rank in the same order (torch.distributed.new_group is collective)
        self.pg, self.rbs, self.cols = {}, {}, {}
        for c, ranks in enumerate(self.groups):
            key = tuple(ranks)
            if key not in self.pg:
                self.pg[key] = dist.new_group(list(ranks)) if len(ranks) > 1 else None
                R = len(ranks)
                r = 1 if shard == "giant" else (R if shard == "baby" else (rb if rb and R % rb == 0 else fd.grid_rb(R)))
                self.rbs[key] = r
                self.cols[key] = fd.grid_groups(dist, ranks, r) if r > 1 and R > 1 else {}

    def _zero(self, ci):
        ck = self.ck
        return ck.encoder.encode_double_vector_batch(ck.ctx, np.zeros((self.G, ck.slots)), ck.scale, chain_index=ci)

    def _rows(self, ranks):
        import fhespear_dist as fd
        R, idx, rb = len(ranks), ranks.index(self.rank), self.rbs[tuple(ranks)]
        if rb == 1:
            return [g * self.G + b for g in fd.giant_groups(self.B, R, idx) for b in range(self.G) if g * self.G + b < self.D]
        return fd.grid_rows(self.G, self.B, self.D, R, rb, idx)

    def matmul(self, ct, M, ranks, baby=None):
        """bg:435-485 for one chunk over `ranks` (this rank among them): the rescaled output on ranks[0]."""
        import fhespear_dist as fd
        ck, ph = self.ck, self.ck.ph
        G, B, D, ci = self.G, self.B, self.D, ct.chain_index()
        if len(ranks) == 1:
            return matmul(ck, ct, M, D, baby if baby is not None else baby_steps(ck, ct, G))
        key = tuple(ranks)
        rows = self._rows(ranks)
        pts = dict(zip(rows, ck.encoder.encode_matrix_diagonals(ck.ctx, M, G, ck.scale, chain_index=ci, rows=rows)))
        zero = self._zero(ci)
        if self.rbs[key] == 1:
            return fd.bsgs_giant_sharded(ph, ck.ctx, baby if baby is not None else baby_steps(ck, ct, G), pts, G, B, D,
                                         ck.gk, zero, self.dist, self.device, ranks=ranks, group=self.pg[key])
        return fd.bsgs_grid_sharded(ph, ck.ctx, ct, pts, G, B, D, ck.gk, zero[0], self.dist, self.rbs[key], self.device,
                                    ranks=ranks, group=self.pg[key], col_groups=self.cols[key])

    def block(self, ct_x, W_key, W_val):
        """x -> x + W_val^T ((W_key^T x)^2) over the ranks; ct_x on rank 0, the output on rank 0."""
        import fhespear_dist as fd
        ck, ph, D, F, dist, me, dev = self.ck, self.ck.ph, self.D, self.F, self.dist, self.rank, self.device
        cx = fd.broadcast_ciphertext(ph, ck.ctx, ct_x if me == 0 else None, 0, dist, dev)
        baby = None
        if self.baby_mode == "broadcast" and self.shard == "giant":   # G baby steps computed once
            mine = baby_steps(ck, cx, self.G) if me == 0 else None
            baby = fd.broadcast_ciphertexts(ph, ck.ctx, mine, 0, dist, dev, self.G)
        elif any(len(r) == 1 and me in r for r in self.groups) or self.shard == "giant":
            baby = baby_steps(ck, cx, self.G)            # shared by every chunk this rank computes whole
        sq = {}
        for c, ranks in enumerate(self.groups):          # key chunks (tf:38-55) + square (tf:57-61)
            if me not in ranks:
                continue
            lo, hi = c * D, min(c * D + D, F)
            if hi - lo == D and not HOST_DIAGONALS[0]:
                M = W_key[:, lo:hi].T
            else:
                M = np.zeros((D, D))
                M[:hi - lo, :] = W_key[:, lo:hi].T
            k = self.matmul(cx, M, ranks, baby if len(ranks) == 1 or self.shard == "giant" else None)
            if me == ranks[0]:
                s = ph.relinearize(ck.ctx, ph.multiply(ck.ctx, k, k), ck.rlk)
                sq[c] = ph.rescale_to_next(ck.ctx, s)
        parts = {}
        for c, ranks in enumerate(self.groups):          # value chunks (tf:65-91)
            if me not in ranks:
                continue
            s = sq.get(c) if me == ranks[0] else None
            if len(ranks) > 1:
                s = fd.broadcast_ciphertext(ph, ck.ctx, s, ranks[0], dist, dev, group=self.pg[tuple(ranks)])
            lo, hi = c * D, min(c * D + D, F)
            if hi - lo == D and not HOST_DIAGONALS[0]:
                M = W_val[lo:hi, :].T
            else:
                M = np.zeros((D, D))
                M[:, :hi - lo] = W_val[lo:hi, :].T
            p = self.matmul(s, M, ranks)
            if me == ranks[0]:
                parts[c] = p
        acc = None
        for c, ranks in enumerate(self.groups):          # parts to rank 0, added in chunk order
            got = fd.send_ciphertext(ph, ck.ctx, parts.get(c), ranks[0], 0, dist, dev)
            if me == 0:
                if acc is None:
                    acc = got
                else:
                    acc, got = align(ph, ck.ctx, acc, got)
                    acc = ph.add(ck.ctx, acc, got)
        if me != 0:
            return None
        xa, acc = align(ph, ck.ctx, ct_x, acc)           # tf:96-109
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


def ct_digest(ct):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(ct.to_numpy()).tobytes()).hexdigest()


def chain_over_ranks(ph, N, L0, P, D, F, blocks, bootstrap, dist, rank, world, device, shard="giant", rb=None,
                     baby_mode="recompute", seed=42, log=None, record_first=False):
    """`blocks` FFN blocks (random weights from `seed`, the same on every rank) on rank 0's chain:
    FfnRanks over the ranks when `dist` is given (any world), else the one-rank ffn_block -- limb-identical.
    tf:239-266: a bootstrap (+ one rescale) before a block whenever fewer than 4 levels remain, its linear
    transforms' giant groups over every rank.  Returns {block_seconds, bootstrap_seconds, chain_index,
    max_err, corr (per block, decrypted vs the plaintext chain: tf:272-298's pass criterion), ct_sha256 (rank 0),
    setup_s, bootstrap_before (block indices)}; every block and bootstrap is bracketed by a device
    synchronisation and (over ranks) a barrier.  `dist.point("block<b>")` / `point("bootstrap")` mark the stage
    boundaries when the caller's dist has them (bench.py's FailureFence).  record_first (one rank, no dist):
    the chain's first BSGS call -- block 0, key chunk 0 -- exported after the chain as `first_bsgs` {ct_in,
    ct_out, pts} limbs (bench.py checks it against the CPU port)."""
    rng = np.random.default_rng(seed)
    t_setup = time.perf_counter()
    ck = Ckks(ph, N, L0, P, D, bootstrap=bootstrap)
    x = rng.normal(0, 0.1, D)
    ct = ck.encrypt_replicated(x) if rank == 0 else None
    ref = x.copy()
    fr = FfnRanks(ck, D, F, dist, rank, world, shard, rb, baby_mode, device) if dist is not None else None
    ck.ctx.synchronize()
    t_setup = time.perf_counter() - t_setup
    times, boots, cis, errs, corrs, boot_at = [], [], [], [], [], []
    point = getattr(dist, "point", None) or (lambda stage: None)
    if record_first and dist is None:
        RECORD[0] = {}

    def sync():
        ck.ctx.synchronize()
        if dist is not None:
            dist.barrier()
    for b in range(blocks):
        point(f"block{b}")
        Wk = rng.normal(0, 0.02, (D, F))
        Wv = rng.normal(0, 0.02, (F, D))
        if bootstrap:   # tf:239-266: fewer than 4 levels left -> bootstrap (+ one rescale)
            need = int(rank == 0 and (ck.L0 - 1) - ct.chain_index() < 4)
            if dist is not None:
                import torch
                flag = torch.tensor([need], dtype=torch.int64, device="cpu" if dist.get_backend() == "gloo" else device)
                dist.broadcast(flag, src=0)
                need = int(flag.item())
            if need:
                point("bootstrap")
                sync()
                t0 = time.perf_counter()
                if dist is None:
                    ct = ck.ph.rescale_to_next(ck.ctx, ck.bootstrap(ct))
                else:                          # its linear transforms' giant groups over every rank
                    if rank == 0:
                        while ct.coeff_modulus_size() > 2:
                            ct = ck.ph.mod_switch_to_next(ck.ctx, ct)
                    out = ck.bt.bootstrap_ranks(ck.ctx, ct if rank == 0 else None, dist, device)
                    ct = ck.ph.rescale_to_next(ck.ctx, out) if rank == 0 else None
                sync()
                boots.append(time.perf_counter() - t0)
                boot_at.append(b)
        sync()
        t0 = time.perf_counter()
        ct = fr.block(ct, Wk, Wv) if fr is not None else ffn_block(ck, ct, Wk, Wv, D, F)
        sync()
        times.append(time.perf_counter() - t0)
        ref = plain_ffn(ref, Wk, Wv)
        if rank == 0:
            dec = ck.decrypt(ct, D)
            errs.append(float(np.max(np.abs(dec - ref))))
            corrs.append(float(np.corrcoef(dec, ref)[0, 1]))
            cis.append(ct.chain_index())
            if log:
                log(f"block {b}: {1e3 * times[-1]:.1f} ms chain_index={cis[-1]} max_err={errs[-1]:.3e} "
                    f"corr={corrs[-1]:.8f}")
    res = {"block_seconds": times, "bootstrap_seconds": boots, "bootstrap_before": boot_at, "setup_s": t_setup}
    if rank == 0:
        res.update(chain_index=cis, max_err=errs, corr=corrs, ct_sha256=ct_digest(ct))
    if RECORD[0] is not None:
        r = RECORD[0]
        RECORD[0] = None
        if "ct_out" in r:
            res["first_bsgs"] = {"ct_in": r["ct_in"].to_numpy(), "ct_out": r["ct_out"].to_numpy(),
                                 "pts": [p.to_numpy() for p in r["pts"]]}
        del r
    del fr, ct, ck
    return res


def run_ranks(ph, a, dist, rank, world, device):
    """--blocks FFN blocks through chain_over_ranks; rank 0 prints the per-block times, the decrypted error
    against the plaintext chain and the final ciphertext's limb digest."""
    r = chain_over_ranks(ph, a.N, a.L0, a.P, a.D, a.F, a.blocks, a.bootstrap, dist, rank, world, device, a.shard,
                         a.rb, a.baby_mode, log=lambda m: print(m, flush=True))
    if rank == 0:
        print(f"ffn world {world} shard {a.shard if dist is not None else 'none'} babies {a.baby_mode}: "
              f"mean block {1e3 * np.mean(r['block_seconds']):.1f} ms, bootstraps {len(r['bootstrap_seconds'])}, "
              f"ct_sha256 {r['ct_sha256']}", flush=True)


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
    ap.add_argument("--dist", action="store_true",
                    help="blocks over ranks (torchrun; SURVEY §8e Config 5): FfnRanks, even at world 1")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"))
    ap.add_argument("--shard", default="giant", choices=("giant", "grid", "baby"))
    ap.add_argument("--rb", type=int, default=None)
    ap.add_argument("--baby-mode", default="recompute", choices=("recompute", "broadcast"))
    a = ap.parse_args()
    HOST_DIAGONALS[0] = a.host_diagonals
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.dist or world > 1:
        import torch
        import torch.distributed as dist
        rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
        if a.backend == "nccl":               # RCCL over xGMI, one GPU per rank
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:                                 # gloo: host-staged exchange (ranks may share a GPU)
            dist.init_process_group("gloo")
            local = int(os.environ.get("FHESPEAR_DEVICE", local))
        os.environ["FHESPEAR_DEVICE"] = str(local)
        import pyPhantom as ph
        run_ranks(ph, a, dist, rank, world, f"cuda:{local}")
        dist.barrier()
        dist.destroy_process_group()
        return
    import pyPhantom as ph
    if a.blocks and os.environ.get("FFN_DIGEST"):   # the one-rank reference of --dist runs
        run_ranks(ph, a, None, 0, 1, "cuda:0")
        return
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
