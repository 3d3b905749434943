"""Latency-mode BSGS: one matvec's giant groups split over the ranks, partial
ciphertexts summed mod q_i on rank 0 over RCCL (fhespear_dist.bsgs_giant_sharded), checked
limb-for-limb against the one-GPU fused BSGS (bg:459) on rank 0.

Every rank builds the same context, keys, input encryption (deterministic from the seeds) and
diagonals; each computes the baby steps of the input (hoisted) and its share of the giant groups.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/giant_shard.py            # RCCL
    FHESPEAR_DEVICE=0 torchrun --nproc-per-node 2 ... tools/giant_shard.py --backend gloo --N 4096 --L0 6 --D 256
"""
import argparse
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))

import fhespear_dist as fd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--L0", type=int, default=36)
    ap.add_argument("--P", type=int, default=3)
    ap.add_argument("--D", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"))
    ap.add_argument("--mode", default="giant", choices=("giant", "baby", "grid"),
                    help="shard the giant groups (baby steps replicated), the baby steps (reduce-scatter "
                         "of every group's partial inner products, fhespear_dist.bsgs_baby_sharded), or both "
                         "(an rb x rg grid, fhespear_dist.bsgs_grid_sharded)")
    ap.add_argument("--rb", type=int, default=1, help="grid mode: baby-step shares (divides the world size)")
    ap.add_argument("--simulate-world", type=int, nargs="*", default=[],
                    help="also time one rank's share of the compute at these world sizes (on this GPU alone)")
    ap.add_argument("--simulate-grid", nargs="*", default=[],
                    help="also time one rank's compute on rb x rg grids given as 'rbxrg' (e.g. 2x4), with its "
                         "phases; the reduce-scatter then runs on a 1-rank group (a copy)")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
        local = int(os.environ.get("FHESPEAR_DEVICE", local % max(1, torch.cuda.device_count())))
    rank = dist.get_rank()
    import pyPhantom as ph

    N, D = a.N, a.D
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(a.P)
    parms.set_galois_elts(sorted(set(ph.get_elts_from_steps(list(range(1, G)) + [g * G for g in range(1, B)], N))))
    parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (a.L0 + a.P)))
    ctx = ph.context(parms, device=local)
    sk = ph.secret_key(ctx, seed=77)
    gk = sk.create_galois_keys(ctx)
    enc = ph.ckks_encoder(ctx)
    scale = 2.0 ** 59
    x = np.random.default_rng(1).normal(0, 0.1, D)
    ct = sk.encrypt_symmetric(ctx, enc.encode_double_vector(ctx, np.tile(x, (N // 2) // D), scale))
    level = ct.chain_index()
    pts = ph.random_plaintexts(ctx, 5, D, level, scale)
    zero = enc.encode_double_vector_batch(ctx, np.zeros((G, N // 2)), scale, chain_index=level)
    dev = f"cuda:{local}"

    def sharded():
        if a.mode == "baby":
            return fd.bsgs_baby_sharded(ph, ctx, ct, pts, G, B, D, gk, zero[0], dist, dev)
        if a.mode == "grid":
            return fd.bsgs_grid_sharded(ph, ctx, ct, pts, G, B, D, gk, zero[0], dist, a.rb, dev, col_groups=cols)
        baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
        return fd.bsgs_giant_sharded(ph, ctx, baby, pts, G, B, D, gk, zero, dist, dev)

    def barrier():
        ctx.synchronize()
        dist.barrier()

    cols = fd.grid_groups(dist, range(world), a.rb) if a.mode == "grid" else None

    y = sharded()
    exact = None
    if rank == 0:
        baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
        ref = ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
        exact = bool(np.array_equal(y.to_numpy(), ref.to_numpy())) and y.scale() == ref.scale() \
            and y.chain_index() == ref.chain_index()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        sharded()
    barrier()
    t_sh = (time.perf_counter() - t0) / a.reps
    if rank == 0:
        t0 = time.perf_counter()
        for _ in range(a.reps):
            baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
            ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B, D, gk)
        ctx.synchronize()
        t_one = (time.perf_counter() - t0) / a.reps
        print(f"{a.mode}-sharded BSGS N={N} L0={a.L0} D={D} (G={G}, B={B}) over {world} ranks "
              f"({a.backend}): bit-exact vs one-GPU fused BSGS: {exact}; "
              f"sharded {1e3 * t_sh:.2f} ms/matvec, one GPU {1e3 * t_one:.2f} ms/matvec", flush=True)
    if rank == 0 and a.simulate_world:
        # one rank's compute at world size W (rank 0 holds the largest share), measured alone:
        # baby steps + its giant groups + the root's rescale; the RCCL reduce is not included
        for W in a.simulate_world:
            grp = fd.giant_groups(B, W, 0)
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                if a.mode == "baby":   # rank 0's baby share, all groups' partial products, its giant groups
                    bs = fd.baby_steps_share(G, W, 0)
                    baby = [ct if b == 0 else ph.rotate(ctx, ct, b, gk) for b in bs]
                    parts = ph.bsgs_inner_products(ctx, baby, [pts[g * G + b] if g * G + b < D else zero[0]
                                                               for g in range(B) for b in bs], len(bs), B)
                    elts = [ph.get_elt_from_step(g * G, N) if g else 1 for g in grp]
                    ph.rescale_to_next(ctx, ph.bsgs_giant_steps(ctx, [parts[g] for g in grp], elts, gk))
                else:
                    baby = [ct] + [ph.rotate(ctx, ct, b, gk) for b in range(1, G)]
                    ph.rescale_to_next(ctx, fd.bsgs_giant_partial(ph, ctx, baby, pts, G, D, grp, gk, zero))
            ctx.synchronize()
            print(f"  per-rank compute at world {W} ({len(grp)} of {B} giant groups): "
                  f"{1e3 * (time.perf_counter() - t0) / a.reps:.2f} ms/matvec", flush=True)
    if rank == 0 and a.simulate_grid:
        # rank (0, 0)'s share on an rb x rg grid: its baby share, the partial inner products of its
        # column, the giant steps of its slice, the final reduce and the root's rescale.  Alone on this
        # GPU the two collectives keep their local part (the staging copies and the mod-q reduction of
        # this rank's slice) without the xGMI transfer itself.
        for spec in a.simulate_grid:
            rb, rg = (int(v) for v in spec.lower().split("x"))
            tm = {}
            t0 = time.perf_counter()
            for _ in range(a.reps):
                fd.bsgs_grid_sharded(ph, ctx, ct, pts, G, B, D, gk, zero[0], dist, rb, dev, timings=tm,
                                     sim_grid=(rb, rg))
            ctx.synchronize()
            dt = (time.perf_counter() - t0) / a.reps
            print(f"  grid {rb}x{rg} rank (0,0): {1e3 * dt:.2f} ms/matvec; phases (ms) " +
                  ", ".join(f"{k} {1e3 * v / a.reps:.2f}" for k, v in tm.items()), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0 and not exact:
        sys.exit(1)


if __name__ == "__main__":
    main()
