"""Multi-GPU plumbing for the 8-projection RWKV block (BASELINE configs[3]/[4]).

One process per GPU (torchrun); backend "nccl" = RCCL over xGMI on MI355X, "gloo" in CPU tests.
The data path has exactly two exchange steps, both on flat int64 views of ciphertext limbs:

  * gather_to_root   -- every rank's output ciphertext(s) to rank 0 (the "client" decrypts there);
  * broadcast_from   -- one rank's ciphertext limbs to all (baby steps shared by projections with
                        the same input, e.g. the FFN key pair, bg:563, north_star "computed once and
                        broadcast").

Projections are assigned round-robin (projection p -> rank p % world).  The reference runs the
block's 8 BSGS calls serially in one process (bg:784-892); which of them are independent:
r, k, v (same input x) -> o -> ffn key pair (shared input, shared baby steps) -> ffn value pair.

Latency mode: one matvec's B giant groups split over the ranks
(`giant_groups`); each rank computes its groups' rotated inner sums without the rescale
(`bsgs_giant_partial`, one fused linear transform), the partial ciphertexts are summed mod q_i on
the root (`modular_reduce_sum`: RCCL int64 sum, then one reduction) and the root rescales.  Every
giant term is an exact residue (the library sums giant steps before ModDown exactly), so the result
is limb-identical to the one-GPU fused BSGS.
"""
from __future__ import annotations

# block stage structure of bg.client_aided_block (bg:784-892): projections per stage
RWKV_BLOCK_STAGES = (("r", "k", "v"), ("o",), ("ffn_key_0", "ffn_key_1"), ("ffn_val_0", "ffn_val_1"))
RWKV_BLOCK_PROJECTIONS = tuple(p for st in RWKV_BLOCK_STAGES for p in st)


def owner(p: int, world: int) -> int:
    return p % world


def my_projections(n: int, world: int, rank: int) -> list[int]:
    return [p for p in range(n) if owner(p, world) == rank]


def stage_assignment(world: int, rank: int):
    """For each block stage, the projections this rank computes (round-robin inside the stage)."""
    out = []
    for stage in RWKV_BLOCK_STAGES:
        out.append([name for i, name in enumerate(stage) if i % world == rank])
    return out


def gather_to_root(dist, tensor, world: int, rank: int, root: int = 0):
    """All ranks' `tensor` (same shape) -> list on root (None elsewhere)."""
    import torch
    lst = [torch.empty_like(tensor) for _ in range(world)] if rank == root else None
    dist.gather(tensor, lst, dst=root)
    return lst


def broadcast_from(dist, tensor, src: int):
    dist.broadcast(tensor, src=src)
    return tensor


def modular_reduce_sum(dist, tensor, moduli_per_row, root: int = 0, group=None):
    """Sum of residues across the ranks of `group` (default: all), reduced mod q_i per limb row on
    the global rank `root` (giant-step sharding, §8e(2)).  RCCL's integer sum is not modular; with
    <= 15 ranks and 59-bit residues the plain int64 sum stays < 2^63, so one final reduction on the
    root is exact."""
    import torch
    if dist.get_world_size(group) > 15:
        raise ValueError("modular_reduce_sum: > 15 ranks could overflow int64 with 59-bit residues")
    dist.reduce(tensor, dst=root, group=group)
    if dist.get_rank() == root:
        q = torch.as_tensor(moduli_per_row, dtype=torch.int64, device=tensor.device).view(-1, 1)
        t = tensor.view(q.shape[0], -1)
        t.remainder_(q)
    return tensor


def stage_groups(n_proj: int, world: int):
    """Latency mode for one block stage: its n_proj projections -> contiguous, balanced groups of
    ranks (sizes differ by <= 1), each group sharding one projection's giant steps.  None when
    there are fewer ranks than projections (the stage is dealt round-robin instead)."""
    if world < n_proj:
        return None
    base, extra = divmod(world, n_proj)
    out, lo = [], 0
    for i in range(n_proj):
        s = base + (1 if i < extra else 0)
        out.append(list(range(lo, lo + s)))
        lo += s
    return out


# ------------------------------------------------------------------ giant-step sharding (§8e(2))
def giant_groups(B: int, world: int, rank: int) -> list[int]:
    """Contiguous, balanced share of the giant groups 0..B-1 for `rank` (sizes differ by <= 1)."""
    if world > B:
        raise ValueError(f"giant_groups: {world} ranks for {B} giant groups")
    base, extra = divmod(B, world)
    lo = rank * base + min(rank, extra)
    return list(range(lo, lo + base + (1 if rank < extra else 0)))


def bsgs_giant_partial(ph, ctx, baby, pts, G: int, D: int, groups, gk, zero_pts):
    """sum_{g in groups} rot_{gG}( sum_b baby[b] (.) pts[gG + b] ), not rescaled (bg:468-483 for a
    subset of g).  `pts` maps a diagonal index to its plaintext (a list, or a dict holding only this
    rank's diagonals); `zero_pts` = G encodings of 0 at the diagonals' level, which fill the identity
    group fhs_linear_transform requires when g = 0 is not ours and pad a short last group."""
    elts, flat = [1], []
    if groups and groups[0] == 0:
        first, rest = [0], groups[1:]
    else:
        first, rest = [], groups
        flat.extend(zero_pts[:G])
    for g in first + list(rest):
        if g:
            elts.append(ph.get_elt_from_step(g * G, ctx.N))
        for b in range(G):
            k = g * G + b
            flat.append(pts[k] if k < D else zero_pts[b])
    return ph.linear_transform(ctx, baby, flat, G, elts, gk, rescale=False)


def bsgs_giant_sharded(ph, ctx, baby, pts, G: int, B: int, D: int, gk, zero_pts, dist, device="cuda",
                       ranks=None, group=None):
    """One matvec with its giant groups split over `ranks` (global ranks of process group `group`;
    default: every rank), gloo staging through host memory.  Returns the rescaled output ciphertext
    on ranks[0], None elsewhere; limb-identical to ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B,
    D, gk).  `pts` need only hold this rank's diagonals."""
    import torch
    me = dist.get_rank()
    ranks = list(range(dist.get_world_size())) if ranks is None else list(ranks)
    share = giant_groups(B, len(ranks), ranks.index(me))
    part = bsgs_giant_partial(ph, ctx, baby, pts, G, D, share, gk, zero_pts)
    ci, scale, l = part.chain_index(), part.scale(), part.coeff_modulus_size()
    buf = torch.empty(2 * l * ctx.N, dtype=torch.int64, device=device)
    torch.cuda.synchronize()                      # torch's earlier use of the allocation is done
    ph.ciphertext_copy_to_device(ctx, part, buf.data_ptr())
    rows = [int(q) for q in ctx.primes[:l]] * 2   # [comp][limb] rows, limb t mod q_t
    if dist.get_backend(group) == "gloo":
        h = buf.cpu()
        modular_reduce_sum(dist, h, rows, root=ranks[0], group=group)
        buf.copy_(h)
    else:
        modular_reduce_sum(dist, buf, rows, root=ranks[0], group=group)
    if me != ranks[0]:
        return None
    torch.cuda.synchronize()
    total = ph.ciphertext_from_device(ctx, buf.data_ptr(), 2, ci, scale)
    return ph.rescale_to_next(ctx, total)
