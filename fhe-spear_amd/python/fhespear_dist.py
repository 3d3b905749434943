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


def modular_reduce_sum(dist, tensor, moduli_per_row, root: int = 0):
    """Sum of residues across ranks, reduced mod q_i per limb row (giant-step sharding, §8e(2)).
    RCCL's integer sum is not modular; with < 8 ranks and 59-bit residues the plain int64 sum
    stays < 2^63, so one final reduction on the root is exact."""
    import torch
    if dist.get_world_size() > 15:
        raise ValueError("modular_reduce_sum: > 15 ranks could overflow int64 with 59-bit residues")
    dist.reduce(tensor, dst=root)
    if dist.get_rank() == root:
        q = torch.as_tensor(moduli_per_row, dtype=torch.int64, device=tensor.device).view(-1, 1)
        t = tensor.view(q.shape[0], -1)
        t.remainder_(q)
    return tensor
