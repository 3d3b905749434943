"""Giant-step sharding of one BSGS matvec over ranks (fhespear_dist)."""
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))

import fhespear_dist as fd  # noqa: E402


@pytest.mark.parametrize("B,world", [(45, 1), (45, 2), (45, 8), (32, 8), (7, 7), (16, 3)])
def test_giant_groups_partition(B, world):
    shares = [fd.giant_groups(B, world, r) for r in range(world)]
    assert sorted(g for s in shares for g in s) == list(range(B))
    sizes = [len(s) for s in shares]
    assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 1
    assert all(s == list(range(s[0], s[0] + len(s))) for s in shares)


def test_giant_groups_rejects_more_ranks_than_groups():
    with pytest.raises(ValueError):
        fd.giant_groups(4, 8, 0)


def test_stage_groups_eight_rank_block_layout():
    """Latency-mode layout of the RWKV block's stages at 8 GPUs (HISTORY.md §6): r/k/v 3+3+2,
    o 8, each FFN pair 4+4; fewer ranks than projections -> None (dealt instead)."""
    assert fd.stage_groups(3, 8) == [[0, 1, 2], [3, 4, 5], [6, 7]]
    assert fd.stage_groups(1, 8) == [list(range(8))]
    assert fd.stage_groups(2, 8) == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert fd.stage_groups(3, 2) is None
    for n, w in [(3, 4), (2, 5), (1, 1), (3, 3)]:
        gs = fd.stage_groups(n, w)
        assert sorted(r for g in gs for r in g) == list(range(w))
        assert max(map(len, gs)) - min(map(len, gs)) <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("D", [256, 200])   # 200: short last giant group, padded with zero diagonals
def test_giant_sharded_bsgs_bit_exact_two_ranks(require_gpu, D):
    """Two ranks on one GPU (gloo, host-staged reduce): the root's rescaled sum of the ranks'
    partial giant sums equals the one-GPU fused BSGS limb for limb."""
    env = dict(os.environ, FHESPEAR_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(29551 + D % 7), str(REPO / "tools" / "giant_shard.py"),
           "--backend", "gloo", "--N", "4096", "--L0", "6", "--P", "3", "--D", str(D), "--reps", "1"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert re.search(r"bit-exact vs one-GPU fused BSGS: True", out.stdout), out.stdout[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("world,D", [(2, 256), (3, 200), (4, 256)])
def test_baby_sharded_bsgs_bit_exact(require_gpu, world, D):
    """Baby-step sharding: each rank rotates its share of the baby steps, forms every
    giant group's partial inner product, a reduce-scatter hands each rank its groups' inner products,
    the owners' giant sums are reduced mod q_i on the root -- limb-identical to the one-GPU fused BSGS.
    `world` ranks share one GPU (gloo, host-staged collectives)."""
    env = dict(os.environ, FHESPEAR_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(29601 + world), str(REPO / "tools" / "giant_shard.py"),
           "--backend", "gloo", "--mode", "baby", "--N", "4096", "--L0", "6", "--P", "3", "--D", str(D), "--reps", "1"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert re.search(r"bit-exact vs one-GPU fused BSGS: True", out.stdout), out.stdout[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("world,rb,D", [(4, 2, 256), (6, 3, 200), (4, 1, 200)])
def test_grid_sharded_bsgs_bit_exact(require_gpu, world, rb, D):
    """Baby x giant grid (fhespear_dist.bsgs_grid_sharded): rb baby shares x world/rb giant columns,
    reduce-scatter inside each column's process group, giant steps of each rank's slice, modular sum
    on the root -- limb-identical to the one-GPU fused BSGS (rb = 1: giant-step sharding through the
    inner-products / giant-steps entries).  `world` ranks share one GPU (gloo)."""
    env = dict(os.environ, FHESPEAR_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(29621 + world + 10 * rb), str(REPO / "tools" / "giant_shard.py"),
           "--backend", "gloo", "--mode", "grid", "--rb", str(rb), "--N", "4096", "--L0", "6", "--P", "3", "--D", str(D),
           "--reps", "1"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert re.search(r"bit-exact vs one-GPU fused BSGS: True", out.stdout), out.stdout[-2000:]


@pytest.mark.gpu
def test_baby_sharded_bsgs_over_rccl_world1(require_gpu):
    """bsgs_baby_sharded through RCCL at world 1 (reduce_scatter_tensor + int64 reduce + event-ordered
    copies), bit-exact vs the fused BSGS."""
    env = dict(os.environ, FHESPEAR_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29591", str(REPO / "tools" / "giant_shard.py"),
           "--backend", "nccl", "--mode", "baby", "--N", "4096", "--L0", "6", "--P", "3", "--D", "256", "--reps", "1"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert re.search(r"bit-exact vs one-GPU fused BSGS: True", out.stdout), out.stdout[-2000:]


@pytest.mark.parametrize("G,world", [(46, 1), (46, 2), (46, 8), (16, 3), (5, 5)])
def test_baby_steps_share_partition(G, world):
    shares = [fd.baby_steps_share(G, world, r) for r in range(world)]
    assert sorted(b for s in shares for b in s) == list(range(G))
    assert max(map(len, shares)) - min(map(len, shares)) <= 1
    D = 45 * G - 3                          # short last giant group
    rows = [set(fd.baby_sharded_rows(G, 45, D, world, r)) for r in range(world)]
    assert sorted(k for r in rows for k in r) == list(range(D))


@pytest.mark.parametrize("world,rb", [(8, 2), (8, 4), (6, 3), (4, 1), (3, 3)])
def test_grid_rows_partition(world, rb):
    """Every diagonal is needed by exactly one rank of an rb x rg grid, and a rank's rows are its baby
    share's columns of its giant column's groups."""
    G, B = 46, 45
    D = B * G - 3
    rows = [fd.grid_rows(G, B, D, world, rb, r) for r in range(world)]
    assert sorted(k for r in rows for k in r) == list(range(D))
    assert fd.grid_rows(G, B, D, world, world, 1) == fd.baby_sharded_rows(G, B, D, world, 1)
    with pytest.raises(ValueError):
        fd.grid_shape(world, world + 1)
    rb_, rg = fd.grid_shape(world, rb)
    for j in range(rg):                      # each column's slices: contiguous, in slot order, none empty
        n = len(fd.giant_groups(B, rg, j))
        sl = fd.column_shares(n, rb_)
        assert [x for s in sl for x in s] == list(range(n)) and all(sl)
        assert all(s[0] == r * len(sl[0]) for r, s in enumerate(sl))
    with pytest.raises(ValueError):
        fd.column_shares(5, 4)               # ceil(5/4) = 2 per slice leaves the 4th rank empty


@pytest.mark.gpu
def test_giant_sharded_bsgs_over_rccl_world1(require_gpu):
    """bsgs_giant_sharded through RCCL (backend nccl) at world 1: the int64 reduce, the event-ordered
    copies between the library stream and torch's stream, and the root's rescale, bit-exact vs the
    fused BSGS."""
    env = dict(os.environ, FHESPEAR_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29561", str(REPO / "tools" / "giant_shard.py"),
           "--backend", "nccl", "--N", "4096", "--L0", "6", "--P", "3", "--D", "256", "--reps", "1"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert re.search(r"bit-exact vs one-GPU fused BSGS: True", out.stdout), out.stdout[-2000:]


def test_modular_reduce_sum_exact_beyond_int64_bound():
    """60-bit moduli at world 9: a plain int64 sum of residues could pass 2^63, so the helper must
    switch to the gathered modular sum; world-9 gloo run on CPU, result vs Python ints."""
    assert fd.int64_sum_is_exact(15, [(1 << 59) - 55])
    assert not fd.int64_sum_is_exact(9, [(1 << 60) - 93])
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "9",
           "--master-addr", "127.0.0.1", "--master-port", "29581", str(Path(__file__).parent / "_reduce_worker.py")]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert "reduce exact: True" in out.stdout, out.stdout[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("N,first_unrotated", [(4096, True), (4096, False), (16384, False)])
def test_bsgs_giant_steps_matches_oracle(require_gpu, N, first_unrotated):
    """ph.bsgs_giant_steps (the baby-sharded mode's giant half, fhs_bsgs_giant_steps): the sum of the
    rotated inner products, key switches summed before one ModDown, equals the oracle's sum of
    individually key-switched rotations (bg:478-483) limb for limb -- with and without an unrotated
    first term, and at N = 16384 (half-limb kernel forms)."""
    import numpy as np
    import pyPhantom as ph
    from oracle.oracle import Oracle, galois_elt
    L0, P, S = 6, 3, 31
    steps = [0, 8, 16, 24] if first_unrotated else [8, 16, 24]
    elts = [1 if s == 0 else galois_elt(s, N) for s in steps]
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(P)
    parms.set_galois_elts(sorted(e for e in elts if e != 1))
    primes = ph.create_coeff_modulus(N, [59] * (L0 + P))
    parms.set_coeff_modulus(primes)
    ctx = ph.context(parms)
    sk = ph.secret_key(ctx, seed=S)
    gk = sk.create_galois_keys(ctx)
    o = Oracle(N, [int(q) for q in primes], P)
    s = o.gen_secret(S)
    rng = np.random.default_rng(N + len(steps))
    cts = [o.encrypt_symmetric(S, j + 1, s, o.encode(rng.standard_normal(N // 2), 2.0 ** 40, L0))
           for j in range(len(steps))]
    got = ph.bsgs_giant_steps(ctx, [ph.ciphertext_from_numpy(ctx, c, 1, 2.0 ** 40) for c in cts], elts, gk)
    want = None
    for c, e in zip(cts, elts):
        t = c if e == 1 else o.rotate_elt(c, o.gen_galois_key(S, s, e), e)
        want = t if want is None else o.add(want, t)
    assert got.chain_index() == 1 and got.scale() == 2.0 ** 40
    assert np.array_equal(got.to_numpy(), want)
    with pytest.raises(ValueError):
        ph.bsgs_giant_steps(ctx, [ph.ciphertext_from_numpy(ctx, c, 1, 2.0 ** 40) for c in cts[:2]], [elts[-1], 1], gk)
