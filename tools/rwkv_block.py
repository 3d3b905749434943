"""Client-aided RWKV-7 block (BASELINE configs[2]/[3]: 8 BSGS projections per block) over pyPhantom.

A restatement of the reference caller scripts/bootstrap_generation.py (bg) -- client_aided_block
(bg:756-899), fhe_projection_bsgs (bg:545-659), fhe_matmul_bsgs[_complex] (bg:435-542),
pre_encode_block (bg:265-333), plaintext_block (bg:902-980) -- so the block runs on the GPU box,
where the reference does not travel.  The reference's own script runs unchanged against this backend
where it is present.  Weights are synthetic (random init of RWKVBlockWeights'
shapes, bg:662-716): there is no checkpoint and no network.

The server side of one block is 8 BSGS matvecs in four dependent stages (fhespear_dist.RWKV_BLOCK_STAGES):
r, k, v (own inputs) -> o -> ffn key pair (one input, shared baby steps, complex-packed output
chunks) -> ffn value pair (conjugate trick, own complex-packed inputs).  With --preencoded the
diagonals of all 8 projections stay resident in HBM (8 x 9.66 GB at cfg3: fits in 288 GB, where
the reference had to offload them to host memory on an 80 GB A100, tex:1074).

Multi-GPU (cfg4, torchrun): one process per GPU; every stage's projections are dealt round-robin to
ranks; rank 0 is the client -- it encrypts the stage inputs and broadcasts the ciphertext limbs,
each rank runs its projections, the output ciphertexts are gathered to rank 0 over RCCL and
decrypted there.  Ranks share the secret key seed only so that rank 0 can
decrypt what the others computed; no rank but 0 encrypts or decrypts.

    python tools/rwkv_block.py [--N 16384 --L0 36 --P 3 --D 2048 --F 8192 --blocks 1 --preencoded]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/rwkv_block.py --preencoded
"""
import argparse
import hashlib
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))

from ffn_block import bsgs_params  # noqa: E402
import fhespear_dist  # noqa: E402


# ------------------------------------------------------------------ client-side math (bg:719-741)
def layer_norm(x, weight, bias, eps=1e-5):
    return (x - np.mean(x)) / np.sqrt(np.var(x) + eps) * weight + bias


def group_norm(x, n_groups, weight, bias, eps=64e-5):
    g = x.reshape(n_groups, -1)
    out = (g - g.mean(axis=1, keepdims=True)) / np.sqrt(g.var(axis=1, keepdims=True) + eps)
    return out.reshape(-1) * weight + bias


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-np.clip(x, -500, 500)))


class BlockWeights:
    """RWKVBlockWeights' fields (bg:662-716), random-initialised at trained-model-like magnitudes.
    Matrices are stored [in, out] as load_weights transposes them."""

    def __init__(self, rng, block_idx, D, F, n_head):
        self.D, self.F, self.n_head, self.head_size, self.block_idx = D, F, n_head, D // n_head, block_idx
        n = rng.standard_normal
        u = rng.uniform
        self.ln1_w, self.ln1_b = 1 + 0.1 * n(D), 0.1 * n(D)
        self.ln2_w, self.ln2_b = 1 + 0.1 * n(D), 0.1 * n(D)
        self.ln_x_w, self.ln_x_b = 1 + 0.1 * n(D), 0.1 * n(D)
        for f in ("x_r", "x_k", "x_v", "x_g", "x_w", "x_a", "x_k_ffn", "k_k", "k_a"):
            setattr(self, f, u(0, 1, D))
        self.w0, self.w1, self.w2 = 0.5 * n(D), 0.1 * n((D, 64)), 0.1 * n((64, D))
        self.a0, self.a1, self.a2 = 0.5 * n(D), 0.1 * n((D, 64)), 0.1 * n((64, D))
        self.v0, self.v1, self.v2 = 0.5 * n(D), 0.1 * n((D, 32)), 0.1 * n((32, D))
        self.r_k = 0.1 * n((n_head, self.head_size))
        self.g1, self.g2 = n((D, 128)) / np.sqrt(D), n((128, D)) / np.sqrt(128)
        for f in ("W_r", "W_k", "W_v", "W_o"):
            setattr(self, f, n((D, D)) / np.sqrt(D))
        self.W_key_ffn = n((D, F)) / np.sqrt(D)
        self.W_val_ffn = n((F, D)) / np.sqrt(F) * 0.25


def _mix(block, x, x_prev_att):
    x_ln = layer_norm(x, block.ln1_w, block.ln1_b)
    xx = x_prev_att - x_ln
    return x_ln, {k: x_ln + xx * getattr(block, "x_" + k) for k in ("r", "k", "v", "g", "w", "a")}


def _wkv(block, xs, r, k, v, state, v_first):
    """bg:808-858 (the client's WKV state update, group norm and gating), shared by both paths."""
    H, hs, D = block.n_head, block.head_size, block.D
    r_h, k_h, v_h = r.reshape(H, hs), k.reshape(H, hs), v.reshape(H, hs)
    w_h = sigmoid(block.w0 + np.tanh(xs["w"] @ block.w1) @ block.w2).reshape(H, hs)
    decay = np.exp(-np.exp(-0.5) * w_h)
    a_h = sigmoid(block.a0 + (xs["a"] @ block.a1) @ block.a2).reshape(H, hs)
    kk_h = k_h * block.k_k.reshape(H, hs)
    kk_h = kk_h / (np.linalg.norm(kk_h, axis=1, keepdims=True) + 1e-12)
    k_h = k_h * (1.0 + (a_h - 1.0) * block.k_a.reshape(H, hs))
    if block.block_idx == 0:
        v_first_out = v.copy()
    else:
        v = v + (v_first - v) * sigmoid(block.v0 + (xs["v"] @ block.v1) @ block.v2)
        v_h = v.reshape(H, hs)
        v_first_out = v_first
    # every head at once (bg:838-845 loop over heads): sa = S (-kk), S' = S diag(decay) + sa (kk a)^T + v k^T,
    # wkv = S' r
    # the two rank-1 updates as one batched (hs x 2) @ (2 x hs) product, added in place: two 1 MB arrays per
    # call instead of five (the client's share of the block is allocation-bound on a loaded host)
    sa = np.matmul(state, -kk_h[:, :, None])[:, :, 0]
    new_state = np.matmul(np.stack([sa, v_h], axis=2), np.stack([kk_h * a_h, k_h], axis=1))
    new_state += state * decay[:, None, :]
    wkv_heads = np.matmul(new_state, r_h[:, :, None])[:, :, 0]
    wkv = group_norm(wkv_heads.reshape(D), H, block.ln_x_w, block.ln_x_b)
    wkv = wkv + ((r_h * k_h * block.r_k).sum(axis=1, keepdims=True) * v_h).reshape(D)
    g = sigmoid(xs["g"] @ block.g1) @ block.g2
    return wkv * g, new_state, v_first_out


def plaintext_block(block, x, x_prev_att, x_prev_ffn, state, v_first):
    """bg:902-980"""
    x_ln, xs = _mix(block, x, x_prev_att)
    gated, new_state, v_first_out = _wkv(block, xs, xs["r"] @ block.W_r, xs["k"] @ block.W_k,
                                         xs["v"] @ block.W_v, state, v_first)
    x = x + gated @ block.W_o
    x_ffn_ln = layer_norm(x, block.ln2_w, block.ln2_b)
    x_k_ffn = x_ffn_ln + (x_prev_ffn - x_ffn_ln) * block.x_k_ffn
    x = x + (np.maximum(x_k_ffn @ block.W_key_ffn, 0.0) ** 2) @ block.W_val_ffn
    return x, x_ln, x_ffn_ln, new_state, v_first_out


# ------------------------------------------------------------------ server side (pyPhantom)
def _diag_rows(M, D, G, slots):
    """bg:198-203 + bg:365-378: d_k[j] = M[j, (j+k) mod D], giant group g rolled by gG, tiled."""
    j = np.arange(D)
    d = M[j[None, :], (j[None, :] + j[:, None]) % D]
    for g in range(1, (D + G - 1) // G):
        s, e = g * G, min((g + 1) * G, D)
        d[s:e] = np.roll(d[s:e], g * G, axis=1)
    reps, rem = divmod(slots, D)
    return np.concatenate([np.tile(d, (1, reps)), d[:, :rem]], axis=1) if rem else np.tile(d, (1, reps))


class Server:
    """The CKKSBootstrapContext members the client-aided block uses (bg:61-147, skip_bootstrap):
    Galois keys for the BSGS elements of D only (bg:79-88; the power-of-two rotation keys serve the
    non-BSGS fhe_projection and are left out)."""

    def __init__(self, ph, N, L0, P, D, seed=11, device=0):
        self.ph, self.N, self.L0, self.D, self.device, self.seed = ph, N, L0, D, device, seed
        G, B = bsgs_params(D)
        self.G, self.B = G, B
        steps = list(range(1, G)) + [g * G for g in range(1, B)]
        parms = ph.params(ph.scheme_type.ckks)
        parms.set_poly_modulus_degree(N)
        parms.set_special_modulus_size(P)
        parms.set_galois_elts(sorted(set(ph.get_elts_from_steps(steps, N))))
        parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (L0 + P)))
        self.ctx = ph.context(parms, device=device)
        self.sk = ph.secret_key(self.ctx, seed=seed)
        self.encoder = ph.ckks_encoder(self.ctx)
        self.gk = self.sk.create_galois_keys(self.ctx)
        self.scale = 2.0 ** 59
        self.diag_scale = self.scale if L0 > 2 else 2.0 ** 29         # bg:102-104
        self.slots = N // 2
        self.level = 1                                                 # fresh encryption's chain index

    # bg:124-143
    def encrypt_replicated(self, x):
        reps = -(-self.slots // len(x))
        pt = self.encoder.encode_double_vector(self.ctx, np.tile(x, reps)[:self.slots], self.scale)
        return self.sk.encrypt_symmetric(self.ctx, pt)

    def encrypt_replicated_complex(self, xr, xi):
        z = np.asarray(xr) + 1j * np.asarray(xi)
        reps = -(-self.slots // len(z))
        pt = self.encoder.encode_complex_vector(self.ctx, np.tile(z, reps)[:self.slots], self.scale)
        return self.sk.encrypt_symmetric(self.ctx, pt)

    def decrypt_vec(self, ct, n):
        return np.array(self.encoder.decode_double_vector(self.ctx, self.sk.decrypt(self.ctx, ct)))[:n]

    def decrypt_vec_complex(self, ct, n):
        return np.array(self.encoder.decode_complex_vector(self.ctx, self.sk.decrypt(self.ctx, ct)))[:n]

    # the client's calls of one stage batched: encode + encrypt of all its inputs in one library pass, decrypt
    # + decode of all its outputs in one (one synchronisation) -- the same values as one at a time
    def encrypt_replicated_batch(self, xs, cplx=False):
        reps = -(-self.slots // len(xs[0]))
        rows = np.stack([np.tile(np.asarray(x), reps)[:self.slots] for x in xs])
        rows = rows.astype(np.complex128) if cplx else rows.astype(np.float64)
        # encode + encrypt_symmetric of each row (bg:53-58) in one library pass: the same ciphertexts
        return self.sk.encode_encrypt_batch(self.ctx, rows, self.scale)

    def decrypt_vecs(self, cts, n):
        """complex slots [len(cts), n] (real parts for real-packed outputs)"""
        # decrypt + decode_complex_vector of each (bg:784-892's decrypt_vec) in one library pass: the same doubles
        return self.sk.decrypt_decode_batch(self.ctx, cts, n)

    # bg:361-432
    def encode_real(self, M, rows=None):
        if rows is None:   # rows built on the GPU from M (limb-identical to the numpy rows below)
            return self.encoder.encode_matrix_diagonals(self.ctx, M, self.G, self.diag_scale, chain_index=self.level)
        d = _diag_rows(M, self.D, self.G, self.slots)
        return self.encoder.encode_double_vector_batch(self.ctx, d if rows is None else d[rows], self.diag_scale,
                                                       chain_index=self.level)

    def encode_complex(self, M1, M2, rows=None):
        if rows is None:
            return self.encoder.encode_matrix_diagonals(self.ctx, M1, self.G, self.diag_scale, chain_index=self.level,
                                                        M2=M2)
        z = _diag_rows(M1, self.D, self.G, self.slots) + 1j * _diag_rows(M2, self.D, self.G, self.slots)
        return self.encoder.encode_complex_vector_batch(self.ctx, z if rows is None else z[rows], self.diag_scale,
                                                        chain_index=self.level)

    def baby(self, ct):
        """bg:215-220"""
        return [ct] + [self.ph.rotate(self.ctx, ct, b, self.gk) for b in range(1, self.G)]

    def matmul(self, baby, pts):
        """bg:435-542 through bsgs_multiply_accumulate (the fused path the reference prefers, bg:462)"""
        return self.ph.bsgs_multiply_accumulate(self.ctx, baby, pts, self.G, self.B, self.D, self.gk)


def projection_matrices(block):
    """The 8 BSGS operands of one block (bg:265-333 pre_encode_block, same chunking as bg:545-659),
    as (name, kind, matrices): kind 'real' -> M, 'complex' -> (M1, M2)."""
    D, F = block.D, block.F
    out = [(n, "real", (getattr(block, "W_" + n).T,)) for n in ("r", "k", "v", "o")]
    n_chunks = -(-F // D)
    if n_chunks % 2:
        raise ValueError("rwkv_block: F/D must be even (complex-packed chunk pairs, bg:567-592)")
    for p in range(n_chunks // 2):           # bg:567-592: output chunks c, c+1 -> real / imag
        ms = []
        for c in (2 * p, 2 * p + 1):
            M = np.zeros((D, D))
            cols = min(D, F - c * D)
            M[:cols, :] = block.W_key_ffn[:, c * D:c * D + cols].T
            ms.append(M)
        out.append((f"ffn_key_{p}", "complex", tuple(ms)))
    for p in range(n_chunks // 2):           # bg:627-646: conjugate trick, input chunks c, c+1
        ms = []
        for i, c in enumerate((2 * p, 2 * p + 1)):
            M = np.zeros((D, D))
            rows = min(D, F - c * D)
            M[:, :rows] = (-1) ** i * block.W_val_ffn[c * D:c * D + rows, :].T
            ms.append(M)
        out.append((f"ffn_val_{p}", "complex", tuple(ms)))
    return out


class BlockRunner:
    """Server projections of client_aided_block, local or over ranks (cfg4).  Over ranks, a stage's
    projections are dealt round-robin (one projection per rank: throughput), or with split=True
    (latency mode) each projection gets a group of ranks that shard its giant
    steps (fhespear_dist.stage_groups / bsgs_giant_sharded); a stage with more projections than
    ranks is dealt."""

    def __init__(self, srv, block, preencoded, dist=None, rank=0, world=1, split=False, baby_mode="recompute",
                 shard="giant", rb=None):
        self.srv, self.block, self.pre, self.dist, self.rank, self.world = srv, block, preencoded, dist, rank, world
        if shard not in ("giant", "baby", "grid"):
            raise ValueError(f"shard {shard!r}: 'giant' (baby steps replicated), 'baby' (reduce-scatter) or 'grid'")
        # latency mode's split of one projection over its rank group: its giant groups (every rank
        # rotates all baby steps), its baby steps (fhespear_dist.bsgs_baby_sharded) or both
        # (fhespear_dist.bsgs_grid_sharded, rb = fhespear_dist.grid_rb(group size) baby shares)
        self.shard = shard
        if baby_mode not in ("recompute", "broadcast"):
            raise ValueError(f"baby_mode {baby_mode!r}: 'recompute' or 'broadcast'")
        # baby steps of an input several ranks need: every rank computes them ("recompute"), or the
        # first of those ranks computes them and broadcasts the G ciphertexts (north_star: "computed
        # once and broadcast"; 434 MB at cfg2) -- limb-identical either way
        self.baby_mode = baby_mode if dist is not None else "recompute"
        self.mats = {n: (k, m) for n, k, m in projection_matrices(block)}
        if set(self.mats) != set(fhespear_dist.RWKV_BLOCK_PROJECTIONS):
            raise ValueError("rwkv_block: this runner expects F = 4 D (8 projections, RWKV-7)")
        self.assign = fhespear_dist.stage_assignment(world, rank)
        self.host_coll = dist is not None and dist.get_backend() == "gloo"
        # latency mode: per stage, [(projection, ranks, process group)] or None (dealt)
        self.layout = [None] * len(fhespear_dist.RWKV_BLOCK_STAGES)
        self.share = {}                      # projection -> giant groups this rank computes
        self.grid = {}                       # projection -> (rb, column process groups) in grid mode
        if split and dist is not None:
            for i, names in enumerate(fhespear_dist.RWKV_BLOCK_STAGES):
                groups = fhespear_dist.stage_groups(len(names), world)
                if groups is None:
                    continue
                lay = []
                for n, ranks in zip(names, groups):   # every rank creates every group, same order
                    pg = dist.new_group(ranks) if len(ranks) > 1 else None
                    lay.append((n, ranks, pg))
                    rb_n = None
                    if shard == "grid":   # baby shares: the caller's, when it divides the group, else the model's
                        rb_n = rb if rb and len(ranks) % rb == 0 else fhespear_dist.grid_rb(len(ranks))
                    if rb_n is not None and len(ranks) > 1:
                        self.grid[n] = (rb_n, fhespear_dist.grid_groups(dist, ranks, rb_n))
                    if rank in ranks:
                        R, me = len(ranks), ranks.index(rank)
                        if shard == "giant":
                            self.share[n] = fhespear_dist.giant_groups(srv.B, R, me)
                        elif shard == "baby":
                            self.share[n] = fhespear_dist.baby_sharded_rows(srv.G, srv.B, srv.D, R, me)
                        else:
                            self.share[n] = fhespear_dist.grid_rows(srv.G, srv.B, srv.D, R, rb_n, me)
                self.layout[i] = lay
                self.assign[i] = [n for n, ranks, _ in lay if rank in ranks]
            self.zero = srv.encoder.encode_double_vector_batch(srv.ctx, np.zeros((srv.G, srv.slots)), srv.diag_scale,
                                                               chain_index=srv.level)
        # dealt stages: ranks owning projections that share an input -> (ranks, process group)
        self.share_groups = {}
        if self.baby_mode == "broadcast":
            for i, names in enumerate(fhespear_dist.RWKV_BLOCK_STAGES):
                if self.layout[i] is not None:
                    continue
                for shared in fhespear_dist.RWKV_SHARED_INPUTS:
                    if not set(shared) <= set(names):
                        continue
                    owners = sorted({names.index(n) % world for n in shared})
                    if len(owners) > 1:
                        self.share_groups[(i, shared)] = (owners, dist.new_group(owners))
        mine = {n for st in self.assign for n in st}
        self.pts = {}
        if preencoded:                       # bg:1124-1174 --preencoded, resident in HBM
            for n in mine:
                self.pts[n] = self._encode(n)

    def _rows(self, name):
        """diagonal indices this rank needs for `name` (its giant groups' share, or all D)"""
        if name not in self.share:
            return None
        if self.shard != "giant":
            return self.share[name]
        G, D = self.srv.G, self.srv.D
        return [g * G + b for g in self.share[name] for b in range(G) if g * G + b < D]

    def _encode(self, name):
        kind, ms = self.mats[name]
        rows = self._rows(name)
        if rows is None:
            return self.srv.encode_real(*ms) if kind == "real" else self.srv.encode_complex(*ms)
        pts = self.srv.encode_real(*ms, rows=rows) if kind == "real" else self.srv.encode_complex(*ms, rows=rows)
        return dict(zip(rows, pts))

    def _pts(self, name):
        return self.pts[name] if self.pre else self._encode(name)

    def _pack(self, ct, buf):
        """ciphertext limbs + its scale (float64 bits in the last word) into an int64 device buffer,
        ordered against torch's stream with events (fhespear_dist.to_buffer)."""
        fhespear_dist.to_buffer(self.srv.ph, self.srv.ctx, ct, buf)
        buf[-1:].copy_(_scale_word(ct.scale(), buf))

    def _unpack(self, buf, ci):
        import torch
        scale = float(buf[-1:].cpu().view(torch.float64).item())
        return fhespear_dist.from_buffer(self.srv.ph, self.srv.ctx, buf, 2, ci, scale)

    def _buf(self, ci):
        import torch
        l = self.srv.L0 + 1 - ci
        return torch.empty(2 * l * self.srv.N + 1, dtype=torch.int64, device=f"cuda:{self.srv.device}")

    def _shared_babies(self, ct, ranks, pg):
        """Baby steps of `ct` (bg:215-220) computed on ranks[0] and broadcast over `pg` to the other
        ranks of `ranks`, as one buffer of G ciphertexts (rotations keep ct's level and scale)."""
        import torch
        srv = self.srv
        G, ci = srv.G, ct.chain_index()
        words = 2 * (srv.L0 + 1 - ci) * srv.N
        buf = torch.empty(G * words + 1, dtype=torch.int64, device=f"cuda:{srv.device}")
        src = ranks[0]
        if self.rank == src:
            babies = srv.baby(ct)
            for b, c in enumerate(babies):
                fhespear_dist.to_buffer(srv.ph, srv.ctx, c, buf[b * words:(b + 1) * words])
            buf[-1:].copy_(_scale_word(ct.scale(), buf))
        if self.host_coll:
            h = buf.cpu()
            self.dist.broadcast(h, src=src, group=pg)
            if self.rank != src:
                buf.copy_(h)
        else:
            self.dist.broadcast(buf, src=src, group=pg)
        if self.rank == src:
            return babies
        scale = float(buf[-1:].cpu().view(torch.float64).item())
        return [fhespear_dist.from_buffer(srv.ph, srv.ctx, buf[b * words:(b + 1) * words], 2, ci, scale)
                for b in range(G)]

    def _bcast_ct(self, ct):
        """rank 0's ciphertext -> every rank (RCCL broadcast over xGMI)."""
        srv = self.srv
        buf = self._buf(srv.level)
        if self.rank == 0:
            self._pack(ct, buf)
        if self.host_coll:                   # gloo (shared-GPU rehearsal): stage through host
            h = buf.cpu()
            fhespear_dist.broadcast_from(self.dist, h, 0)
            buf.copy_(h)
        else:
            fhespear_dist.broadcast_from(self.dist, buf, 0)
        return self._unpack(buf, srv.level)

    def stage(self, idx, inputs):
        """Run stage idx.  inputs: name -> (ciphertext on rank 0 | None elsewhere, shared key).  Returns
        name -> output ciphertext on rank 0."""
        srv = self.srv
        names = fhespear_dist.RWKV_BLOCK_STAGES[idx]
        point = getattr(self.dist, "point", None)
        if point is not None:                # stage boundary (bench.py's FailureFence: check + injection)
            point(f"stage{idx}")
        cts = {}
        for n in names:                      # distinct input ciphertexts in first-use order
            key = inputs[n][1]
            if key not in cts:
                cts[key] = inputs[n][0] if self.dist is None else self._bcast_ct(inputs[n][0])
        if self.layout[idx] is not None:
            return self._stage_split(idx, inputs, cts)
        mine = names if self.dist is None else self.assign[idx]
        babies = {}
        for (i, shared), (ranks, pg) in self.share_groups.items():
            if i == idx and self.rank in ranks:   # computed on ranks[0], broadcast to the others
                key = inputs[shared[0]][1]
                babies[key] = self._shared_babies(cts[key], ranks, pg)
        outs = {}
        for n in mine:
            key = inputs[n][1]
            if key not in babies:            # baby steps computed once per input (bg:563 shared)
                babies[key] = srv.baby(cts[key])
            outs[n] = srv.matmul(babies[key], self._pts(n))
        if self.dist is None:
            return outs
        return self._gather(names, outs)

    def _stage_split(self, idx, inputs, cts):
        """Latency mode: each projection's rank group shards its giant steps; the group roots send
        the rescaled outputs to rank 0 (the client)."""
        import torch
        srv, ph = self.srv, self.srv.ph
        dev = f"cuda:{srv.device}"
        res = {}
        for n, ranks, pg in self.layout[idx]:
            if self.rank not in ranks:
                continue
            if self.shard == "baby" and len(ranks) > 1:   # no replicated baby rotations
                out = fhespear_dist.bsgs_baby_sharded(ph, srv.ctx, cts[inputs[n][1]], self._pts(n), srv.G, srv.B,
                                                      srv.D, srv.gk, self.zero[0], self.dist, dev, ranks=ranks, group=pg)
                if out is not None:
                    res[n] = out
                continue
            if self.shard == "grid" and len(ranks) > 1:
                rb, cols = self.grid[n]
                out = fhespear_dist.bsgs_grid_sharded(ph, srv.ctx, cts[inputs[n][1]], self._pts(n), srv.G, srv.B,
                                                      srv.D, srv.gk, self.zero[0], self.dist, rb, dev, ranks=ranks,
                                                      group=pg, col_groups=cols)
                if out is not None:
                    res[n] = out
                continue
            if self.baby_mode == "broadcast" and len(ranks) > 1:
                baby = self._shared_babies(cts[inputs[n][1]], ranks, pg)
            else:
                baby = srv.baby(cts[inputs[n][1]])
            pts = self._pts(n)
            if len(ranks) == 1:
                out = srv.matmul(baby, [pts[k] for k in range(srv.D)] if isinstance(pts, dict) else pts)
            else:
                out = fhespear_dist.bsgs_giant_sharded(ph, srv.ctx, baby, pts, srv.G, srv.B, srv.D, srv.gk,
                                                       self.zero, self.dist, dev, ranks=ranks, group=pg)
            if out is not None:
                res[n] = out
        ci = srv.level + 1
        got = {}
        for n, ranks, _ in self.layout[idx]:          # group roots -> rank 0 (point to point)
            src = ranks[0]
            if src == 0:
                if self.rank == 0:
                    got[n] = res[n]
                continue
            if self.rank == src:
                buf = self._buf(ci)
                self._pack(res[n], buf)
                if self.host_coll:
                    self.dist.send(buf.cpu(), dst=0)
                else:
                    self.dist.send(buf, dst=0)
            elif self.rank == 0:
                buf = self._buf(ci)
                if self.host_coll:
                    h = buf.cpu()
                    self.dist.recv(h, src=src)
                    buf.copy_(h)
                else:
                    self.dist.recv(buf, src=src)
                got[n] = self._unpack(buf, ci)
        return got

    def _gather(self, names, outs):
        """Output ciphertexts -> rank 0 (RCCL gather); projection i of the stage lives on rank i % world."""
        srv = self.srv
        ci = srv.level + 1
        res = {}
        for r in range(-(-len(names) // self.world)):
            buf = self._buf(ci)
            local = [n for i, n in enumerate(names) if i // self.world == r and i % self.world == self.rank]
            if local:
                self._pack(outs[local[0]], buf)
            if self.host_coll:
                got = fhespear_dist.gather_to_root(self.dist, buf.cpu(), self.world, self.rank)
                got = [g.to(buf.device) for g in got] if got is not None else None
            else:
                got = fhespear_dist.gather_to_root(self.dist, buf, self.world, self.rank)
            if self.rank == 0:
                for i, n in enumerate(names):
                    if i // self.world == r:
                        res[n] = self._unpack(got[i % self.world], ci)
        return res


def _scale_word(scale, like):
    import torch
    return torch.tensor([scale], dtype=torch.float64).view(torch.int64).to(like.device)


def _enc(srv, xs, cplx=False):
    """the stage's inputs encrypted together when the server batches (Server), else one at a time"""
    if hasattr(srv, "encrypt_replicated_batch"):
        return srv.encrypt_replicated_batch(xs, cplx)
    return [srv.encrypt_replicated_complex(x.real, x.imag) if cplx else srv.encrypt_replicated(x) for x in xs]


def _dec(srv, cts, n):
    if hasattr(srv, "decrypt_vecs"):
        return srv.decrypt_vecs(cts, n)
    return np.stack([srv.decrypt_vec_complex(c, n) for c in cts])


def client_aided_block(run, x, x_prev_att, x_prev_ffn, state, v_first):
    """bg:756-899 with the server projections dealt by `run` (BlockRunner).  The client (rank 0)
    computes; other ranks return None for the activations but take part in every stage.
    Timings (seconds): server_<stage> = the stage's projections alone (input broadcast, matvecs, output
    gather); client_encrypt / client_decrypt = the client's encode+encrypt and decrypt+decode calls (one
    batch per stage); client_numpy = its float64 math (layer norms, WKV state, gates)."""
    srv, block, client = run.srv, run.block, run.rank == 0
    D = block.D
    t = {"client_encrypt": 0.0, "client_decrypt": 0.0, "client_numpy": 0.0}
    sync = srv.ctx.synchronize
    clock = time.perf_counter

    def timed(key, fn, *args):
        sync()
        t0 = clock()
        r = fn(*args)
        sync()
        t[key] = t.get(key, 0.0) + clock() - t0
        return r

    def enc(xs, cplx=False):
        return timed("client_encrypt", _enc, srv, xs, cplx) if client else [None] * len(xs)

    def dec(cts):
        return timed("client_decrypt", _dec, srv, cts, D)

    t0 = clock()
    x_ln = xs = None
    if client:
        x_ln, xs = _mix(block, x, x_prev_att)
    t["client_numpy"] += clock() - t0
    cts = enc([xs[n] for n in ("r", "k", "v")] if client else [0, 0, 0])
    outs = timed("server_rkv", run.stage, 0, {n: (c, n) for n, c in zip(("r", "k", "v"), cts)})
    gated = new_state = v_first_out = None
    if client:
        d = dec([outs[n] for n in ("r", "k", "v")]).real
        t0 = clock()
        gated, new_state, v_first_out = _wkv(block, xs, d[0], d[1], d[2], state, v_first)
        t["client_numpy"] += clock() - t0
    (ct_o,) = enc([gated] if client else [0])
    outs = timed("server_wo", run.stage, 1, {"o": (ct_o, "o")})
    x_k_ffn = x_ffn_ln = None
    if client:
        att = dec([outs["o"]])[0].real
        t0 = clock()
        x = x + att
        x_ffn_ln = layer_norm(x, block.ln2_w, block.ln2_b)
        x_k_ffn = x_ffn_ln + (x_prev_ffn - x_ffn_ln) * block.x_k_ffn
        t["client_numpy"] += clock() - t0
    n_pairs = block.F // D // 2
    (ct_k,) = enc([x_k_ffn] if client else [0])
    outs = timed("server_ffn_key", run.stage, 2, {f"ffn_key_{p}": (ct_k, "x_k_ffn") for p in range(n_pairs)})
    fk_sq = None
    if client:
        z = dec([outs[f"ffn_key_{p}"] for p in range(n_pairs)])
        t0 = clock()
        fk = np.empty(block.F)
        for p in range(n_pairs):             # bg:585-587: real -> chunk 2p, imag -> chunk 2p+1
            fk[2 * p * D:(2 * p + 1) * D] = z[p].real
            fk[(2 * p + 1) * D:(2 * p + 2) * D] = z[p].imag
        fk_sq = np.maximum(fk, 0.0) ** 2
        t["client_numpy"] += clock() - t0
    # bg:612-640: Enc(x0 + i x1) against (M0, -M1)
    cts = enc([fk_sq[2 * p * D:(2 * p + 1) * D] + 1j * fk_sq[(2 * p + 1) * D:(2 * p + 2) * D]
               for p in range(n_pairs)] if client else [0] * n_pairs, cplx=True)
    outs = timed("server_ffn_val", run.stage, 3, {f"ffn_val_{p}": (cts[p], f"v{p}") for p in range(n_pairs)})
    if client:
        v_ffn = dec([outs[f"ffn_val_{p}"] for p in range(n_pairs)]).real.sum(axis=0)
        x = x + v_ffn
    return x, x_ln, x_ffn_ln, new_state, v_first_out, t


def run_blocks(ph, args, dist=None, rank=0, world=1, device=0, log=print):
    """Build the server and n blocks, run the client-aided chain and the plaintext chain side by side;
    returns per-block records (server seconds, stage times, max error, corr) on rank 0."""
    H = max(1, args.D // args.head_size)
    rng = np.random.default_rng(args.seed)
    blocks = [BlockWeights(rng, b, args.D, args.F, H) for b in range(args.blocks)]
    t0 = time.perf_counter()
    srv = Server(ph, args.N, args.L0, args.P, args.D, device=device)
    runs = [BlockRunner(srv, b, args.preencoded, dist, rank, world, split=getattr(args, "split", False),
                        baby_mode=getattr(args, "baby_mode", "recompute"), shard=getattr(args, "shard", "giant"), rb=getattr(args, "rb", None))
            for b in blocks]
    srv.ctx.synchronize()
    if rank == 0:
        log(f"setup (keys{', pre-encoded diagonals' if args.preencoded else ''}): {time.perf_counter() - t0:.2f} s")
    x = rng.standard_normal(args.D)
    st = (x.copy(), np.zeros(args.D), np.zeros(args.D), np.zeros((H, args.D // H, args.D // H)), None)
    ref = tuple(v.copy() if v is not None else None for v in st)
    recs = []
    for b, run in enumerate(runs):
        for rep in range(args.reps):
            out = client_aided_block(run, *st)
            tm = out[5]
        st = out[:5]
        ref = plaintext_block(blocks[b], *ref)
        if rank == 0:
            err = float(np.max(np.abs(st[0] - ref[0])))
            corr = float(np.corrcoef(st[0], ref[0])[0, 1])
            sec = sum(v for k, v in tm.items() if k.startswith("server_"))
            rec = dict(block=b, server_seconds=sec, client_seconds=sum(v for k, v in tm.items() if k.startswith("client_")),
                       stages=tm, max_err=err, corr=corr,
                       mag=float(np.max(np.abs(ref[0]))),
                       x_sha256=hashlib.sha256(np.ascontiguousarray(st[0]).tobytes()).hexdigest())
            recs.append(rec)
            log(f"block {b}: server {1e3 * sec:.1f} ms (" + ", ".join(f"{k} {1e3 * v:.1f}" for k, v in tm.items())
                + f")  max_err={err:.3e} |x|={rec['mag']:.2f} corr={corr:.10f}")
    return recs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--L0", type=int, default=36)
    ap.add_argument("--P", type=int, default=3)
    ap.add_argument("--D", type=int, default=2048)
    ap.add_argument("--F", type=int, default=8192)
    ap.add_argument("--head-size", type=int, default=64)
    ap.add_argument("--blocks", type=int, default=1)
    ap.add_argument("--reps", type=int, default=2, help="runs of each block (the last one is reported)")
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--preencoded", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"))
    ap.add_argument("--split", action="store_true",
                    help="latency mode: each stage's projections shard their giant steps over rank groups")
    ap.add_argument("--shard", default="giant", choices=("giant", "baby", "grid"),
                    help="latency mode's split of a projection: giant groups (baby steps replicated), baby steps "
                         "(reduce-scatter of every group's partial inner products) or a baby x giant grid")
    ap.add_argument("--rb", type=int, default=None,
                    help="grid shard: baby shares per projection group (default fhespear_dist.grid_rb)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group even at world 1 (runs the exchange code on one GPU)")
    ap.add_argument("--baby-mode", default="recompute", choices=("recompute", "broadcast"),
                    help="baby steps of an input several ranks need: recomputed by each, or computed once and broadcast")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or a.dist:
        import torch
        import torch.distributed as dist
        if a.backend == "nccl":               # RCCL over xGMI, one GPU per rank
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:                                 # gloo: host-staged exchange (ranks may share a GPU)
            dist.init_process_group("gloo")
            local = int(os.environ.get("FHESPEAR_DEVICE", local % max(1, torch.cuda.device_count())))
    import pyPhantom as ph
    recs = run_blocks(ph, a, dist, rank, world, local)
    if rank == 0:
        s = [r["server_seconds"] for r in recs]
        print(f"world {world}{' split' if a.split else ''} babies {a.baby_mode}: mean server time per block "
              f"{np.mean(s):.4f} s over {len(s)} block(s), final max_err {recs[-1]['max_err']:.3e} "
              f"x_sha256 {recs[-1]['x_sha256']}")
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
