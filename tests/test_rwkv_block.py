"""Client-aided RWKV-7 block (bg:756-899) restated in tools/rwkv_block.py: BASELINE configs[2]/[3].

CPU: the projection chunking (complex-packed FFN key pairs, conjugate-trick FFN value pairs,
bg:545-659) checked against plaintext_block (bg:902-980) through an exact stand-in server.
GPU: the same block through pyPhantom (8 BSGS matvecs) against plaintext_block."""
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))

import rwkv_block as rb  # noqa: E402


@pytest.fixture(scope="module")
def ph(require_gpu):
    import pyPhantom
    return pyPhantom


class _Ctx:
    def synchronize(self):
        pass


class ExactServer:
    """Server's interface over plain complex vectors: encryption is the identity, a plaintext
    'encoding' is the matrix itself, so any chunking / packing mistake shows as a real error."""

    def __init__(self, D, slots):
        self.D, self.slots, self.level, self.ctx, self.device = D, slots, 1, _Ctx(), 0

    def encrypt_replicated(self, x):
        return np.asarray(x, dtype=complex)

    def encrypt_replicated_complex(self, xr, xi):
        return np.asarray(xr) + 1j * np.asarray(xi)

    def decrypt_vec(self, ct, n):
        return ct.real[:n]

    def decrypt_vec_complex(self, ct, n):
        return ct[:n]

    def encode_real(self, M):
        return M.astype(complex)

    def encode_complex(self, M1, M2):
        return M1 + 1j * M2

    def baby(self, ct):
        return ct

    def matmul(self, baby, pts):
        return pts @ baby


@pytest.mark.parametrize("preencoded", [False, True])
def test_block_chunking_matches_plaintext_block(preencoded):
    D, F, H = 32, 128, 4
    rng = np.random.default_rng(0)
    blocks = [rb.BlockWeights(rng, b, D, F, H) for b in range(2)]
    srv = ExactServer(D, 64)
    x = rng.standard_normal(D)
    st = (x, np.zeros(D), np.zeros(D), np.zeros((H, D // H, D // H)), None)
    ref = st
    for blk in blocks:
        run = rb.BlockRunner(srv, blk, preencoded)
        out = rb.client_aided_block(run, *st)
        st = out[:5]
        ref = rb.plaintext_block(blk, *ref)
        assert set(out[5]) == {"server_rkv", "server_wo", "server_ffn_key", "server_ffn_val", "client_encrypt",
                               "client_decrypt", "client_numpy"}
        for a, b in zip(st[:4], ref[:4]):
            np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12)


def test_projection_matrices_shape_and_stages():
    D, F = 16, 64
    blk = rb.BlockWeights(np.random.default_rng(1), 0, D, F, 2)
    names = [n for n, _, _ in rb.projection_matrices(blk)]
    import fhespear_dist
    assert names == list(fhespear_dist.RWKV_BLOCK_PROJECTIONS)
    with pytest.raises(ValueError):
        rb.BlockRunner(ExactServer(D, 32), rb.BlockWeights(np.random.default_rng(1), 0, D, 3 * D, 2), False)


def _run_block_tool(world, backend="gloo", extra=(), port=29541):
    """tools/rwkv_block.py under torch.distributed.run on cuda:0; returns (final max_err, x digest)."""
    import os
    import re
    import subprocess
    env = dict(os.environ, FHESPEAR_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           str(REPO / "tools" / "rwkv_block.py"),
           "--backend", backend, "--N", "2048", "--L0", "4", "--P", "2", "--D", "64", "--F", "256",
           "--head-size", "16", "--blocks", "2", "--reps", "1", "--preencoded"] + list(extra)
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=100 if world <= 4 else 280)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    m = re.search(rf"world {world}.*: .* final max_err ([0-9.e+-]+) x_sha256 ([0-9a-f]+)", out.stdout)
    assert m, out.stdout[-2000:]
    assert all(float(c) > 0.999999 for c in re.findall(r"corr=([0-9.]+)", out.stdout))
    return float(m.group(1)), m.group(2)


_ONE_RANK = {}


def _one_rank_digest():
    if "d" not in _ONE_RANK:
        _ONE_RANK["d"] = _run_block_tool(1, port=29540)[1]
    return _ONE_RANK["d"]


@pytest.mark.gpu
@pytest.mark.parametrize("world,split,babies", [(2, False, "recompute"), (2, False, "broadcast"),
                                                 (2, True, "recompute"), (4, True, "recompute"),
                                                 (4, True, "broadcast")])
def test_block_over_ranks(require_gpu, world, split, babies):
    """cfg4's exchange (stage inputs broadcast from the client rank, output ciphertexts to it) on one
    GPU: gloo stages the limbs through host memory, every rank's context shares cuda:0.  split=True
    is latency mode (giant steps of a projection sharded over a rank group: at world 4 the stages
    split 2+1+1 / 4 / 2+2 / 2+2; at world 2 stage 1 is dealt).  babies="broadcast": the baby steps
    of an input several ranks need are computed on one rank and broadcast (north_star).  Every
    variant must give the one-rank block's output bit for bit (same digest of the decrypted x)."""
    extra = (["--split"] if split else []) + ["--baby-mode", babies]
    err, digest = _run_block_tool(world, extra=extra, port=29541 + world + 10 * split + 20 * (babies == "broadcast"))
    assert err < 1e-4
    assert digest == _one_rank_digest()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_block_over_ranks_baby_sharded(require_gpu, world):
    """Latency mode with the baby steps sharded (BlockRunner shard="baby", fhespear_dist.bsgs_baby_sharded:
    no replicated baby rotations, a reduce-scatter of every giant group's partial inner products):
    the same decrypted block output as one rank, bit for bit."""
    err, digest = _run_block_tool(world, extra=["--split", "--shard", "baby"], port=29561 + world)
    assert err < 1e-4
    assert digest == _one_rank_digest()


@pytest.mark.gpu
def test_block_over_ranks_grid_sharded(require_gpu):
    """Latency mode on a baby x giant grid (BlockRunner shard="grid", rb=2): at world 4 the o projection
    runs on a 2 x 2 grid (column process groups, reduce-scatter inside each), each FFN pair's 2-rank group
    as a 2 x 1 grid (baby shares only), the 1-rank groups whole -- the same decrypted block output as one
    rank, bit for bit."""
    err, digest = _run_block_tool(4, extra=["--split", "--shard", "grid", "--rb", "2"], port=29581)
    assert err < 1e-4
    assert digest == _one_rank_digest()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["dealt", "dealt-broadcast", "giant", "baby", "grid"])
def test_block_over_eight_ranks(require_gpu, mode):
    """cfg4's world size: 8 ranks (gloo, all sharing cuda:0) in every shard mode of BlockRunner.  dealt:
    each stage's projections round-robin (r, k, v on ranks 0-2, o on 0, the FFN pairs on 0-1), with
    "broadcast" the FFN key pair's baby steps computed once and broadcast; giant / baby / grid: latency
    mode, the stages' rank groups 3+3+2 (r, k, v), 8 (o), 4+4, 4+4 (FFN pairs) shard each projection by
    giant groups, by baby steps (reduce-scatter) or on a grid with fhespear_dist.grid_rb(group size)
    baby shares (8x1 for o).  Every mode must give the one-rank block's output bit for bit."""
    extra = {"dealt": [], "dealt-broadcast": ["--baby-mode", "broadcast"], "giant": ["--split"],
             "baby": ["--split", "--shard", "baby"], "grid": ["--split", "--shard", "grid"]}[mode]
    port = 29600 + ["dealt", "dealt-broadcast", "giant", "baby", "grid"].index(mode)
    err, digest = _run_block_tool(8, extra=extra, port=port)
    assert err < 1e-4
    assert digest == _one_rank_digest()


@pytest.mark.gpu
def test_block_exchange_over_rccl_world1(require_gpu):
    """The real transport: backend nccl (RCCL) at world 1 with the process group forced on, so the
    input broadcast, the output gather and the event ordering between the library stream and torch's
    stream (fhespear_dist.to_buffer / from_buffer) run on hardware; the output must equal the
    no-process-group run bit for bit."""
    err, digest = _run_block_tool(1, backend="nccl", extra=["--dist"], port=29571)
    assert err < 1e-4
    assert digest == _one_rank_digest()


@pytest.mark.gpu
def test_client_aided_block_on_gpu(ph):
    """2 blocks, N = 2048, L0 = 4, D = 64, F = 256: every projection a fused BSGS on the GPU."""
    import argparse
    a = argparse.Namespace(N=2048, L0=4, P=2, D=64, F=256, head_size=16, blocks=2, reps=1, seed=5,
                           preencoded=True)
    recs = rb.run_blocks(ph, a, log=lambda *_: None)
    assert len(recs) == 2
    for r in recs:
        assert r["corr"] > 0.999999, r
        assert r["max_err"] < 1e-4 * max(1.0, r["mag"]), r
