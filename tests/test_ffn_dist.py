"""The fully-encrypted FFN chain (test_fully_enc_bsgs.py:26-118, BASELINE configs[4]) over ranks
(tools/ffn_block.py FfnRanks, SURVEY.md §8e "Config 5"): the F/D key chunks and value chunks dealt over
rank groups, each chunk's BSGS sharded inside its group (giant groups, a baby x giant grid, or baby
steps), the square / relinearize / rescale on the chunk owners, the value chunks' outputs added on rank
0.  Gloo with every rank sharing cuda:0 (the driver's 8-GPU node is the real transport); the final
ciphertext after two blocks must be limb-identical to the one-rank chain."""
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
ARGS = ["--N", "2048", "--L0", "10", "--P", "2", "--D", "64", "--F", "128", "--blocks", "2"]
_REF = {}


def _digest(out):
    m = re.search(r"ct_sha256 ([0-9a-f]{64})", out.stdout)
    assert m, out.stdout[-2000:] + out.stderr[-3000:]
    errs = [float(e) for e in re.findall(r"max_err=([0-9.e+-]+)", out.stdout)]
    assert errs and max(errs) < 1e-3, out.stdout[-2000:]
    return m.group(1)


# the bootstrapping chain (tf:233-298): N = 1024, L0 = 24, P = 3, level budget (2, 2) (bootstrap depth 16);
# seven blocks use up the fresh levels, so a bootstrap runs before the eighth, its CoeffToSlot / SlotToCoeff
# groups over the ranks
BOOT_ARGS = ["--N", "1024", "--L0", "24", "--P", "3", "--D", "16", "--F", "32", "--blocks", "8", "--bootstrap"]


def _one_rank(args=None):
    args = ARGS if args is None else args
    key = " ".join(args)
    if key not in _REF:
        env = dict(os.environ, FHESPEAR_DEVICE="0", FFN_DIGEST="1")
        out = subprocess.run([sys.executable, str(REPO / "tools" / "ffn_block.py")] + args, env=env,
                             capture_output=True, text=True, timeout=200)
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
        _REF[key] = _digest(out)
    return _REF[key]


def _ranks(world, extra, port, args=None):
    env = dict(os.environ, FHESPEAR_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(REPO / "tools" / "ffn_block.py"),
           "--dist", "--backend", "gloo"] + (ARGS if args is None else args) + list(extra)
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    if args is BOOT_ARGS:
        assert re.search(r"bootstraps [1-9]", out.stdout), out.stdout[-2000:]
    return _digest(out)


@pytest.mark.gpu
@pytest.mark.parametrize("world,extra", [
    (1, []),                                                    # FfnRanks at world 1: no sharding
    (2, []),                                                    # one key / value chunk per rank
    (2, ["--baby-mode", "broadcast"]),
    (3, ["--shard", "giant"]),                                  # groups [0, 1], [2]
    (4, ["--shard", "giant"]),                                  # groups [0, 1], [2, 3], giant-sharded
    (4, ["--shard", "giant", "--baby-mode", "broadcast"]),
    (4, ["--shard", "grid", "--rb", "2"]),                      # each group a 2 x 1 grid
    (4, ["--shard", "baby"]),
])
def test_ffn_chain_over_ranks_is_limb_identical(require_gpu, world, extra):
    import zlib
    port = 29700 + 20 * world + zlib.crc32(" ".join(extra).encode()) % 20
    assert _ranks(world, extra, port) == _one_rank()


@pytest.mark.gpu
@pytest.mark.parametrize("world,extra", [(2, []), (4, ["--shard", "grid", "--rb", "2"])])
def test_ffn_chain_with_bootstrap_over_ranks_is_limb_identical(require_gpu, world, extra):
    """The chain with a bootstrap in it: the FFN chunks over the ranks as above, and the bootstrap's
    CoeffToSlot / SlotToCoeff linear transforms with their giant groups dealt over every rank
    (ckks_bootstrapper.bootstrap_ranks, fhespear_dist.linear_transform_sharded) -- the final ciphertext
    limb-identical to the one-rank chain's."""
    assert _ranks(world, extra, 29800 + 10 * world, BOOT_ARGS) == _one_rank(BOOT_ARGS)
