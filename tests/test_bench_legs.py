"""bench.py's legs on the GPU at test size: the measured RWKV-block leg with its CPU limb check
(VERDICT r2 next #1), so the code path the driver's bench line takes is covered by the suite."""
import argparse
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


@pytest.mark.gpu
def test_block_leg_with_cpu_limb_check(require_gpu):
    """bench.run_block on a small block (N=4096, L0=6, D=64, F=256): timing fields, the decrypted output
    against the plaintext block, and the r projection's server call recorded in the block and
    recomputed by the CPU port (cpu_check_block_projection) -- limb for limb."""
    import bench
    import pyPhantom as ph
    args = argparse.Namespace(split=False, block_dealt=False, config="cfg2")
    res = bench.run_block(args, ph, None, 0, 1, 0, 1, 1, capture=True, config="block_small")
    cap = res.pop("_capture")
    assert res["sec_per_block"] > 0 and set(res["stages_ms"]) == {"server_rkv", "server_wo", "server_ffn_key",
                                                                   "server_ffn_val", "client_encrypt",
                                                                   "client_decrypt", "client_numpy"}
    assert res["client_ms"] > 0 and res["server_ms"] > 0
    assert cap["ct_in"].shape == (2, 6, 4096) and cap["ct_out"].shape == (2, 5, 4096) and len(cap["pts"]) == 64
    par = bench.cpu_check_block_projection(cap)
    assert par["r_projection_limbs_match_cpu_port"], par
