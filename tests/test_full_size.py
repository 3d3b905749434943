"""BASELINE configs[2] and configs[4] at their full sizes on one MI355X:

- cfg3: one client-aided RWKV-7 block (bg:756-899; tools/rwkv_block.py), d = 2048, d_ffn = 8192,
  N = 16384, L0 = 36, P = 3, the diagonals of all 8 projections pre-encoded and resident (77 GB),
  against the plaintext block (bg:902-980);
- cfg5: test_fully_enc_bsgs.py's 24-block chain (tf:233-298; tools/ffn_block.py), d = 2048,
  F = 4096, N = 32768, L0 = 36, P = 3, bootstrapping whenever fewer than 4 levels remain, against the
  plaintext chain with the reference's pass criterion corr > 0.999 (tf:298).

Both are property checks (size-independent): the limb-level parity of the same code paths is in
test_golden_replay.py and test_gpu_parity.py."""
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))


@pytest.mark.gpu
def test_cfg3_rwkv_block_full_size(require_gpu):
    import pyPhantom as ph
    import rwkv_block as rb
    D, F = 2048, 8192
    H = D // 64
    rng = np.random.default_rng(5)
    block = rb.BlockWeights(rng, 1, D, F, H)
    srv = rb.Server(ph, 16384, 36, 3, D)
    run = rb.BlockRunner(srv, block, True)
    assert srv.ctx.memory_in_use() > 8 * D * 36 * 16384 * 8     # all 8 projections resident
    x = rng.standard_normal(D)
    st = (x, np.zeros(D), np.zeros(D), np.zeros((H, 64, 64)), rng.standard_normal(D))
    out = rb.client_aided_block(run, *st)
    ref = rb.plaintext_block(block, *st)
    for got, want in zip(out[:5], ref):
        assert np.max(np.abs(got - want)) < 1e-6 * max(1.0, float(np.max(np.abs(want))))
    assert float(np.corrcoef(out[0], ref[0])[0, 1]) > 0.999999


@pytest.mark.gpu
def test_cfg5_ffn_chain_24_blocks_n32768(require_gpu):
    import pyPhantom as ph
    import ffn_block as fb
    D, F, blocks = 2048, 4096, 24
    ck = fb.Ckks(ph, 32768, 36, 3, D, bootstrap=True)
    x_cal, Wk, Wv = fb.calibrated_weights(np.random.default_rng(42), D, F, blocks)
    recs = fb.run_chain(ck, x_cal, Wk, Wv, D, F, True, log=lambda *a: None)
    assert len(recs) == blocks, "chain stopped early (out of levels)"
    assert sum(r["bootstrap_seconds"] is not None for r in recs) >= 3
    assert recs[-1]["corr"] > 0.999                                   # tf:298
    assert all(r["corr"] > 0.999 for r in recs)
