"""Error contract the reference relies on: device OOM surfaces as RuntimeError whose
text contains "out of memory" (bg:1164-1166 falls back to on-the-fly encoding on it), a failed
batch leaves no HBM behind, and a process holding more than 100 GB of cached device
blocks exits cleanly (round-1 exit-handler crash)."""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def ph(require_gpu):
    import pyPhantom
    return pyPhantom


def _ctx(ph, N=16384, L0=36, P=3):
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(P)
    parms.set_galois_elts([ph.get_elt_from_step(1, N)])
    parms.set_coeff_modulus(ph.create_coeff_modulus(N, [59] * (L0 + P)))
    return ph.context(parms)


@pytest.mark.gpu
def test_oom_in_batch_is_runtime_error_and_frees_partial_batch(ph):
    """random_plaintexts of more plaintexts than HBM holds (4.72 MB each at N = 16384, L0 = 36:
    70000 = 330 GB > 288 GB): RuntimeError("... out of memory ..."), every plaintext the batch had
    already created is released, and the context keeps working."""
    ctx = _ctx(ph)
    before = ctx.memory_in_use()
    with pytest.raises(RuntimeError, match="out of memory"):
        ph.random_plaintexts(ctx, 3, 70000, 1, 2.0 ** 59)
    ctx.synchronize()
    assert ctx.memory_in_use() == before
    pts = ph.random_plaintexts(ctx, 4, 8, 1, 2.0 ** 59)     # the context still allocates
    assert len(pts) == 8 and pts[0].coeff_modulus_size() == 36


@pytest.mark.gpu
def test_oom_in_batch_encode_with_hbm_held_elsewhere(ph):
    """The reference's pre-encoding loop (bg:1124-1170) hits OOM inside encode_double_vector_batch
    when another allocation holds the HBM: same exception text, nothing left allocated."""
    import torch
    ctx = _ctx(ph)
    enc = ph.ckks_encoder(ctx)
    before = ctx.memory_in_use()
    free, _ = torch.cuda.mem_get_info(0)
    hold = torch.empty(int(free) - (3 << 30), dtype=torch.uint8, device="cuda:0")   # leave ~3 GB
    try:
        rows = np.random.default_rng(0).normal(0, 0.02, (1024, 8192))     # 1024 x 4.72 MB = 4.8 GB
        with pytest.raises(RuntimeError, match="out of memory"):
            enc.encode_double_vector_batch(ctx, rows, 2.0 ** 59, chain_index=1)
        ctx.synchronize()
        assert ctx.memory_in_use() == before
    finally:
        del hold
        torch.cuda.empty_cache()


@pytest.mark.gpu
def test_exit_with_100gb_cache_returns_zero(require_gpu):
    """The round-1 crash: a 13-block d = 2048 FFN chain (bootstrapped) with the device-block cache uncapped
    (FHESPEAR_CACHE_BYTES = 200 GB) segfaulted in the HIP runtime's exit handler.  Each context now
    owns its memory pool, destroyed with the context and trimmed by an atexit hook that runs before
    the runtime's; the process must exit with status 0."""
    env = dict(os.environ, FHESPEAR_DEVICE="0", FHESPEAR_CACHE_BYTES=str(200 * 10 ** 9))
    cmd = [sys.executable, "-X", "faulthandler", str(REPO / "tools" / "ffn_block.py"), "--N", "16384", "--L0", "36",
           "--P", "3", "--D", "2048", "--F", "4096", "--blocks", "13", "--bootstrap"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, f"rc {out.returncode}\n" + out.stdout[-2000:] + out.stderr[-3000:]


@pytest.mark.gpu
def test_failed_flush_drops_the_queue_and_marks_its_outputs_lost(ph):
    """The round-5 world-8 rehearsal's rank-0 abort (gpurun_out/r05l): a flush of queued rotations failed out of
    memory in its workspace, the queue kept its pointers, the caller destroyed the objects (their blocks went back
    to the device when the cache was trimmed) and a later flush launched the key switch on freed memory -- an
    illegal address at exit.  Now a failed flush empties the queue: the error surfaces as RuntimeError("... out of
    memory ..."), the queued outputs are marked lost (every later use raises instead of reading undefined limbs),
    destroying the inputs launches nothing, and the context keeps working (bit-exact rotations afterwards)."""
    from oracle.oracle import Oracle
    N, L0, P = 4096, 6, 3
    parms = ph.params(ph.scheme_type.ckks)
    parms.set_poly_modulus_degree(N)
    parms.set_special_modulus_size(P)
    parms.set_galois_elts(sorted(set(ph.get_elts_from_steps([1, 2], N))))
    primes = ph.create_coeff_modulus(N, [59] * (L0 + P))
    parms.set_coeff_modulus(primes)
    ctx = ph.context(parms)
    sk = ph.secret_key(ctx, seed=5)
    gk = sk.create_galois_keys(ctx)
    o = Oracle(N, [int(q) for q in primes], P)
    s = o.gen_secret(5)
    rng = np.random.default_rng(2)
    a = np.stack([np.stack([rng.integers(0, int(primes[i]), N, dtype=np.uint64) for i in range(L0)]) for _ in range(2)])
    ct = ph.ciphertext_from_numpy(ctx, a, 1, 2.0 ** 40)
    r1, r2 = ph.rotate(ctx, ct, 1, gk), ph.rotate(ctx, ct, 2, gk)     # queued, not yet launched
    ph.debug_fail_next_flushes(ctx, 1)
    with pytest.raises(RuntimeError, match="out of memory"):
        ph.add(ctx, ct, ct)                                              # its entry flushes the queue: fails
    del ct                                                               # nothing queued references it now
    ctx.synchronize()
    for r in (r1, r2):
        with pytest.raises(ValueError, match="lost"):
            r.to_numpy()
        with pytest.raises(ValueError, match="lost"):
            ph.add(ctx, r, r)
    del r1, r2
    ct = ph.ciphertext_from_numpy(ctx, a, 1, 2.0 ** 40)
    e = ph.get_elt_from_step(1, N)
    assert np.array_equal(ph.rotate(ctx, ct, 1, gk).to_numpy(), o.rotate_elt(a, o.gen_galois_key(5, s, e), e))
    ctx.synchronize()
