"""Where a client-aided RWKV block's time goes beyond its 8 matvecs (cfg3): encrypt / decrypt /
decode / baby steps / fused BSGS, each synchronised and timed alone.

    python tools/debug/block_overhead.py
"""
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tools"))
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))

import rwkv_block as rb  # noqa: E402


def main():
    import pyPhantom as ph
    D, F, N = 2048, 8192, 16384
    srv = rb.Server(ph, N, 36, 3, D)
    rng = np.random.default_rng(1)
    blk = rb.BlockWeights(rng, 1, D, F, D // 64)
    pts = srv.encode_real(blk.W_r.T)
    x = rng.standard_normal(D)
    sync = srv.ctx.synchronize

    def t(fn, reps=5):
        fn()
        sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        sync()
        return (time.perf_counter() - t0) / reps * 1e3, r

    te, ct = t(lambda: srv.encrypt_replicated(x))
    tb, baby = t(lambda: srv.baby(ct))
    tm, y = t(lambda: srv.matmul(baby, pts))
    tbm, _ = t(lambda: srv.matmul(srv.baby(ct), pts))
    tdp, ptd = t(lambda: srv.sk.decrypt(srv.ctx, y))
    tdc, _ = t(lambda: srv.encoder.decode_double_vector(srv.ctx, ptd))
    td, _ = t(lambda: srv.decrypt_vec(y, D))
    tec, _ = t(lambda: srv.encrypt_replicated_complex(x, x))
    tdcc, _ = t(lambda: srv.decrypt_vec_complex(y, D))
    print(f"encrypt_replicated {te:.2f} ms, complex {tec:.2f}; baby steps {tb:.2f}; fused BSGS {tm:.2f}; "
          f"baby+BSGS {tbm:.2f}; decrypt {tdp:.2f} + decode {tdc:.2f} = decrypt_vec {td:.2f}; complex {tdcc:.2f}")


if __name__ == "__main__":
    main()
