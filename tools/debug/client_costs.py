"""Where the client-aided block's client time goes (bench.py rwkv_block.client_ms):
each client call of one cfg3 block stage timed alone (synchronised, median of 7), batched as
client_aided_block issues them, plus the host-side marks of one batched decode (FHESPEAR_HOST_TRACE).

    python tools/debug/client_costs.py
"""
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tools"))
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))
os.environ.setdefault("FHESPEAR_PARITY_RNG", "1")

import rwkv_block as rb  # noqa: E402


def main():
    import pyPhantom as ph
    D, F, N = 2048, 8192, 16384
    srv = rb.Server(ph, N, 36, 3, D)
    rng = np.random.default_rng(1)
    blk = rb.BlockWeights(rng, 1, D, F, D // 64)
    sync = srv.ctx.synchronize
    xs = [rng.standard_normal(D) for _ in range(3)]
    zs = [rng.standard_normal(D) + 1j * rng.standard_normal(D) for _ in range(2)]

    def t(name, fn, reps=7):
        fn()
        sync()
        ts = []
        for _ in range(reps):
            sync()
            t0 = time.perf_counter()
            r = fn()
            sync()
            ts.append(time.perf_counter() - t0)
        print(f"{name:44s} {1e3 * float(np.median(ts)):7.3f} ms", flush=True)
        return r

    cts3 = t("encrypt_replicated_batch(3 real)", lambda: srv.encrypt_replicated_batch(xs))
    t("encrypt_replicated_batch(1 real)", lambda: srv.encrypt_replicated_batch(xs[:1]))
    t("encrypt_replicated_batch(2 complex)", lambda: srv.encrypt_replicated_batch(zs, True))
    t("encode_double_vector_batch(3) alone", lambda: srv.encoder.encode_double_vector_batch(
        srv.ctx, np.stack([np.tile(x, 4) for x in xs]), srv.scale))
    t("encrypt_replicated x3 (one at a time)", lambda: [srv.encrypt_replicated(x) for x in xs])
    # outputs as the server returns them: one level down (after the BSGS rescale)
    outs = [ph.rescale_to_next(srv.ctx, c) for c in cts3]
    t("decrypt_vecs(3)", lambda: srv.decrypt_vecs(outs, D))
    t("decrypt_vecs(1)", lambda: srv.decrypt_vecs(outs[:1], D))
    pts = t("sk.decrypt x3", lambda: [srv.sk.decrypt(srv.ctx, c) for c in outs])
    t("decode_batch(3) alone", lambda: srv.encoder.decode_batch(srv.ctx, pts, D))
    t("decode_complex_vector x3 (one at a time)", lambda: [srv.encoder.decode_complex_vector(srv.ctx, p) for p in pts])
    x = rng.standard_normal(D)
    st = (x, np.zeros(D), np.zeros(D), np.zeros((D // 64, 64, 64)), rng.standard_normal(D))
    x_ln, mixes = t("numpy _mix", lambda: rb._mix(blk, x, st[1]))
    t("numpy _wkv", lambda: rb._wkv(blk, mixes, xs[0], xs[1], xs[2], st[3], st[4]))
    t("numpy layer_norm", lambda: rb.layer_norm(x, blk.ln2_w, blk.ln2_b))
    print("one decrypt_vecs(3) with host marks:", flush=True)
    os.environ["FHESPEAR_HOST_TRACE"] = "1"   # read per call by the library's HostTrace
    srv.decrypt_vecs(outs, D)
    os.environ.pop("FHESPEAR_HOST_TRACE")


if __name__ == "__main__":
    main()
