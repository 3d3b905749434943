"""Locate the segfault seen at process exit after tools/ffn_block.py --D 2048 --bootstrap: runs a short
chain, then releases the objects one group at a time with a marker line before and after each step.

    python -X faulthandler -u tools/debug/exit_crash.py [--bootstrap] [--blocks 2]
"""
import argparse
import atexit
import gc
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tools"))
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))

import ffn_block as fb  # noqa: E402


def mark(s):
    print(f"[exit_crash] {s}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--D", type=int, default=2048)
    ap.add_argument("--F", type=int, default=4096)
    ap.add_argument("--blocks", type=int, default=2)
    ap.add_argument("--bootstrap", action="store_true")
    a = ap.parse_args()
    import pyPhantom as ph
    atexit.register(mark, "atexit handler")
    rng = np.random.default_rng(42)
    ck = fb.Ckks(ph, a.N, 36, 3, a.D, bootstrap=a.bootstrap)
    x_cal, Wk, Wv = fb.calibrated_weights(rng, a.D, a.F, a.blocks)
    recs = fb.run_chain(ck, x_cal, Wk, Wv, a.D, a.F, a.bootstrap)
    mark(f"chain done ({len(recs)} blocks)")
    ck.ctx.synchronize()
    del recs
    gc.collect()
    mark("records freed")
    if ck.bt is not None:
        ck.bt = None
        gc.collect()
        mark("bootstrapper freed")
    ck.gk = None
    ck.rlk = None
    gc.collect()
    mark("keys freed")
    ck.sk = None
    ck.encoder = None
    gc.collect()
    mark("secret key / encoder freed")
    ctx = ck.ctx
    ck.ctx = None
    del ck
    gc.collect()
    mark("ckks holder freed (context still referenced)")
    ctx.synchronize()
    del ctx
    ph._default_ctx = None
    gc.collect()
    mark("context released by Python (FHESPEAR_TRACE_LIFETIME=1 shows whether the library freed it)")


if __name__ == "__main__":
    main()
    mark("main returned")
