#!/usr/bin/env python3
"""Oracle digest of bench.py's timed workload: the SHA-256 of the output limbs
of the exact matvec the bench times, computed here by the C oracle alone (oracle/ckks_oracle.c, the
restatement of bg:464-485 and the CKKS ops) -- never by the GPU -- and committed to
tests/golden/manifest.json under "bench_digests".  bench.py hashes its last timed output and reports
`parity.<config>_sha256_match`, so every driver bench run is also a full-size limb-parity check.

Workload (bench.py, rank 0): secret key seed 1000; the G-1 baby and B-1 giant Galois keys of that key;
input = fresh symmetric encryption (counter 0) of random_plaintext(10000, 0) at the top level; D
diagonals random_plaintext(2, k) (i.i.d. uniform limbs mod q_i); baby steps
rotate(ct, b); y = rescale(sum_g rot_{gG}(sum_b baby_b (.) pt_{gG+b})).  The oracle rotates one
rotation at a time (non-hoisted, as the reference issues them); the library hoists -- same limbs.

At N > 1 rank r of bench.py runs the same workload with seeds (1000 + r, 10000 + r, 2 + r); --rank r
writes that rank's digest as "<config>_rank<r>" (bench.py limb-checks every gathered output on rank 0).

    python3 tests/golden/make_bench_digest.py cfg2 [--workers 8] [--mode exact|seal] [--rank r]
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))

from oracle.oracle import Oracle, create_coeff_modulus, galois_elt  # noqa: E402

CONFIGS = {"cfg2": (16384, 36, 3, 2048), "cfg1": (8192, 24, 3, 1024), "small": (4096, 6, 3, 256),
           "cfg5mv": (32768, 36, 3, 2048)}
SK_SEED, INPUT_SEED, DIAG_SEED = 1000, 10000, 2

_W = {}


def _setup(N, primes, P, mode, sk_seed):
    key = (N, tuple(primes), P, mode, sk_seed)
    if key not in _W:
        o = Oracle(N, primes, P)
        if mode == "seal":
            o.set_key_switch_mode("seal")
        _W.clear()
        _W[key] = (o, o.gen_secret(sk_seed))
    return _W[key]


def _task(t):
    kind, idx, N, primes, P, mode, G, D, path, rank = t
    sk_seed, diag_seed = SK_SEED + rank, DIAG_SEED + rank
    o, s = _setup(N, primes, P, mode, sk_seed)
    arr = np.load(path, mmap_mode="r")
    if kind == "baby":
        ct = np.array(arr[0])
        return idx, o.rotate(ct, o.gen_galois_key(sk_seed, s, galois_elt(idx, N)), idx)
    l = arr.shape[2]
    inner = None
    for b in range(G):
        k = idx * G + b
        if k >= D:
            break
        term = o.multiply_plain(np.array(arr[b]), o.random_plaintext(diag_seed, k, l))
        inner = term if inner is None else o.add(inner, term)
    if idx > 0:
        inner = o.rotate(inner, o.gen_galois_key(sk_seed, s, galois_elt(idx * G, N)), idx * G)
    return idx, inner


def digest(cfg, workers, mode="exact", rank=0):
    N, L0, P, D = CONFIGS[cfg]
    if mode == "seal":
        P = 1
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    bits = [59] * (L0 + P)
    primes = [int(q) for q in create_coeff_modulus(N, bits)]
    o, s = _setup(N, primes, P, mode, SK_SEED + rank)
    pt = o.random_plaintext(INPUT_SEED + rank, 0, L0)
    ct = o.encrypt_symmetric(SK_SEED + rank, 0, s, pt)
    t0 = time.time()
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as td:
        p0 = os.path.join(td, "ct.npy")
        np.save(p0, ct[None])
        with ctx.Pool(workers) as pool:
            baby = dict(pool.map(_task, [("baby", b, N, primes, P, mode, G, D, p0, rank) for b in range(1, G)], chunksize=1))
            baby[0] = ct
            pb = os.path.join(td, "baby.npy")
            np.save(pb, np.stack([baby[b] for b in range(G)]))
            del baby
            giant = pool.map(_task, [("giant", g, N, primes, P, mode, G, D, pb, rank) for g in range(B)], chunksize=1)
    acc = None
    for _, term in sorted(giant, key=lambda r: r[0]):
        acc = term if acc is None else o.add(acc, term)
    y = np.ascontiguousarray(o.rescale(acc))
    return {"sha256": hashlib.sha256(y.tobytes()).hexdigest(), "shape": list(y.shape), "N": N, "L0": L0, "P": P,
            "D": D, "G": G, "B": B, "key_switch_mode": mode, "sk_seed": SK_SEED + rank,
            "input_seed": INPUT_SEED + rank, "diag_seed": DIAG_SEED + rank, "oracle_seconds": round(time.time() - t0, 1),
            "generator": "tests/golden/make_bench_digest.py (C oracle only)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=sorted(CONFIGS))
    ap.add_argument("--workers", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--mode", default="exact", choices=["exact", "seal"])
    ap.add_argument("--rank", type=int, default=0, help="bench.py rank r's workload (seeds + r)")
    ap.add_argument("--no-write", action="store_true")
    a = ap.parse_args()
    rec = digest(a.config, a.workers, a.mode, a.rank)
    print(json.dumps(rec))
    if not a.no_write:
        mf = REPO / "tests" / "golden" / "manifest.json"
        man = json.loads(mf.read_text())
        key = a.config + ("" if a.mode == "exact" else "_" + a.mode) + (f"_rank{a.rank}" if a.rank else "")
        man.setdefault("bench_digests", {})[key] = rec
        mf.write_text(json.dumps(man, indent=1) + "\n")


if __name__ == "__main__":
    main()
