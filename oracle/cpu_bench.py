"""CPU-baseline worker for bench.py's `cpu_baseline` leg (TEST INFRASTRUCTURE: runs the oracle,
never the product).  Spawned one per core by bench.cpu_baseline; never touches the GPU."""
import time

import numpy as np

from oracle.oracle import Oracle, galois_elt


def worker(N, primes, P, G, nr, nd, seed, barrier, out, reps=1):
    """Set up a context, a Galois key and random operands, wait for all workers, then `reps` times
    time `nr` rotations (oracle/ckks_oracle.c ock_rotate) and `nd` multiply_plain+add pairs."""
    L0 = len(primes) - P
    o = Oracle(N, primes, P)
    s = o.gen_secret(5 + seed)
    key = o.gen_galois_key(5 + seed, s, galois_elt(G, N))
    rng = np.random.default_rng(9 + seed)
    ct = np.stack([np.stack([rng.integers(0, primes[i], N, dtype=np.uint64) for i in range(L0)]) for _ in range(2)])
    pt = np.stack([rng.integers(0, primes[i], N, dtype=np.uint64) for i in range(L0)])
    barrier.wait()
    tr, td = [], []
    for rep in range(reps + 1):   # rep 0 is the warmup
        t0 = time.perf_counter()
        for _ in range(nr):
            o.rotate(ct, key, G)
        t1 = time.perf_counter()
        acc = o.multiply_plain(ct, pt)
        for _ in range(nd - 1):
            acc = o.add(acc, o.multiply_plain(ct, pt))
        t2 = time.perf_counter()
        if rep:
            tr.append(t1 - t0)
            td.append(t2 - t1)
    out.put((tr, td))
