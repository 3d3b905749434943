"""Worker for tests/test_full_size.py::test_full_matvec_bit_exact_vs_oracle (spawned, CPU only):
one baby rotation, or one giant group's oracle inner product + rotation, of the full-size matvec."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from oracle.oracle import Oracle, galois_elt  # noqa: E402

_O = {}


def _oracle(N, primes, P, seed):
    key = (N, tuple(primes), P)
    if key not in _O:
        o = Oracle(N, primes, P)
        _O.clear()
        _O[key] = (o, o.gen_secret(seed))
    return _O[key]


def run(task):
    """('baby', b): oracle rotation of the input by b == the GPU's hoisted baby step b (bool).
    ('giant', g): rot_{gG}(sum_b baby_b (.) pt_{gG+b}) with the oracle (bg:464-483), limbs."""
    kind, idx, N, primes, P, seed, pt_seed, G, D, baby_path = task
    o, s = _oracle(N, primes, P, seed)
    baby = np.load(baby_path, mmap_mode="r")
    if kind == "baby":
        key = o.gen_galois_key(seed, s, galois_elt(idx, N))
        return idx, bool(np.array_equal(o.rotate(np.array(baby[0]), key, idx), baby[idx]))
    l = baby.shape[2]
    g = idx
    inner = None
    for b in range(G):
        k = g * G + b
        if k >= D:
            break
        term = o.multiply_plain(np.array(baby[b]), o.random_plaintext(pt_seed, k, l))
        inner = term if inner is None else o.add(inner, term)
    if g > 0:
        inner = o.rotate(inner, o.gen_galois_key(seed, s, galois_elt(g * G, N)), g * G)
    return g, inner
