"""ctypes wrapper of oracle/cpu_port.c -- bench.py's CPU baseline (kind "port").

TEST INFRASTRUCTURE: used by bench.py's cpu_baseline leg and by tests/, never by the product path.
The matvec is the reference loop bg:464-485 with its baby steps bg:215-220, one rotation at a time
(non-hoisted, as the reference's CPU path issues them), computed with SEAL-class CPU arithmetic
(Harvey NTT, Shoup/Barrett) on OpenMP threads.  Keys, diagonals and the input ciphertext are made by
the oracle (oracle/ckks_oracle.c) with the bench's seeds, so the port's output limbs can be checked
against the oracle digest of the same workload (tests/golden/manifest.json bench_digests).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

from oracle.oracle import Oracle, create_coeff_modulus, galois_elt

HERE = Path(__file__).resolve().parent
_u64p = C.POINTER(C.c_uint64)
_lib = None


def lib():
    global _lib
    if _lib is None:
        p = HERE / "_build" / "libcpu_port.so"
        if not p.is_file():
            import subprocess
            subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)
        L = C.CDLL(str(p))
        L.cpx_create.restype = C.c_void_p
        L.cpx_create.argtypes = [C.c_uint64, _u64p, C.c_int, C.c_int]
        L.cpx_destroy.argtypes = [C.c_void_p]
        L.cpx_rotate.argtypes = [C.c_void_p, _u64p, _u64p, C.c_uint64, C.c_int, _u64p]
        L.cpx_matvec.argtypes = [C.c_void_p, _u64p, C.c_int, C.POINTER(_u64p), C.POINTER(_u64p), C.POINTER(_u64p),
                                 C.c_int, C.c_int, C.c_int, _u64p]
        L.cpx_threads.restype = C.c_int
        L.cpx_set_threads.argtypes = [C.c_int]
        L.cpx_set_ks_mode.argtypes = [C.c_void_p, C.c_int]
        L.cpx_set_ks_mode.restype = C.c_int
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(_u64p)


class CpuPort:
    def __init__(self, N, primes, P, threads=None, mode="exact"):
        self.N, self.P, self.L0 = N, P, len(primes) - P
        if threads:
            lib().cpx_set_threads(int(threads))
        arr = np.ascontiguousarray(np.array(primes, dtype=np.uint64))
        self._h = lib().cpx_create(N, _p(arr), len(primes), P)
        if mode not in ("exact", "seal") or lib().cpx_set_ks_mode(self._h, int(mode == "seal")):
            raise ValueError(f"key-switch mode {mode!r} (seal needs P = 1)")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().cpx_destroy(self._h)
            self._h = None

    @staticmethod
    def threads():
        return int(lib().cpx_threads())

    def rotate(self, ct, key, step):
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = np.empty_like(ct)
        lib().cpx_rotate(self._h, _p(ct), _p(np.ascontiguousarray(key)), galois_elt(step, self.N), ct.shape[1], _p(out))
        return out

    def matvec(self, ct, baby_keys, giant_keys, pts, G, B, D):
        """baby_keys[b] (b = 1..G-1), giant_keys[g] (g = 1..B-1): oracle-layout keys; pts: D arrays
        [l][N].  Returns rescale(sum_g rot_{gG}(sum_b rot_b(ct) (.) pts[gG+b]))."""
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        l = ct.shape[1]
        out = np.empty((2, l - 1, self.N), dtype=np.uint64)
        bk = (_u64p * G)(*([None] + [_p(baby_keys[b]) for b in range(1, G)]))
        gk = (_u64p * B)(*([None] + [_p(giant_keys[g]) for g in range(1, B)]))
        pp = (_u64p * D)(*[_p(p) for p in pts])
        lib().cpx_matvec(self._h, _p(ct), l, bk, gk, pp, G, B, D, _p(out))
        return out


def cgroup_cpu_quota():
    """CPUs allowed by the cgroup's CPU bandwidth limit (cgroup v2 cpu.max, v1 cfs_quota), None if
    unlimited or unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def usable_cores():
    """What this process may run on: the affinity mask, the cgroup quota, and the pool's share
    (OMP_NUM_THREADS; the GPU box sets 16 -- its CPU share of the 8-GPU node)."""
    env = os.environ.get("OMP_NUM_THREADS")
    return {"affinity": len(os.sched_getaffinity(0)), "cgroup_quota": cgroup_cpu_quota(),
            "omp_num_threads": int(env) if env and env.isdigit() and int(env) > 0 else None,
            "os_cpu_count": os.cpu_count()}


def box_threads():
    """The host cores this process may use: OMP_NUM_THREADS when set (16 on the GPU box, its CPU
    share of the node), else the affinity mask bounded by the cgroup quota."""
    u = usable_cores()
    if u["omp_num_threads"]:
        return u["omp_num_threads"]
    n = u["affinity"]
    return max(1, min(n, int(u["cgroup_quota"]))) if u["cgroup_quota"] else n


def baseline(N, L0, P, D, reps=3, threads=None, sk_seed=1000, input_seed=10000, diag_seed=2, mode="exact"):
    """Time `reps` full matvecs (after one untimed one) of the bench's workload on `threads` cores;
    returns (seconds per matvec for each rep, output limbs of the last rep, setup seconds, threads).
    mode="seal" (P = 1): SEAL's switch_key_inplace convention, as bench.py's seal_mode leg."""
    threads = threads or box_threads()
    t_setup = time.perf_counter()
    primes = [int(q) for q in create_coeff_modulus(N, [59] * (L0 + P))]
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    o = Oracle(N, primes, P)
    if mode == "seal":
        o.set_key_switch_mode("seal")
    s = o.gen_secret(sk_seed)
    with ThreadPoolExecutor(threads) as ex:   # the oracle's C calls release the GIL
        bk = dict(zip(range(1, G), ex.map(lambda b: o.gen_galois_key(sk_seed, s, galois_elt(b, N)), range(1, G))))
        gk = dict(zip(range(1, B), ex.map(lambda g: o.gen_galois_key(sk_seed, s, galois_elt(g * G, N)), range(1, B))))
        pts = list(ex.map(lambda k: o.random_plaintext(diag_seed, k, L0), range(D)))
    ct = o.encrypt_symmetric(sk_seed, 0, s, o.random_plaintext(input_seed, 0, L0))
    port = CpuPort(N, primes, P, threads, mode)
    t_setup = time.perf_counter() - t_setup
    port.matvec(ct, bk, gk, pts, G, B, D)      # untimed: first-touch of the scratch buffers
    secs = []
    y = None
    for _ in range(reps):
        t0 = time.perf_counter()
        y = port.matvec(ct, bk, gk, pts, G, B, D)
        secs.append(time.perf_counter() - t0)
    return secs, y, t_setup, threads


def sha256(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
