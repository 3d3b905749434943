"""ctypes wrapper over the C parity oracle (oracle/ckks_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product (fhe-spear_amd/).  See ckks_oracle.h for what each
function restates and which reference file:line it follows.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "libckks_oracle.so"

_u64p = C.POINTER(C.c_uint64)
_dblp = C.POINTER(C.c_double)


def build(quiet: bool = True) -> Path:
    """Compile the oracle with gcc (Makefile next to this file)."""
    out = subprocess.run(["make", "-C", str(HERE)], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        L.ock_ctx_create.restype = C.c_void_p
        L.ock_ctx_create.argtypes = [C.c_uint64, _u64p, C.c_int, C.c_int]
        L.ock_ctx_set_ks_mode.argtypes = [C.c_void_p, C.c_int]
        L.ock_random_plaintext.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, _u64p]
        L.ock_ctx_set_ks_mode.restype = C.c_int
        L.ock_ctx_destroy.argtypes = [C.c_void_p]
        L.ock_create_coeff_modulus.argtypes = [C.c_uint64, C.POINTER(C.c_int), C.c_int, _u64p]
        L.ock_galois_elt_from_step.restype = C.c_uint64
        L.ock_galois_elt_from_step.argtypes = [C.c_int, C.c_uint64]
        for name in ("ock_splitmix64",):
            getattr(L, name).restype = C.c_uint64
            getattr(L, name).argtypes = [C.c_uint64]
        L.ock_chacha20_block.argtypes = [C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.ock_pk_rng_key.argtypes = [C.c_char_p, C.c_char_p]
        L.ock_pk_rng_key_gen.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p]
        L.ock_rnd.restype = C.c_uint64
        L.ock_rnd.argtypes = [C.c_uint64, C.c_uint64]
        vp = C.c_void_p
        L.ock_ntt_fwd.argtypes = [vp, _u64p, C.c_int]
        L.ock_ntt_inv.argtypes = [vp, _u64p, C.c_int]
        L.ock_apply_galois_ntt.argtypes = [vp, _u64p, _u64p, C.c_uint64]
        for name in ("ock_add", "ock_sub", "ock_multiply_plain", "ock_add_plain"):
            getattr(L, name).argtypes = [vp, _u64p, _u64p, _u64p, C.c_int, C.c_int]
        L.ock_negate.argtypes = [vp, _u64p, _u64p, C.c_int, C.c_int]
        L.ock_multiply.argtypes = [vp, _u64p, _u64p, _u64p, C.c_int]
        L.ock_rescale_to_next.argtypes = [vp, _u64p, _u64p, C.c_int, C.c_int]
        L.ock_keyswitch.argtypes = [vp, _u64p, _u64p, C.c_int, _u64p, _u64p]
        L.ock_rotate.argtypes = [vp, _u64p, _u64p, C.c_uint64, C.c_int, _u64p]
        L.ock_relinearize.argtypes = [vp, _u64p, _u64p, C.c_int, _u64p]
        L.ock_rotate_hoisted.argtypes = [vp, _u64p, C.POINTER(_u64p), _u64p, C.c_int, C.c_int, C.POINTER(_u64p)]
        L.ock_mod_raise.argtypes = [vp, _u64p, C.c_int, C.c_int, _u64p]
        L.ock_scalar.argtypes = [vp, C.c_int, _u64p, _u64p, _u64p, C.c_int, C.c_int]
        L.ock_centered_count_test.argtypes = [_u64p, _u64p, C.c_int]
        L.ock_centered_count_test.restype = C.c_int
        L.ock_seeded_uniform.argtypes = [C.c_uint64, C.c_int, C.c_uint64, C.c_uint64]
        L.ock_seeded_uniform.restype = C.c_uint64
        L.ock_bsgs_loop.argtypes = [vp, C.POINTER(_u64p), C.POINTER(_u64p), C.POINTER(_u64p),
                                    C.c_int, C.c_int, C.c_int, C.c_int, _u64p]
        L.ock_gen_secret.argtypes = [vp, C.c_char_p, _u64p]
        L.ock_gen_switch_key.argtypes = [vp, C.c_char_p, C.c_uint64, _u64p, _u64p, _u64p]
        L.ock_gen_galois_key.argtypes = [vp, C.c_char_p, _u64p, C.c_uint64, _u64p]
        L.ock_gen_relin_key.argtypes = [vp, C.c_char_p, _u64p, _u64p]
        L.ock_gen_public_key.argtypes = [vp, C.c_char_p, _u64p, _u64p]
        L.ock_encrypt_symmetric.argtypes = [vp, C.c_char_p, C.c_uint64, _u64p, _u64p, C.c_int, _u64p]
        L.ock_encrypt_asymmetric.argtypes = [vp, C.c_char_p, C.c_uint64, _u64p, _u64p, C.c_int, _u64p]
        L.ock_decrypt.argtypes = [vp, _u64p, _u64p, C.c_int, C.c_int, _u64p]
        L.ock_encode_complex.argtypes = [vp, _dblp, C.c_size_t, C.c_double, C.c_int, _u64p]
        L.ock_decode_complex.argtypes = [vp, _u64p, C.c_int, C.c_double, _dblp]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(_u64p)


def create_coeff_modulus(N: int, bits) -> list[int]:
    bits = list(bits)
    arr = (C.c_int * len(bits))(*bits)
    out = np.zeros(len(bits), dtype=np.uint64)
    rc = lib().ock_create_coeff_modulus(N, arr, len(bits), _p(out))
    if rc != 0:
        raise ValueError(f"create_coeff_modulus failed rc={rc}")
    return [int(x) for x in out]


def centered_count(y, qs) -> int:
    y = np.ascontiguousarray(np.asarray(y, dtype=np.uint64))
    q = np.ascontiguousarray(np.asarray(qs, dtype=np.uint64))
    return int(lib().ock_centered_count_test(_p(y), _p(q), len(y)))


def key_bytes(seed: int) -> bytes:
    """Secret-key PRF key: the integer seed as 32 little-endian bytes (pyPhantom.secret_key)."""
    return int(seed).to_bytes(32, "little")


def chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    """ock_chacha20_block (RFC 8439 §2.3) on byte strings: 64 output bytes."""
    k = (C.c_uint32 * 8)(*np.frombuffer(key, dtype="<u4").tolist())
    n = (C.c_uint32 * 3)(*np.frombuffer(nonce, dtype="<u4").tolist())
    out = (C.c_uint32 * 16)()
    lib().ock_chacha20_block(k, counter, n, out)
    return np.array(out[:], dtype="<u4").tobytes()


def _sm64_for_tests(x: int) -> int:
    return int(lib().ock_splitmix64(x))


def pk_rng_key(key32: bytes, gen: int = 0) -> bytes:
    """Mask key of the gen-th public key generated from the secret key `key32` (fhs_gen_public_key)."""
    out = C.create_string_buffer(32)
    lib().ock_pk_rng_key_gen(key32, gen, out)
    return out.raw


def seeded_uniform(key: int, prime_idx: int, n: int, q: int) -> int:
    """ock_seeded_uniform: the switching-key `a` sampler (rejection from SplitMix64 top bits)."""
    return int(lib().ock_seeded_uniform(key, prime_idx, n, q))


def galois_elt(step: int, N: int) -> int:
    return int(lib().ock_galois_elt_from_step(step, N))


class Oracle:
    """Parameter set + tables.  primes: key-level list (L0 data primes, then P special)."""

    def __init__(self, N: int, primes, special: int):
        self.N = N
        self.primes = [int(q) for q in primes]
        self.P = special
        self.L0 = len(self.primes) - special
        self.K = len(self.primes)
        arr = np.array(self.primes, dtype=np.uint64)
        self._h = lib().ock_ctx_create(N, _p(arr), len(self.primes), special)
        if not self._h:
            raise ValueError("bad oracle parameters")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.ock_ctx_destroy(h)
            self._h = None

    @property
    def dnum(self):
        return (self.L0 + self.P - 1) // self.P

    # --- transforms
    def ntt(self, limb: np.ndarray, prime_idx: int) -> np.ndarray:
        a = np.ascontiguousarray(limb, dtype=np.uint64).copy()
        lib().ock_ntt_fwd(self._h, _p(a), prime_idx)
        return a

    def intt(self, limb: np.ndarray, prime_idx: int) -> np.ndarray:
        a = np.ascontiguousarray(limb, dtype=np.uint64).copy()
        lib().ock_ntt_inv(self._h, _p(a), prime_idx)
        return a

    def random_plaintext(self, seed: int, k: int, l: int):
        """pyPhantom.random_plaintexts(ctx, seed, ...)[k] at l limbs (test data)."""
        out = np.empty((l, self.N), dtype=np.uint64)
        lib().ock_random_plaintext(self._h, seed, k, l, _p(out))
        return out

    def set_key_switch_mode(self, mode: str):
        """'exact' (default: exact centred ModUp, ModDown without rounding) or 'seal' (P = 1:
        SEAL's switch_key_inplace, ock_ctx_set_ks_mode)."""
        if lib().ock_ctx_set_ks_mode(self._h, {"exact": 0, "seal": 1}[mode]) != 0:
            raise ValueError("seal key switching needs special_modulus_size 1")

    def galois_ntt(self, limb: np.ndarray, elt: int) -> np.ndarray:
        a = np.ascontiguousarray(limb, dtype=np.uint64)
        out = np.empty_like(a)
        lib().ock_apply_galois_ntt(self._h, _p(a), _p(out), elt)
        return out

    # --- ciphertext ops; ct arrays are (ncomp, l, N) uint64
    def _bin(self, fn, a, b, ncomp, l, out_shape=None):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        b = np.ascontiguousarray(b, dtype=np.uint64)
        out = np.empty(out_shape or a.shape, dtype=np.uint64)
        fn(self._h, _p(a), _p(b), _p(out), ncomp, l)
        return out

    def add(self, a, b):
        return self._bin(lib().ock_add, a, b, a.shape[0], a.shape[1])

    def sub(self, a, b):
        return self._bin(lib().ock_sub, a, b, a.shape[0], a.shape[1])

    def negate(self, a):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        out = np.empty_like(a)
        lib().ock_negate(self._h, _p(a), _p(out), a.shape[0], a.shape[1])
        return out

    def multiply_plain(self, ct, pt):
        return self._bin(lib().ock_multiply_plain, ct, pt, ct.shape[0], ct.shape[1])

    def add_plain(self, ct, pt):
        return self._bin(lib().ock_add_plain, ct, pt, ct.shape[0], ct.shape[1])

    def multiply(self, a, b):
        l = a.shape[1]
        a = np.ascontiguousarray(a, dtype=np.uint64)
        b = np.ascontiguousarray(b, dtype=np.uint64)
        out = np.empty((3, l, self.N), dtype=np.uint64)
        lib().ock_multiply(self._h, _p(a), _p(b), _p(out), l)
        return out

    def rescale(self, ct):
        ncomp, l, N = ct.shape
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = np.empty((ncomp, l - 1, N), dtype=np.uint64)
        lib().ock_rescale_to_next(self._h, _p(ct), _p(out), ncomp, l)
        return out

    def mod_raise(self, ct):
        """ckks_bootstrapper ModRaise: limb q0 lifted centred to all L0 limbs (ock_mod_raise)."""
        ncomp, l, N = ct.shape
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = np.empty((ncomp, self.L0, N), dtype=np.uint64)
        lib().ock_mod_raise(self._h, _p(ct), l, ncomp, _p(out))
        return out

    def scalar(self, ct, k: int, add: bool):
        """ct * k (add=False) or ct + k into component 0 (add=True) for the integer k."""
        ncomp, l, N = ct.shape
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        res = np.array([int(k) % int(self.primes[i]) for i in range(l)], dtype=np.uint64)
        out = np.empty_like(ct)
        lib().ock_scalar(self._h, 1 if add else 0, _p(ct), _p(res), _p(out), ncomp, l)
        return out

    def keyswitch(self, a, key):
        l = a.shape[0]
        a = np.ascontiguousarray(a, dtype=np.uint64)
        key = np.ascontiguousarray(key, dtype=np.uint64)
        o0 = np.empty((l, self.N), dtype=np.uint64)
        o1 = np.empty_like(o0)
        lib().ock_keyswitch(self._h, _p(a), _p(key), l, _p(o0), _p(o1))
        return o0, o1

    def rotate(self, ct, gkey, step: int):
        l = ct.shape[1]
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = np.empty_like(ct)
        lib().ock_rotate(self._h, _p(ct), _p(np.ascontiguousarray(gkey)), galois_elt(step, self.N), l, _p(out))
        return out

    def rotate_elt(self, ct, gkey, elt: int):
        l = ct.shape[1]
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = np.empty_like(ct)
        lib().ock_rotate(self._h, _p(ct), _p(np.ascontiguousarray(gkey)), elt, l, _p(out))
        return out

    def rotate_hoisted(self, ct, keys, elts):
        l = ct.shape[1]
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        keys = [np.ascontiguousarray(k, dtype=np.uint64) for k in keys]
        e = np.ascontiguousarray(np.asarray(elts, dtype=np.uint64))
        outs = [np.empty_like(ct) for _ in keys]
        KA = (_u64p * len(keys))(*[_p(k) for k in keys])
        OA = (_u64p * len(outs))(*[_p(o) for o in outs])
        lib().ock_rotate_hoisted(self._h, _p(ct), KA, _p(e), len(keys), l, OA)
        return outs

    def relinearize(self, ct3, rlk):
        l = ct3.shape[1]
        ct3 = np.ascontiguousarray(ct3, dtype=np.uint64)
        out = np.empty((2, l, self.N), dtype=np.uint64)
        lib().ock_relinearize(self._h, _p(ct3), _p(np.ascontiguousarray(rlk)), l, _p(out))
        return out

    def bsgs_loop(self, baby, pts, gkeys_by_giant, G, B, D):
        """bg:464-485 restated.  gkeys_by_giant[g] is the key for step g*G (entry 0 unused)."""
        l = baby[0].shape[1]
        baby = [np.ascontiguousarray(b, dtype=np.uint64) for b in baby]
        pts = [np.ascontiguousarray(p, dtype=np.uint64) for p in pts]
        keys = [np.ascontiguousarray(k, dtype=np.uint64) if k is not None else baby[0] for k in gkeys_by_giant]
        BA = (_u64p * len(baby))(*[_p(b) for b in baby])
        PA = (_u64p * len(pts))(*[_p(p) for p in pts])
        KA = (_u64p * len(keys))(*[_p(k) for k in keys])
        out = np.empty((2, l - 1, self.N), dtype=np.uint64)
        lib().ock_bsgs_loop(self._h, BA, PA, KA, G, B, D, l, _p(out))
        return out

    # --- keys / encryption.  `seed` is the secret key's PRF key as an integer (< 2^256), the same
    # 32 little-endian bytes pyPhantom.secret_key(ctx, seed) hands to fhs_secret_key_create.
    def gen_secret(self, seed: int):
        s = np.empty((self.K, self.N), dtype=np.uint64)
        lib().ock_gen_secret(self._h, key_bytes(seed), _p(s))
        return s

    def key_shape(self):
        return (self.dnum, 2, self.K, self.N)

    def switch_key_seeds(self, seed: int, stream_base: int):
        """The public a_j seeds a switching key stores (one per digit): w0 of block 0 of stream
        stream_base | 2j (fhs_host.hip gen_switch_key)."""
        out = []
        for j in range(self.dnum):
            sid = stream_base | (2 * j)
            blk = chacha20_block(key_bytes(seed), 0, (sid & 0xFFFFFFFF).to_bytes(4, "little") +
                                 (sid >> 32).to_bytes(4, "little") + (0x31534846).to_bytes(4, "little"))
            out.append(int.from_bytes(blk[:8], "little"))
        return out

    def gen_galois_key(self, seed: int, s, elt: int):
        k = np.empty(self.key_shape(), dtype=np.uint64)
        lib().ock_gen_galois_key(self._h, key_bytes(seed), _p(s), elt, _p(k))
        return k

    def gen_relin_key(self, seed: int, s):
        k = np.empty(self.key_shape(), dtype=np.uint64)
        lib().ock_gen_relin_key(self._h, key_bytes(seed), _p(s), _p(k))
        return k

    def gen_public_key(self, seed: int, s):
        pk = np.empty((2, self.L0, self.N), dtype=np.uint64)
        lib().ock_gen_public_key(self._h, key_bytes(seed), _p(s), _p(pk))
        return pk

    def encrypt_symmetric(self, seed: int, counter: int, s, pt):
        l = pt.shape[0]
        ct = np.empty((2, l, self.N), dtype=np.uint64)
        lib().ock_encrypt_symmetric(self._h, key_bytes(seed), counter, _p(s), _p(np.ascontiguousarray(pt)), l, _p(ct))
        return ct

    def encrypt_asymmetric(self, seed: int, counter: int, pk, pt, pk_gen: int = 0):
        """`seed`: the SECRET key's seed; the masks come from the public key's own PRF key
        (pk_rng_key of the pk_gen-th public key made from that secret key), as in fhs_gen_public_key."""
        l = pt.shape[0]
        ct = np.empty((2, l, self.N), dtype=np.uint64)
        lib().ock_encrypt_asymmetric(self._h, pk_rng_key(key_bytes(seed), pk_gen), counter, _p(np.ascontiguousarray(pk)),
                                     _p(np.ascontiguousarray(pt)), l, _p(ct))
        return ct

    def decrypt(self, s, ct):
        ncomp, l, N = ct.shape
        pt = np.empty((l, N), dtype=np.uint64)
        lib().ock_decrypt(self._h, _p(s), _p(np.ascontiguousarray(ct)), ncomp, l, _p(pt))
        return pt

    def encode(self, values, scale: float, l: int):
        z = np.asarray(values)
        zc = np.zeros((len(z), 2), dtype=np.float64)
        zc[:, 0] = np.real(z)
        zc[:, 1] = np.imag(z) if np.iscomplexobj(z) else 0.0
        zc = np.ascontiguousarray(zc)
        pt = np.empty((l, self.N), dtype=np.uint64)
        lib().ock_encode_complex(self._h, zc.ctypes.data_as(_dblp), len(z), scale, l, _p(pt))
        return pt

    def decode(self, pt, scale: float):
        l = pt.shape[0]
        z = np.empty((self.N // 2, 2), dtype=np.float64)
        lib().ock_decode_complex(self._h, _p(np.ascontiguousarray(pt)), l, scale, z.ctypes.data_as(_dblp))
        return z[:, 0] + 1j * z[:, 1]
