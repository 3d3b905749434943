"""pyPhantom -- drop-in replacement for FHE-SPEAR's `pyPhantom` module on AMD MI355X.

The reference imports `pyPhantom` (fhe_common.py:9-17, scripts/bootstrap_generation.py:13-14,
test_fully_enc_bsgs.py:13-14, fhe_rwkv_inference.py:7-9); it was the pybind11 module built from
gpu/phantom_binding.cu (pb) over the CUDA library PhantomFHE.  This module keeps that Python
surface (names, argument order, return-new-object semantics, exceptions) and binds it with ctypes
to libfhespear_hip.so, whose C ABI is include/fhespear.h.  All arithmetic runs in hand-written
gfx950 HIP kernels; there is no CPU fallback: importing this module without the library raises
ImportError, and creating a context without an AMD GPU raises RuntimeError.

Fork-only symbols the reference probes with try/except AttributeError are
implemented: bsgs_multiply_accumulate (bg:459), encode_*_vector_batch (bg:382, 423),
offload_plaintexts / upload_plaintexts / bsgs_from_cpu (bg:336-358, 449), ciphertext.chain_index /
scale / coeff_modulus_size, and ckks_bootstrapper (bootstrap.py; the fork's is un-vendored, so its
limbs are unpinned -- DESIGN.md §5).
"""
from __future__ import annotations

import ctypes as C
import enum
import os
import sys
import threading
from pathlib import Path

import numpy as np

__version__ = "fhespear-mi355x-0.1"

_HERE = Path(__file__).resolve().parent
_LIB_CANDIDATES = [
    os.environ.get("FHESPEAR_LIB", ""),
    str(_HERE.parent.parent / "lib" / "libfhespear_hip.so"),
]


def _share_torch_hip_runtime():
    """One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7,
    but libtorch_hip asks for it as `libamdhip64.so`, so the loader never matches it against
    /opt/rocm's copy).  When this library loads first it binds /opt/rocm's runtime, a later
    `import torch` loads a second runtime, and torch.cuda then reports "No HIP GPUs are available"
    -- while the reference callers import torch first (fhe_common.py:5, bg:6) and so share torch's.
    Loading torch's runtime here (if torch is installed; torch itself is not imported) makes both
    orders bind the same one.  FHESPEAR_HIP_RUNTIME=system keeps /opt/rocm's."""
    if os.environ.get("FHESPEAR_HIP_RUNTIME", "torch") != "torch":
        return None
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.submodule_search_locations:
        return None
    rt = Path(list(spec.submodule_search_locations)[0]) / "lib" / "libamdhip64.so"
    if not rt.is_file():
        return None
    C.CDLL(str(rt), mode=C.RTLD_GLOBAL)
    return str(rt)


HIP_RUNTIME = _share_torch_hip_runtime()


def _load():
    for p in _LIB_CANDIDATES:
        if p and Path(p).is_file():
            return C.CDLL(p), p
    raise ImportError(
        "pyPhantom (MI355X backend): libfhespear_hip.so not found; build it with "
        "`make -C fhe-spear_amd` or `python -c 'import __graft_entry__ as g; g.build()'`")


_lib, LIB_PATH = _load()

_vp = C.c_void_p
_u64 = C.c_uint64
_u64p = C.POINTER(C.c_uint64)
_dblp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)

_SIGS = {
    "fhs_last_error": (C.c_char_p, []),
    "fhs_version": (C.c_char_p, []),
    "fhs_device_count": (C.c_int, []),
    "fhs_device_pci_bus_id": (C.c_int, [C.c_int, C.c_char_p, C.c_int]),
    "fhs_create_coeff_modulus": (C.c_int, [_u64, _ip, C.c_int, _u64p]),
    "fhs_galois_elt_from_step": (_u64, [C.c_int, _u64]),
    "fhs_context_create": (C.c_int, [_u64, _u64p, C.c_int, C.c_int, _u64p, C.c_int, C.c_int, C.POINTER(_vp)]),
    "fhs_context_destroy": (C.c_int, [_vp]),
    "fhs_context_info": (C.c_int, [_vp, _u64p, _ip, _ip, _ip]),
    "fhs_context_galois_elts": (C.c_int, [_vp, _u64p]),
    "fhs_synchronize": (C.c_int, [_vp]),
    "fhs_memory_in_use": (C.c_int, [_vp, _u64p]),
    "fhs_secret_key_create": (C.c_int, [_vp, C.c_char_p, C.POINTER(_vp)]),
    "fhs_secret_key_destroy": (C.c_int, [_vp]),
    "fhs_gen_public_key": (C.c_int, [_vp, _vp, C.POINTER(_vp)]),
    "fhs_gen_relin_key": (C.c_int, [_vp, _vp, C.POINTER(_vp)]),
    "fhs_create_galois_keys": (C.c_int, [_vp, _vp, _u64p, C.c_int, C.POINTER(_vp)]),
    "fhs_public_key_destroy": (C.c_int, [_vp]),
    "fhs_relin_key_destroy": (C.c_int, [_vp]),
    "fhs_galois_keys_destroy": (C.c_int, [_vp]),
    "fhs_galois_keys_has": (C.c_int, [_vp, _u64, _ip]),
    "fhs_galois_key_export": (C.c_int, [_vp, _vp, _u64, _u64p]),
    "fhs_relin_key_export": (C.c_int, [_vp, _vp, _u64p]),
    "fhs_secret_key_export": (C.c_int, [_vp, _vp, _u64p]),
    "fhs_galois_keys_import": (C.c_int, [_vp, _u64p, C.c_int, _u64p, C.POINTER(_vp)]),
    "fhs_relin_key_import": (C.c_int, [_vp, _u64p, C.POINTER(_vp)]),
    "fhs_secret_key_import": (C.c_int, [_vp, _u64p, C.POINTER(_vp)]),
    "fhs_context_set_key_switch_mode": (C.c_int, [_vp, C.c_int]),
    "fhs_context_key_switch_mode": (C.c_int, [_vp, _ip]),
    "fhs_seal_hoist_stats": (C.c_int, [_vp, _u64p, _u64p]),
    "fhs_public_key_export": (C.c_int, [_vp, _vp, _u64p]),
    "fhs_galois_keys_bytes": (C.c_int, [_vp, _u64p]),
    "fhs_ciphertext_destroy": (C.c_int, [_vp]),
    "fhs_plaintext_destroy": (C.c_int, [_vp]),
    "fhs_ciphertext_info": (C.c_int, [_vp, _ip, _ip, _ip, _dblp]),
    "fhs_ciphertext_set_scale": (C.c_int, [_vp, C.c_double]),
    "fhs_plaintext_info": (C.c_int, [_vp, _ip, _ip, _dblp]),
    "fhs_ciphertext_export": (C.c_int, [_vp, _vp, _u64p]),
    "fhs_ciphertext_import": (C.c_int, [_vp, _u64p, C.c_int, C.c_int, C.c_double, C.POINTER(_vp)]),
    "fhs_plaintext_export": (C.c_int, [_vp, _vp, _u64p]),
    "fhs_plaintext_import": (C.c_int, [_vp, _u64p, C.c_int, C.c_double, C.POINTER(_vp)]),
    "fhs_ciphertext_device_ptr": (C.c_int, [_vp, C.POINTER(_vp), _u64p]),
    "fhs_encode": (C.c_int, [_vp, _dblp, C.c_size_t, C.c_double, C.c_int, C.POINTER(_vp)]),
    "fhs_encode_batch": (C.c_int, [_vp, _dblp, C.c_size_t, C.c_size_t, C.c_double, C.c_int, C.POINTER(_vp)]),
    "fhs_encode_real": (C.c_int, [_vp, _dblp, C.c_size_t, C.c_double, C.c_int, C.POINTER(_vp)]),
    "fhs_encode_real_batch": (C.c_int, [_vp, _dblp, C.c_size_t, C.c_size_t, C.c_double, C.c_int, C.POINTER(_vp)]),
    "fhs_decode": (C.c_int, [_vp, _vp, _dblp]),
    "fhs_decode_batch": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _dblp]),
    "fhs_encrypt_symmetric": (C.c_int, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "fhs_encrypt_symmetric_batch": (C.c_int, [_vp, _vp, _vp, C.c_int, _vp]),
    "fhs_encode_encrypt_symmetric_batch": (C.c_int, [_vp, _vp, _dblp, C.c_size_t, C.c_size_t, C.c_int, C.c_double,
                                                     C.c_int, _vp]),
    "fhs_decrypt_decode_batch": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int, _dblp]),
    "fhs_encrypt_asymmetric": (C.c_int, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "fhs_decrypt": (C.c_int, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "fhs_add": (C.c_int, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "fhs_sub": (C.c_int, [_vp, _vp, _vp, C.c_int, C.POINTER(_vp)]),
    "fhs_negate": (C.c_int, [_vp, _vp, C.POINTER(_vp)]),
    "fhs_add_plain": (C.c_int, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "fhs_sub_plain": (C.c_int, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "fhs_multiply_plain": (C.c_int, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "fhs_multiply": (C.c_int, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "fhs_relinearize": (C.c_int, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "fhs_rescale_to_next": (C.c_int, [_vp, _vp, C.POINTER(_vp)]),
    "fhs_mod_switch_to_next": (C.c_int, [_vp, _vp, C.POINTER(_vp)]),
    "fhs_mod_switch_to": (C.c_int, [_vp, _vp, C.c_int, C.POINTER(_vp)]),
    "fhs_plain_mod_switch_to_next": (C.c_int, [_vp, _vp, C.POINTER(_vp)]),
    "fhs_plain_mod_switch_to": (C.c_int, [_vp, _vp, C.c_int, C.POINTER(_vp)]),
    "fhs_rotate": (C.c_int, [_vp, _vp, C.c_int, _vp, C.POINTER(_vp)]),
    "fhs_apply_galois": (C.c_int, [_vp, _vp, _u64, _vp, C.POINTER(_vp)]),
    "fhs_rotate_many": (C.c_int, [_vp, C.POINTER(_vp), _ip, C.c_int, _vp, C.POINTER(_vp)]),
    "fhs_bsgs_multiply_accumulate": (C.c_int, [_vp, C.POINTER(_vp), C.c_int, C.POINTER(_vp), C.c_int, C.c_int, _vp,
                                               C.POINTER(_vp)]),
    "fhs_offload_plaintexts": (C.c_int, [_vp, C.POINTER(_vp), C.c_int, _u64p]),
    "fhs_upload_plaintexts": (C.c_int, [_vp, _u64p, C.c_int, C.c_int, C.c_double, C.POINTER(_vp)]),
    "fhs_bsgs_from_cpu": (C.c_int, [_vp, C.POINTER(_vp), C.c_int, _u64p, C.c_int, C.c_int, C.c_int, C.c_double, _vp,
                                    C.POINTER(_vp)]),
    "fhs_bsgs_inner_products": (C.c_int, [_vp, C.POINTER(_vp), C.c_int, C.POINTER(_vp), C.c_int, C.POINTER(_vp)]),
    "fhs_bsgs_giant_steps": (C.c_int, [_vp, C.POINTER(_vp), C.c_int, _u64p, _vp, C.POINTER(_vp)]),
    "fhs_bsgs_inner_products_device": (C.c_int, [_vp, C.POINTER(_vp), C.c_int, C.POINTER(_vp), C.c_int, _vp]),
    "fhs_bsgs_giant_steps_device": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.c_double, _u64p, _vp, C.POINTER(_vp)]),
    "fhs_linear_transform": (C.c_int, [_vp, C.POINTER(_vp), C.c_int, C.POINTER(_vp), C.c_int, C.c_int, _u64p, _vp,
                                       C.c_int, C.POINTER(_vp)]),
    "fhs_multiply_const": (C.c_int, [_vp, _vp, C.c_double, C.c_double, C.POINTER(_vp)]),
    "fhs_add_const": (C.c_int, [_vp, _vp, C.c_double, C.POINTER(_vp)]),
    "fhs_mod_raise": (C.c_int, [_vp, _vp, C.POINTER(_vp)]),
    "fhs_bootstrap_evalmod": (C.c_int, [_vp, _vp, _vp, _dblp, _dblp, C.c_int, C.c_int, C.c_int, C.POINTER(_vp)]),
    "fhs_encode_precise": (C.c_int, [_vp, _dblp, C.c_size_t, C.c_size_t, C.c_double, C.c_int, C.POINTER(_vp)]),
    "fhs_encode_diagonals": (C.c_int, [_vp, _dblp, _dblp, C.c_int, C.c_int, C.c_double, C.c_int, C.POINTER(_vp)]),
    "fhs_encode_diagonals_ex": (C.c_int, [_vp, _vp, _vp, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int,
                                          C.POINTER(_vp)]),
    "fhs_encode_diagonals_rows": (C.c_int, [_vp, _vp, _vp, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int,
                                            _vp, C.c_int, C.POINTER(_vp)]),
    "fhs_host_alloc": (C.c_int, [_u64, C.POINTER(_vp)]),
    "fhs_host_free": (C.c_int, [_vp]),
    "fhs_random_plaintexts": (C.c_int, [_vp, _u64, C.c_int, C.c_int, C.c_double, C.POINTER(_vp)]),
    "fhs_event_record": (C.c_int, [_vp, C.POINTER(_vp)]),
    "fhs_event_elapsed": (C.c_int, [_vp, _vp, C.POINTER(C.c_float)]),
    "fhs_event_destroy": (C.c_int, [_vp]),
    "fhs_kernel_timer": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_float), _ip, C.c_int]),
    "fhs_kernel_timer_arm": (C.c_int, [_vp, C.c_uint32]),
    "fhs_ciphertext_copy_to_device": (C.c_int, [_vp, _vp, _vp]),
    "fhs_ciphertext_from_device": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.c_double, C.POINTER(_vp)]),
    "fhs_ciphertext_copy_to_device_async": (C.c_int, [_vp, _vp, _vp]),
    "fhs_ciphertext_from_device_async": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.c_double, C.POINTER(_vp)]),
    "fhs_context_stream": (C.c_int, [_vp, C.POINTER(_vp)]),
    "fhs_staging_stats": (C.c_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "fhs_debug_fail_next_flushes": (C.c_int, [_vp, C.c_int]),
}
# Fork-only symbols the reference probes with try/except AttributeError (bg:449-461, 382-391): if
# the library lacks one (an older build, or FHESPEAR_DISABLE_SYMBOLS for tests), the Python names
# below are removed at the end of this module, so the reference takes its documented fallback (the
# upload + fused path, or the pure-Python BSGS loop / per-row encode) instead of failing on import.
_OPTIONAL = {
    "fhs_bsgs_multiply_accumulate": ("bsgs_multiply_accumulate",),
    "fhs_bsgs_from_cpu": ("bsgs_from_cpu", "bsgs_complete_from_cpu"),
    "fhs_upload_plaintexts": ("upload_plaintexts",),
    "fhs_offload_plaintexts": ("offload_plaintexts",),
    "fhs_encode_real_batch": ("ckks_encoder.encode_double_vector_batch",),
    "fhs_encode_batch": ("ckks_encoder.encode_complex_vector_batch",),
}
_DISABLED = {x.strip() for x in os.environ.get("FHESPEAR_DISABLE_SYMBOLS", "").split(",") if x.strip()}
_MISSING = []
for _name, (_res, _args) in _SIGS.items():
    try:
        if _name in _DISABLED:
            raise AttributeError(_name)
        _f = getattr(_lib, _name)
    except AttributeError:
        if _name in _OPTIONAL:
            _MISSING.append(_name)
            continue
        raise ImportError(f"pyPhantom: {LIB_PATH} lacks the required symbol {_name}") from None
    _f.restype = _res
    _f.argtypes = _args

_OOM, _HIP, _NODEV = 2, 3, 7


def _check(rc: int, what: str = ""):
    if rc == 0:
        return
    msg = (_lib.fhs_last_error() or b"").decode(errors="replace")
    if rc in (_OOM, _HIP, _NODEV):
        raise RuntimeError(f"{what}: {msg}" if what else msg)
    raise ValueError(f"{what}: {msg}" if what else msg)


def _u64_arr(values):
    a = np.ascontiguousarray(np.asarray(values, dtype=np.uint64))
    return a, a.ctypes.data_as(_u64p)


# ------------------------------------------------------------------ enums / params (pb:56-92)
class scheme_type(enum.IntEnum):
    none = 0
    bgv = 1
    bfv = 2
    ckks = 3


class mul_tech_type(enum.IntEnum):
    none = 0
    behz = 1
    hps = 2
    hps_overq = 3
    hps_overq_leveled = 4


class sec_level_type(enum.IntEnum):
    none = 0
    tc128 = 1
    tc192 = 2
    tc256 = 3


class modulus(int):
    """pb:78 modulus(uint64)."""

    def value(self):
        return int(self)


def create_coeff_modulus(poly_modulus_degree, bit_sizes):
    """pb:81 CoeffModulus::Create: largest primes = 1 mod 2N of each bit size, descending."""
    bits = [int(b) for b in bit_sizes]
    arr = (C.c_int * len(bits))(*bits)
    out = np.zeros(len(bits), dtype=np.uint64)
    _check(_lib.fhs_create_coeff_modulus(int(poly_modulus_degree), arr, len(bits), out.ctypes.data_as(_u64p)),
           "create_coeff_modulus")
    return [modulus(int(x)) for x in out]


def get_elt_from_step(step, poly_modulus_degree):
    """pb:124 Galois element 5^step mod 2N (left rotation by `step`)."""
    return int(_lib.fhs_galois_elt_from_step(int(step), int(poly_modulus_degree)))


def get_elts_from_steps(steps, poly_modulus_degree):
    """pb:126"""
    return [get_elt_from_step(s, poly_modulus_degree) for s in steps]


class params:
    """pb:85-92 EncryptionParameters (CKKS only)."""

    def __init__(self, scheme=scheme_type.ckks):
        if int(scheme) != int(scheme_type.ckks):
            raise ValueError("only scheme_type.ckks is supported by the MI355X backend")
        self.scheme = scheme
        self.poly_modulus_degree = None
        self.special_modulus_size = 1
        self.galois_elts = None
        self.coeff_modulus = None
        self.mul_tech = mul_tech_type.none

    def set_poly_modulus_degree(self, n):
        self.poly_modulus_degree = int(n)

    def set_special_modulus_size(self, p):
        self.special_modulus_size = int(p)

    def set_galois_elts(self, elts):
        self.galois_elts = [int(e) for e in elts]

    def set_coeff_modulus(self, mods):
        self.coeff_modulus = [int(q) for q in mods]

    def set_mul_tech(self, t):
        self.mul_tech = t

    def set_plain_modulus(self, _m):
        raise ValueError("plain modulus is a BFV/BGV parameter; CKKS only")


class cuda_stream:
    """pb:94 placeholder: each context owns one HIP stream."""


def _default_device():
    for k in ("FHESPEAR_DEVICE", "LOCAL_RANK"):
        if os.environ.get(k, "").strip():
            return int(os.environ[k])
    return 0


class context:
    """pb:96 PhantomContext(params): uploads NTT / base-conversion tables to the GPU."""

    def __init__(self, p: params, device: int | None = None):
        if p.poly_modulus_degree is None or p.coeff_modulus is None:
            raise ValueError("params need poly_modulus_degree and coeff_modulus")
        primes, pp = _u64_arr(p.coeff_modulus)
        if p.galois_elts:
            elts, ep = _u64_arr(p.galois_elts)
            ne = len(p.galois_elts)
        else:
            elts, ep, ne = None, None, 0
        h = _vp()
        self.device = _default_device() if device is None else int(device)
        _check(_lib.fhs_context_create(p.poly_modulus_degree, pp, len(p.coeff_modulus), p.special_modulus_size, ep, ne,
                                       self.device, C.byref(h)), "context")
        self._h = h
        self.params = p
        self.N = p.poly_modulus_degree
        self.P = p.special_modulus_size
        self.L0 = len(p.coeff_modulus) - self.P
        self.primes = list(p.coeff_modulus)
        global _default_ctx
        _default_ctx = self

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            _lib is not None and _lib.fhs_context_destroy(h)
            self._h = None

    def synchronize(self):
        _check(_lib.fhs_synchronize(self._h), "synchronize")

    def memory_in_use(self):
        v = _u64()
        _check(_lib.fhs_memory_in_use(self._h, C.byref(v)))
        return int(v.value)

    def limbs(self, chain_index):
        return self.L0 + 1 - chain_index

    def set_key_switch_mode(self, mode):
        """Key-switch convention (extension): 'exact' (default: exact centred ModUp,
        ModDown without rounding -- rotations of one input share a ModUp) or 'seal' (special_modulus_size
        1 only: SEAL's switch_key_inplace -- per-limb lift without centring, automorphism before the
        decomposition, ModDown rounded; batched rotations of one input still share one decomposition,
        corrected to SEAL's limbs per Galois key -- see seal_hoist_stats)."""
        modes = {"exact": 0, "seal": 1}
        if mode not in modes:
            raise ValueError("key switch mode: 'exact' or 'seal'")
        _check(_lib.fhs_context_set_key_switch_mode(self._h, modes[mode]), "set_key_switch_mode")

    def key_switch_mode(self):
        v = C.c_int()
        _check(_lib.fhs_context_key_switch_mode(self._h, C.byref(v)), "key_switch_mode")
        return ("exact", "seal")[v.value]

    def seal_hoist_stats(self):
        """(hoisted, fallback): key-switch flushes in the SEAL convention that shared one decomposition per
        input, and those that fell back to SEAL's per-rotation decomposition (a digit coefficient was 0)."""
        h, f = C.c_uint64(), C.c_uint64()
        _check(_lib.fhs_seal_hoist_stats(self._h, C.byref(h), C.byref(f)), "seal_hoist_stats")
        return int(h.value), int(f.value)

    def galois_elts(self):
        """The Galois elements keys are made for (the params' set, or the SEAL/Phantom default
        +-2^k steps and conjugation when none was set)."""
        n, L0, P, ne = _u64(), C.c_int(), C.c_int(), C.c_int()
        _check(_lib.fhs_context_info(self._h, C.byref(n), C.byref(L0), C.byref(P), C.byref(ne)), "context_info")
        out = np.empty(ne.value, dtype=np.uint64)
        _check(_lib.fhs_context_galois_elts(self._h, out.ctypes.data_as(_u64p)), "context_galois_elts")
        return [int(e) for e in out]


_default_ctx = None


# ------------------------------------------------------------------ objects (pb:157-163)
class plaintext:
    def __init__(self, _ctx=None, _h=None):
        self._ctx = _ctx
        self._h = _h

    def __del__(self):
        if getattr(self, "_h", None):
            _lib is not None and _lib.fhs_plaintext_destroy(self._h)
            self._h = None

    def _info(self):
        ci, l, sc = C.c_int(), C.c_int(), C.c_double()
        _check(_lib.fhs_plaintext_info(self._h, C.byref(ci), C.byref(l), C.byref(sc)))
        return ci.value, l.value, sc.value

    def chain_index(self):
        return self._info()[0]

    def scale(self):
        return self._info()[2]

    def coeff_modulus_size(self):
        return self._info()[1]

    def to_numpy(self):
        ci, l, _ = self._info()
        out = np.empty((l, self._ctx.N), dtype=np.uint64)
        _check(_lib.fhs_plaintext_export(self._ctx._h, self._h, out.ctypes.data_as(_u64p)), "export")
        return out


class ciphertext:
    def __init__(self, _ctx=None, _h=None):
        self._ctx = _ctx
        self._h = _h

    def __del__(self):
        if getattr(self, "_h", None):
            _lib is not None and _lib.fhs_ciphertext_destroy(self._h)
            self._h = None

    def _info(self):
        n, ci, l, sc = C.c_int(), C.c_int(), C.c_int(), C.c_double()
        _check(_lib.fhs_ciphertext_info(self._h, C.byref(n), C.byref(ci), C.byref(l), C.byref(sc)))
        return n.value, ci.value, l.value, sc.value

    def chain_index(self):
        return self._info()[1]

    def scale(self):
        return self._info()[3]

    def set_scale(self, s):
        """pb:163"""
        _check(_lib.fhs_ciphertext_set_scale(self._h, float(s)))

    def coeff_modulus_size(self):
        return self._info()[2]

    def size(self):
        return self._info()[0]

    def to_numpy(self):
        n, ci, l, _ = self._info()
        out = np.empty((n, l, self._ctx.N), dtype=np.uint64)
        _check(_lib.fhs_ciphertext_export(self._ctx._h, self._h, out.ctypes.data_as(_u64p)), "export")
        return out


def ciphertext_from_numpy(ctx, limbs, chain_index, scale):
    a = np.ascontiguousarray(limbs, dtype=np.uint64)
    h = _vp()
    _check(_lib.fhs_ciphertext_import(ctx._h, a.ctypes.data_as(_u64p), a.shape[0], int(chain_index), float(scale),
                                      C.byref(h)), "ciphertext import")
    return ciphertext(ctx, h)


def plaintext_from_numpy(ctx, limbs, chain_index, scale):
    a = np.ascontiguousarray(limbs, dtype=np.uint64)
    h = _vp()
    _check(_lib.fhs_plaintext_import(ctx._h, a.ctypes.data_as(_u64p), int(chain_index), float(scale), C.byref(h)),
           "plaintext import")
    return plaintext(ctx, h)


def _ct(ctx, fn, *args, what=""):
    h = _vp()
    _check(fn(ctx._h, *args, C.byref(h)), what)
    return ciphertext(ctx, h)


def _pt(ctx, fn, *args, what=""):
    h = _vp()
    _check(fn(ctx._h, *args, C.byref(h)), what)
    return plaintext(ctx, h)


# ------------------------------------------------------------------ keys (pb:100-122)
class public_key:
    def __init__(self, _ctx=None, _h=None):
        self._ctx, self._h = _ctx, _h

    def __del__(self):
        if getattr(self, "_h", None):
            _lib is not None and _lib.fhs_public_key_destroy(self._h)
            self._h = None

    def encrypt_asymmetric(self, ctx, pt):
        """pb:112-116"""
        return _ct(ctx, _lib.fhs_encrypt_asymmetric, self._h, pt._h, what="encrypt_asymmetric")


class relin_key:
    def __init__(self, _ctx=None, _h=None):
        self._ctx, self._h = _ctx, _h

    def __del__(self):
        if getattr(self, "_h", None):
            _lib is not None and _lib.fhs_relin_key_destroy(self._h)
            self._h = None


class galois_key:
    def __init__(self, _ctx=None, _h=None):
        self._ctx, self._h = _ctx, _h

    def __del__(self):
        if getattr(self, "_h", None):
            _lib is not None and _lib.fhs_galois_keys_destroy(self._h)
            self._h = None

    def has(self, elt):
        v = C.c_int()
        _check(_lib.fhs_galois_keys_has(self._h, int(elt), C.byref(v)))
        return bool(v.value)

    def nbytes(self):
        v = _u64()
        _check(_lib.fhs_galois_keys_bytes(self._h, C.byref(v)))
        return int(v.value)

    def export(self, elt):
        c = self._ctx
        dnum = (c.L0 + c.P - 1) // c.P
        out = np.empty((dnum, 2, c.L0 + c.P, c.N), dtype=np.uint64)
        _check(_lib.fhs_galois_key_export(c._h, self._h, int(elt), out.ctypes.data_as(_u64p)), "galois key export")
        return out


def _fresh_seed():
    s = os.environ.get("FHESPEAR_SEED", "").strip()
    if s:
        return int(s, 0)
    return int.from_bytes(os.urandom(32), "little")


class secret_key:
    """pb:100-110 PhantomSecretKey.  All secret randomness (s, errors, encryption masks) is drawn
    from ChaCha20 keyed by 256 bits: by default os.urandom(32) (or
    FHESPEAR_SEED); `seed` (extension, an integer < 2^256, its 32 little-endian bytes are the key)
    makes key generation and encryption deterministic for tests."""

    def __init__(self, ctx, seed=None):
        self._ctx = ctx
        self.seed = _fresh_seed() if seed is None else int(seed)
        if not 0 <= self.seed < 1 << 256:
            raise ValueError("secret_key: seed must be an integer in [0, 2^256)")
        h = _vp()
        _check(_lib.fhs_secret_key_create(ctx._h, self.seed.to_bytes(32, "little"), C.byref(h)), "secret_key")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            _lib is not None and _lib.fhs_secret_key_destroy(self._h)
            self._h = None

    def gen_publickey(self, ctx):
        h = _vp()
        _check(_lib.fhs_gen_public_key(ctx._h, self._h, C.byref(h)), "gen_publickey")
        return public_key(ctx, h)

    def gen_relinkey(self, ctx):
        h = _vp()
        _check(_lib.fhs_gen_relin_key(ctx._h, self._h, C.byref(h)), "gen_relinkey")
        return relin_key(ctx, h)

    def create_galois_keys(self, ctx, elts=None):
        h = _vp()
        if elts:
            a, ap = _u64_arr(elts)
            _check(_lib.fhs_create_galois_keys(ctx._h, self._h, ap, len(a), C.byref(h)), "create_galois_keys")
        else:
            _check(_lib.fhs_create_galois_keys(ctx._h, self._h, None, 0, C.byref(h)), "create_galois_keys")
        return galois_key(ctx, h)

    def encrypt_symmetric(self, ctx, pt):
        return _ct(ctx, _lib.fhs_encrypt_symmetric, self._h, pt._h, what="encrypt_symmetric")

    def encrypt_symmetric_batch(self, ctx, pts):
        """fhs_encrypt_symmetric_batch: the same ciphertexts as encrypt_symmetric over `pts` in order, with
        the samplers and NTTs run once over the batch."""
        n = len(pts)
        if n == 0:
            return []
        ins = (_vp * n)(*[p._h for p in pts])
        outs = (_vp * n)()
        _check(_lib.fhs_encrypt_symmetric_batch(ctx._h, self._h, ins, n, outs), "encrypt_symmetric_batch")
        return [ciphertext(ctx, _vp(outs[i])) for i in range(n)]

    def encode_encrypt_batch(self, ctx, mat, scale, chain_index=1):
        """Extension: one ciphertext per row of `mat` (real rows: encode_double_vector_batch, complex rows:
        encode_complex_vector_batch) encrypted with this key -- the same ciphertexts as encoding then
        encrypt_symmetric_batch, in one pass without plaintexts (fhs_encode_encrypt_symmetric_batch)."""
        cplx = np.iscomplexobj(mat)
        m = np.ascontiguousarray(np.asarray(mat, dtype=np.complex128 if cplx else np.float64))
        if m.ndim != 2:
            raise ValueError("encode_encrypt_batch expects a 2-D array (count, values)")
        count, n = m.shape
        if count == 0:
            return []
        outs = (_vp * count)()
        _check(_lib.fhs_encode_encrypt_symmetric_batch(ctx._h, self._h, m.ctypes.data_as(_dblp), count, n,
                                                       0 if cplx else 1, float(scale), int(chain_index), outs),
               "encode_encrypt_batch")
        return [ciphertext(ctx, _vp(outs[i])) for i in range(count)]

    def decrypt_decode_batch(self, ctx, cts, nslots=None):
        """Extension: decrypt each ciphertext and decode its first `nslots` slots (default all) -- the
        values of decrypt + ckks_encoder.decode_batch, without plaintexts (fhs_decrypt_decode_batch);
        complex array [len(cts), nslots]."""
        n = ctx.N // 2 if nslots is None else int(nslots)
        out = np.empty((len(cts), n, 2), dtype=np.float64)
        hs = (_vp * max(1, len(cts)))(*[c._h for c in cts])
        _check(_lib.fhs_decrypt_decode_batch(ctx._h, self._h, hs, len(cts), n, out.ctypes.data_as(_dblp)),
               "decrypt_decode_batch")
        return out[..., 0] + 1j * out[..., 1]

    def decrypt(self, ctx, ct):
        return _pt(ctx, _lib.fhs_decrypt, self._h, ct._h, what="decrypt")

    def export(self):
        c = self._ctx
        out = np.empty((c.L0 + c.P, c.N), dtype=np.uint64)
        _check(_lib.fhs_secret_key_export(c._h, self._h, out.ctypes.data_as(_u64p)), "secret key export")
        return out


# ------------------------------------------------------------------ encoder (pb:128-156)
class ckks_encoder:
    def __init__(self, ctx):
        self._ctx = ctx

    def slot_count(self):
        return self._ctx.N // 2

    @staticmethod
    def _vals(values, cplx):
        a = np.asarray(values)
        if cplx:
            a = np.ascontiguousarray(a, dtype=np.complex128)
            return a.view(np.float64).reshape(a.shape + (2,)) if a.ndim else a
        return np.ascontiguousarray(a, dtype=np.float64)

    def encode_double_vector(self, ctx, values, scale, chain_index=1):
        v = self._vals(values, False)
        return _pt(ctx, _lib.fhs_encode_real, v.ctypes.data_as(_dblp), v.shape[0], float(scale), int(chain_index),
                   what="encode_double_vector")

    def encode_complex_vector(self, ctx, values, scale, chain_index=1):
        v = np.ascontiguousarray(np.asarray(values, dtype=np.complex128))
        return _pt(ctx, _lib.fhs_encode, v.ctypes.data_as(_dblp), v.shape[0], float(scale), int(chain_index),
                   what="encode_complex_vector")

    def _batch(self, ctx, mat, scale, chain_index, cplx, precise=False):
        if precise:
            cplx = True
        m = np.ascontiguousarray(np.asarray(mat, dtype=np.complex128 if cplx else np.float64))
        if m.ndim != 2:
            raise ValueError("batch encode expects a 2-D array (count, values)")
        count, n = m.shape
        hs = (_vp * count)()
        fn = _lib.fhs_encode_precise if precise else (_lib.fhs_encode_batch if cplx else _lib.fhs_encode_real_batch)
        _check(fn(ctx._h, m.ctypes.data_as(_dblp), count, n, float(scale), int(chain_index), hs), "encode batch")
        return [plaintext(ctx, _vp(hs[i])) for i in range(count)]

    def encode_double_vector_batch(self, ctx, mat, scale, chain_index=1):
        """bg:382: one plaintext per row of `mat` (D diagonals x slots)."""
        return self._batch(ctx, mat, scale, chain_index, False)

    def encode_complex_vector_batch(self, ctx, mat, scale, chain_index=1, precise=False):
        """bg:423.  precise=True (extension): long-double canonical embedding with exact rounding
        (fhs_encode_precise), for constant plaintexts such as the bootstrap transforms."""
        return self._batch(ctx, mat, scale, chain_index, True, precise)

    def encode_matrix_diagonals(self, ctx, M, G, scale, chain_index=1, M2=None, rows=None):
        """Extension (no reference symbol): the caller-side pipeline of bg:198-203 + bg:361-432 --
        diagonals of the D x D matrix M (complex-packed with M2: bg:394-432), giant group g rolled by
        g G, tiled to the slots, encoded -- on the GPU from the matrix itself.  Limb-identical to
        encode_double_vector_batch / encode_complex_vector_batch of the numpy-prepared rows.
        rows (sharded matvecs): encode only these diagonal indices, returned in that order."""
        def view(X):   # (pointer, leading dimension, transposed) of a float64 2-D view, copying only if needed
            X = np.asarray(X)
            if X.dtype != np.float64:
                X = X.astype(np.float64)
            if X.ndim != 2 or X.shape[0] != X.shape[1]:
                raise ValueError("encode_matrix_diagonals: M must be square")
            s0, s1 = X.strides
            if s1 == 8 and s0 >= 8 * X.shape[1] and s0 % 8 == 0:
                return X, s0 // 8, 0
            if s0 == 8 and s1 >= 8 * X.shape[0] and s1 % 8 == 0:   # e.g. W[:, lo:hi].T
                return X, s1 // 8, 1
            X = np.ascontiguousarray(X)
            return X, X.shape[1], 0
        A, lda, ta = view(M)
        B2, ldb, tb = view(M2) if M2 is not None else (None, lda, ta)
        if B2 is not None and (B2.shape != A.shape or (ldb, tb) != (lda, ta)):
            A, B2 = np.ascontiguousarray(A), np.ascontiguousarray(B2)
            lda, ta = A.shape[1], 0
        D = A.shape[0]
        if rows is not None:
            r = np.ascontiguousarray(np.asarray(rows, dtype=np.int32))
            hs = (_vp * max(1, len(r)))()
            _check(_lib.fhs_encode_diagonals_rows(ctx._h, _vp(A.ctypes.data),
                                                  None if B2 is None else _vp(B2.ctypes.data), int(lda), int(ta), D,
                                                  int(G), float(scale), int(chain_index), _vp(r.ctypes.data), len(r),
                                                  hs), "encode_matrix_diagonals")
            return [plaintext(ctx, _vp(hs[i])) for i in range(len(r))]
        hs = (_vp * D)()
        _check(_lib.fhs_encode_diagonals_ex(ctx._h, _vp(A.ctypes.data), None if B2 is None else _vp(B2.ctypes.data),
                                            int(lda), int(ta), D, int(G), float(scale), int(chain_index), hs),
               "encode_matrix_diagonals")
        return [plaintext(ctx, _vp(hs[i])) for i in range(D)]

    def _decode(self, ctx, pt):
        out = np.empty((ctx.N // 2, 2), dtype=np.float64)
        _check(_lib.fhs_decode(ctx._h, pt._h, out.ctypes.data_as(_dblp)), "decode")
        return out

    def decode_double_vector(self, ctx, pt):
        return self._decode(ctx, pt)[:, 0].tolist()

    def decode_complex_vector(self, ctx, pt):
        z = self._decode(ctx, pt)
        return (z[:, 0] + 1j * z[:, 1]).tolist()

    def decode_batch(self, ctx, pts, nslots=None):
        """Extension: the first `nslots` slots (default all) of every plaintext, with one device
        synchronisation for the batch (fhs_decode_batch); complex array [len(pts), nslots] -- the same
        values decode_complex_vector gives."""
        n = ctx.N // 2 if nslots is None else int(nslots)
        out = np.empty((len(pts), n, 2), dtype=np.float64)
        hs = (_vp * max(1, len(pts)))(*[p._h for p in pts])
        _check(_lib.fhs_decode_batch(ctx._h, hs, len(pts), n, out.ctypes.data_as(_dblp)), "decode_batch")
        return out[..., 0] + 1j * out[..., 1]


# ------------------------------------------------------------------ evaluator (pb:165-205)
def add(ctx, a, b):
    return _ct(ctx, _lib.fhs_add, a._h, b._h, what="add")


def sub(ctx, a, b, negate=False):
    return _ct(ctx, _lib.fhs_sub, a._h, b._h, 1 if negate else 0, what="sub")


def negate(ctx, a):
    return _ct(ctx, _lib.fhs_negate, a._h, what="negate")


def add_many(ctx, cts, *_):
    cts = list(cts)
    if not cts:
        raise ValueError("add_many: empty list")
    r = cts[0]
    for c in cts[1:]:
        r = add(ctx, r, c)
    return r


def add_plain(ctx, a, p):
    return _ct(ctx, _lib.fhs_add_plain, a._h, p._h, what="add_plain")


def sub_plain(ctx, a, p):
    return _ct(ctx, _lib.fhs_sub_plain, a._h, p._h, what="sub_plain")


def multiply_plain(ctx, a, p):
    return _ct(ctx, _lib.fhs_multiply_plain, a._h, p._h, what="multiply_plain")


def multiply(ctx, a, b):
    return _ct(ctx, _lib.fhs_multiply, a._h, b._h, what="multiply")


def relinearize(ctx, a, rk):
    return _ct(ctx, _lib.fhs_relinearize, a._h, rk._h, what="relinearize")


def multiply_and_relin(ctx, a, b, rk):
    return relinearize(ctx, multiply(ctx, a, b), rk)


def rescale_to_next(ctx, a):
    return _ct(ctx, _lib.fhs_rescale_to_next, a._h, what="rescale_to_next")


def mod_switch_to_next(ctx, x):
    if isinstance(x, plaintext):
        return _pt(ctx, _lib.fhs_plain_mod_switch_to_next, x._h, what="mod_switch_to_next")
    return _ct(ctx, _lib.fhs_mod_switch_to_next, x._h, what="mod_switch_to_next")


def mod_switch_to(ctx, x, chain_index):
    if isinstance(x, plaintext):
        return _pt(ctx, _lib.fhs_plain_mod_switch_to, x._h, int(chain_index), what="mod_switch_to")
    return _ct(ctx, _lib.fhs_mod_switch_to, x._h, int(chain_index), what="mod_switch_to")


def rotate(ctx, a, step, gk):
    """pb:203: left rotation of the N/2 slots by `step` (out[j] = in[j + step])."""
    return _ct(ctx, _lib.fhs_rotate, a._h, int(step), gk._h, what="rotate")


def apply_galois(ctx, a, elt, gk):
    return _ct(ctx, _lib.fhs_apply_galois, a._h, int(elt), gk._h, what="apply_galois")


def hoisting(ctx, a, gk, steps):
    """pb:205: all rotations of one ciphertext (batched in one key-switch launch)."""
    steps = [int(s) for s in steps]
    n = len(steps)
    ins = (_vp * n)(*([a._h] * n))
    st = (C.c_int * n)(*steps)
    outs = (_vp * n)()
    _check(_lib.fhs_rotate_many(ctx._h, ins, st, n, gk._h, outs), "hoisting")
    return [ciphertext(ctx, _vp(outs[i])) for i in range(n)]


def bsgs_multiply_accumulate(ctx, ct_baby, pts, G, B, D, gk):
    """bg:459 / bg:515 fused BSGS; limb-identical to the loop bg:464-485 (incl. final rescale)."""
    G, B, D = int(G), int(B), int(D)
    bb = (_vp * G)(*[c._h for c in ct_baby[:G]])
    pp = (_vp * D)(*[p._h for p in pts[:D]])
    return _ct(ctx, _lib.fhs_bsgs_multiply_accumulate, bb, G, pp, D, B, gk._h, what="bsgs_multiply_accumulate")


def bsgs_inner_products(ctx, ct_baby, pts, G, B):
    """Extension: the Hadamard half of bsgs_multiply_accumulate alone -- [sum_b baby[b] * pts[g G + b]
    for g < B], not rotated, not rescaled (fhs_bsgs_inner_products)."""
    G, B = int(G), int(B)
    if len(pts) != G * B:
        raise ValueError(f"bsgs_inner_products: {len(pts)} plaintexts for G={G}, B={B}")
    bb = (_vp * G)(*[c._h for c in ct_baby[:G]])
    pp = (_vp * (G * B))(*[p._h for p in pts])
    hs = (_vp * B)()
    _check(_lib.fhs_bsgs_inner_products(ctx._h, bb, G, pp, B, hs), "bsgs_inner_products")
    return [ciphertext(ctx, _vp(hs[g])) for g in range(B)]


def bsgs_inner_products_to_device(ctx, ct_baby, pts, G, B, dst_ptr):
    """Extension: bsgs_inner_products written to caller device memory (group g at dst_ptr + g 2 l N
    words), ordered on the context stream (fhs_bsgs_inner_products_device)."""
    G, B = int(G), int(B)
    if len(pts) != G * B:
        raise ValueError(f"bsgs_inner_products_to_device: {len(pts)} plaintexts for G={G}, B={B}")
    bb = (_vp * G)(*[c._h for c in ct_baby[:G]])
    pp = (_vp * (G * B))(*[p._h for p in pts])
    _check(_lib.fhs_bsgs_inner_products_device(ctx._h, bb, G, pp, B, _vp(int(dst_ptr))), "bsgs_inner_products_to_device")


def bsgs_giant_steps_from_device(ctx, src_ptr, k, chain_index, scale, elts, gk):
    """Extension: bsgs_giant_steps over k terms in caller device memory (term j at src_ptr + j 2 l N
    words), ordered on the context stream (fhs_bsgs_giant_steps_device)."""
    if len(elts) != int(k):
        raise ValueError(f"bsgs_giant_steps_from_device: {k} terms for {len(elts)} Galois elements")
    e, ep = _u64_arr(elts)
    return _ct(ctx, _lib.fhs_bsgs_giant_steps_device, _vp(int(src_ptr)), int(k), int(chain_index), float(scale), ep,
               gk._h, what="bsgs_giant_steps_from_device")


def bsgs_giant_steps(ctx, inners, elts, gk):
    """Extension: the giant-step half of bsgs_multiply_accumulate alone -- sum_j galois_{elts[j]}(inners[j])
    with the key switches summed before one ModDown, not rescaled (fhs_bsgs_giant_steps).  Only elts[0]
    may be 1 (an unrotated term)."""
    k = len(inners)
    if k != len(elts) or k < 1:
        raise ValueError(f"bsgs_giant_steps: {k} inner products for {len(elts)} Galois elements")
    hh = (_vp * k)(*[c._h for c in inners])
    e, ep = _u64_arr(elts)
    return _ct(ctx, _lib.fhs_bsgs_giant_steps, hh, k, ep, gk._h, what="bsgs_giant_steps")


# ------------------------------------------------------------------ bootstrapping primitives
def linear_transform(ctx, ct_baby, pts, G, giant_elts, gk, rescale=True):
    """Generalised fused BSGS (CoeffToSlot / SlotToCoeff groups of ckks_bootstrapper):
    [rescale]( sum_g galois_{giant_elts[g]}( sum_b baby[b] * pts[g G + b] ) ), giant_elts[0] = 1."""
    G, B = int(G), len(giant_elts)
    D = len(pts)
    bb = (_vp * G)(*[c._h for c in ct_baby[:G]])
    pp = (_vp * D)(*[p._h for p in pts])
    e, ep = _u64_arr(giant_elts)
    return _ct(ctx, _lib.fhs_linear_transform, bb, G, pp, D, B, ep, gk._h, 1 if rescale else 0,
               what="linear_transform")


def multiply_const(ctx, a, value, const_scale=1.0):
    """a * round(value * const_scale) (exact integer constant); scale *= const_scale."""
    return _ct(ctx, _lib.fhs_multiply_const, a._h, float(value), float(const_scale), what="multiply_const")


def add_const(ctx, a, value):
    """a + value (encoded as round(value * a.scale) in every slot)."""
    return _ct(ctx, _lib.fhs_add_const, a._h, float(value), what="add_const")


def mod_raise(ctx, a):
    """Bootstrapping ModRaise: limb q0 lifted (centred) to all L0 data limbs, chain index 1."""
    return _ct(ctx, _lib.fhs_mod_raise, a._h, what="mod_raise")


def bootstrap_evalmod(ctx, y, rk, cc, cs, r, cheb_depth):
    """ckks_bootstrapper EvalMod in one library call (bootstrap.py Bootstrapper._evalmod's op sequence)."""
    a = np.ascontiguousarray(cc, dtype=np.float64)
    b = np.ascontiguousarray(cs, dtype=np.float64)
    if a.shape != b.shape:
        raise ValueError("bootstrap_evalmod: coefficient arrays differ in length")
    return _ct(ctx, _lib.fhs_bootstrap_evalmod, y._h, rk._h, a.ctypes.data_as(_dblp), b.ctypes.data_as(_dblp),
               len(a), int(r), int(cheb_depth), what="bootstrap_evalmod")


class _HostPlaintexts(np.ndarray):
    """uint64 (count, limbs, N) array in pinned host memory; remembers its context."""


class _PinnedBuffer:
    def __init__(self, nbytes):
        p = _vp()
        _check(_lib.fhs_host_alloc(int(nbytes), C.byref(p)), "pinned host allocation")
        self.ptr = p

    def __del__(self):
        if getattr(self, "ptr", None):
            _lib.fhs_host_free(self.ptr)
            self.ptr = None


def offload_plaintexts(pts):
    """bg:339: copy pre-encoded plaintexts to pinned host memory.
    Returns (data, chain_index, scale, coeff_modulus_size, poly_modulus_degree) (bg:348)."""
    pts = list(pts)
    ctx = pts[0]._ctx
    ci, l, sc = pts[0]._info()
    buf = _PinnedBuffer(8 * len(pts) * l * ctx.N)
    raw = np.ctypeslib.as_array(C.cast(buf.ptr, _u64p), shape=(len(pts), l, ctx.N))
    data = raw.view(_HostPlaintexts)
    data._buf = buf
    data._ctx = ctx
    hs = (_vp * len(pts))(*[p._h for p in pts])
    _check(_lib.fhs_offload_plaintexts(ctx._h, hs, len(pts), raw.ctypes.data_as(_u64p)), "offload_plaintexts")
    return data, ci, sc, l, ctx.N


def _ctx_of(data):
    ctx = getattr(data, "_ctx", None) or _default_ctx
    if ctx is None:
        raise ValueError("no context")
    return ctx


def _host_diagonals(ctx, data, chain_index, coeff_modulus_size, poly_modulus_degree, count, what):
    """Validate a host array of plaintext limbs (count, limbs, N) against the context before the
    device DMA reads count * limbs * N words from it (bg:348 tuple: chain_index, coeff_modulus_size,
    poly_modulus_degree)."""
    a = np.ascontiguousarray(data, dtype=np.uint64)
    l = ctx.L0 + 1 - int(chain_index)
    if a.ndim != 3:
        raise ValueError(f"{what}: expected a (count, limbs, N) array, got shape {a.shape}")
    if int(coeff_modulus_size) != l or a.shape[1] != l:
        raise ValueError(f"{what}: chain_index {chain_index} has {l} limbs, but coeff_modulus_size is "
                         f"{coeff_modulus_size} and the array has {a.shape[1]}")
    if int(poly_modulus_degree) != ctx.N or a.shape[2] != ctx.N:
        raise ValueError(f"{what}: poly_modulus_degree {poly_modulus_degree} / array width {a.shape[2]} "
                         f"differ from the context's N = {ctx.N}")
    if count is not None and a.shape[0] < count:
        raise ValueError(f"{what}: {a.shape[0]} plaintexts given, {count} needed")
    return a


def upload_plaintexts(data, chain_index, scale, coeff_modulus_size, poly_modulus_degree):
    """bg:349: host -> device; returns a list of plaintexts."""
    ctx = _ctx_of(data)
    a = _host_diagonals(ctx, data, chain_index, coeff_modulus_size, poly_modulus_degree, None, "upload_plaintexts")
    n = a.shape[0]
    if n < 1:
        raise ValueError("upload_plaintexts: empty array")
    hs = (_vp * n)()
    _check(_lib.fhs_upload_plaintexts(ctx._h, a.ctypes.data_as(_u64p), n, int(chain_index), float(scale), hs),
           "upload_plaintexts")
    return [plaintext(ctx, _vp(hs[i])) for i in range(n)]


def bsgs_from_cpu(ctx, ct_baby, data, chain_index, scale, coeff_modulus_size, poly_modulus_degree, G, B, D, gk):
    """bg:449: BSGS with the diagonals streamed from host memory."""
    G, B, D = int(G), int(B), int(D)
    a = _host_diagonals(ctx, data, chain_index, coeff_modulus_size, poly_modulus_degree, D, "bsgs_from_cpu")
    bb = (_vp * G)(*[c._h for c in ct_baby[:G]])
    return _ct(ctx, _lib.fhs_bsgs_from_cpu, bb, G, a.ctypes.data_as(_u64p), D, B, int(chain_index), float(scale),
               gk._h, what="bsgs_from_cpu")


def bsgs_complete_from_cpu(ctx, ct_x, data, chain_index, scale, coeff_modulus_size, poly_modulus_degree, G, B, D,
                           gk):
    """bg:244 (fork-only, called from _parallel_bsgs_projections' thread pool): the baby steps of
    ct_x (bg:215-220, one hoisted key-switch inside the library) then bsgs_from_cpu.  Safe from
    several threads on one context: every library call holds the context's lock."""
    G = int(G)
    baby = [ct_x] + [rotate(ctx, ct_x, b, gk) for b in range(1, G)]
    return bsgs_from_cpu(ctx, baby, data, chain_index, scale, coeff_modulus_size, poly_modulus_degree, G, B, D, gk)


# ------------------------------------------------------------------ measurement helpers
def random_plaintexts(ctx, seed, count, chain_index, scale):
    hs = (_vp * count)()
    _check(_lib.fhs_random_plaintexts(ctx._h, int(seed), int(count), int(chain_index), float(scale), hs),
           "random_plaintexts")
    return [plaintext(ctx, _vp(hs[i])) for i in range(count)]


def galois_keys_from_numpy(ctx, keys):
    """{galois element: [dnum][2][L0+P][N] uint64} -> galois_key (import of keys made elsewhere, e.g.
    SEAL's KSwitchKeys: component 0 = b_j = -a_j s + e_j + P g_j s', component 1 = a_j; the layout
    galois_key.export returns)."""
    elts = sorted(int(e) for e in keys)
    want = _switch_key_shape(ctx)
    for e in elts:
        _check_key_shape(keys[e], want, f"galois_keys_from_numpy: key for element {e}")
    arr = np.ascontiguousarray(np.stack([np.asarray(keys[e], dtype=np.uint64) for e in elts]))
    e_arr = np.array(elts, dtype=np.uint64)
    h = _vp()
    _check(_lib.fhs_galois_keys_import(ctx._h, e_arr.ctypes.data_as(_u64p), len(elts), arr.ctypes.data_as(_u64p),
                                       C.byref(h)), "galois_keys_from_numpy")
    return galois_key(ctx, h)


def _switch_key_shape(ctx):
    """(dnum, 2, L0+P, N): the layout the C side reads without a length (fhs_*_import)."""
    return (-(-ctx.L0 // ctx.P), 2, ctx.L0 + ctx.P, ctx.N)


def _check_key_shape(arr, want, what):
    shape = tuple(np.shape(arr))
    if shape != tuple(want):
        raise ValueError(f"{what}: shape {shape}, this context needs {tuple(want)}")


def relin_key_from_numpy(ctx, key):
    """[dnum][2][L0+P][N] -> relin_key (the galois_keys_from_numpy layout)."""
    _check_key_shape(key, _switch_key_shape(ctx), "relin_key_from_numpy")
    a = np.ascontiguousarray(key, dtype=np.uint64)
    h = _vp()
    _check(_lib.fhs_relin_key_import(ctx._h, a.ctypes.data_as(_u64p), C.byref(h)), "relin_key_from_numpy")
    return relin_key(ctx, h)


def secret_key_from_numpy(ctx, s_ntt):
    """[L0+P][N] NTT-form secret -> secret_key (its encryption randomness: a fresh 256-bit key)."""
    _check_key_shape(s_ntt, (ctx.L0 + ctx.P, ctx.N), "secret_key_from_numpy")
    a = np.ascontiguousarray(s_ntt, dtype=np.uint64)
    sk = secret_key.__new__(secret_key)
    sk._ctx, sk.seed = ctx, None
    h = _vp()
    _check(_lib.fhs_secret_key_import(ctx._h, a.ctypes.data_as(_u64p), C.byref(h)), "secret_key_from_numpy")
    sk._h = h
    return sk


class Event:
    def __init__(self, ctx):
        h = _vp()
        _check(_lib.fhs_event_record(ctx._h, C.byref(h)), "event")
        self._h = h

    def elapsed_ms(self, later):
        v = C.c_float()
        _check(_lib.fhs_event_elapsed(self._h, later._h, C.byref(v)), "event elapsed")
        return float(v.value)

    def __del__(self):
        if getattr(self, "_h", None):
            _lib is not None and _lib.fhs_event_destroy(self._h)
            self._h = None


KERNEL_IDS = {"k_bsgs_inner": 0, "k_modup": 1, "k_ks_ip": 2, "k_moddown": 3, "k_ks_intt": 4,
              "k_ks_special_intt": 5, "k_giant_sum": 6, "k_giant_final": 7, "rescale": 8}


def kernel_timer_arm(ctx, names=None):
    """Record HIP events around every launch of the named kernels (None = all, [] = off)."""
    ids = KERNEL_IDS.values() if names is None else [KERNEL_IDS[n] for n in names]
    mask = 0
    for i in ids:
        mask |= 1 << i
    _check(_lib.fhs_kernel_timer_arm(ctx._h, mask), "kernel_timer_arm")


def kernel_timer_read(ctx, reset=False):
    """{kernel: (ms, launches)} accumulated since the last reset."""
    out = {}
    for name, kid in KERNEL_IDS.items():
        ms, n = C.c_float(), C.c_int()
        _check(_lib.fhs_kernel_timer(ctx._h, kid, C.byref(ms), C.byref(n), 0), "kernel_timer")
        out[name] = (float(ms.value), int(n.value))
    if reset:
        _check(_lib.fhs_kernel_timer(ctx._h, -1, None, None, 1), "kernel_timer")
    return out


def debug_fail_next_flushes(ctx, count=1):
    """Testing hook: the next `count` flushes of queued rotations fail as out of memory (their outputs are
    marked lost and the queue is dropped: fhs_debug_fail_next_flushes)."""
    _check(_lib.fhs_debug_fail_next_flushes(ctx._h, int(count)), "debug_fail_next_flushes")


def staging_stats(ctx):
    """(segment re-entries, re-entries that waited for the GPU) of the context's descriptor ring."""
    a, b = C.c_uint64(), C.c_uint64()
    _check(_lib.fhs_staging_stats(ctx._h, C.byref(a), C.byref(b)), "staging_stats")
    return int(a.value), int(b.value)


def ciphertext_copy_to_device(ctx, ct, dst_ptr, sync=True):
    """Ciphertext limbs -> caller-owned HBM.  sync=False only enqueues the copy on the context stream
    (context_stream); the caller orders its streams with events (fhespear_dist.to_buffer)."""
    fn = _lib.fhs_ciphertext_copy_to_device if sync else _lib.fhs_ciphertext_copy_to_device_async
    _check(fn(ctx._h, ct._h, _vp(int(dst_ptr))), "copy_to_device")


def ciphertext_from_device(ctx, src_ptr, ncomp, chain_index, scale, sync=True):
    fn = _lib.fhs_ciphertext_from_device if sync else _lib.fhs_ciphertext_from_device_async
    h = _vp()
    _check(fn(ctx._h, _vp(int(src_ptr)), int(ncomp), int(chain_index), float(scale), C.byref(h)), "from_device")
    return ciphertext(ctx, h)


def context_stream(ctx):
    """The context's HIP stream handle (int), e.g. for torch.cuda.ExternalStream."""
    h = _vp()
    _check(_lib.fhs_context_stream(ctx._h, C.byref(h)), "context_stream")
    return int(h.value or 0)


from . import bootstrap as _bootstrap  # noqa: E402


class ckks_bootstrapper(_bootstrap.Bootstrapper):
    """bg:72-74, 112-116, 149-154: CKKS bootstrapping (pyPhantom/bootstrap.py) on the GPU ops."""


ckks_bootstrapper._ph = sys.modules[__name__]


def device_count():
    return int(_lib.fhs_device_count())


def device_pci_bus_id(device):
    """PCI bus id of HIP device `device` (extension: the multi-rank bench line's device check)."""
    buf = C.create_string_buffer(64)
    _check(_lib.fhs_device_pci_bus_id(int(device), buf, 64), "device_pci_bus_id")
    return buf.value.decode()


_lock = threading.Lock()

for _name in _MISSING:   # absent optional symbols -> AttributeError for the reference's fallbacks
    for _py in _OPTIONAL[_name]:
        _owner, _, _attr = _py.rpartition(".")
        if _owner:
            delattr(globals()[_owner], _attr)
        else:
            del globals()[_attr]
