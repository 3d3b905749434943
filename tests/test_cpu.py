"""CPU-only tests (no GPU): the parity oracle against known answers, algebraic identities and the
golden fixtures generated from the reference's own BSGS orchestration; the C-ABI library loads and
exports every symbol include/fhespear.h declares; the product fails loudly without a GPU; the
multi-process (gloo, world_size 2) exchange steps of the 8-projection block."""
import hashlib
import json
import re
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
GOLDEN = REPO / "tests" / "golden"


@pytest.fixture(scope="module")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


# ------------------------------------------------------------------ known answers
def test_seal_coeff_modulus_known_answers(orc):
    # SEAL CoeffModulus::BFVDefault(4096 / 8192) are Create() outputs for these bit sizes
    assert orc.create_coeff_modulus(4096, [36, 36, 37]) == [0xffffee001, 0xffffc4001, 0x1ffffe0001]
    assert orc.create_coeff_modulus(8192, [43, 43, 44, 44, 44]) == [
        0x7fffffd8001, 0x7fffffc8001, 0xfffffffc001, 0xffffff6c001, 0xfffffebc001]
    qs = orc.create_coeff_modulus(16384, [59] * 39)
    assert qs == sorted(qs, reverse=True) and all((q - 1) % 32768 == 0 and q < 2 ** 59 for q in qs)


def test_galois_elements_match_reference_formula(orc):
    N = 16384
    for s in (1, 2, 45, 46, 44 * 46, 4095):
        assert orc.galois_elt(s, N) == pow(5, s, 2 * N)          # bg:24
    assert orc.galois_elt(0, N) == 2 * N - 1                    # bg:21 conjugation
    assert orc.galois_elt(-1, N) == pow(5, N // 2 - 1, 2 * N)


# ------------------------------------------------------------------ algebraic identities
def _psi(q, N):
    # minimal primitive 2N-th root (brute force over odd powers of a generator)
    for c in range(2, 1000):
        g = pow(c, (q - 1) // (2 * N), q)
        if pow(g, N, q) == q - 1:
            return min(pow(g, 2 * k + 1, q) for k in range(N))


def _rev(i, bits):
    return int(format(i, f"0{bits}b")[::-1], 2)


def test_ntt_is_evaluation_at_odd_powers(orc):
    N = 256
    qs = orc.create_coeff_modulus(N, [50, 50])
    o = orc.Oracle(N, qs, 1)
    rng = np.random.default_rng(0)
    a = rng.integers(0, qs[0], N, dtype=np.uint64)
    A = o.ntt(a, 0)
    psi = _psi(qs[0], N)
    for i in (0, 1, 7, 100, 255):
        x = pow(psi, 2 * _rev(i, 8) + 1, qs[0])
        assert int(A[i]) == sum(int(a[k]) * pow(x, k, qs[0]) for k in range(N)) % qs[0]
    assert np.array_equal(o.intt(A, 0), a)


def test_galois_ntt_is_coefficient_automorphism(orc):
    N = 256
    qs = orc.create_coeff_modulus(N, [50, 50])
    o = orc.Oracle(N, qs, 1)
    q = qs[0]
    rng = np.random.default_rng(1)
    a = rng.integers(0, q, N, dtype=np.uint64)
    elt = orc.galois_elt(3, N)
    b = np.zeros(N, dtype=np.uint64)
    for i in range(N):                     # X^i -> X^(i*elt) mod (X^N + 1)
        j = (i * elt) % (2 * N)
        v = int(a[i])
        if j >= N:
            j -= N
            v = (q - v) % q
        b[j] = v
    assert np.array_equal(o.galois_ntt(o.ntt(a, 0), elt), o.ntt(b, 0))


def test_encode_rotate_multiply_semantics(orc):
    N, L0, P = 1024, 6, 3
    qs = orc.create_coeff_modulus(N, [59] * (L0 + P))
    o = orc.Oracle(N, qs, P)
    s = o.gen_secret(3)
    rng = np.random.default_rng(2)
    x = rng.normal(0, 0.5, N // 2)
    sc = 2.0 ** 40
    pt = o.encode(x, sc, L0)
    assert np.max(np.abs(o.decode(pt, sc).real - x)) < 1e-9
    ct = o.encrypt_symmetric(3, 0, s, pt)
    for st in (1, 5, -2):
        r = o.rotate(ct, o.gen_galois_key(3, s, orc.galois_elt(st, N)), st)
        assert np.max(np.abs(o.decode(o.decrypt(s, r), sc).real - np.roll(x, -st))) < 1e-6
    sq = o.rescale(o.relinearize(o.multiply(ct, ct), o.gen_relin_key(3, s)))
    assert np.max(np.abs(o.decode(o.decrypt(s, sq), sc * sc / qs[L0 - 1]).real - x * x)) < 1e-3


# ------------------------------------------------------------------ golden fixtures
def _golden(name):
    man = json.loads((GOLDEN / "manifest.json").read_text())
    return man["cases"][name], np.load(GOLDEN / man["cases"][name]["file"])


@pytest.mark.parametrize("case", ["bsgs_real_n512", "bsgs_complex_n512", "bsgs_real_n1024_p1"])
def test_oracle_reproduces_reference_bsgs_golden(orc, case):
    meta, z = _golden(case)
    N, P, D, G, B = (meta[k] for k in ("N", "P", "D", "G", "B"))
    primes = [int(q) for q in z["primes"]]
    o = orc.Oracle(N, primes, P)
    s = o.gen_secret(meta["sk_seed"])
    assert hashlib.sha256(s.tobytes()).hexdigest() == meta["secret_sha256"]
    keys = [None] + [o.gen_galois_key(meta["sk_seed"], s, e) for e in meta["giant_elts"]]
    for e, k in zip(meta["giant_elts"][:2], keys[1:3]):
        assert hashlib.sha256(k.tobytes()).hexdigest() == meta["giant_key_sha256"][str(e)]
    out = o.bsgs_loop(list(z["baby"]), list(z["pts"]), keys, G, B, D)
    assert np.array_equal(out, z["out"])
    # baby steps are rotations of the input (bg:215-220)
    for b in (1, G - 1):
        assert np.array_equal(o.rotate(z["ct_in"], o.gen_galois_key(meta["sk_seed"], s, orc.galois_elt(b, N)), b),
                              z["baby"][b])
    assert meta["op_counts"]["rotate"] == B - 1 and meta["op_counts"]["multiply_plain"] == D
    dec = o.decode(o.decrypt(s, out), meta["scale_out"])[:D]
    want = z["ref"]
    got = dec if meta["complex"] else dec.real
    assert np.max(np.abs(got - want)) < 1e-9


def test_golden_ffn_meets_reference_pass_criterion():
    meta, z = _golden("ffn_n1024")
    assert all(c > 0.999 for c in meta["corr"])          # tf:298
    for b in range(meta["blocks"]):
        assert np.corrcoef(z["dec"][b], z["ref"][b])[0, 1] > 0.999


# ------------------------------------------------------------------ C ABI / product boundary
def _declared_symbols():
    hdr = (REPO / "include" / "fhespear.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(fhs_[a-z0-9_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    import ctypes
    lib_path = REPO / "fhe-spear_amd" / "lib" / "libfhespear_hip.so"
    if not lib_path.exists():
        import __graft_entry__
        __graft_entry__.build()
    lib = ctypes.CDLL(str(lib_path))
    syms = _declared_symbols()
    assert len(syms) > 60
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_product_host_helpers_agree_with_oracle(orc):
    sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))
    import pyPhantom as ph
    for N, bits in ((4096, [36, 36, 37]), (16384, [59] * 39), (32768, [60] + [40] * 9 + [60])):
        assert [int(q) for q in ph.create_coeff_modulus(N, bits)] == orc.create_coeff_modulus(N, bits)
    for s in (1, 46, -3, 0):
        assert ph.get_elt_from_step(s, 16384) == orc.galois_elt(s, 16384)


def test_product_fails_loudly_without_gpu():
    sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))
    import pyPhantom as ph
    if ph.device_count() > 0:
        pytest.skip("a GPU is present")
    p = ph.params(ph.scheme_type.ckks)
    p.set_poly_modulus_degree(1024)
    p.set_special_modulus_size(1)
    p.set_coeff_modulus(ph.create_coeff_modulus(1024, [50, 50]))
    with pytest.raises(RuntimeError, match="no HIP device"):
        ph.context(p)


# ------------------------------------------------------------------ multi-process exchange (gloo)
def _worker(rank, world, port, q):
    import os
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))
    import fhespear_dist as fd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        td = fd.TimedDist(dist)          # the bench's exchange log (every call below goes through it)
        td.start()
        mine = fd.my_projections(8, world, rank)
        t = torch.full((4,), rank * 10 + len(mine), dtype=torch.int64)
        got = fd.gather_to_root(td, t, world, rank)
        b = torch.arange(4, dtype=torch.int64) if rank == 1 else torch.zeros(4, dtype=torch.int64)
        fd.broadcast_from(td, b, src=1)
        big = torch.full((2048,), rank, dtype=torch.int64)
        fd.broadcast_from(td, big, src=0)
        primes = [(1 << 59) - 55, (1 << 59) - 99]
        r = torch.tensor([[primes[0] - 1 - rank, 5], [primes[1] - 2, 7 + rank]], dtype=torch.int64)
        fd.modular_reduce_sum(td, r.view(-1), primes)
        td.stop()
        fd.broadcast_from(td, b, src=1)   # not logged
        ids = fd.gather_identities(td, {"local_rank": rank, "pci_bus_id": f"0000:0{rank}:00.0"})
        q.put((rank, mine, None if got is None else [x.tolist() for x in got], b.tolist(),
               r.tolist() if rank == 0 else None, fd.stage_assignment(world, rank), td.summary(per=1), ids,
               int(big[0])))
    finally:
        dist.destroy_process_group()


def test_two_rank_exchange_gloo():
    import torch.multiprocessing as mp
    import random
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == [0, 2, 4, 6] and res[1][1] == [1, 3, 5, 7]
    assert res[0][2] == [[4] * 4, [14] * 4]
    assert res[0][3] == res[1][3] == [0, 1, 2, 3]
    p0, p1 = (1 << 59) - 55, (1 << 59) - 99
    assert res[0][4] == [[(2 * p0 - 3) % p0, 10], [(2 * p1 - 4) % p1, 15]]
    assert res[0][5] == [["r", "v"], ["o"], ["ffn_key_0"], ["ffn_val_0"]]
    assert res[1][5] == [["k"], [], ["ffn_key_1"], ["ffn_val_1"]]
    # exchange log schema (bench.py exchange_per_step / exchange_per_block_rank0): per kind calls, MB, ms;
    # transfers under 4 KiB are the _small kinds
    for rk in (0, 1):
        ex = res[rk][6]
        assert set(ex) == {"gather_small", "broadcast_small", "broadcast", "reduce_small"}, ex
        assert ex["broadcast"]["calls"] == 1 and ex["broadcast"]["MB"] == round(2048 * 8 / 1e6, 3)
        assert all(set(v) == {"calls", "MB", "ms"} and v["ms"] >= 0 for v in ex.values())
    assert res[1][8] == 0
    assert res[0][7] == res[1][7] == [{"local_rank": 0, "pci_bus_id": "0000:00:00.0"},
                                      {"local_rank": 1, "pci_bus_id": "0000:01:00.0"}]


# ------------------------------------------------------------------ exact centred ModUp / hoisting
def test_centered_count_exact_including_near_half(orc):
    from math import prod
    rng = np.random.default_rng(11)
    for ns in (1, 2, 3, 4):
        qs = orc.create_coeff_modulus(1 << 14, [59] * ns)
        Q = prod(qs)
        for trial in range(3000):
            y = [int(rng.integers(0, q)) for q in qs]
            if ns > 1 and trial % 2:       # steer sum_u y_u/q_u to within a few ulp of k + 1/2
                f = sum(y[u] / qs[u] for u in range(ns - 1))
                tgt = (np.floor(f) + 1.5 - f) % 1.0
                y[-1] = (int(tgt * qs[-1]) + int(rng.integers(-3, 4))) % qs[-1]
            X = sum(yu * (Q // qu) for yu, qu in zip(y, qs))
            assert orc.centered_count(y, qs) == (2 * X + Q) // (2 * Q)


def test_hoisted_rotations_bit_identical_to_individual(orc):
    N, L0, P = 1024, 6, 3
    qs = orc.create_coeff_modulus(N, [59] * (L0 + P))
    o = orc.Oracle(N, qs, P)
    s = o.gen_secret(8)
    rng = np.random.default_rng(4)
    for l in (6, 4):
        ct = np.stack([np.stack([rng.integers(0, qs[i], N, dtype=np.uint64) for i in range(l)]) for _ in range(2)])
        steps = [1, 2, 5, -1]
        elts = [orc.galois_elt(k, N) for k in steps]
        keys = [o.gen_galois_key(8, s, e) for e in elts]
        for h, k, e in zip(o.rotate_hoisted(ct, keys, elts), keys, elts):
            assert np.array_equal(h, o.rotate_elt(ct, k, e))


def _lib():
    import ctypes
    lib_path = REPO / "fhe-spear_amd" / "lib" / "libfhespear_hip.so"
    if not lib_path.exists():
        import __graft_entry__
        __graft_entry__.build()
    return ctypes.CDLL(str(lib_path))


def test_pseudo_mersenne_reduction_matches_bigint(orc):
    """The kernels' q = 2^b - d folds (fhs_modarith.h pm_reduce128) against Python big ints, on
    the reference's 59-bit chain (all eligible), on 60-bit primes, and on adversarial inputs
    (all-ones, multiples of q, q-1 products, 2^128 - 1)."""
    import ctypes
    lib = _lib()
    lib.fhs_debug_reduce128.argtypes = [ctypes.c_uint64] * 3 + [ctypes.POINTER(ctypes.c_uint64),
                                                              ctypes.POINTER(ctypes.c_int)]
    rng = np.random.default_rng(7)
    primes = orc.create_coeff_modulus(16384, [59] * 39) + orc.create_coeff_modulus(32768, [60] * 4) \
        + orc.create_coeff_modulus(4096, [36] * 3)
    out, used = ctypes.c_uint64(), ctypes.c_int()
    n_pm = 0
    for q in primes:
        xs = [(1 << 128) - 1, q * q - 1, (q - 1) ** 2, q << 64, ((1 << 128) // q) * q, (1 << 64) - 1, 0, q]
        xs += [int(a) << 64 | int(b) for a, b in rng.integers(0, 2 ** 63, size=(200, 2), dtype=np.int64)]
        xs += [((int(a) << 64) | int(b)) * 4 % (1 << 128) for a, b in rng.integers(0, 2 ** 63, size=(50, 2), dtype=np.int64)]
        for x in xs:
            assert lib.fhs_debug_reduce128(q, x & ((1 << 64) - 1), x >> 64, ctypes.byref(out), ctypes.byref(used)) == 0
            assert out.value == x % q, (q, x)
        n_pm += used.value
        if q.bit_length() == 59 and q in primes[:39]:
            assert used.value == 1, "reference 59-bit chain must take the pseudo-Mersenne path"
    assert n_pm >= 43


def test_modup_xform_matches_centred_extension(orc):
    """ModUp's X form (fhs_modarith.h centered_x_pack + convert3x_value, the routines k_centered_x and
    modup_convert3x run, here on the host through fhs_debug_modup_xform) against the centred extension
    in big integers: X = sum_u y_u Q/q_u - round(.) Q, X mod m -- on cfg2's chain (every digit, every
    target), with extreme residues and sums steered to within a few ulp of k + 1/2."""
    import ctypes
    from math import prod
    lib = _lib()
    U64 = ctypes.c_uint64
    lib.fhs_debug_modup_xform.argtypes = [ctypes.POINTER(U64), ctypes.POINTER(U64), U64, ctypes.POINTER(U64)]
    qs = orc.create_coeff_modulus(16384, [59] * 39)
    rng = np.random.default_rng(23)
    out = U64()
    for j in range(12):
        q3 = qs[3 * j:3 * j + 3]
        Q = prod(q3)
        cases = [[0, 0, 0], [q - 1 for q in q3], [q3[0] - 1, 0, 0], [0, 0, q3[2] - 1]]
        for trial in range(40):
            y = [int(rng.integers(0, q)) for q in q3]
            if trial % 2:   # steer sum_u y_u/q_u next to k + 1/2
                f = y[0] / q3[0] + y[1] / q3[1]
                y[2] = (int(((np.floor(f) + 1.5 - f) % 1.0) * q3[2]) + int(rng.integers(-3, 4))) % q3[2]
            cases.append(y)
        targets = [t for t in range(39) if t // 3 != j]
        for y in cases:
            S = sum(yu * (Q // qu) for yu, qu in zip(y, q3))
            X = S - ((2 * S + Q) // (2 * Q)) * Q
            assert 2 * abs(X) < Q
            for t in targets[:: max(1, len(targets) // 9)] if y not in cases[:4] else targets:
                assert lib.fhs_debug_modup_xform((U64 * 3)(*q3), (U64 * 3)(*y), qs[t], ctypes.byref(out)) == 0
                assert out.value == X % qs[t], (j, t, y)


def test_modup_xform_on_60_bit_primes(orc):
    """The X form's edge: with 60-bit primes q = 2^60 - d, |X| < Q_S/2 < 2^179 and
    U = X + 2^179 < 2^180 fill the three 60-bit words.  Residues at y = q - 1, zero, and sums steered to
    both sides of every rounding threshold k + 1/2 (k = 0, 1, 2) against big integers; a residue >= q
    (outside centered_x_pack's three thresholds) is rejected, not mis-rounded."""
    import ctypes
    from math import prod
    lib = _lib()
    U64 = ctypes.c_uint64
    lib.fhs_debug_modup_xform.argtypes = [ctypes.POINTER(U64), ctypes.POINTER(U64), U64, ctypes.POINTER(U64)]
    qs = orc.create_coeff_modulus(16384, [60] * 15)
    assert all((1 << 59) < q < (1 << 60) for q in qs)
    rng = np.random.default_rng(41)
    out = U64()
    for j in range(3):
        q3 = qs[3 * j:3 * j + 3]
        Q = prod(q3)
        targets = [t for t in range(15) if t // 3 != j]
        cases = [[q - 1 for q in q3], [0, 0, 0], [q3[0] - 1, q3[1] - 1, 0]]
        for k in range(3):   # S / Q next to k + 1/2, from below and above
            for delta in (-2, -1, 0, 1, 2):
                y = [int(rng.integers(0, q)) for q in q3]
                f = y[0] / q3[0] + y[1] / q3[1]
                target = (k + 0.5 - f) % 1.0
                y[2] = (int(target * q3[2]) + delta) % q3[2]
                cases.append(y)
        for y in cases:
            S = sum(yu * (Q // qu) for yu, qu in zip(y, q3))
            X = S - ((2 * S + Q) // (2 * Q)) * Q
            assert 2 * abs(X) < Q and abs(X) < 2 ** 179 and X + 2 ** 179 < 2 ** 180
            for t in targets:
                assert lib.fhs_debug_modup_xform((U64 * 3)(*q3), (U64 * 3)(*y), qs[t], ctypes.byref(out)) == 0
                assert out.value == X % qs[t], (j, t, y)
        bad = [q3[0], 0, 0]
        assert lib.fhs_debug_modup_xform((U64 * 3)(*q3), (U64 * 3)(*bad), qs[targets[0]], ctypes.byref(out)) != 0


def test_moddown_xform_matches_fast_base_conversion(orc):
    """ModDown's X form (k_special_x + moddown_convert3x, the same __host__ __device__ routines through
    fhs_debug_moddown_xform) against big integers: (sum_k y_k P/p_k) mod q_i, the fast base conversion's
    value, on cfg2's 3 special primes into every data prime, with extreme residues."""
    import ctypes
    from math import prod
    lib = _lib()
    U64 = ctypes.c_uint64
    lib.fhs_debug_moddown_xform.argtypes = [ctypes.POINTER(U64), ctypes.POINTER(U64), U64, ctypes.POINTER(U64)]
    qs = orc.create_coeff_modulus(16384, [59] * 39)
    p3, data = qs[36:], qs[:36]
    P = prod(p3)
    rng = np.random.default_rng(29)
    out = U64()
    cases = [[0, 0, 0], [p - 1 for p in p3]] + [[int(rng.integers(0, p)) for p in p3] for _ in range(60)]
    for y in cases:
        Y = sum(yk * (P // pk) for yk, pk in zip(y, p3))
        for q in data:
            assert lib.fhs_debug_moddown_xform((U64 * 3)(*p3), (U64 * 3)(*y), q, ctypes.byref(out)) == 0
            assert out.value == Y % q, (q, y)


def test_device_ntt_passes_emulated_match_direct_evaluation(tmp_path):
    """fhs_ntt.h's forward (Harvey and lazy) and inverse passes, compiled for the host through a
    shim header and run thread-by-thread between barriers, against a direct O(N^2) evaluation
    a(psi^(2 rev(i) + 1)) -- the same convention the oracle pins (test_ntt_is_evaluation_at_odd_powers).
    The Shoup products take their plain C form here (FHS_ASM_SHOUP=0): the default form is gfx950
    inline asm, pinned bit-exact against the oracle by the GPU tests."""
    import subprocess
    exe = tmp_path / "ntt_emu"
    subprocess.run(["g++", "-O2", "-std=c++17", "-DFHS_ASM_SHOUP=0", f"-I{REPO / 'tools/debug/shim'}", f"-I{REPO / 'fhe-spear_amd/csrc'}",
                    str(REPO / "tools/debug/ntt_emu.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout


def test_wave_local_passes_touch_only_their_waves_elements(tmp_path):
    """The barriers fhs_ntt.h's wave-local passes drop (fwd_from / inv_from with WL, the wave-local exits
    and heads the ModUp / INTT kernels rely on) are safe: with fhs_ntt.h's own ntt_pass run thread by thread
    and the LDS array diffed, every element a thread touches after a dropped barrier was written by its own
    wave (64 lanes, or every thread of a one-wave transform) -- tools/debug/wl_check.cpp."""
    import subprocess
    exe = tmp_path / "wl_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-DFHS_ASM_SHOUP=0", f"-I{REPO / 'tools/debug/shim'}",
                    f"-I{REPO / 'fhe-spear_amd/csrc'}", str(REPO / "tools/debug/wl_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout


def _sm64(x):
    M = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & M
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
    return x ^ (x >> 31)


def test_seeded_key_sampler_spec(orc):
    """Switching-key `a` components are regenerated on the GPU from a seed (fhs_modarith.h
    seeded_uniform_x); the oracle's sampler must follow the written spec exactly, including the
    rejection path (forced here with q just above a power of two, so about half the tries reject)."""
    from oracle.oracle import seeded_uniform
    G, M = 0x9E3779B97F4A7C15, (1 << 64) - 1

    def spec(key, pi, n, q):
        bits = q.bit_length()
        kx = (key + (((pi << 20) | n) * G)) & M
        m = 0
        while True:
            v = _sm64((kx + ((m << 40) * G)) & M) >> (64 - bits)
            if v < q:
                return v
            m += 1

    q59 = orc.create_coeff_modulus(16384, [59] * 2)[0]
    for q in (q59, (1 << 58) + 3, 97):
        for key in (0, 1, 0xDEADBEEFCAFEF00D):
            for pi, n in ((0, 0), (3, 1), (38, 16383), (5, 777)):
                assert seeded_uniform(key, pi, n, q) == spec(key, pi, n, q)


def test_chacha20_rfc8439_block_vector(orc):
    """The secret-randomness PRF is ChaCha20: RFC 8439 §2.3.2 test vector
    (key 00..1f, nonce 00:00:00:09:00:00:00:4a:00:00:00:00, block counter 1)."""
    out = orc.chacha20_block(bytes(range(32)), 1, bytes.fromhex("000000090000004a00000000"))
    assert out.hex() == ("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
                         "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def _sm64_inverse(z):
    """Inverse of SplitMix64's finaliser (the round-1 sampler), used to run the ADVICE r1 attack."""
    M = (1 << 64) - 1

    def unxorshift(x, k):
        y = x
        for _ in range(64 // k + 1):
            y = x ^ (y >> k)
        return y & M
    z = unxorshift(z, 31)
    z = (z * pow(0x94D049BB133111EB, -1, 1 << 64)) & M
    z = unxorshift(z, 27)
    z = (z * pow(0xBF58476D1CE4E5B9, -1, 1 << 64)) & M
    z = unxorshift(z, 30)
    return (z - 0x9E3779B97F4A7C15) & M


def test_switching_key_seeds_do_not_reveal_the_secret_key(orc):
    """round 1 stored each a_j seed as sm64(sk_seed ^ sm64(stream)), so inverting
    SplitMix64 on a published key gave sk.  The seeds are now ChaCha20 outputs under the 256-bit
    secret key: the same inversion yields nothing that regenerates s, and the key has 256 bits
    (two keys sharing their low 64 bits differ)."""
    from oracle.oracle import Oracle, _sm64_for_tests
    N, primes, P = 1024, [int(q) for q in orc.create_coeff_modulus(1024, [40] * 4)], 1
    o = Oracle(N, primes, P)
    seed = 0x1234_5678_9ABC_DEF0_0FED_CBA9_8765_4321_1122_3344_5566_7788_99AA_BBCC_DDEE_FF00
    s = o.gen_secret(seed)
    elt = orc.galois_elt(1, N)
    stream = (4 << 56) | (elt << 16)
    assert _sm64_inverse(_sm64_for_tests(0x0123456789ABCDEF)) == 0x0123456789ABCDEF   # the inverse is right
    seeds = o.switch_key_seeds(seed, stream)
    for j, sj in enumerate(seeds):
        guess = _sm64_inverse(sj) ^ _sm64_for_tests(stream | (2 * j))   # round-1 recovery
        assert not np.array_equal(o.gen_secret(guess), s)
    s_low = o.gen_secret(seed & ((1 << 64) - 1))
    assert not np.array_equal(s_low, s)


@pytest.mark.parametrize("case", ["client_aided_n256", "ffn_replay_n256"])
def test_recorded_reference_calls_replay_on_the_oracle(orc, case):
    """The fixtures the GPU replay tests use (tests/test_golden_replay.py) are self-consistent on
    the CPU: the oracle re-encodes every recorded plaintext to the recorded SHA-256, and re-running
    each recorded BSGS call (baby steps bg:215-220 + loop bg:464-485) on its recorded input gives
    the recorded output limbs."""
    man = json.loads((GOLDEN / "manifest.json").read_text())["cases"][case]
    z = np.load(GOLDEN / man["file"])
    N, P, D = man["N"], man["P"], man["D"]
    o = orc.Oracle(N, [int(q) for q in z["primes"]], P)
    s = o.gen_secret(man["sk_seed"])
    G = int(np.ceil(np.sqrt(D)))
    B = int(np.ceil(D / G))
    baby_keys = {b: o.gen_galois_key(man["sk_seed"], s, orc.galois_elt(b, N)) for b in range(1, G)}
    giant_keys = [None] + [o.gen_galois_key(man["sk_seed"], s, orc.galois_elt(g * G, N)) for g in range(1, B)]
    for i, c in enumerate(man["calls"]):
        l = o.L0 + 1 - c["pt_level"]
        pts = [o.encode(r, c["pt_scale"], l) for r in z[f"c{i}_rows"]]
        assert hashlib.sha256(np.ascontiguousarray(np.stack(pts)).tobytes()).hexdigest() == c["pt_sha256"]
        ct = z[f"c{i}_ct_in"]
        baby = [ct] + [o.rotate(ct, baby_keys[b], b) for b in range(1, G)]
        assert np.array_equal(o.bsgs_loop(baby, pts, giant_keys, G, B, D), z[f"c{i}_out"]), f"call {i}"


def test_bench_digest_recomputed_by_the_oracle(orc):
    """bench.py's parity field compares its output limbs with tests/golden/manifest.json's
    bench_digests, which only the C oracle writes (tests/golden/make_bench_digest.py): the small
    configuration's digest is recomputed here from scratch, and the committed full-size records carry
    the bench's seeds and shapes."""
    sys.path.insert(0, str(GOLDEN))
    import make_bench_digest as mbd
    man = json.loads((GOLDEN / "manifest.json").read_text())["bench_digests"]
    rec = mbd.digest("small", 2)
    assert rec["sha256"] == man["small"]["sha256"]
    import bench
    for cfg in ("cfg2", "cfg1"):
        r = man[cfg]
        N, L0, P, D = mbd.CONFIGS[cfg]
        assert (r["N"], r["L0"], r["P"], r["D"]) == (bench.CONFIGS[cfg]["N"], bench.CONFIGS[cfg]["L0"],
                                                     bench.CONFIGS[cfg]["P"], bench.CONFIGS[cfg]["D"])
        assert (r["sk_seed"], r["input_seed"], r["diag_seed"]) == (bench.SK_SEED, bench.INPUT_SEED, bench.DIAG_SEED)
        assert r["shape"] == [2, L0 - 1, N] and r["key_switch_mode"] == "exact"


def test_cpu_port_matches_oracle(orc):
    """bench.py's CPU baseline (oracle/cpu_port.c: Harvey NTT, Shoup/Barrett, OpenMP) computes the
    oracle's limbs: single non-hoisted rotations at two rings, and the whole small bench matvec
    against the oracle-made digest of tests/golden/manifest.json."""
    from oracle import cpu_port as cp
    for N, L0, P in ((2048, 4, 2), (4096, 6, 3)):
        primes = [int(q) for q in orc.create_coeff_modulus(N, [59] * (L0 + P))]
        o = orc.Oracle(N, primes, P)
        s = o.gen_secret(7)
        ct = o.encrypt_symmetric(7, 0, s, o.random_plaintext(3, 0, L0))
        port = cp.CpuPort(N, primes, P, 2)
        for st in (1, 3, -5):
            k = o.gen_galois_key(7, s, orc.galois_elt(st, N))
            assert np.array_equal(port.rotate(ct, k, st), o.rotate(ct, k, st)), (N, st)
    import bench
    secs, y, _, _ = cp.baseline(4096, 6, 3, 256, reps=1, threads=2, sk_seed=bench.SK_SEED,
                                input_seed=bench.INPUT_SEED, diag_seed=bench.DIAG_SEED)
    man = json.loads((GOLDEN / "manifest.json").read_text())["bench_digests"]
    assert cp.sha256(y) == man["small"]["sha256"]


def test_cpu_port_seal_mode_matches_oracle(orc):
    """The SEAL-convention CPU baseline (bench.py seal_mode.cpu_baseline: cpu_port in SEAL mode, P = 1)
    computes the oracle's SEAL-mode limbs: single rotations and a whole small BSGS matvec (bg:464-485,
    every rotation non-hoisted) against the oracle's own loop."""
    from oracle import cpu_port as cp
    N, L0, P, D, seed = 2048, 5, 1, 36, 9
    primes = [int(q) for q in orc.create_coeff_modulus(N, [59] * (L0 + P))]
    o = orc.Oracle(N, primes, P)
    o.set_key_switch_mode("seal")
    s = o.gen_secret(seed)
    ct = o.encrypt_symmetric(seed, 0, s, o.random_plaintext(3, 0, L0))
    port = cp.CpuPort(N, primes, P, 2, mode="seal")
    for st in (1, 6, -3):
        k = o.gen_galois_key(seed, s, orc.galois_elt(st, N))
        assert np.array_equal(port.rotate(ct, k, st), o.rotate(ct, k, st)), st
    G, B = 6, 6
    pts = [o.random_plaintext(4, k, L0) for k in range(D)]
    bk = {b: o.gen_galois_key(seed, s, orc.galois_elt(b, N)) for b in range(1, G)}
    gk = {g: o.gen_galois_key(seed, s, orc.galois_elt(g * G, N)) for g in range(1, B)}
    baby = [ct] + [o.rotate(ct, bk[b], b) for b in range(1, G)]
    want = o.bsgs_loop(baby, pts, [None] + [gk[g] for g in range(1, B)], G, B, D)
    assert np.array_equal(port.matvec(ct, bk, gk, pts, G, B, D), want)
    with pytest.raises(ValueError):
        cp.CpuPort(N, [int(q) for q in orc.create_coeff_modulus(N, [59] * 6)], 2, 2, mode="seal")


def test_bench_block_projection_check_on_cpu(orc):
    """bench.py's block-leg limb check (cpu_check_block_projection) accepts the oracle's own loop
    output for a recorded call and rejects a one-limb change (small ring, no GPU)."""
    import bench
    N, L0, P, D, seed = 4096, 6, 3, 64, 11
    primes = [int(q) for q in orc.create_coeff_modulus(N, [59] * (L0 + P))]
    o = orc.Oracle(N, primes, P)
    s = o.gen_secret(seed)
    G, B = bench.bsgs_params(D)
    ct = o.encrypt_symmetric(seed, 1, s, o.random_plaintext(5, 0, L0))
    pts = [o.random_plaintext(6, k, L0) for k in range(D)]
    bk = {b: o.gen_galois_key(seed, s, orc.galois_elt(b, N)) for b in range(1, G)}
    gkeys = [None] + [o.gen_galois_key(seed, s, orc.galois_elt(g * G, N)) for g in range(1, B)]
    baby = [ct] + [o.rotate(ct, bk[b], b) for b in range(1, G)]
    want = o.bsgs_loop(baby, pts, gkeys, G, B, D)
    cap = dict(ct_in=ct, ct_out=want, pts=pts, N=N, L0=L0, P=P, D=D, sk_seed=seed)
    assert bench.cpu_check_block_projection(cap)["r_projection_limbs_match_cpu_port"]
    bad = want.copy()
    bad[1, 0, 0] ^= 1
    assert not bench.cpu_check_block_projection(dict(cap, ct_out=bad))["r_projection_limbs_match_cpu_port"]

