"""The sparse form of tiled slot vectors (fhs_kernels.hip k_enc_period / k_encode / k_ntt_fwd_from_dbl_sp), checked
on the CPU in exact and float arithmetic at small rings -- the identities the GPU path relies on:

1. CKKS encoding: a slot vector of period d = (N/2)/t is the encoding of m(X) = p(X^t), p the encoding of its first
   period in the ring of dimension M = N/t (coefficients off the multiples of t vanish);
2. the encoder's slot positions: bin enc_pos_N[j] >> log t of the N/2-point FFT input is the M-ring's bin enc_pos_M[j]
   (fhs_host.hip builds enc_pos; k_encode's sparse branch shifts it);
3. the NTT: the N-point negacyclic NTT (bit-reversed order, psi the 2N-th root) of p(X^t) is the M-point NTT of p with
   phi = psi^t -- whose bit-reversed twiddle table is the first M entries of psi's -- each value repeated t times.
"""
import numpy as np
import pytest


def _bitrev(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


def _enc_pos(N):
    """fhs_host.hip: ep[j] = bitrev((5^j mod 2N - 1) / 4, log2(N/2))."""
    H, logH = N // 2, (N // 2).bit_length() - 1
    e5, out = 1, []
    for _ in range(H):
        out.append(_bitrev((e5 - 1) // 4, logH))
        e5 = (e5 * 5) % (2 * N)
    return out


def _encode_exact(z, N):
    """m with m(zeta^(5^j)) = z_j for j < N/2 (and conjugates), zeta = exp(i pi / N): the CKKS canonical embedding
    inverse by a direct linear solve (no FFT), as real coefficients."""
    H = N // 2
    zeta = np.exp(1j * np.pi / N)
    roots = [zeta ** pow(5, j, 2 * N) for j in range(H)]
    roots += [np.conj(r) for r in roots]
    V = np.array([[r ** k for k in range(N)] for r in roots])
    vals = np.concatenate([z, np.conj(z)])
    return np.linalg.solve(V, vals).real


@pytest.mark.parametrize("N,t", [(32, 2), (64, 4), (128, 8)])
def test_tiled_vector_encodes_as_p_of_x_to_the_t(N, t):
    rng = np.random.default_rng(N + t)
    M, d = N // t, N // 2 // t
    first = rng.normal(0, 1, d) + 1j * rng.normal(0, 1, d)
    m = _encode_exact(np.tile(first, t), N)
    p = _encode_exact(first, M)
    off = np.arange(N) % t != 0
    assert np.max(np.abs(m[off])) < 1e-9
    assert np.allclose(m[::t], p, atol=1e-9)


@pytest.mark.parametrize("N", [64, 1024, 32768])
def test_sparse_slot_positions_are_the_small_rings(N):
    ep = _enc_pos(N)
    for s in (1, 2, 3):
        M = N >> s
        if M < 4:
            continue
        epm = _enc_pos(M)
        assert [ep[j] >> s for j in range(M // 2)] == epm


def _primitive_2n_root(q, n2):
    """the minimal primitive n2-th root of unity mod q (q = 1 mod n2), as SEAL / the oracle pick psi"""
    order = q - 1
    fac, x, f = set(), order, 2
    while f * f <= x:
        while x % f == 0:
            fac.add(f)
            x //= f
        f += 1
    if x > 1:
        fac.add(x)
    for g in range(2, q):
        if all(pow(g, order // f, q) != 1 for f in fac):
            break
    w = pow(g, order // n2, q)
    best, cur = None, w
    for k in range(1, n2, 2):   # the primitive n2-th roots are w^k, k odd
        best = cur if best is None or cur < best else best
        cur = cur * w * w % q
    return best


def _ntt_negacyclic(a, q, psi):
    """out[j] = a(psi^(2 rev(j) + 1)): the SEAL / Phantom bit-reversed evaluation order"""
    n = len(a)
    bits = n.bit_length() - 1
    out = []
    for j in range(n):
        x = pow(psi, 2 * _bitrev(j, bits) + 1, q)
        acc, xp = 0, 1
        for c in a:
            acc = (acc + c * xp) % q
            xp = xp * x % q
        out.append(acc)
    return out


@pytest.mark.parametrize("N,t", [(32, 2), (64, 4), (64, 8)])
def test_sparse_ntt_is_the_small_ntt_repeated(N, t):
    q = 7681                                  # 7681 = 1 mod 512: an NTT prime for every N here
    assert (q - 1) % (2 * N) == 0
    psi = _primitive_2n_root(q, 2 * N)
    M = N // t
    rng = np.random.default_rng(N * t)
    p = [int(v) for v in rng.integers(0, q, M)]
    spread = [0] * N
    for k, v in enumerate(p):
        spread[k * t] = v
    big = _ntt_negacyclic(spread, q, psi)
    phi = pow(psi, t, q)
    small = _ntt_negacyclic(p, q, phi)
    assert big == [small[j >> (t.bit_length() - 1)] for j in range(N)]
    # the M-point transform's bit-reversed twiddles are the first M of the N-point table
    logN, logM = N.bit_length() - 1, M.bit_length() - 1
    assert [pow(psi, _bitrev(i, logN), q) for i in range(M)] == [pow(phi, _bitrev(i, logM), q) for i in range(M)]
