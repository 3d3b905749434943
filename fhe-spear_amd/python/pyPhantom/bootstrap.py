"""CKKS bootstrapping for the MI355X backend: `pyPhantom.ckks_bootstrapper`.

Reference surface (the fork's C++ bootstrapper is un-vendored -- SURVEY.md §2.4, §8c, §8f row 4):
  scripts/bootstrap_generation.py:72-74    ckks_bootstrapper.get_galois_elements(N, 0, level_budget)
  scripts/bootstrap_generation.py:112-116  ckks_bootstrapper(encoder); .setup(ctx, level_budget);
                                           .keygen(ctx, sk); ckks_bootstrapper.get_bootstrap_depth(budget)
  scripts/bootstrap_generation.py:149-154  ct mod-switched down to 2 limbs, then bt.bootstrap(ctx, ct)
  test_fully_enc_bsgs.py:243-262           output "at scale ~ (2^bits)^2, must rescale" once
  paper/main.tex:698, 1138                 CoeffToSlot / EvalMod / SlotToCoeff, level budget [2, 2]
Its limbs are therefore not pinnable (parity unpinned); the algorithm below is the
public CKKS bootstrapping recipe (Cheon-Han-Kim-Kim-Song 2018; the FFT-factored linear transforms
of Chen-Chillotti-Song 2019 evaluated with BSGS; EvalMod as a low-frequency exp(i theta) series
raised to a power of two by repeated squaring, in the spirit of Han-Ki 2020's double angle) laid
out for this library's fused kernels.

Pipeline (n = N/2 slots, q0 = first prime, Delta_in = input scale):
  0. pre-scale (2 limbs -> 1): multiply by the integer c = round(q0 q1 2^-k / Delta_in), rescale
     by q1: the message now sits at Delta' = q0 2^-k, so |m| Delta'/q0 <= |m| 2^-k is small.
  1. ModRaise (fhs_mod_raise): centred lift of the q0 limb to all L0 limbs.  The ciphertext now
     decrypts to t = m' + q0 I, |I| < K; its scale is declared q0 so slot j = E(t/q0)_j.
  2. CoeffToSlot: (1/(2K)) E^-1, factored into budget[0] merged groups of inverse butterflies
     (bit-reversed output order, which SlotToCoeff undoes); each group is one fused BSGS linear
     transform (fhs_linear_transform: hoisted baby steps, giant steps summed before ModDown).
     Unit-magnitude (unnormalised) butterflies; the 1/(2K n) rides on the declared scale so x
     stays at ~2^72 through the key switches, then one integer product brings it to ~q.
  3. real/imaginary split with the conjugation automorphism (Galois element 2N-1) and the exact
     monomial -X^(N/2) (= -i in every slot): re, im hold x/K with x = t/q0 in [-K, K].
  4. EvalMod on both: Chebyshev interpolants of cos and sin of 2 pi K y / 2^r (degree 63, one
     basis, scale-exact Paterson-Stockmeyer split on T_8, T_16, T_32), then r complex squarings
     of w0 = c + i s (exp(2 pi i x / 2^r) -> exp(2 pi i x)): Im = sin(2 pi x) ~ 2 pi m'/q0.
  5. recombine re + i im, SlotToCoeff: (q0 / (2 pi Delta')) E in budget[1] merged butterfly
     groups; the last group is not rescaled and its plaintext scale makes the output scale
     exactly Delta_in * q_next, so the caller's one rescale_to_next (tf:252) returns Delta_in.
K = smallest power of two >= 8 sigma with sigma = sqrt(h/12 + 1/12), h = 2N/3 the expected Hamming
weight of the uniform ternary secret, and r = log2 K - 2 (the interpolant spans 4 cosine periods).
"""
from __future__ import annotations

import math
from fractions import Fraction

import numpy as np

CHEB_DEGREE = 63          # depth 7: babies T_1..T_7 at depth <= 3, leaves at 4, giants T_8, T_16, T_32
CHEB_DEPTH = 7
PRESCALE_BITS = 13        # Delta' = q0 2^-13: sine error (2 pi |m| 2^-13)^2 / 6 relative


# ----------------------------------------------------------------------------- parameters
def slot_exponents(N):
    """g_j = 5^j mod 2N, j < N/2: slot j of a plaintext is m(zeta^{g_j}) / scale."""
    n = N // 2
    g = np.empty(n, dtype=np.int64)
    e = 1
    for j in range(n):
        g[j] = e
        e = (e * 5) % (2 * N)
    return g


def mod_bound(N):
    """K: |I| < K for t = m' + q0 I after ModRaise, I ~ sum of ~2N/3 uniforms in [-1/2, 1/2)."""
    sigma = math.sqrt((2.0 * N / 3.0 + 1.0) / 12.0)
    return 1 << max(1, math.ceil(math.log2(8.0 * sigma)))


def double_angles(N):
    """r: the Chebyshev interpolant covers K / 2^r = 4 periods of the cosine (degree 63 reaches
    ~1e-14 there), the r doublings amplify its error (and the noise) by <= 4^r."""
    return max(1, int(round(math.log2(mod_bound(N)))) - 2)


def split_budget(logn, groups):
    """Stages (log2 of half block size, 0..logn-1) split into `groups` contiguous runs, sizes as even
    as possible, the larger runs on the low (small-stride) stages."""
    groups = max(1, min(int(groups), logn))
    base, extra = divmod(logn, groups)
    sizes = [base + (1 if i < extra else 0) for i in range(groups)]
    runs, s = [], 0
    for z in sizes:
        runs.append(list(range(s, s + z)))
        s += z
    return runs


def bootstrap_depth(N, level_budget):
    """Levels consumed by bootstrap() plus the caller's one rescale_to_next (tf:252):
    CoeffToSlot groups (+1: the scale-down product after them, see setup) + Chebyshev (7)
    + r double angles + SlotToCoeff groups."""
    return int(level_budget[0]) + 1 + CHEB_DEPTH + double_angles(N) + int(level_budget[1])


# ----------------------------------------------------------------------------- special FFT
def butterfly(N, h, inverse):
    """Stage with half block size h (block m = 2h) of E = B^(n) ... B^(2) P_bitrev as a diagonal
    form {offset: vector}: y = sum_o d_o * rot(x, o), rot(x, o)_j = x_{(j+o) mod n}.
    Forward: y_p = x_p + w_j x_{p+h}, y_{p+h} = x_p - w_j x_{p+h} (p = block start + j, j < h),
    w_j = exp(2 pi i (5^j mod 4m) / 4m)."""
    n = N // 2
    m = 2 * h
    p = np.arange(n)
    j = p % m
    first = j < h
    jj = np.where(first, j, j - h)
    w = np.exp(2j * np.pi * ((slot_exponents(N)[jj] % (4 * m)) / (4.0 * m)))
    if not inverse:
        a = np.where(first, 1.0 + 0j, -w)
        b = np.where(first, w, 0j)
        c = np.where(first, 0j, 1.0 + 0j)
    else:
        a = np.where(first, 0.5 + 0j, -0.5 / w)
        b = np.where(first, 0.5 + 0j, 0j)
        c = np.where(first, 0j, 0.5 / w)
    out = {0: a}
    out[h % n] = out.get(h % n, 0) + b
    out[(-h) % n] = out.get((-h) % n, 0) + c
    return out


def compose(second, first, n):
    """Diagonal form of (second o first)."""
    out = {}
    for o2, d2 in second.items():
        for o1, d1 in first.items():
            o = (o1 + o2) % n
            v = d2 * np.roll(d1, -o2)
            out[o] = out[o] + v if o in out else v
    return out


def apply_diag(diags, x):
    n = x.shape[0]
    y = np.zeros(n, dtype=np.complex128)
    for o, d in diags.items():
        y += d * np.roll(x, -o)
    return y


def stc_groups(N, budget):
    """SlotToCoeff (bit-reversed coefficients -> slots) as merged diagonal forms, application order."""
    n, logn = N // 2, int(math.log2(N // 2))
    mats = []
    for run in split_budget(logn, budget):
        M = None
        for s in run:                     # h = 2^s, applied smallest first
            B = butterfly(N, 1 << s, False)
            M = B if M is None else compose(B, M, n)
        mats.append(M)
    return mats


def cts_groups(N, budget):
    """CoeffToSlot (slots -> bit-reversed coefficients, E^-1 without P_bitrev) in application order."""
    n, logn = N // 2, int(math.log2(N // 2))
    mats = []
    for run in reversed(split_budget(logn, budget)):
        M = None
        for s in reversed(run):           # largest block first
            B = butterfly(N, 1 << s, True)
            M = B if M is None else compose(B, M, n)
        mats.append(M)
    return mats


def bitrev_perm(n):
    bits = int(math.log2(n))
    return np.array([int(format(i, f"0{bits}b")[::-1], 2) if bits else 0 for i in range(n)])


def embed(N, v):
    """E(v)_j = sum_i v_i zeta^{g_j i} (i < n): the decode map (slots) of coefficient pairs
    v_i = m_i + i m_{i+n}.  Via one 2N-point FFT."""
    n = N // 2
    buf = np.zeros(2 * N, dtype=np.complex128)
    buf[:n] = v
    F = np.fft.ifft(buf) * (2 * N)    # sum_i v_i exp(+2 pi i k i / 2N)
    return F[slot_exponents(N)]


# ----------------------------------------------------------------------------- BSGS layout
class LinearStage:
    """One merged group as a fused BSGS call: baby steps rot(x, b delta), b in [b_lo, b_lo + G);
    giant groups g (identity group first); plaintext (g, b) = rot(d_{(gG+b) delta}, -gG delta)."""

    def __init__(self, N, diags, scale_factor=1.0):
        n = N // 2
        self.N, self.n = N, n
        offs = sorted(diags)
        signed = [o if o <= n // 2 else o - n for o in offs]
        nz = [abs(s) for s in signed if s]
        delta = 0
        for s in nz:
            delta = math.gcd(delta, s)
        delta = delta or 1
        ks = {s // delta: diags[o] * scale_factor for s, o in zip(signed, offs)}
        kmin, kmax = min(ks), max(ks)
        best = None
        for lg in range(0, 7):            # G <= 64 (k_bsgs_inner's LDS slice)
            G = 1 << lg
            b_lo = -(G // 2)
            groups = sorted({(k - b_lo) // G for k in ks})
            cost = (G - 1) + 3 * (len(groups) - 1)    # a giant step costs its own ModUp
            if best is None or cost < best[0]:
                best = (cost, G, b_lo, groups)
        _, G, b_lo, groups = best
        groups.sort(key=lambda g: (g != 0, g))        # identity group first (kernel convention)
        if groups[0] != 0:
            groups.insert(0, 0)
        self.delta, self.G, self.b_lo, self.groups = delta, G, b_lo, groups
        self.baby_steps = [(b_lo + i) * delta for i in range(G)]
        self.giant_steps = [g * G * delta for g in groups]
        zero = np.zeros(n, dtype=np.complex128)
        vals = []
        for g in groups:
            for i in range(G):
                k = g * G + b_lo + i
                d = ks.get(k)
                vals.append(zero if d is None else np.roll(d, g * G * delta))
        self.values = np.array(vals)                  # (len(groups) * G, n)

    def rotation_steps(self):
        return [s for s in self.baby_steps if s % self.n] + [s for s in self.giant_steps if s % self.n]

    def apply(self, x):
        """Float model of the fused call (test helper)."""
        babies = [np.roll(x, -s) for s in self.baby_steps]
        y = np.zeros(self.n, dtype=np.complex128)
        for gi, (g, gs) in enumerate(zip(self.groups, self.giant_steps)):
            inner = sum(self.values[gi * self.G + i] * babies[i] for i in range(self.G))
            y += np.roll(inner, -gs)
        return y


def galois_steps(N, level_budget):
    """Rotation steps (signed) every linear stage of the bootstrap uses."""
    steps = set()
    for M in cts_groups(N, level_budget[0]) + stc_groups(N, level_budget[1]):
        steps.update(LinearStage(N, M).rotation_steps())
    return sorted(steps)


# ----------------------------------------------------------------------------- EvalMod polynomial
def evalmod_coeffs(N, degree=CHEB_DEGREE):
    """Chebyshev interpolants (y in [-1, 1]) of cos and sin of a y, a = 2 pi K / 2^r: the real and
    imaginary parts of w0 = exp(2 pi i x / 2^r) for x = K y.  Parities are exact (odd / even
    coefficients zeroed), so each polynomial uses half of the leaf products."""
    K, r = mod_bound(N), double_angles(N)
    a = 2 * np.pi * K / (1 << r)
    cc = np.polynomial.chebyshev.chebinterpolate(lambda y: np.cos(a * y), degree)
    cs = np.polynomial.chebyshev.chebinterpolate(lambda y: np.sin(a * y), degree)
    cc[1::2] = 0.0
    cs[0::2] = 0.0
    return cc, cs


def cheb_split(c, m):
    """p = L + T_m H for deg p < 2m: T_{m+j} = 2 T_m T_j - T_{m-j} (j >= 1), T_m = T_m T_0."""
    c = list(c) + [0.0] * (2 * m - len(c))
    H = [c[m]] + [2.0 * c[m + j] for j in range(1, m)]
    L = list(c[:m])
    for j in range(1, m):
        L[m - j] -= c[m + j]
    return L, H


def exact_round(x):
    """round half away from zero of a double, exactly (std::round); an int."""
    f = Fraction(float(x))
    return math.floor(f + Fraction(1, 2)) if f >= 0 else -math.floor(-f + Fraction(1, 2))


# ----------------------------------------------------------------------------- the bootstrapper
class Bootstrapper:
    """Backend-agnostic orchestration; `_ph` is the pyPhantom-shaped module whose ops run it
    (pyPhantom on the GPU; tests also run it over the CPU oracle shim for limb parity)."""

    _ph = None

    def __init__(self, encoder):
        self.encoder = encoder
        self.ctx = None
        self.level_budget = None

    # -- static surface (bg:73, bg:115)
    @staticmethod
    def get_galois_elements(N, slots=0, level_budget=(2, 2)):
        """Galois elements bootstrap() needs: the CoeffToSlot / SlotToCoeff BSGS rotations and
        conjugation (2N-1).  `slots` = 0 or N/2 (full packing; sparse packing is not implemented)."""
        N = int(N)
        if slots not in (0, None, N // 2):
            raise ValueError("ckks_bootstrapper: only full slot packing (slots = 0 or N/2) is supported")
        elts = {(pow(5, s % (N // 2), 2 * N)) for s in galois_steps(N, level_budget)}
        elts.add(2 * N - 1)
        return sorted(elts)

    @staticmethod
    def get_bootstrap_depth(level_budget=(2, 2), N=16384):
        return bootstrap_depth(N, level_budget)

    # -- setup (bg:113): plans and plaintexts
    def setup(self, ctx, level_budget=(2, 2)):
        ph = self._ph
        self.ctx = ctx
        self.level_budget = [int(level_budget[0]), int(level_budget[1])]
        N, L0 = ctx.N, ctx.L0
        self.N, self.n = N, N // 2
        self.K, self.r = mod_bound(N), double_angles(N)
        depth = bootstrap_depth(N, self.level_budget)
        if L0 < depth + 1:
            raise ValueError(f"ckks_bootstrapper: L0 = {L0} data primes cannot hold a bootstrap of depth {depth}")
        self.primes = [int(q) for q in ctx.primes]
        self.q0 = self.primes[0]
        self.cheb = evalmod_coeffs(N)
        # CoeffToSlot: (1/(2K)) E^-1 = E^H / (2K n).  Key-switching noise is absolute (~2^10 per
        # coefficient), and CtS's output x/(2K) carries x (|x| < K) whose error EvalMod and the
        # message ratio amplify by 2 pi 2^k sqrt(n): so the transform runs with unit-magnitude
        # (unnormalised) butterflies and the 1/(2K n) is carried by the declared scale of the
        # ModRaised ciphertext (q0 2K n, an exact power-of-two multiple): x sits at scale ~2^72
        # through every CtS key switch.  One exact integer constant product + rescale then brings
        # the scale back to ~q before EvalMod (the bootstrap's one extra level).
        self.cts = []
        ci = 1
        logn = int(math.log2(self.n))
        runs = list(reversed(split_budget(logn, self.level_budget[0])))
        for gi, M in enumerate(cts_groups(N, self.level_budget[0])):
            st = LinearStage(N, M, 2.0 ** len(runs[gi]))
            st.ci = ci
            st.pt_scale = float(self._q_drop(ci))
            st.pts = self._encode_stage(st)
            self.cts.append(st)
            ci += 1
        self.ci_scale_down = ci
        ci += 1
        self.ci_evalmod = ci
        ci_end = ci + CHEB_DEPTH + self.r              # Chebyshev + double angles
        # SlotToCoeff: (q0 / (2 pi Delta'_nom)) E, Delta'_nom = q0 2^-k (the constant rides on the
        # last group; bootstrap() corrects the output scale by Delta'/Delta'_nom exactly)
        self.stc_const = float(2.0 ** PRESCALE_BITS / (2 * np.pi))
        self.stc = []
        groups = stc_groups(N, self.level_budget[1])
        for gi, M in enumerate(groups):
            last = gi == len(groups) - 1
            st = LinearStage(N, M, self.stc_const if last else 1.0)
            st.ci = ci_end + gi
            st.last = last
            st.pt_scale = float(self._q_drop(st.ci))
            st.pts = self._encode_stage(st)
            self.stc.append(st)
        self.ci_out = ci_end + len(groups) - 1
        # exact monomials +-X^(N/2) (= +-i in every slot) at the split / recombination levels
        self.pt_minus_i = self.encoder.encode_complex_vector(ctx, np.full(self.n, -1j), 1.0,
                                                             chain_index=self.ci_scale_down)
        self.pt_plus_i = self.encoder.encode_complex_vector(ctx, np.full(self.n, 1j), 1.0, chain_index=ci_end)
        return self

    def keygen(self, ctx, sk):
        """bg:114: relinearisation key and the bootstrap Galois keys."""
        self.rlk = sk.gen_relinkey(ctx)
        self.gk = sk.create_galois_keys(ctx, self.get_galois_elements(ctx.N, 0, self.level_budget))
        return self

    def _q_drop(self, ci):
        """prime removed by rescale_to_next from chain index ci (L0 + 1 - ci limbs)."""
        return self.primes[self.ctx.L0 - ci]

    def _encode_stage(self, st):
        return self.encoder.encode_complex_vector_batch(self.ctx, st.values, st.pt_scale, chain_index=st.ci,
                                                        precise=True)

    # -- building blocks over the backend
    def _linear(self, ct, st, pts, rescale=True):
        ph, ctx = self._ph, self.ctx
        steps = [s for s in st.baby_steps if s % self.n]
        rot = iter(ph.hoisting(ctx, ct, self.gk, steps)) if steps else iter(())
        babies = [ct if s % self.n == 0 else next(rot) for s in st.baby_steps]
        elts = [1 if s % self.n == 0 else pow(5, s % self.n, 2 * self.N) for s in st.giant_steps]
        return ph.linear_transform(ctx, babies, pts, st.G, elts, self.gk, rescale)

    def _mul(self, a, b):
        ph, ctx = self._ph, self.ctx
        ci = max(a.chain_index(), b.chain_index())
        if a.chain_index() < ci:
            a = ph.mod_switch_to(ctx, a, ci)
        if b.chain_index() < ci:
            b = ph.mod_switch_to(ctx, b, ci)
        return ph.rescale_to_next(ctx, ph.relinearize(ctx, ph.multiply(ctx, a, b), self.rlk))

    def _scalar(self, a, value, ci, scale):
        """value * a landing exactly at (chain index ci, scale): one constant product + rescale."""
        ph, ctx = self._ph, self.ctx
        if a.chain_index() > ci - 1:
            raise ValueError("bootstrap: scalar product target level too low")
        if a.chain_index() < ci - 1:
            a = ph.mod_switch_to(ctx, a, ci - 1)
        r = ph.rescale_to_next(ctx, ph.multiply_const(ctx, a, float(value),
                                                      scale * self._q_drop(ci - 1) / a.scale()))
        r.set_scale(scale)
        return r

    def _align(self, a, ci, scale):
        if a.chain_index() == ci and abs(a.scale() - scale) <= 1e-9 * scale:
            return a
        return self._scalar(a, 1.0, ci, scale)

    def _cheb_basis(self, y):
        T = {1: y}

        def get(k):
            if k in T:
                return T[k]
            a = 1 << (k.bit_length() - 1) if k & (k - 1) else k // 2   # split k = a + b, a >= b
            b = k - a
            if a == b:
                P = self._mul(get(a), get(a))
                P2 = self._ph.add(self.ctx, P, P)
                T[k] = self._ph.add_const(self.ctx, P2, -1.0)
            else:
                P = self._mul(get(a), get(b))
                P2 = self._ph.add(self.ctx, P, P)
                T[k] = self._ph.sub(self.ctx, P2, self._align(get(a - b), P2.chain_index(), P2.scale()))
            return T[k]

        for k in (2, 3, 4, 5, 6, 7, 8, 16, 32):
            get(k)
        return T

    def _cheb_eval(self, c, T, ci, scale):
        """sum_k c_k T_k landing exactly at (ci, scale)."""
        ph, ctx = self._ph, self.ctx
        deg = len(c) - 1
        while deg > 0 and c[deg] == 0.0:
            deg -= 1
        if deg < 8:
            acc = None
            for k in [k for k in range(1, deg + 1) if c[k] != 0.0] or [1]:
                t = self._scalar(T[k], c[k] if k <= deg else 0.0, ci, scale)
                acc = t if acc is None else ph.add(ctx, acc, t)
            return ph.add_const(ctx, acc, float(c[0])) if c[0] != 0.0 else acc
        m = 1 << (deg.bit_length() - 1)               # largest power of two <= deg (>= 8)
        L, H = cheb_split(c[:deg + 1], m)
        Tm = T[m]
        h = self._cheb_eval(H, T, ci - 1, scale * self._q_drop(ci - 1) / Tm.scale())
        P = self._mul(h, Tm)
        P.set_scale(scale)
        return ph.add(ctx, P, self._cheb_eval(L, T, ci, scale))

    def _evalmod(self, y):
        """sin(2 pi x) for y = x / K: w0 = cos + i sin of 2 pi x / 2^r from two Chebyshev series on
        one basis, then r complex squarings (c, s) -> ((c + s)(c - s), 2 c s).  Squaring on the
        unit circle amplifies an error by 2 per step, where the cosine double angle 2c^2 - 1
        amplifies it by up to 4: 2^r instead of 4^r on everything before (measured 2^21 total)."""
        ph, ctx = self._ph, self.ctx
        cc, cs = self.cheb
        if hasattr(ph, "bootstrap_evalmod"):      # the same op sequence, orchestrated in the library
            return ph.bootstrap_evalmod(ctx, y, self.rlk, cc, cs, self.r, CHEB_DEPTH)
        T = self._cheb_basis(y)
        ci = y.chain_index() + CHEB_DEPTH
        c = self._cheb_eval(list(cc), T, ci, y.scale())
        s = self._cheb_eval(list(cs), T, ci, y.scale())
        for step in range(self.r):
            P = self._mul(c, s)
            if step < self.r - 1:
                c = self._mul(ph.add(ctx, c, s), ph.sub(ctx, c, s))
            s = ph.add(ctx, P, P)
        return s

    # -- stages of bootstrap() (separate so tools/debug/bootstrap_stages.py can audit each)
    def _prescale(self, ct):
        """2 limbs at Delta_in -> 1 limb at Delta' = Delta_in c / q1 ~ q0 2^-k (exact integer c)."""
        ph, ctx = self._ph, self.ctx
        l = ct.coeff_modulus_size()
        if l < 2:
            raise ValueError("ckks_bootstrapper: input needs at least 2 limbs (q0 q1) for the pre-scale step")
        x = ph.mod_switch_to(ctx, ct, ctx.L0 - 1) if l > 2 else ct
        q0, q1 = self.primes[0], self.primes[1]
        c = exact_round(q0 * (q1 / ct.scale()) * 2.0 ** -PRESCALE_BITS)
        return ph.rescale_to_next(ctx, ph.multiply_const(ctx, x, 1.0, float(c)))

    def _mod_raise(self, x):
        """decrypts to t = m' + q0 I; declared scale q0 2K n so slot j = E(t / q0)_j / (2K n)."""
        r = self._ph.mod_raise(self.ctx, x)
        r.set_scale(float(self.q0) * 2 * self.K * self.n)
        return r

    def _coeff_to_slot(self, x):
        """-> bit-reversed (x_lo + i x_hi) / (2K) (x = t / q0), still at the high scale ~q0 2K n."""
        for st in self.cts:
            x = self._linear(x, st, st.pts, True)
        return x

    def _split(self, x):
        """-> (x_lo / K, x_hi / K) as real slot vectors at scale ~q0: conjugation and the exact
        monomial -X^(N/2) at the high scale (the conjugation's key switch noise is absolute), then
        one exact integer constant product + rescale each (no forced nominal scale: a 2^-38
        bookkeeping error would be 2^-30 on x)."""
        ph, ctx = self._ph, self.ctx
        conj = ph.apply_galois(ctx, x, 2 * self.N - 1, self.gk)
        re = ph.add(ctx, x, conj)
        im = ph.multiply_plain(ctx, ph.sub(ctx, x, conj), self.pt_minus_i)
        k = exact_round(self.q0 * (self._q_drop(x.chain_index()) / x.scale()))
        return tuple(ph.rescale_to_next(ctx, ph.multiply_const(ctx, v, 1.0, float(k))) for v in (re, im))

    def _slot_to_coeff(self, re, im, d_prime):
        ph, ctx = self._ph, self.ctx
        y = ph.add(ctx, re, ph.multiply_plain(ctx, im, ph.mod_switch_to(ctx, self.pt_plus_i, im.chain_index())))
        for st in self.stc:
            if y.chain_index() != st.ci:
                y = ph.mod_switch_to(ctx, y, st.ci)
            y = self._linear(y, st, st.pts, not st.last)
        # the last group is not rescaled (output at ~Delta^2, tf:250-252 rescales); the nominal
        # SlotToCoeff constant assumed Delta' = q0 2^-k: fold the exact ratio into the scale
        y.set_scale(y.scale() * d_prime / (self.q0 * 2.0 ** -PRESCALE_BITS))
        return y

    # -- over ranks (SURVEY.md §8e Config 5): the CoeffToSlot / SlotToCoeff transforms sharded
    def _linear_ranks(self, x, st, rescale, dist, device, ranks, group):
        """_linear with its giant groups split over `ranks` (fhespear_dist.linear_transform_sharded): x on
        ranks[0] (None elsewhere) is broadcast, every rank rotates the baby steps and sums its groups,
        the partial sums meet on ranks[0].  The same limbs as _linear."""
        import fhespear_dist as fd
        ph, ctx = self._ph, self.ctx
        x = fd.broadcast_ciphertext(ph, ctx, x, ranks[0], dist, device, group)
        steps = [s for s in st.baby_steps if s % self.n]
        rot = iter(ph.hoisting(ctx, x, self.gk, steps)) if steps else iter(())
        babies = [x if s % self.n == 0 else next(rot) for s in st.baby_steps]
        elts = [1 if s % self.n == 0 else pow(5, s % self.n, 2 * self.N) for s in st.giant_steps]
        if getattr(st, "zero_pts", None) is None:   # the identity group of a rank that has another's groups
            st.zero_pts = self.encoder.encode_complex_vector_batch(ctx, np.zeros((st.G, self.n)), st.pt_scale,
                                                                   chain_index=st.ci)
        return fd.linear_transform_sharded(ph, ctx, babies, st.pts, st.G, elts, self.gk, rescale, st.zero_pts, dist,
                                           device, ranks, group)

    def bootstrap_ranks(self, ctx, ct, dist, device, ranks=None, group=None):
        """bootstrap() over the ranks of `group` (global ranks `ranks`, default all): ct on ranks[0], None
        elsewhere; every rank calls.  The pre-scale, ModRaise, conjugation split and EvalMod run on ranks[0];
        each CoeffToSlot / SlotToCoeff linear stage is one fused transform whose giant groups are dealt over
        the ranks.  Returns the bootstrapped ciphertext on ranks[0] (None elsewhere), limb-identical to
        bootstrap()."""
        if self.ctx is None:
            raise ValueError("ckks_bootstrapper: call setup() and keygen() first")
        ph = self._ph
        ranks = list(range(dist.get_world_size())) if ranks is None else list(ranks)
        root = dist.get_rank() == ranks[0]
        x = d_prime = None
        if root:
            x = self._prescale(ct)
            d_prime = x.scale()
            x = self._mod_raise(x)
        for st in self.cts:
            x = self._linear_ranks(x, st, True, dist, device, ranks, group)
        y = None
        if root:
            re, im = self._split(x)
            re, im = self._evalmod(re), self._evalmod(im)
            y = ph.add(self.ctx, re, ph.multiply_plain(self.ctx, im,
                                                        ph.mod_switch_to(self.ctx, self.pt_plus_i, im.chain_index())))
        for st in self.stc:
            if root and y.chain_index() != st.ci:
                y = ph.mod_switch_to(self.ctx, y, st.ci)
            y = self._linear_ranks(y, st, not st.last, dist, device, ranks, group)
        if not root:
            return None
        y.set_scale(y.scale() * d_prime / (self.q0 * 2.0 ** -PRESCALE_BITS))
        return y

    # -- bg:154
    def bootstrap(self, ctx, ct):
        if self.ctx is None:
            raise ValueError("ckks_bootstrapper: call setup() and keygen() first")
        x = self._prescale(ct)
        d_prime = x.scale()
        x = self._coeff_to_slot(self._mod_raise(x))
        re, im = self._split(x)
        return self._slot_to_coeff(self._evalmod(re), self._evalmod(im), d_prime)
