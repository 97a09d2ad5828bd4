"""Pure-Python big-int restatement of the dusk-plonk hot path — TEST INFRASTRUCTURE ONLY.

This module is an oracle: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may use it, and only as the checker. The
product path (``dusk_plonk_amd``) never imports it.

What it restates (the code itself lives in un-vendored crates):

* BLS12-381 scalar field ``Fr`` in Montgomery form with R = 2^256.  Pinned by the
  reference: ``src/lib.rs:583-588`` hard-codes Montgomery(-1); ``permutation.rs:311-313``
  builds K1..K3 with ``to_mont_form``.
* ``Fft`` (poly-commit, absent): ``Fft::new(k)`` with ``elements[i] = w^i``
  (``permutation.rs:148,913-946``), ``dft``/``idft`` natural order in and out
  (``permutation.rs:1031-1076`` pins ``idft`` as the exact inverse), ``coset_dft`` /
  ``coset_idft`` over g*H with g = 7 (the Fr multiplicative generator, "assumed",
  SURVEY.md §8c), the nested family w_n = w_8n^8 (``quotient_poly.rs:160``).
  w_k = ROOT_OF_UNITY^(2^(32-k)), ROOT_OF_UNITY = 7^((r-1)/2^32) — the zkcrypto/dusk
  bls12_381 convention.
* ``compute_vanishing_poly_over_coset`` (``key.rs:291``): v_h[i] = (g*w_8n^i)^n - 1.
* G1 of BLS12-381 (y^2 = x^3 + 4 over Fp), the KZG commit = MSM over the SRS prefix
  (``prover.rs:133-136`` etc.), ``PlonkParams::setup`` = [tau^i]G1.

Parity status: r, R and K1..K3 are pinned by reference files; NTT/MSM numeric
outputs are mathematically unique given (w, g, SRS) but no reference test holds
a numeric vector for them ("parity partially unpinned").
"""
from __future__ import annotations

import numpy as np

# --------------------------------------------------------------------------- Fr
R_MOD = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
FR_BITS = 255
FR_R = 1 << 256
FR_RINV = pow(FR_R, -1, R_MOD)
TWO_ADICITY = 32
FR_GENERATOR = 7  # multiplicative generator, also the coset shift g
ROOT_OF_UNITY = pow(FR_GENERATOR, (R_MOD - 1) >> TWO_ADICITY, R_MOD)

# permutation.rs:28-30
K1, K2, K3 = 7, 13, 17

# lib.rs:583-588 — Montgomery(-1), the in-tree pin of R = 2^256
MINUS_ONE_MONT_LIMBS = (0xFFFFFFFD00000003, 0xFB38EC08FFFB13FC,
                        0x99AD88181CE5880F, 0x5BC8F5F97CD877D8)

# --------------------------------------------------------------------------- Fp / G1
P_MOD = int("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f624"
            "1eabfffeb153ffffb9feffffffffaaab", 16)
FP_R = 1 << 384
G1_B = 4
G1_GEN = (
    int("17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac58"
        "6c55e83ff97a1aeffb3af00adb22c6bb", 16),
    int("08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3ed"
        "d03cc744a2888ae40caa232946c5e7e1", 16),
)
G1_WORDS = 13  # x[6], y[6] Montgomery u64 limbs + u64 infinity flag (include/plk.h)


def fr_to_mont(x: int) -> int:
    return (x % R_MOD) * FR_R % R_MOD


def fr_from_mont(x: int) -> int:
    return x * FR_RINV % R_MOD


def fp_to_mont(x: int) -> int:
    return (x % P_MOD) * FP_R % P_MOD


def fp_from_mont(x: int) -> int:
    return x * pow(FP_R, -1, P_MOD) % P_MOD


def omega(k: int) -> int:
    """Primitive 2^k-th root of unity, w_k = ROOT^(2^(32-k))."""
    assert 0 <= k <= TWO_ADICITY
    return pow(ROOT_OF_UNITY, 1 << (TWO_ADICITY - k), R_MOD)


# --------------------------------------------------------------------------- packing
def limbs_to_int(row) -> int:
    v = 0
    for i, w in enumerate(row):
        v |= int(w) << (64 * i)
    return v


def int_to_limbs(v: int, n: int):
    return [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)]


def fr_vec_to_np(vals, mont=True) -> np.ndarray:
    """Canonical Fr ints -> uint64[n,4] (Montgomery form by default, the ABI layout)."""
    out = np.zeros((len(vals), 4), dtype=np.uint64)
    for i, v in enumerate(vals):
        out[i] = int_to_limbs(fr_to_mont(v) if mont else v, 4)
    return out


def fr_vec_from_np(arr: np.ndarray, mont=True):
    arr = np.asarray(arr, dtype=np.uint64).reshape(-1, 4)
    vals = [limbs_to_int(r) for r in arr]
    return [fr_from_mont(v) for v in vals] if mont else vals


def g1_vec_to_np(points) -> np.ndarray:
    """Affine points (None = infinity) -> uint64[n,13] (Montgomery Fp)."""
    out = np.zeros((len(points), G1_WORDS), dtype=np.uint64)
    for i, pt in enumerate(points):
        if pt is None:
            out[i, 12] = 1
        else:
            out[i, 0:6] = int_to_limbs(fp_to_mont(pt[0]), 6)
            out[i, 6:12] = int_to_limbs(fp_to_mont(pt[1]), 6)
    return out


def g1_vec_from_np(arr: np.ndarray):
    arr = np.asarray(arr, dtype=np.uint64).reshape(-1, G1_WORDS)
    pts = []
    for row in arr:
        if int(row[12]) != 0:
            pts.append(None)
        else:
            pts.append((fp_from_mont(limbs_to_int(row[0:6])),
                        fp_from_mont(limbs_to_int(row[6:12]))))
    return pts


# --------------------------------------------------------------------------- PRNG
MASK64 = 0xFFFFFFFFFFFFFFFF


class SplitMix64:
    """SplitMix64 — the synthetic-input PRNG. Seed 8349 = the
    reference tests' seed (tests/boolean.rs:21). Does NOT reproduce Rust StdRng."""

    def __init__(self, seed: int):
        self.state = seed & MASK64

    def next_u64(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def fr(self) -> int:
        """Uniform canonical Fr: 4 words LE, top word masked to 255 bits, rejection."""
        while True:
            v = 0
            for i in range(4):
                v |= self.next_u64() << (64 * i)
            v &= (1 << FR_BITS) - 1
            if v < R_MOD:
                return v


# --------------------------------------------------------------------------- NTT
def dft_naive(coeffs, k: int, inverse=False):
    """O(n^2) definition: v_i = sum_j c_j w^(ij) (natural order), zero-padded to n."""
    n = 1 << k
    c = list(coeffs) + [0] * (n - len(coeffs))
    assert len(c) == n
    w = omega(k)
    if inverse:
        w = pow(w, -1, R_MOD)
    out = []
    for i in range(n):
        wi = pow(w, i, R_MOD)
        acc, x = 0, 1
        for j in range(n):
            acc += c[j] * x
            x = x * wi % R_MOD
        out.append(acc % R_MOD)
    if inverse:
        ninv = pow(n, -1, R_MOD)
        out = [v * ninv % R_MOD for v in out]
    return out


def _fft_rec(a, w):
    n = len(a)
    if n == 1:
        return a[:]
    even = _fft_rec(a[0::2], w * w % R_MOD)
    odd = _fft_rec(a[1::2], w * w % R_MOD)
    out = [0] * n
    t = 1
    h = n // 2
    for i in range(h):
        x = odd[i] * t % R_MOD
        out[i] = (even[i] + x) % R_MOD
        out[i + h] = (even[i] - x) % R_MOD
        t = t * w % R_MOD
    return out


def dft(coeffs, k: int):
    """Fft::dft — forward NTT, natural order, input zero-padded to n = 2^k."""
    n = 1 << k
    c = [v % R_MOD for v in coeffs] + [0] * (n - len(coeffs))
    assert len(c) == n, "input longer than the domain"
    return _fft_rec(c, omega(k))


def idft(values, k: int):
    """Fft::idft — inverse NTT, natural order, scaled by n^-1."""
    n = 1 << k
    v = [x % R_MOD for x in values] + [0] * (n - len(values))
    assert len(v) == n
    out = _fft_rec(v, pow(omega(k), -1, R_MOD))
    ninv = pow(n, -1, R_MOD)
    return [x * ninv % R_MOD for x in out]


def coset_dft(coeffs, k: int, g: int = FR_GENERATOR):
    """Fft::coset_dft — evaluate on g*H: scale c_j by g^j, then dft."""
    c = list(coeffs)
    s = 1
    for j in range(len(c)):
        c[j] = c[j] * s % R_MOD
        s = s * g % R_MOD
    return dft(c, k)


def coset_idft(values, k: int, g: int = FR_GENERATOR):
    """Fft::coset_idft — idft, then scale c_j by g^-j."""
    c = idft(values, k)
    ginv = pow(g, -1, R_MOD)
    s = 1
    for j in range(len(c)):
        c[j] = c[j] * s % R_MOD
        s = s * ginv % R_MOD
    return c


def vanishing_poly_over_coset(k8: int, n: int, g: int = FR_GENERATOR):
    """Fft::compute_vanishing_poly_over_coset(n) on the 2^k8 domain (key.rs:291)."""
    N = 1 << k8
    w = omega(k8)
    gn = pow(g, n, R_MOD)
    wn = pow(w, n, R_MOD)
    out, x = [], gn
    for _ in range(N):
        out.append((x - 1) % R_MOD)
        x = x * wn % R_MOD
    return out


def poly_eval(coeffs, x: int) -> int:
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % R_MOD
    return acc


def ruffini(coeffs, z: int):
    """Synthetic division by (X - z), remainder dropped (zksnarks' Coefficients::ruffini,
    absent crate; called through compute_aggregate_witness): q_(i-1) = c_i + z q_i from the
    top coefficient down. len(q) = len(c) - 1."""
    q = [0] * max(len(coeffs) - 1, 0)
    acc = 0
    for i in range(len(coeffs) - 1, 0, -1):
        acc = (coeffs[i] + z * acc) % R_MOD
        q[i - 1] = acc
    return q


def aggregate_witness(polys, point: int, v: int):
    """PlonkParams::compute_aggregate_witness(&[p_0..p_(k-1)], &point, &v)
    (reference call sites src/prover.rs:422-438 and :444-450): the v-power combination
    sum_i v^i p_i (powers 1, v, v^2, .. in slice order), then ruffini(point). Plain ints."""
    m = max((len(p) for p in polys), default=0)
    acc = [0] * m
    vp = 1
    for p in polys:
        for j, c in enumerate(p):
            acc[j] = (acc[j] + vp * c) % R_MOD
        vp = vp * v % R_MOD
    return ruffini(acc, point)


# --------------------------------------------------------------------------- G1
def _fp_inv(x):
    return pow(x, P_MOD - 2, P_MOD)


def g1_is_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - G1_B) % P_MOD == 0


def jac_from_affine(pt):
    if pt is None:
        return (1, 1, 0)
    return (pt[0], pt[1], 1)


def jac_to_affine(P):
    X, Y, Z = P
    if Z % P_MOD == 0:
        return None
    zi = _fp_inv(Z)
    zi2 = zi * zi % P_MOD
    return (X * zi2 % P_MOD, Y * zi2 * zi % P_MOD)


def jac_double(P):
    X, Y, Z = P
    if Z == 0 or Y == 0:
        return (1, 1, 0)
    A = X * X % P_MOD
    B = Y * Y % P_MOD
    C = B * B % P_MOD
    D = 2 * ((X + B) ** 2 - A - C) % P_MOD
    E = 3 * A % P_MOD
    F = E * E % P_MOD
    X3 = (F - 2 * D) % P_MOD
    Y3 = (E * (D - X3) - 8 * C) % P_MOD
    Z3 = 2 * Y * Z % P_MOD
    return (X3, Y3, Z3)


def jac_add(P, Q):
    X1, Y1, Z1 = P
    X2, Y2, Z2 = Q
    if Z1 == 0:
        return Q
    if Z2 == 0:
        return P
    Z1Z1 = Z1 * Z1 % P_MOD
    Z2Z2 = Z2 * Z2 % P_MOD
    U1 = X1 * Z2Z2 % P_MOD
    U2 = X2 * Z1Z1 % P_MOD
    S1 = Y1 * Z2 * Z2Z2 % P_MOD
    S2 = Y2 * Z1 * Z1Z1 % P_MOD
    if U1 == U2:
        if S1 == S2:
            return jac_double(P)
        return (1, 1, 0)
    H = (U2 - U1) % P_MOD
    I = (2 * H) ** 2 % P_MOD
    J = H * I % P_MOD
    rr = 2 * (S2 - S1) % P_MOD
    V = U1 * I % P_MOD
    X3 = (rr * rr - J - 2 * V) % P_MOD
    Y3 = (rr * (V - X3) - 2 * S1 * J) % P_MOD
    Z3 = ((Z1 + Z2) ** 2 - Z1Z1 - Z2Z2) * H % P_MOD
    return (X3, Y3, Z3)


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P_MOD)


def g1_mul(pt, s: int):
    """Scalar multiplication (double-and-add) -> affine."""
    s %= R_MOD
    acc = (1, 1, 0)
    base = jac_from_affine(pt)
    for bit in bin(s)[2:] if s else "":
        acc = jac_double(acc)
        if bit == "1":
            acc = jac_add(acc, base)
    return jac_to_affine(acc)


def g1_add(p, q):
    return jac_to_affine(jac_add(jac_from_affine(p), jac_from_affine(q)))


def msm_naive(points, scalars):
    """sum_i s_i * P_i by per-point double-and-add (the definition; small N only)."""
    acc = (1, 1, 0)
    for pt, s in zip(points, scalars):
        q = g1_mul(pt, s)
        acc = jac_add(acc, jac_from_affine(q))
    return jac_to_affine(acc)


def msm_pippenger(points, scalars, c: int = 8):
    """Bucket method (unsigned windows) — the restated commit for mid-size N."""
    nwin = (FR_BITS + c - 1) // c
    total = (1, 1, 0)
    jpts = [jac_from_affine(p) for p in points]
    for w in reversed(range(nwin)):
        for _ in range(c):
            total = jac_double(total)
        buckets = [(1, 1, 0)] * (1 << c)
        for P, s in zip(jpts, scalars):
            d = (s >> (w * c)) & ((1 << c) - 1)
            if d:
                buckets[d] = jac_add(buckets[d], P)
        run, acc = (1, 1, 0), (1, 1, 0)
        for b in range((1 << c) - 1, 0, -1):
            run = jac_add(run, buckets[b])
            acc = jac_add(acc, run)
        total = jac_add(total, acc)
    return jac_to_affine(total)


def srs_setup(tau: int, count: int):
    """PlonkParams::setup restated: [tau^i]G1 for i < count (affine)."""
    out = []
    t = 1
    for _ in range(count):
        out.append(g1_mul(G1_GEN, t))
        t = t * tau % R_MOD
    return out


def msm_effective_c(c: int) -> int:
    """srs.hip msm_prepare_srs: a c whose every window would be c - 1 bits wide (c = 18:
    15 x 17 = 255) runs as c - 1."""
    return c - 1 if (c - 1) * ((FR_BITS + c - 1) // c) == FR_BITS else c


def msm_window_layout(c: int):
    """The MSM's window layout (srs.hip msm_prepare_srs, round 5 "balanced windows"): W =
    ceil(255 / c) windows covering exactly 255 bits, the top `narrow` = c W - 255 of them
    c - 1 bits wide with their digits scaled by 2 (table rows pre-divided by 2). Returns
    [(bit offset, width, scale shift)] per window."""
    c = msm_effective_c(c)
    W = (FR_BITS + c - 1) // c
    narrow = c * W - FR_BITS
    out, o = [], 0
    for w in range(W):
        nar = w >= W - narrow
        cw = c - 1 if nar else c
        out.append((o, cw, 1 if nar else 0))
        o += cw
    assert o == FR_BITS
    return out


def msm_bucket_part(points, scalars, c: int, part: int, parts: int):
    """The share of bucket range `part` of `parts` of a signed-digit Pippenger MSM with window
    c (plk_commit_batch_dev_part's definition; a checker for the split, not the reference's
    algorithm): sum over the entries whose bucket |d| - 1 lies in [part, part + 1) x
    2^(c-1) / parts of d * 2^(offset) * P_i, with the scalar first brought to [0, (r-1)/2] (s or
    r - s with the digits' signs flipped) and the windows of msm_window_layout (narrow windows'
    digits scaled by 2 into the bucket range, their table rows divided by 2). The shares of all
    parts sum to sum_i s_i P_i. Each entry's contribution is a multiple of its point, so the
    share is a plain MSM with per-point sums of those multiples (affine result, None =
    identity)."""
    layout = msm_window_layout(c)
    B = 1 << (msm_effective_c(c) - 1)
    lo, hi = part * B // parts, (part + 1) * B // parts
    inv2 = pow(2, -1, R_MOD)
    per_point = []
    for s in scalars:
        s %= R_MOD
        neg = s > (R_MOD - 1) // 2
        h = R_MOD - s if neg else s
        acc, carry = 0, 0
        for o, cw, sh in layout:
            val = (h >> o) & ((1 << cw) - 1)
            d = val + carry
            carry = 1 if d > (1 << (cw - 1)) else 0
            d -= (1 << cw) if carry else 0
            mult = pow(2, o, R_MOD)
            if sh:
                d *= 2
                mult = mult * inv2 % R_MOD
            if d and lo <= abs(d) - 1 < hi:
                acc += (-d if neg else d) * mult
        assert carry == 0
        per_point.append(acc % R_MOD)
    return msm_naive(points, per_point)
