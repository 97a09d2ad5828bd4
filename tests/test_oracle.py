"""CPU tests: pin the oracle (oracle/pyref.py, oracle/plk_oracle.c) before trusting it.

1. The reference's in-tree known answers: Montgomery(-1) (lib.rs:583-588), K1..K3 in
   Montgomery form (permutation.rs:28-30,311-313), the sigma-encoding KAT
   (permutation.rs:841-947: elements[i] = w^i, encodings w^i * {1,K1,K2,K3}) and the
   grand-product identities that pin idft as the exact natural-order inverse
   (permutation.rs:957-1088).
2. Definitions: the fast Python NTT against the O(n^2) DFT; MSM against double-and-add.
3. The C oracle against the Python restatement and the committed golden fixtures.
"""
import numpy as np
import pytest

import pyref as P


def fr(v):
    return P.fr_vec_to_np([v])[0]


# ------------------------------------------------------------------ reference KATs
def test_montgomery_minus_one_matches_reference():
    # /root/reference/src/lib.rs:584-587
    assert tuple(int(x) for x in P.fr_vec_to_np([P.R_MOD - 1])[0]) == P.MINUS_ONE_MONT_LIMBS


def test_k_constants_and_generator():
    assert (P.K1, P.K2, P.K3) == (7, 13, 17)
    # 7 generates the 2-adic subgroup: ROOT^(2^31) == -1
    assert pow(P.ROOT_OF_UNITY, 1 << 31, P.R_MOD) == P.R_MOD - 1
    for k in range(0, 33):
        w = P.omega(k)
        assert pow(w, 1 << k, P.R_MOD) == 1
        if k:
            assert pow(w, 1 << (k - 1), P.R_MOD) == P.R_MOD - 1
    # nested family w_n = w_8n^8 (quotient_poly.rs:160)
    for k in range(0, 28):
        assert pow(P.omega(k + 3), 8, P.R_MOD) == P.omega(k)


def test_sigma_encoding_kat():
    """permutation.rs:841-947 restated on the oracle's elements/generator."""
    # the wiring of the reference test (var_one..var_four over 4 gates)
    gates = [(1, 1, 2, 4), (2, 1, 2, 4), (3, 3, 1, 4), (2, 1, 3, 4)]
    wires = {}
    for g, ws in enumerate(gates):
        for col, v in enumerate(ws):
            wires.setdefault(v, []).append((col, g))
    n = 4
    sigma = [[(c, i) for i in range(n)] for c in range(4)]
    for v, lst in wires.items():
        for idx, (col, g) in enumerate(lst):
            sigma[col][g] = lst[(idx + 1) % len(lst)]
    w = P.omega(2)
    elems = [pow(w, i, P.R_MOD) for i in range(n)]
    ks = [1, P.K1, P.K2, P.K3]
    enc = [[ks[c] * elems[i] % P.R_MOD for (c, i) in col] for col in sigma]
    w2, w3 = pow(w, 2, P.R_MOD), pow(w, 3, P.R_MOD)
    K1, K2, K3 = P.K1, P.K2, P.K3
    m = lambda a, b: a * b % P.R_MOD  # noqa: E731
    assert enc[0] == [K1, m(w, K2), m(w2, K1), K2]
    assert enc[1] == [m(w, K1), m(w2, K2), m(w3, K2), 1]
    assert enc[2] == [w, w3, m(w3, K1), w2]
    assert enc[3] == [m(w, K3), m(w2, K3), m(w3, K3), K3]


def test_grand_product_identities():
    """permutation.rs:957-1088: z[0] = 1, z(1) = 1, deg z = n-1, z(Xw)*den = z(X)*num."""
    rng = P.SplitMix64(8349)
    k, n = 3, 8
    beta, gamma = rng.fr(), rng.fr()
    wires = [[rng.fr() for _ in range(n)] for _ in range(4)]
    elems = [pow(P.omega(k), i, P.R_MOD) for i in range(n)]
    ks = [1, P.K1, P.K2, P.K3]
    # identity permutation on a random wiring: shift the 'a' column cyclically
    sig = [[ks[c] * elems[i] % P.R_MOD for i in range(n)] for c in range(4)]
    sig[0] = sig[0][1:] + sig[0][:1]
    num, den = [], []
    for i in range(n):
        a = b = 1
        for c in range(4):
            a = a * (wires[c][i] + beta * ks[c] * elems[i] + gamma) % P.R_MOD
            b = b * (wires[c][i] + beta * sig[c][i] + gamma) % P.R_MOD
        num.append(a)
        den.append(b)
    z = [1]
    for i in range(n - 1):
        z.append(z[-1] * num[i] * pow(den[i], -1, P.R_MOD) % P.R_MOD)
    zc = P.idft(z, k)
    assert P.poly_eval(zc, 1) == 1
    assert zc[-1] != 0  # degree n - 1
    for i in range(n - 1):
        lhs = P.poly_eval(zc, elems[i] * P.omega(k) % P.R_MOD) * den[i] % P.R_MOD
        rhs = P.poly_eval(zc, elems[i]) * num[i] % P.R_MOD
        assert lhs == rhs
    # dft(idft(z)) == z: the evaluation at w^i is z[i]
    assert P.dft(zc, k) == z


def test_python_ntt_matches_definition():
    rng = P.SplitMix64(1)
    for k in range(0, 7):
        x = [rng.fr() for _ in range(1 << k)]
        assert P.dft(x, k) == P.dft_naive(x, k)
        assert P.idft(x, k) == P.dft_naive(x, k, inverse=True)
        assert P.coset_idft(P.coset_dft(x, k), k) == x
        # coset_dft(p) evaluates p at g*w^i
        cd = P.coset_dft(x, k)
        for i in range(1 << k):
            pt = 7 * pow(P.omega(k), i, P.R_MOD) % P.R_MOD
            assert cd[i] == P.poly_eval(x, pt)


def test_python_msm_matches_definition():
    pts = P.srs_setup(987654321, 12)
    rng = P.SplitMix64(2)
    sc = [rng.fr() for _ in range(12)]
    expect = None
    for p_, s in zip(pts, sc):
        expect = P.g1_add(expect, P.g1_mul(p_, s))
    assert P.msm_naive(pts, sc) == expect
    assert P.msm_pippenger(pts, sc, 4) == expect
    # SRS structure: [tau^i]G
    assert pts[3] == P.g1_mul(P.G1_GEN, pow(987654321, 3, P.R_MOD))


# ------------------------------------------------------------------ C oracle
def test_c_oracle_field_matches_python(oracle):
    rng = P.SplitMix64(3)
    for _ in range(50):
        a, b = rng.fr(), rng.fr()
        got = oracle.fr_mul(fr(a), fr(b))
        assert P.fr_vec_from_np(got)[0] == a * b % P.R_MOD
    for k in (1, 5, 20, 23, 32):
        w = np.zeros(4, dtype=np.uint64)
        oracle.lib.orc_fr_omega(k, w.ctypes.data)
        assert P.fr_vec_from_np(w)[0] == P.omega(k)


@pytest.mark.parametrize("k", [0, 1, 2, 3, 4, 5, 6, 8, 10])
def test_c_oracle_ntt_golden(oracle, golden, k):
    g = golden["ntt"]
    x = g[f"k{k}_in"]
    assert np.array_equal(oracle.dft(x, k), g[f"k{k}_dft"])
    assert np.array_equal(oracle.idft(x, k), g[f"k{k}_idft"])
    assert np.array_equal(oracle.coset_dft(x, k), g[f"k{k}_coset_dft"])
    assert np.array_equal(oracle.coset_idft(x, k), g[f"k{k}_coset_idft"])
    assert np.array_equal(oracle.dft(g[f"k{k}_part"], k), g[f"k{k}_part_dft"])
    assert np.array_equal(oracle.coset_dft(g[f"k{k}_part"], k), g[f"k{k}_part_coset_dft"])
    assert np.array_equal(oracle.elements(k), g[f"k{k}_elements"])


def test_c_oracle_vanishing_golden(oracle, golden):
    assert np.array_equal(oracle.vanishing(5, 4), golden["ntt"]["vanish_k5_n4"])


def test_c_oracle_srs_and_msm_golden(oracle, golden):
    g = golden["msm"]
    srs = oracle.srs(g["tau"], 64)
    assert np.array_equal(srs, g["srs"])
    for name in ("random", "zeros", "ones", "minus_one", "sparse", "small", "high_bits"):
        assert np.array_equal(oracle.msm(srs, g[f"{name}_scalars"]), g[f"{name}_result"]), name
    for m in (1, 2, 3, 17, 33):
        got = oracle.msm(srs[:m], g["random_scalars"][:m])
        assert np.array_equal(got, g[f"random_prefix{m}_result"])


def test_c_oracle_ntt_roundtrip_mid(oracle):
    from oracle_lib import random_fr
    for k in (12, 14):
        x = random_fr(1 << k, seed=k)
        assert np.array_equal(oracle.idft(oracle.dft(x, k), k), x)
        assert np.array_equal(oracle.coset_idft(oracle.coset_dft(x, k), k), x)


def test_ruffini_restatement_divides():
    """pyref.ruffini is exact division for p(X) - p(z): q(X)(X - z) + p(z) = p(X), and
    aggregate_witness is ruffini of the v-power combination (prover.rs:422-450)."""
    import random
    import pyref as P
    rng = random.Random(3)
    for m in (0, 1, 2, 7, 40):
        c = [rng.randrange(P.R_MOD) for _ in range(m)]
        z = rng.randrange(P.R_MOD)
        q = P.ruffini(c, z)
        assert len(q) == max(m - 1, 0)
        x = rng.randrange(P.R_MOD)
        if m:
            lhs = (P.poly_eval(q, x) * (x - z) + P.poly_eval(c, z)) % P.R_MOD
            assert lhs == P.poly_eval(c, x)
    polys = [[rng.randrange(P.R_MOD) for _ in range(k)] for k in (5, 9, 3)]
    v, z = rng.randrange(P.R_MOD), rng.randrange(P.R_MOD)
    comb = [0] * 9
    for i, p in enumerate(polys):
        for j, cc in enumerate(p):
            comb[j] = (comb[j] + pow(v, i, P.R_MOD) * cc) % P.R_MOD
    assert P.aggregate_witness(polys, z, v) == P.ruffini(comb, z)
