"""CPU check of the bucket-reduction identities the MSM kernels rely on (msm.hip), with
integers standing in for the bucket sums (the identities are linear, so any abelian group
behaves the same):

* run-sum form (wide bucket sets, k_runsum1/2 + k_bitsum1/2 + host tail):
  sum_b (b+1) S_b = K (sum_r (r+1) Y_r - sum_r Y_r) + sum_r T_r, runs of K buckets,
  Y_r = R_(r,0), T_r = sum_t R_(r,t), R_(r,t) = sum_(t'>=t) S_(rK+t');
* bit-sum form (k_bitsum1/2): sum_u (u+1) S_u = sum_j 2^j T_j with b = 256 g + 16 a + c,
  T_j(g) from row / column sums and the group term (256 g + 1) A_g spread over T_(8+i);
* the top-window-free recoding: signed c-bit digits of a scalar below 2^254 reconstruct it
  with W = ceil(255 / c) windows and never exceed 2^(c-1) (msm.hip digit_at).
"""
import random

import pytest


def weighted(S):
    return sum((b + 1) * s for b, s in enumerate(S))


@pytest.mark.parametrize("K,nruns", [(16, 8), (16, 33), (8, 9), (4, 5), (2, 17)])
def test_run_sum_identity(K, nruns):
    rng = random.Random(K * 1000 + nruns)
    S = [rng.randrange(-10**6, 10**6) if rng.random() > 0.1 else 0 for _ in range(K * nruns)]
    Y, T = [], []
    for r in range(nruns):
        suffix = [sum(S[r * K + t2] for t2 in range(t, K)) for t in range(K)]
        Y.append(suffix[0])
        T.append(sum(suffix))
    assert weighted(S) == K * (weighted(Y) - sum(Y)) + sum(T)


def bitsum_device(S):
    """k_bitsum1 (per group of 256: rows / columns -> T_j(g), A_g) and k_bitsum2."""
    B = len(S)
    G = (B + 255) // 256
    nbits = 8 + (G - 1).bit_length() if G > 1 else 8
    out = []
    for g in range(G):
        sg = [S[256 * g + u] if 256 * g + u < B else 0 for u in range(256)]
        row = [sum(sg[16 * a + c] for c in range(16)) for a in range(16)]
        col = [sum(sg[16 * a + c] for a in range(16)) for c in range(16)]
        t = [sum(col[c] for c in range(16) if (c >> j) & 1) for j in range(4)]
        t += [sum(row[a] for a in range(16) if (a >> i) & 1) for i in range(4)]
        out.append((t, sum(row)))
    T = []
    for j in range(nbits):
        if j < 8:
            T.append(sum(o[0][j] for o in out) + (sum(o[1] for o in out) if j == 0 else 0))
        else:
            T.append(sum(o[1] for g, o in enumerate(out) if (g >> (j - 8)) & 1))
    return sum((1 << j) * T[j] for j in range(nbits))


@pytest.mark.parametrize("B", [256, 1024, 4096])
def test_bitsum_identity(B):
    rng = random.Random(B)
    S = [rng.randrange(-10**6, 10**6) for _ in range(B)]
    assert bitsum_device(S) == weighted(S)


def digits(s, c, W):
    """msm.hip digit_at over all windows (carry threaded)."""
    out, carry = [], 0
    for w in range(W):
        val = (s >> (w * c)) & ((1 << c) - 1) if w * c < 256 else 0
        d = val + carry
        if d > (1 << (c - 1)):
            d -= 1 << c
            carry = 1
        else:
            carry = 0
        out.append(d)
    return out, carry


@pytest.mark.parametrize("c", [8, 10, 13, 15, 16, 17, 20])
def test_signed_recoding(c):
    W = (255 + c - 1) // c
    rng = random.Random(c)
    cases = [0, 1, (1 << 254) - 1, (1 << 253) + 12345] + [rng.randrange(1 << 254) for _ in range(200)]
    for s in cases:
        d, carry = digits(s, c, W)
        assert carry == 0
        assert all(abs(x) <= 1 << (c - 1) for x in d)
        assert sum(x << (w * c) for w, x in enumerate(d)) == s


def run_bits_lone(B, run_lanes=65536, kmax=4, kmin=1):
    """msm.hip run_bits for a lone MSM: the largest rb <= 4 with B >> rb >= 2^16 run lanes."""
    rb = kmax
    while rb > kmin and (B >> rb) < run_lanes:
        rb -= 1
    return rb


def reduce_wide(S):
    """The wide path's reduction of a bucket array as the kernels + host tail compute it:
    run sums (k_runsum1/2), bit sums over the runs (k_bitsum1/2), K (sum (r+1) Y_r - sum Y_r)
    + sum T_r; also returns sum_r Y_r (= sum_b S_b)."""
    B = len(S)
    K = 1 << run_bits_lone(B)
    Y, T = [], []
    for r in range(B // K):
        suffix = [sum(S[r * K + t2] for t2 in range(t, K)) for t in range(K)]
        Y.append(suffix[0])
        T.append(sum(suffix))
    return K * (bitsum_device(Y) - sum(Y)) + sum(T), sum(Y)


@pytest.mark.parametrize("c,parts", [(17, 2), (17, 4), (18, 8), (20, 8), (20, 32)])
def test_bucket_parts_identity(c, parts):
    """msm_run_batch's bucket-range parts (plk_commit_batch_dev_part): part p keeps the digits
    of buckets [b_lo, b_lo + B/parts), b_lo = p B / parts (k_chist / k_cscatter: b - b_lo
    unsigned < B/parts, digit 0 wrapping out of range), reduces them as a wide set of B/parts
    buckets and adds b_lo sum_b S_b on the host; the parts' shares sum to sum_b (b+1) S_b.
    Integers mod r stand in for the points (the identities are linear): the whole MSM
    sum_i s_i P_i with the signed recoding, the scalar halving and the balanced windows
    (srs.hip msm_prepare_srs: the top c W - 255 windows c - 1 bits wide, digits x 2)."""
    rng = random.Random(c * 100 + parts)
    W = (255 + c - 1) // c
    narrow = c * W - 255  # balanced windows: the top `narrow` are c - 1 bits, digits x 2
    r_mod = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    q = r_mod  # the group order: r P = 0 is what makes the scalar halving exact
    n = 40
    P = [rng.randrange(q) for _ in range(n)]
    sc = [rng.randrange(r_mod) for _ in range(n - 4)] + [0, 1, r_mod - 1, (r_mod - 1) // 2 + 1]
    B = 1 << (c - 1)
    inv2 = pow(2, -1, q)
    entries = {}  # bucket -> sum of signed table values
    for s, p in zip(sc, P):
        neg = s > (r_mod - 1) // 2
        h = r_mod - s if neg else s
        o, carry = 0, 0
        for w in range(W):
            nar = w >= W - narrow
            cw = c - 1 if nar else c
            d = ((h >> o) & ((1 << cw) - 1)) + carry
            carry = 1 if d > 1 << (cw - 1) else 0
            d -= (1 << cw) if carry else 0
            tv = pow(2, o, q) * p % q
            if nar:  # digit_at scales a narrow window's digit by 2, its table row is halved
                d *= 2
                tv = tv * inv2 % q
            o += cw
            if d == 0:
                continue
            assert abs(d) <= B
            sign = (d < 0) != neg
            entries[abs(d) - 1] = (entries.get(abs(d) - 1, 0) + (-tv if sign else tv)) % q
        assert o == 255 and carry == 0
    want = sum(s * p for s, p in zip(sc, P)) % q
    Bp = B // parts
    total = 0
    for part in range(parts):
        b_lo = part * Bp
        S = [0] * Bp
        for b, v in entries.items():
            bb = (b - b_lo) & 0xFFFFFFFF  # the kernels' unsigned range test
            if bb < Bp:
                S[bb] = v
        local, ssum = reduce_wide(S)
        assert local == sum((b + 1) * v for b, v in enumerate(S))
        total += local + b_lo * ssum
    assert total % q == want


@pytest.mark.parametrize("c", [8, 10, 13, 15, 16, 17, 18, 19, 20, 22])
def test_balanced_windows_recoding_and_load(c):
    """srs.hip's balanced windows: the signed digits of the layout (oracle/pyref.py
    msm_window_layout) reconstruct every scalar < 2^254 with no final carry, stay within the
    bucket range after the narrow windows' x 2, and — the point of the layout — every run of
    two buckets receives the same expected number of entries (no hot buckets)."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "oracle"))
    import pyref as P
    layout = P.msm_window_layout(c)
    B = 1 << (P.msm_effective_c(c) - 1)
    rng = random.Random(c)
    load = [0] * B
    for s in [0, 1, (1 << 254) - 1] + [rng.randrange(1 << 254) for _ in range(300)]:
        carry, back = 0, 0
        for o, cw, sh in layout:
            d = ((s >> o) & ((1 << cw) - 1)) + carry
            carry = 1 if d > 1 << (cw - 1) else 0
            d -= (1 << cw) if carry else 0
            back += d << o
            b = abs(d << sh) - 1
            assert -1 <= b < B
            if b >= 0:
                load[b] += 1
        assert carry == 0 and back == s
    # expected entries per bucket: a wide window's |d| is uniform on [1, 2^(c-1)], a narrow
    # one's doubled digit lands on odd-indexed buckets only (b = 2|d| - 1): runs of 2 even out
    exp = [0.0] * B
    for o, cw, sh in layout:
        for b in range(B):
            exp[b] += (1.0 / B) if not sh else (2.0 / B if b % 2 == 1 else 0.0)
    runs = [exp[2 * r] + exp[2 * r + 1] for r in range(B // 2)]
    assert max(runs) - min(runs) < 1e-9


def test_balanced_windows_exist_only_for_supported_c():
    """c W - 255 narrow windows need (c - 1) W <= 255: true for every c srs.hip accepts
    (8 .. 20 and 22; choose_c refuses PLK_MSM_C = 21 / 23)."""
    for c in range(8, 24):
        W = (255 + c - 1) // c
        assert ((c - 1) * W <= 255) == (c not in (21, 23)), c
