"""GPU parity of the SRS setup and the MSM / KZG commit (PlonkParams) through the C ABI.

Bit-exact canonical affine outputs against the golden fixtures (Python double-and-add)
and the C oracle (Jacobian Pippenger), over random and skewed scalars, SRS prefixes,
points at infinity; commit's degree error (the reference's negative-test path,
prover.rs:262-265); linearity and [tau]-structure at 2^20 without the oracle.
"""
import numpy as np
import pytest

import pyref as P
from oracle_lib import random_fr

pytestmark = pytest.mark.gpu


def fr_int(v):
    return P.fr_vec_to_np([v])


@pytest.fixture(scope="module")
def srs_small(plk, gpu_ctx, golden):
    return plk.PlonkParams.setup(6, golden["msm"]["tau"], gpu_ctx, n_points=64)


def test_srs_setup_matches_golden(srs_small, golden):
    assert np.array_equal(srs_small.points(), golden["msm"]["srs"])


def test_msm_golden(srs_small, golden):
    g = golden["msm"]
    for name in ("random", "zeros", "ones", "minus_one", "sparse", "small", "high_bits"):
        got = srs_small.msm(g[f"{name}_scalars"]).words
        assert np.array_equal(got, g[f"{name}_result"]), name
    for m in (1, 2, 3, 17, 33):
        got = srs_small.msm(g["random_scalars"][:m]).words
        assert np.array_equal(got, g[f"random_prefix{m}_result"]), m


def test_commit_strips_trailing_zeros_and_errs_past_srs(plk, srs_small, golden):
    g = golden["msm"]
    sc = g["random_scalars"]
    padded = np.concatenate([sc, np.zeros((40, 4), dtype=np.uint64)])
    assert np.array_equal(srs_small.commit(plk.Coefficients(padded)).words, g["random_result"])
    too_long = padded.copy()
    too_long[70] = fr_int(5)[0]
    with pytest.raises(plk.PlonkError) as e:
        srs_small.commit(plk.Coefficients(too_long))
    assert e.value.status == plk.PLK_E_DEGREE
    assert srs_small.commit(plk.Coefficients(np.zeros((0, 4), np.uint64))).is_identity


@pytest.mark.parametrize("logn", [7, 10, 12, 14, 16, 18])
def test_msm_vs_oracle(plk, gpu_ctx, oracle, logn):
    n = 1 << logn
    tau = random_fr(1, seed=logn)[0]
    pp = plk.PlonkParams.setup(logn, tau, gpu_ctx, n_points=n + 8)
    pts = pp.points()
    # logn = 16, 18: c = 17 (15 windows, 2^16 buckets: the wide-set sort and run-sum
    # reduction of msm.hip); below 2^16 the LDS-histogram path (srs.hip choose_c)
    if logn <= 12:  # the SRS itself against the oracle's setup
        assert np.array_equal(pts, oracle.srs(tau, n + 8))
    sc = random_fr(n, seed=1000 + logn)
    assert np.array_equal(pp.msm(sc).words, oracle.msm(pts, sc))
    # skewed scalar sets: all equal, tiny, sparse selector-like, -1
    cases = {
        "all_one": np.tile(fr_int(1), (n, 1)),
        "all_same": np.tile(sc[:1], (n, 1)),
        "tiny": P.fr_vec_to_np([i % 5 for i in range(n)]),
        "sparse": np.where((np.arange(n) % 17 == 0)[:, None], sc, 0).astype(np.uint64),
        "minus_one": np.tile(fr_int(P.R_MOD - 1), (n, 1)),
        # around the half-range recoding boundary (msm.hip scalar_half: s > (r-1)/2 -> r - s)
        "half_boundary": P.fr_vec_to_np([
            [(P.R_MOD - 1) // 2, (P.R_MOD + 1) // 2, (P.R_MOD - 1) // 2 - 1, (P.R_MOD + 3) // 2,
             1 << 253, P.R_MOD - (1 << 253), (1 << 254) - 1, P.R_MOD - 2][i % 8] for i in range(n)]),
    }
    for name, s in cases.items():
        assert np.array_equal(pp.msm(s).words, oracle.msm(pts, s)), name
    # commit over a shorter prefix and with len > n (degree error)
    m = n // 2 + 3
    assert np.array_equal(pp.commit(plk.Coefficients(sc[:m])).words, oracle.msm(pts[:m], sc[:m]))


@pytest.mark.parametrize("tau", [1, P.R_MOD - 1])
def test_msm_repeated_points(plk, gpu_ctx, oracle, tau):
    """tau = 1 makes every SRS point G, tau = -1 alternates G and -G: buckets then receive
    the same point (the accumulation's doubling branch) and a point with its negation (the
    infinity branch) — the exceptional cases of the XYZZ mixed addition."""
    n = 1 << 10
    pp = plk.PlonkParams.setup(10, fr_int(tau)[0], gpu_ctx, n_points=n)
    pts = pp.points()
    sc = random_fr(n, seed=77)
    few = np.tile(random_fr(3, seed=78), (n // 3 + 1, 1))[:n].copy()
    cases = {"random": sc, "all_same": np.tile(sc[:1], (n, 1)), "three_values": few,
             "all_one": np.tile(fr_int(1), (n, 1))}
    for name, s in cases.items():
        assert np.array_equal(pp.msm(s).words, oracle.msm(pts, s)), name


def test_srs_with_infinity_points(plk, gpu_ctx, oracle):
    n = 300
    pp0 = plk.PlonkParams.setup(8, random_fr(1, seed=5)[0], gpu_ctx, n_points=n)
    pts = pp0.points()
    pts[[3, 100, 299]] = 0
    pts[[3, 100, 299], 12] = 1
    pp = plk.PlonkParams.load(pts, gpu_ctx)
    sc = random_fr(n, seed=6)
    assert np.array_equal(pp.msm(sc).words, oracle.msm(pts, sc))


def test_commit_dev_and_stats(plk, gpu_ctx, oracle):
    import torch
    n = 1 << 12
    pp = plk.PlonkParams.setup(12, random_fr(1, seed=11)[0], gpu_ctx, n_points=n + 8)
    sc = random_fr(n + 8, seed=12)
    sc[n:] = 0
    d = torch.from_numpy(sc.view(np.int64)).cuda()
    torch.cuda.synchronize()
    got = pp.commit_dev(d.data_ptr(), n + 8, torch.cuda.current_stream().cuda_stream)
    assert np.array_equal(got.words, oracle.msm(pp.points(), sc))
    ms, adds, c = pp.last_msm_stats()
    assert ms > 0 and adds > 0 and c > 0


@pytest.mark.slow
def test_msm_2_20_vs_oracle(plk, gpu_ctx, oracle):
    """BASELINE configs[2] at its full size: a 2^20-point MSM over the bench SRS (c = 20: 13
    windows of the window table, the wide-bucket sort and run-sum reduction) bit-exact
    against the C oracle's Pippenger, random and sparse scalars."""
    import os
    n = 1 << 20
    pp = plk.PlonkParams.setup(20, random_fr(1, seed=20)[0], gpu_ctx)
    pts = pp.points(0, n)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    sc = random_fr(n, seed=23)
    assert np.array_equal(pp.msm(sc).words, oracle.msm(pts, sc, threads))
    sparse = np.where((np.arange(n) % 29 == 0)[:, None], sc, 0).astype(np.uint64)
    assert np.array_equal(pp.msm(sparse).words, oracle.msm(pts, sparse, threads))


@pytest.mark.slow
def test_msm_2_20_properties(plk, gpu_ctx):
    """2^20: linearity commit(a) + commit(b) == commit(a + b), and commit(e_i) == g1[i]."""
    n = 1 << 20
    pp = plk.PlonkParams.setup(20, random_fr(1, seed=20)[0], gpu_ctx)
    a = random_fr(n, seed=21)
    b = random_fr(n, seed=22)
    ca = pp.commit(plk.Coefficients(a))
    cb = pp.commit(plk.Coefficients(b))
    ai = P.fr_vec_from_np(a[:4])
    # a + b computed limb-wise in Python on the whole vector is slow; use the GPU-free
    # identity sum_i (a_i + b_i) G_i with numpy big-int on object arrays
    ab = np.empty_like(a)
    A = a.astype(object)
    B = b.astype(object)
    va = A[:, 0] + (A[:, 1] << 64) + (A[:, 2] << 128) + (A[:, 3] << 192)
    vb = B[:, 0] + (B[:, 1] << 64) + (B[:, 2] << 128) + (B[:, 3] << 192)
    vs = (va + vb) % P.R_MOD  # Montgomery form is linear
    for j in range(4):
        ab[:, j] = np.array([(int(v) >> (64 * j)) & 0xFFFFFFFFFFFFFFFF for v in vs], dtype=np.uint64)
    cab = pp.commit(plk.Coefficients(ab))
    pa = P.g1_vec_from_np(ca.words)[0]
    pb = P.g1_vec_from_np(cb.words)[0]
    assert P.g1_vec_from_np(cab.words)[0] == P.g1_add(pa, pb)
    assert ai  # keep the prefix decode exercised
    # unit vectors pick single SRS points, including the last one
    for i in (0, 1, 12345, n - 1, n + 7):
        e = np.zeros((i + 1, 4), dtype=np.uint64)
        e[i] = fr_int(1)[0]
        assert np.array_equal(pp.commit(plk.Coefficients(e)).words[:12], pp.points(i, 1)[0, :12])


def test_commit_batch_dev(plk, gpu_ctx, oracle):
    """Independent commits as one batch (the prover's wire / quotient / opening groups):
    different lengths, a zero polynomial, and one slot past the SRS (degree error)."""
    import torch
    n = 1 << 11
    pp = plk.PlonkParams.setup(11, random_fr(1, seed=31)[0], gpu_ctx, n_points=n + 8)
    pts = pp.points()
    lens = [n, n + 3, 17, n // 2, 1, n + 8]
    polys = [random_fr(m, seed=40 + i) for i, m in enumerate(lens)]
    polys[4][:] = 0  # zero polynomial -> identity
    bad = random_fr(n + 20, seed=99)  # longer than the SRS with a non-zero tail
    devs = [torch.from_numpy(p.view(np.int64)).cuda() for p in polys + [bad]]
    torch.cuda.synchronize()
    res = pp.commit_batch_dev([(d.data_ptr(), d.shape[0]) for d in devs],
                              torch.cuda.current_stream().cuda_stream, raise_on_error=False)
    for i, p in enumerate(polys):
        assert np.array_equal(res[i].words, oracle.msm(pts[: p.shape[0]], p)), i
    assert isinstance(res[-1], plk.PlonkError) and res[-1].status == plk.PLK_E_DEGREE
    # more than one batch worth of slots (>16) goes through in chunks
    many = [random_fr(64, seed=200 + i) for i in range(20)]
    dm = [torch.from_numpy(p.view(np.int64)).cuda() for p in many]
    torch.cuda.synchronize()
    out = pp.commit_batch_dev([(d.data_ptr(), 64) for d in dm],
                              torch.cuda.current_stream().cuda_stream)
    for i, p in enumerate(many):
        assert np.array_equal(out[i].words, oracle.msm(pts[:64], p)), i


@pytest.mark.parametrize("c,logn", [(17, 10), (20, 12), (18, 14), (19, 14), (20, 16)])
def test_msm_wide_buckets_vs_oracle(plk, gpu_ctx, oracle, monkeypatch, c, logn):
    """Wide bucket sets (2^(c-1) > 32 K buckets: the two-level radix sort, the per-bin
    counting sort and the run-sum bucket reduction of msm.hip) at small sizes, forced with
    PLK_MSM_C: most buckets empty or single, skewed and adversarial scalar sets, batches."""
    import torch
    monkeypatch.setenv("PLK_MSM_C", str(c))
    n = 1 << logn
    tau = random_fr(1, seed=300 + logn)[0]
    pp = plk.PlonkParams.setup(logn, tau, gpu_ctx, n_points=n + 8)
    pts = pp.points()
    sc = random_fr(n, seed=400 + logn)
    cases = {
        "random": sc,
        "all_one": np.tile(fr_int(1), (n, 1)),
        "all_same": np.tile(sc[:1], (n, 1)),
        "tiny": P.fr_vec_to_np([i % 5 for i in range(n)]),
        "sparse": np.where((np.arange(n) % 17 == 0)[:, None], sc, 0).astype(np.uint64),
        "minus_one": np.tile(fr_int(P.R_MOD - 1), (n, 1)),
        "high_bits": P.fr_vec_to_np([(1 << 253) + 7 * i for i in range(n)]),
    }
    for name, s in cases.items():
        assert np.array_equal(pp.msm(s).words, oracle.msm(pts, s)), name
    # a batch of independent commits (slots) with different lengths and a degree error
    lens = [n, n + 3, 17, n // 2, 1]
    polys = [random_fr(m, seed=500 + i) for i, m in enumerate(lens)]
    polys[4][:] = 0
    bad = random_fr(n + 20, seed=599)
    devs = [torch.from_numpy(p.view(np.int64)).cuda() for p in polys + [bad]]
    torch.cuda.synchronize()
    res = pp.commit_batch_dev([(d.data_ptr(), d.shape[0]) for d in devs],
                              torch.cuda.current_stream().cuda_stream, raise_on_error=False)
    for i, p in enumerate(polys):
        assert np.array_equal(res[i].words, oracle.msm(pts[: p.shape[0]], p)), i
    assert isinstance(res[-1], plk.PlonkError) and res[-1].status == plk.PLK_E_DEGREE


@pytest.mark.parametrize("c,logn", [(11, 12), (12, 13), (13, 12), (13, 14), (14, 14)])
def test_msm_narrow_balanced_windows_vs_oracle(plk, gpu_ctx, oracle, monkeypatch, c, logn):
    """Narrow bucket sets with balanced windows (c W - 255 top windows one bit narrower,
    digits x 2): the window sizes choose_c now takes at 2^13 / 2^14 points (12, 13) and their
    neighbours, through the one-dispatch sort (<= 8192 scalars) and the k_hist / k_sort_small
    / k_scatter path (more), with skewed scalar sets and a batch with a degree error."""
    import torch
    monkeypatch.setenv("PLK_MSM_C", str(c))
    n = 1 << logn
    tau = random_fr(1, seed=800 + c)[0]
    pp = plk.PlonkParams.setup(logn, tau, gpu_ctx, n_points=n + 8)
    pts = pp.points()
    sc = random_fr(n + 8, seed=810 + logn)
    cases = {
        "random": sc,
        "all_same": np.tile(sc[:1], (n + 8, 1)),
        "sparse": np.where((np.arange(n + 8) % 13 == 0)[:, None], sc, 0).astype(np.uint64),
        "minus_one": np.tile(fr_int(P.R_MOD - 1), (n + 8, 1)),
        "high_bits": P.fr_vec_to_np([(1 << 253) + 5 * i for i in range(n + 8)]),
    }
    for name, s in cases.items():
        assert np.array_equal(pp.msm(s).words, oracle.msm(pts, s)), name
    lens = [n + 3, n // 2, 7]
    polys = [random_fr(m, seed=820 + i) for i, m in enumerate(lens)]
    bad = random_fr(n + 20, seed=829)  # longer than the SRS: PLK_E_DEGREE
    devs = [torch.from_numpy(p.view(np.int64)).cuda() for p in polys + [bad]]
    torch.cuda.synchronize()
    res = pp.commit_batch_dev([(d.data_ptr(), d.shape[0]) for d in devs],
                              torch.cuda.current_stream().cuda_stream, raise_on_error=False)
    for i, p in enumerate(polys):
        assert np.array_equal(res[i].words, oracle.msm(pts[: p.shape[0]], p)), i
    assert isinstance(res[-1], plk.PlonkError) and res[-1].status == plk.PLK_E_DEGREE


@pytest.mark.parametrize("tau", [1, P.R_MOD - 1])
def test_msm_wide_buckets_repeated_points(plk, gpu_ctx, oracle, monkeypatch, tau):
    """Wide bucket sets with tau = +-1 (every SRS point G or -G): equal and opposite points
    meet in the accumulation and the run sums (doubling / infinity branches)."""
    monkeypatch.setenv("PLK_MSM_C", "20")
    n = 1 << 10
    pp = plk.PlonkParams.setup(10, fr_int(tau)[0], gpu_ctx, n_points=n)
    pts = pp.points()
    sc = random_fr(n, seed=79)
    few = np.tile(random_fr(3, seed=80), (n // 3 + 1, 1))[:n].copy()
    for name, s in {"random": sc, "three_values": few, "all_one": np.tile(fr_int(1), (n, 1))}.items():
        assert np.array_equal(pp.msm(s).words, oracle.msm(pts, s)), name


@pytest.mark.parametrize("quad", ["0", "1", "2"])
@pytest.mark.parametrize("c,logn", [(None, 10), (None, 12), (17, 10), (20, 12)])
def test_msm_tail_forms(plk, gpu_ctx, oracle, monkeypatch, quad, c, logn):
    """The forms of the reduction trees (k_bucket_sum / k_bitsum1 / k_bitsum2, msm.hip):
    one lane per addition, the quad-cooperative g1r_add_quad, and quads in k_bitsum2 only
    (PLK_TAIL_QUAD = 0 / 1 / 2),
    on the narrow (default c) and wide (forced c) bucket paths. tau = 1 makes every SRS point
    G, so equal partial sums meet inside the trees (the quad addition's doubling repair) and
    opposite ones cancel (its infinity cases); plus random and sparse scalar sets."""
    monkeypatch.setenv("PLK_TAIL_QUAD", quad)
    if c:
        monkeypatch.setenv("PLK_MSM_C", str(c))
    n = 1 << logn
    for tau in (fr_int(1)[0], random_fr(1, seed=700 + logn)[0]):
        pp = plk.PlonkParams.setup(logn, tau, gpu_ctx, n_points=n)
        pts = pp.points()
        sc = random_fr(n, seed=701 + logn)
        cases = {
            "random": sc,
            "two_values": np.tile(random_fr(2, seed=702), (n // 2, 1)),
            "tiny": P.fr_vec_to_np([i % 3 for i in range(n)]),
            "sparse": np.where((np.arange(n) % 29 == 0)[:, None], sc, 0).astype(np.uint64),
            "plus_minus": P.fr_vec_to_np([(1 if i % 2 else P.R_MOD - 1) for i in range(n)]),
        }
        for name, s in cases.items():
            assert np.array_equal(pp.msm(s).words, oracle.msm(pts, s)), (name, quad)


@pytest.mark.parametrize("c,logn,parts", [(20, 6, 2), (20, 6, 8), (20, 6, 32), (17, 6, 4)])
def test_msm_bucket_parts_vs_pyref(plk, gpu_ctx, golden, monkeypatch, c, logn, parts):
    """plk_commit_batch_dev_part: EVERY part's share equals the restated split
    (oracle/pyref.py msm_bucket_part: same recoding, halving and top-window spread), and the
    shares fold to the golden MSM. c forced on the golden 64-point SRS (wide bucket sets)."""
    import torch
    import pyref as P
    monkeypatch.setenv("PLK_MSM_C", str(c))
    g = golden["msm"]
    pp = plk.PlonkParams.setup(logn, g["tau"], gpu_ctx, n_points=64)
    pts = P.g1_vec_from_np(g["srs"])
    for name in ("random", "minus_one", "high_bits"):
        sc = g[f"{name}_scalars"]
        d = torch.from_numpy(sc.view(np.int64)).cuda()
        torch.cuda.synchronize()
        shares = []
        for q in range(parts):
            got = pp.commit_batch_dev([(d.data_ptr(), sc.shape[0])], part=q, parts=parts)[0]
            if q in (0, 1, parts - 1):  # pyref shares are slow: spot-check three parts
                want = P.g1_vec_to_np([P.msm_bucket_part(pts, P.fr_vec_from_np(sc), c, q, parts)])[0]
                assert np.array_equal(got.words, want), (name, q)
            shares.append(got.words)
        assert np.array_equal(plk.plonk.g1_sum(np.stack(shares)).words, g[f"{name}_result"]), name


def test_msm_bucket_parts_2_20(plk, gpu_ctx):
    """The bench's configs[2] MSM (2^20 points, c = 20) as 8 bucket-range parts: the folded
    shares equal the unsharded commit (itself checked against the oracle in
    test_msm_2_20_vs_oracle); invalid part counts are refused."""
    import torch
    k = 20
    tau = random_fr(1, seed=2020)[0]
    pp = plk.PlonkParams.setup(k, tau, gpu_ctx)
    n = 1 << k
    sc = random_fr(n, seed=4242)
    d = torch.from_numpy(sc.view(np.int64)).cuda()
    torch.cuda.synchronize()
    full = pp.commit_batch_dev([(d.data_ptr(), n)])[0]
    for parts in (2, 8):
        shares = [pp.commit_batch_dev([(d.data_ptr(), n)], part=q, parts=parts)[0].words
                  for q in range(parts)]
        assert np.array_equal(plk.plonk.g1_sum(np.stack(shares)).words, full.words), parts
    for parts in (3, 64):
        with pytest.raises(plk.PlonkError) as e:
            pp.commit_batch_dev([(d.data_ptr(), n)], part=0, parts=parts)
        assert e.value.status == plk.PLK_E_ARG


def test_msm_bucket_parts_degree_error(plk, gpu_ctx, golden, monkeypatch):
    """A polynomial longer than the SRS fails with PLK_E_DEGREE in every part."""
    import torch
    monkeypatch.setenv("PLK_MSM_C", "20")
    g = golden["msm"]
    pp = plk.PlonkParams.setup(6, g["tau"], gpu_ctx, n_points=64)
    bad = np.concatenate([g["random_scalars"], random_fr(9, seed=5)])
    d = torch.from_numpy(bad.view(np.int64)).cuda()
    torch.cuda.synchronize()
    for q in range(4):
        r = pp.commit_batch_dev([(d.data_ptr(), bad.shape[0])], raise_on_error=False, part=q, parts=4)
        assert isinstance(r[0], plk.PlonkError) and r[0].status == plk.PLK_E_DEGREE
