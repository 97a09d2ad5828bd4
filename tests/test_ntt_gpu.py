"""GPU parity of the NTT family (poly_commit::Fft) through the C ABI.

Bit-exact against the golden fixtures (Python big-int restatement) and the C oracle at
every size up to 2^16 for all four transforms; size-independent properties (round trips,
linearity, evaluation at a point) at 2^20 and 2^23 (the 8n domain of n = 2^20).
"""
import numpy as np
import pytest

from oracle_lib import random_fr

pytestmark = pytest.mark.gpu


def test_golden_vectors(plk, gpu_ctx, golden):
    g = golden["ntt"]
    for k in (0, 1, 2, 3, 4, 5, 6, 8, 10):
        f = plk.Fft(k, gpu_ctx)
        x = plk.Coefficients(g[f"k{k}_in"])
        assert np.array_equal(f.dft(x).values, g[f"k{k}_dft"]), k
        assert np.array_equal(f.idft(plk.PointsValue(x.values)).values, g[f"k{k}_idft"]), k
        assert np.array_equal(f.coset_dft(x).values, g[f"k{k}_coset_dft"]), k
        assert np.array_equal(f.coset_idft(plk.PointsValue(x.values)).values,
                              g[f"k{k}_coset_idft"]), k
        part = plk.Coefficients(g[f"k{k}_part"])
        assert np.array_equal(f.dft(part).values, g[f"k{k}_part_dft"]), k
        assert np.array_equal(f.coset_dft(part).values, g[f"k{k}_part_coset_dft"]), k
        assert np.array_equal(f.elements, g[f"k{k}_elements"]), k
    f5 = plk.Fft(5, gpu_ctx)
    assert np.array_equal(f5.compute_vanishing_poly_over_coset(4).values, g["vanish_k5_n4"])


@pytest.mark.parametrize("k", list(range(0, 17)))
def test_all_transforms_vs_oracle(plk, gpu_ctx, oracle, k):
    n = 1 << k
    f = plk.Fft(k, gpu_ctx)
    x = random_fr(n, seed=100 + k)
    for direction, coset, name in ((1, 0, "dft"), (-1, 0, "idft"), (1, 1, "coset_dft"),
                                   (-1, 1, "coset_idft")):
        want = oracle.ntt(x, k, direction, bool(coset))
        got = getattr(f, name)(plk.Coefficients(x)).values
        assert np.array_equal(got, want), (k, name)
    # ragged input, zero padded (len n+2 polys go into 8n domains in the prover)
    m = max(1, (3 * n) // 4 + 1) if n > 1 else 1
    assert np.array_equal(f.dft(plk.Coefficients(x[:m])).values, oracle.dft(x[:m], k))
    assert np.array_equal(f.coset_dft(plk.Coefficients(x[:m])).values, oracle.coset_dft(x[:m], k))


@pytest.mark.parametrize("k", [12, 17, 20])
def test_idft_multipass_identity_rows(plk, gpu_ctx, oracle, k):
    """A multi-pass plain idft carries n^-1 on its last pass' inter-pass twiddles
    (pass_tw_inv_last, round 5), so the j = 0 / k = 0 entries of that table are n^-1, not one
    (ntt.hip: the multiply must stay unconditional). idft(all ones) = (1, 0, ..., 0) puts all
    of the result on row 0; a skipped identity entry would leave n there."""
    import pyref as P
    n = 1 << k
    f = plk.Fft(k, gpu_ctx)
    delta = np.zeros((n, 4), dtype=np.uint64)
    delta[0] = P.fr_vec_to_np([1])[0]
    ones = oracle.dft(delta, k)
    assert np.array_equal(ones, np.repeat(delta[:1], n, axis=0))
    assert np.array_equal(f.idft(plk.PointsValue(ones)).values, delta)
    x = random_fr(n, seed=7 + k)
    assert np.array_equal(f.idft(plk.PointsValue(x)).values, oracle.idft(x, k))


def test_empty_and_zero_inputs(plk, gpu_ctx):
    f = plk.Fft(6, gpu_ctx)
    z = np.zeros((0, 4), dtype=np.uint64)
    for fn in (f.dft, f.idft, f.coset_dft, f.coset_idft):
        assert not fn(plk.Coefficients(z)).values.any()
    with pytest.raises(ValueError):
        f.dft(plk.Coefficients(random_fr(65, seed=1)))


def test_domain_accessors(plk, gpu_ctx, oracle):
    import pyref as P
    for k in (1, 9, 12, 16, 20):
        f = plk.Fft(k, gpu_ctx)
        assert f.size() == 1 << k
        assert P.fr_vec_from_np(f.generator())[0] == P.omega(k)
        assert P.fr_vec_from_np(f.generator_inv())[0] == pow(P.omega(k), -1, P.R_MOD)
        assert P.fr_vec_from_np(f.size_inv())[0] == pow(1 << k, -1, P.R_MOD)
        if k <= 16:
            assert np.array_equal(f.elements, oracle.elements(k))
    f = plk.Fft(15, gpu_ctx)
    assert np.array_equal(f.compute_vanishing_poly_over_coset(1 << 12).values,
                          oracle.vanishing(15, 1 << 12))


def test_sigma_encoding_on_gpu_elements(plk, gpu_ctx):
    """permutation.rs:913-946: encodings use fft.elements = w^i of the GPU domain."""
    import pyref as P
    f = plk.Fft(2, gpu_ctx)
    el = P.fr_vec_from_np(f.elements)
    w = P.fr_vec_from_np(f.generator())[0]
    assert el == [1, w, w * w % P.R_MOD, pow(w, 3, P.R_MOD)]


@pytest.mark.slow
# every plan shape past 2^16: 2^17 / 2^18 two passes (9 + 8, 9 + 9), 2^19 7 + 6 + 6, 2^20
# 7 + 7 + 6, 2^21 7 + 7 + 7 (an odd radix in every pass: the radix-2 stage on the loaded
# registers in each), 2^22 8 + 7 + 7, 2^23 8 + 8 + 7
@pytest.mark.parametrize("k", [17, 18, 19, 20, 21, 22, 23])
def test_large_properties(plk, gpu_ctx, oracle, k):
    import pyref as P
    n = 1 << k
    f = plk.Fft(k, gpu_ctx)
    x = random_fr(n, seed=7 + k)
    y = random_fr(n, seed=8 + k)
    X = f.dft(plk.Coefficients(x)).values
    # round trips
    assert np.array_equal(f.idft(plk.PointsValue(X)).values, x)
    CX = f.coset_dft(plk.Coefficients(x)).values
    assert np.array_equal(f.coset_idft(plk.PointsValue(CX)).values, x)
    # linearity: dft(x + y) == dft(x) + dft(y)  (checked at sampled indices)
    xs = P.fr_vec_from_np(x[:64])
    ys = P.fr_vec_from_np(y[:64])
    s = P.fr_vec_to_np([(a + b) % P.R_MOD for a, b in zip(xs, ys)] + [0] * 0)
    xy = x.copy()
    xy[:64] = s
    xy[64:] = 0
    xo = x.copy()
    xo[64:] = 0
    yo = y.copy()
    yo[:] = 0
    yo[:64] = y[:64]
    D1 = f.dft(plk.Coefficients(xy)).values
    D2 = f.dft(plk.Coefficients(xo)).values
    D3 = f.dft(plk.Coefficients(yo)).values
    idx = np.random.default_rng(k).integers(0, n, 32)
    for i in idx:
        a, b, c = (P.fr_vec_from_np(D[i:i + 1])[0] for D in (D1, D2, D3))
        assert a == (b + c) % P.R_MOD
    # evaluation: X[i] = x(w^i), CX[i] = x(g w^i) at sampled i (full Horner in Python on a
    # short prefix polynomial)
    w = P.omega(k)
    pre = P.fr_vec_from_np(x[:64])
    xs_short = x.copy()
    xs_short[64:] = 0
    Xs = f.dft(plk.Coefficients(xs_short)).values
    CXs = f.coset_dft(plk.Coefficients(xs_short)).values
    for i in idx[:8]:
        pt = pow(w, int(i), P.R_MOD)
        assert P.fr_vec_from_np(Xs[i:i + 1])[0] == P.poly_eval(pre, pt)
        assert P.fr_vec_from_np(CXs[i:i + 1])[0] == P.poly_eval(pre, 7 * pt % P.R_MOD)
    if k <= 20:  # the C oracle finishes 2^20 in about a second
        assert np.array_equal(X, oracle.dft(x, k))
        assert np.array_equal(CX, oracle.coset_dft(x, k))


def test_device_entry_points(plk, gpu_ctx, oracle):
    import torch
    k = 14
    n = 1 << k
    f = plk.Fft(k, gpu_ctx)
    x = random_fr(n, seed=3)
    d = torch.from_numpy(x.view(np.int64)).cuda()
    out = torch.empty_like(d)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream().cuda_stream
    f.ntt_dev(d.data_ptr(), out.data_ptr(), n, 1, True, stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), oracle.coset_dft(x, k))
    # in place, inverse, with a caller-owned scratch buffer
    scratch = torch.empty((2 * n, 4), dtype=torch.int64, device="cuda")
    f.ntt_dev(out.data_ptr(), out.data_ptr(), n, -1, True, stream, scratch.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), x)


@pytest.mark.parametrize("k", [5, 12, 20])
def test_device_null_input(plk, gpu_ctx, k):
    """plk_ntt_dev with len_in = 0 and no input buffer (a zero polynomial): every transform
    writes n zeros. The pass kernel's loads are unconditional, so the host points them at a
    live table (ntt.hip `no_input`); single- and multi-pass plans."""
    import torch
    n = 1 << k
    f = plk.Fft(k, gpu_ctx)
    out = torch.full((n, 4), -1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for direction, coset in ((1, False), (1, True), (-1, False), (-1, True)):
        out.fill_(-1)
        f.ntt_dev(0, out.data_ptr(), 0, direction, coset, stream)
        torch.cuda.synchronize()
        assert not out.cpu().numpy().any(), (k, direction, coset)


@pytest.mark.parametrize("k", [6, 12, 16, 20])
def test_zero_padded_first_pass(plk, gpu_ctx, oracle, k):
    """Inputs of at most n/8 + n/R coefficients take the closed-form first stages of the
    first pass (ntt.hip PRUNE): lengths around both edges of that range, vs the C oracle."""
    n = 1 << k
    f = plk.Fft(k, gpu_ctx)
    x = random_fr(n, seed=300 + k)
    lens = {0, 1, 2, n // 8 - 1, n // 8, n // 8 + 1, n // 8 + 3, n // 8 + n // 64,
            n // 8 + n // 64 + 1, n // 8 + n // 128, n // 8 + n // 256, n // 8 + n // 256 + 1}
    if k == 20:
        lens = {n // 8, n // 8 + 3, n // 8 + n // 128, n // 8 + n // 128 + 1}
    for m in sorted(v for v in lens if 0 <= v <= n):
        xm = x[:m]
        assert np.array_equal(f.dft(plk.Coefficients(xm)).values, oracle.dft(xm, k)), (k, m)
        assert np.array_equal(f.coset_dft(plk.Coefficients(xm)).values,
                              oracle.coset_dft(xm, k)), (k, m)


_OPT_IN_SCRIPT = r"""
import sys
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/tests"]
import dusk_plonk_amd as plk
from oracle_lib import random_fr
ctx = plk.Context.default(0)
out = {}
for k in (16, 18, 20):
    f = plk.Fft(k, ctx)
    x = random_fr(1 << k, seed=900 + k)
    out[f"x{k}"] = x
    out[f"dft{k}"] = f.dft(plk.Coefficients(x)).values
    out[f"idft{k}"] = f.idft(plk.PointsValue(x)).values
    out[f"cdft{k}"] = f.coset_dft(plk.Coefficients(x[: (3 << k) // 4])).values
    out[f"cidft{k}"] = f.coset_idft(plk.PointsValue(x)).values
np.savez(sys.argv[2], **out)
"""


def test_opt_in_plans_vs_oracle(tmp_path, oracle):
    """The opt-in NTT plan (a process-wide environment switch, so in a child process): radix
    up to 2^10 (PLK_NTT_MAX_LR: 2^18 / 2^20 in two passes, 1-column tiles, > 64 KiB of LDS
    for the pruned first pass) — bit-exact against the oracle like the default plans."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    f = tmp_path / "out.npz"
    env = dict(os.environ, PLK_NTT_MAX_LR="10")
    subprocess.run([sys.executable, "-c", _OPT_IN_SCRIPT, str(root), str(f)], env=env, check=True,
                   timeout=240)
    d = np.load(f)
    for k in (16, 18, 20):
        x = d[f"x{k}"]
        assert np.array_equal(d[f"dft{k}"], oracle.ntt(x, k, 1, False)), k
        assert np.array_equal(d[f"idft{k}"], oracle.ntt(x, k, -1, False)), k
        assert np.array_equal(d[f"cdft{k}"], oracle.coset_dft(x[: (3 << k) // 4], k)), k
        assert np.array_equal(d[f"cidft{k}"], oracle.ntt(x, k, -1, True)), k
