"""The primitive entry points added at the §8b boundary in round 4:
* plk_aggregate_witness[_dev] — PlonkParams::compute_aggregate_witness
  (/root/reference/src/prover.rs:422-438 at z, :444-450 at z·ω): (Σ vⁱ pᵢ) ÷ (X − z),
  checked against the pure-Python restatement (oracle/pyref.py aggregate_witness, the
  classical top-down synthetic division — a different algorithm from the GPU's scaled
  suffix scan);
* plk_ntt_stream — host plk_ntt on the caller's stream (§8b signature), several threads
  with their own streams sharing ONE Fft, against the C oracle."""
import concurrent.futures as cf

import numpy as np
import pytest

from oracle_lib import random_fr

pytestmark = pytest.mark.gpu


def _ints(a):
    import pyref as P
    return P.fr_vec_from_np(a)


def _np(vals):
    import pyref as P
    return P.fr_vec_to_np(vals)


def _want(polys, z, v):
    import pyref as P
    q = P.aggregate_witness([_ints(p) for p in polys], _ints(z)[0], _ints(v)[0])
    return _np(q) if q else np.zeros((0, 4), dtype=np.uint64)


@pytest.mark.parametrize("lens", [(256, 258, 259, 256, 256, 256, 256, 256, 256),  # the 9 at z
                                  (259, 258, 258, 258),                            # the 4 at zw
                                  (1000,), (3, 1, 0, 17), (2,)])
def test_aggregate_witness_host_vs_oracle(plk, gpu_ctx, lens):
    pp = plk.PlonkParams.setup(4, random_fr(1, seed=1)[0], gpu_ctx)
    polys = [random_fr(m, seed=10 + i) for i, m in enumerate(lens)]
    z, v = random_fr(1, seed=98), random_fr(1, seed=99)
    got = pp.compute_aggregate_witness(polys, z, v).values
    assert np.array_equal(got, _want(polys, z, v))


def test_aggregate_witness_many_terms_and_edge_points(plk, gpu_ctx):
    """More polynomials than one linear-combination pass holds (kMaxTerms = 24), the point
    zero (division by X), v = 0 (only p_0), constant inputs (empty result) and the argument
    checks (non-canonical point)."""
    pp = plk.PlonkParams.setup(4, random_fr(1, seed=1)[0], gpu_ctx)
    polys = [random_fr(64 + 3 * i, seed=200 + i) for i in range(50)]
    z, v = random_fr(1, seed=5), random_fr(1, seed=6)
    assert np.array_equal(pp.compute_aggregate_witness(polys, z, v).values, _want(polys, z, v))
    zero = np.zeros((1, 4), dtype=np.uint64)
    assert np.array_equal(pp.compute_aggregate_witness(polys[:5], zero, v).values,
                          _want(polys[:5], zero, v))
    assert np.array_equal(pp.compute_aggregate_witness(polys[:5], z, zero).values,
                          _want(polys[:5], z, zero))
    assert len(pp.compute_aggregate_witness([random_fr(1, seed=7)], z, v)) == 0
    assert len(pp.compute_aggregate_witness([], z, v)) == 0
    import pyref as P
    bad = np.array([P.int_to_limbs(P.R_MOD, 4)], dtype=np.uint64)  # r itself: not canonical
    with pytest.raises(plk.PlonkError) as e:
        pp.compute_aggregate_witness(polys[:2], bad, v)
    assert e.value.status == plk.PLK_E_ARG


def test_aggregate_witness_dev_2_14(plk, gpu_ctx):
    """The device entry on torch tensors at n = 2^14 with the prover's shapes (9 polys at z,
    lengths n..n+3), on a torch stream, against the oracle."""
    import torch
    n = 1 << 14
    lens = [n, n + 3, n + 2, n + 2, n + 2, n + 2, n, n, n]
    polys = [random_fr(m, seed=300 + i) for i, m in enumerate(lens)]
    z, v = random_fr(1, seed=7), random_fr(1, seed=8)
    dev = [torch.from_numpy(p.view(np.int64)).cuda() for p in polys]
    out = torch.zeros((n + 2, 4), dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        pp = plk.PlonkParams.setup(4, random_fr(1, seed=1)[0], gpu_ctx)
        m = pp.compute_aggregate_witness_dev([(t.data_ptr(), t.shape[0]) for t in dev], z, v,
                                             out.data_ptr(), st.cuda_stream)
    st.synchronize()
    assert m == n + 2
    assert np.array_equal(out.cpu().numpy().view(np.uint64)[:m], _want(polys, z, v))


def test_ntt_stream_threads_share_one_fft(plk, gpu_ctx, oracle):
    """plk_ntt_stream: 4 host threads, each with its own torch stream, run dft / idft /
    coset_dft / coset_idft on ONE shared Fft concurrently (no shared staging buffer); every
    result equals the C oracle's."""
    import torch
    k = 14
    f = plk.Fft(k, gpu_ctx)
    streams = [torch.cuda.Stream() for _ in range(4)]
    xs = [random_fr(1 << k, seed=400 + i) for i in range(8)]
    ops = [("dft", oracle.dft), ("idft", oracle.idft), ("coset_dft", oracle.coset_dft),
           ("coset_idft", oracle.coset_idft)]

    def run(t):
        out = []
        for j in range(t, len(xs), 4):
            name, _ = ops[j % 4]
            cls = plk.Coefficients if "idft" not in name else plk.PointsValue
            out.append((j, getattr(f, name)(cls(xs[j]), stream=streams[t].cuda_stream).values))
        return out

    with cf.ThreadPoolExecutor(4) as ex:
        res = [r for rs in ex.map(run, range(4)) for r in rs]
    assert len(res) == len(xs)
    for j, got in res:
        assert np.array_equal(got, ops[j % 4][1](xs[j], k)), ops[j % 4][0]
    # a short input zero-pads on the stream path too
    short = xs[0][:100]
    assert np.array_equal(f.dft(plk.Coefficients(short), stream=streams[0].cuda_stream).values,
                          oracle.dft(np.vstack([short, np.zeros(((1 << k) - 100, 4), np.uint64)]), k))
